# A/B of compile-time variants on the C4 bench and two tools/bench_scenes.py scenes (parity tests on the first).
# usage: VARIANTS="a:-DX|b:" bash tools/gpu_ab_c4_scenes.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS=${STEPS:-6} bash tools/gpu_ab.sh || exit 1
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > /dev/null 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_scenes.py ${SCENES:-gopher3 bunny70k} > gpurun_out/ab/scenes_$NAME.log 2>&1 || exit 1
done
