# Where C5's time goes: standalone per-kernel times (PT_SIDE_STREAM=0) of timing-probe builds
# (PT_PROBE_NO_VOL / PT_PROBE_NO_SDF: those shapes never hit — wrong images, timing only).
# usage: VARIANTS="base:|novol:-DPT_PROBE_NO_VOL|nosdf:-DPT_PROBE_NO_SDF" bash tools/gpu_probe_c5.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-probec5}; mkdir -p $D
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > $D/build_$NAME.log 2>&1 || exit 1
  PT_SIDE_STREAM=0 timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --json-out $D/c5_$NAME.json > $D/c5_$NAME.log 2>&1 || exit 1
  echo "$NAME: $(python -c "import json;d=json.load(open('$D/c5_$NAME.json'));print(d['value'], d['ms_per_step'], d['config']['kernel_ms_per_step'])")"
done
