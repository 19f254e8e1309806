# A/B of compile-time variants on tools/bench_scenes.py's scenes (the FULL kernels: textures,
# SDF, volume, transformed shapes).  usage: VARIANTS="base:|x:-DFOO" SCENES="sdf_zoo volume" bash tools/gpu_ab_scenes.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > gpurun_out/ab/build_$NAME.log 2>&1 || exit 1
  timeout -k 10 600 python -m pytest tests/test_gpu_shapes_ext.py tests/test_gpu_textures.py -x -q -m gpu > gpurun_out/ab/tests_$NAME.log 2>&1 || exit 1
  timeout -k 10 400 python tools/bench_scenes.py ${SCENES:-textured sdf_zoo volume transformed} > gpurun_out/ab/scenes_$NAME.log 2>&1 || exit 1
done
