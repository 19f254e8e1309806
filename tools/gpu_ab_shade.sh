set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for W in 2 4; do
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="-DPT_SHADE_WAVES=$W" > gpurun_out/build_$W.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --spp 4 --cpu-seconds 0 --no-parity --engine wave --json-out gpurun_out/shade_w$W.json > gpurun_out/shade_w$W.log 2>&1 || exit 1
done
