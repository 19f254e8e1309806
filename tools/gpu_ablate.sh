# timing-only ablation builds of the wavefront kernels (results are NOT valid renders)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablate
for V in base ACC RESERVE; do
  if [ "$V" = base ]; then X=""; else X="-DPT_ABLATE_$V"; fi
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$X" > gpurun_out/ablate/build_$V.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity --json-out gpurun_out/ablate/$V.json > gpurun_out/ablate/$V.log 2>&1 || exit 1
done
