# (1) the dependent-gather microbenchmark's chase mode: K of a 128-B record's eight 16-B pieces per step, 6 waves
#     per SIMD: does a divergent step's time follow its load instructions (a 64-B node would halve a node step's)?
# (2) the instanced-mesh scene: the BLAS private stack sized by the BVH4 budget (current) vs kStackMax (ab/lib_stack64.so),
#     one stream, alternated.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06g; mkdir -p $D
timeout -k 10 120 ./tools/microbench_gather chase > $D/microbench_chase.txt 2>&1 || exit 1
cp ptsharp_amd/libptsharp_hip.so $D/.cur.so || exit 1
for r in 1 2; do
  for L in cur stack64; do
    if [ $L = stack64 ]; then cp ab/lib_stack64.so ptsharp_amd/libptsharp_hip.so; else cp $D/.cur.so ptsharp_amd/libptsharp_hip.so; fi
    PT_SIDE_STREAM=0 timeout -k 10 200 python -u tools/bench_scenes.py instances > $D/${L}_$r.jsonl 2> $D/${L}_$r.log || { cp $D/.cur.so ptsharp_amd/libptsharp_hip.so; exit 1; }
  done
done
cp $D/.cur.so ptsharp_amd/libptsharp_hip.so; rm -f $D/.cur.so
