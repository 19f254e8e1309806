set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_parity.py example3 64 48 4 "0,0 32,0 0,64 32,64" > gpurun_out/g3_dbg.log 2>&1
timeout -k 10 300 python -u tools/debug_parity.py gopher3 64 48 1 "0,0 0,4 3,0" >> gpurun_out/g3_dbg.log 2>&1
bash tools/gpu_quick.sh g3
