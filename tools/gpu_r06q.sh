# k_wf_trace_lanes refill: the two queue loads pinned together (pin) and the next refill's claim sent ahead
# (pinclaim = in-tree): parity subset, same-box C4 A/B against HEAD; then where the C4 and C2 kernels' wave time
# goes (SQ wave-state counters, one --pmc pass each, kernel trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06q; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_mesh1m or refill or lockstep or textures or tiles or bvh" > $D/tests.log 2>&1 || exit 1
LIBS="pin:ab/lib_pin.so base:ab/lib_base.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06q/c4 || exit 1
W="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $W --kernel-trace -d $D/c4w -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c4w.json > $D/c4w.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc $W --kernel-trace -d $D/c2w -o p --output-format csv -- python3 bench.py --workload c2 --spp 16 --steps 1 --warmup 0 --cpu-seconds 0 --no-parity --json-out $D/c2w.json > $D/c2w.log 2>&1 || exit 1
