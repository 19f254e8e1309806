# Shadow rays' last-blocker test (ab/lib_lastb.so, -DPT_LAST_BLOCKER=1) against the current build, same box; its
# parity leg (the bench's own 16-spp oracle sample); then VERDICT r05 #7b's instanced-scene comparison (gpu_r06e).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06f; mkdir -p $D
LIBS="lastb:ab/lib_lastb.so" ROUNDS=2 bash tools/gpu_ab_lib.sh r06f/ab || exit 1
cp ptsharp_amd/libptsharp_hip.so $D/.cur.so && cp ab/lib_lastb.so ptsharp_amd/libptsharp_hip.so &&
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --cpu-seconds 5 --json-out $D/lastb_parity.json > $D/lastb_parity.log 2>&1; rc=$?
cp $D/.cur.so ptsharp_amd/libptsharp_hip.so; rm -f $D/.cur.so
[ $rc = 0 ] || exit $rc
bash tools/gpu_r06e.sh
