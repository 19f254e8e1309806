# A/B of compile-time variants on one box.  Per variant: rebuild, a parity subset (PARITY tests, the
# refill-kernel and C4-tile checks by default), then the C4 bench (STEPS steps), and optionally the C2
# bench (C2=1), the 1/8 share (SHARD=1) and the C5 bench (C5=1); NOBENCH=1 skips the C4 bench.  Stops at the
# first failure.
# usage: VARIANTS="base:|coop:-DPT_COOP=2" bash tools/gpu_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-ab}; mkdir -p $D
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
PARITY=${PARITY:-tests/test_00_gpu_baseline.py::test_c4_mesh1m_tiles tests/test_gpu_parity.py::test_refill_kernels_match_lockstep tests/test_gpu_parity.py::test_side_stream_deep_bvh_spill}
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  echo "== $NAME ($FLAGS)" >> $D/progress.log
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > $D/build_$NAME.log 2>&1 || exit 1
  if [ "$PARITY" != "none" ]; then
    timeout -k 10 600 python -u -m pytest $PARITY -x -q -m gpu --timeout 240 --timeout-method thread > $D/tests_$NAME.log 2>&1 || exit 1
  fi
  [ -z "$NOBENCH" ] && { timeout -k 10 300 python -u bench.py --steps ${STEPS:-16} --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/c4_$NAME.json > $D/c4_$NAME.log 2>&1 || exit 1; }
  [ -n "$C2" ] && { timeout -k 10 300 python -u bench.py --workload c2 --steps 6 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c2_$NAME.json > $D/c2_$NAME.log 2>&1 || exit 1; }
  [ -n "$SHARD" ] && { timeout -k 10 300 python -u bench.py --shard 0/8 --steps 32 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/shard8_$NAME.json > $D/shard8_$NAME.log 2>&1 || exit 1; }
  [ -n "$C5" ] && { timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c5_$NAME.json > $D/c5_$NAME.log 2>&1 || exit 1; }
done
make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc > $D/build_final.log 2>&1
exit 0
