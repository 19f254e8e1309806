set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06a; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "tail_handoffs or 16spp_one_full_chunk" --timeout 300 --timeout-method thread > $D/new_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $D/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --json-out $D/bench_default.json > $D/bench_default.log 2>&1 &&
timeout -k 10 400 python -u bench.py --group --steps 16 --warmup 2 --cpu-seconds 0 --no-parity --json-out $D/bench_group1.json > $D/bench_group1.log 2>&1 &&
LIBS="noshift:ab/lib_noshift.so" ROUNDS=2 BARGS="--width 2048 --height 1024" bash tools/gpu_ab_lib.sh r06a/ab_shift &&
for L in cur r05 cur r05; do
  if [ $L = r05 ]; then cp ptsharp_amd/libptsharp_hip.so $D/cur.so && cp ab/lib_r05.so ptsharp_amd/libptsharp_hip.so; fi
  timeout -k 10 300 python -u bench.py --engine mega --spp 1 --steps 3 --warmup 1 --width 960 --height 540 --cpu-seconds 0 --no-parity --json-out $D/mega_$L.json > $D/mega_$L.log 2>&1; rc=$?
  if [ $L = r05 ]; then cp $D/cur.so ptsharp_amd/libptsharp_hip.so; fi
  [ $rc = 0 ] || exit $rc
  echo "$L $(python -c "import json;j=json.load(open('$D/mega_$L.json'));print(j['value'],j['config']['kernel_ms_per_step'])")" >> $D/mega.txt
done
