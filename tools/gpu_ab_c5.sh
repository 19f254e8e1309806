# Same-box A/B of prebuilt libraries on C5 only (tools/gpu_ab_lib.sh's rounds, C5 bench, 1 step + 1 warm-up).
# usage: LIBS="base:ab/lib_x.so" ROUNDS=2 [TRACE=1] [WORKLOAD=c2|c3] bash tools/gpu_ab_c5.sh TAG
# TRACE=1: one more round per library under rocprofv3 --kernel-trace --stats (per-kernel times, $D/kt_<name>_kernel_stats.csv)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-abc5}; mkdir -p $D
CUR=ptsharp_amd/libptsharp_hip.so
cp $CUR $D/.cur.so || exit 1
W=${WORKLOAD:-c5}
case $W in c2) A="--workload c2 --steps 8 --warmup 1";; c3) A="--workload c3 --steps 16 --warmup 2";; *) A="--workload c5 --steps 1 --warmup 1";; esac
restore() { cp $D/.cur.so $CUR; rm -f $D/.cur.so; }
IFS=' ' read -ra LS <<< "cur:$D/.cur.so ${LIBS:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in "${LS[@]}"; do
    N=${L%%:*}; P=${L#*:}
    cp $P $CUR || { restore; exit 1; }
    timeout -k 10 400 python -u bench.py $A --cpu-seconds 0 --no-parity --json-out $D/c5_${N}_$r.json > $D/c5_${N}_$r.log 2>&1 || { restore; exit 1; }
    echo "$N round $r: $(python -c "import json;j=json.load(open('$D/c5_${N}_$r.json'));print(j['value'],j['config']['kernel_ms_per_step'],j['roofline'].get('volume_march_clock',{}).get('share'))")" >> $D/summary.txt
  done
done
if [ "${TRACE:-0}" = 1 ]; then
  for L in "${LS[@]}"; do
    N=${L%%:*}; P=${L#*:}
    cp $P $CUR || { restore; exit 1; }
    timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_$N -o kt -- python3 bench.py $A --cpu-seconds 0 --no-parity --json-out $D/c5_${N}_trace.json > $D/c5_${N}_trace.log 2>&1 || { restore; exit 1; }
    find $D/kt_$N -name '*kernel_stats.csv' -exec cp {} $D/kt_${N}_kernel_stats.csv \;
  done
fi
restore
exit 0
