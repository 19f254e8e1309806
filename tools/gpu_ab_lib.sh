# Same-box A/B of prebuilt libraries (built on the CPU host, in-tree): the current build against others,
# each C4 bench run alternated (ABAB...), optionally C5 once per library.  The current build is restored.
# usage: LIBS="bvh4:ab/lib_bvh4.so" ROUNDS=2 BARGS="--width 2048 --height 1024" C5="cur bvh4" bash tools/gpu_ab_lib.sh TAG   (C5=all: every library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-ablib}; mkdir -p $D
CUR=ptsharp_amd/libptsharp_hip.so
cp $CUR $D/.cur.so || exit 1
restore() { cp $D/.cur.so $CUR; rm -f $D/.cur.so; }
IFS=' ' read -ra LS <<< "cur:$D/.cur.so ${LIBS:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in "${LS[@]}"; do
    N=${L%%:*}; P=${L#*:}
    cp $P $CUR || { restore; exit 1; }
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-16} --warmup 2 --cpu-seconds 0 --no-parity ${BARGS:-} --json-out $D/c4_${N}_$r.json > $D/c4_${N}_$r.log 2>&1 || { restore; exit 1; }
    echo "$N round $r: $(python -c "import json;j=json.load(open('$D/c4_${N}_$r.json'));print(j['value'],j['config']['kernel_ms_per_step'])")" >> $D/summary.txt
  done
done
if [ -n "$C5" ]; then   # C5="all" or a list of the names to run C5 on
  for L in "${LS[@]}"; do
    N=${L%%:*}; P=${L#*:}
    [ "$C5" != all ] && [[ " $C5 " != *" $N "* ]] && continue
    cp $P $CUR || { restore; exit 1; }
    timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --json-out $D/c5_$N.json > $D/c5_$N.log 2>&1 || { restore; exit 1; }
    echo "$N c5: $(python -c "import json;j=json.load(open('$D/c5_$N.json'));print(j['value'],j['config']['kernel_ms_per_step'])")" >> $D/summary.txt
  done
fi
restore
exit 0
