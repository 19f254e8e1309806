# Same-box A/B of prebuilt libraries on tools/bench_scenes.py scenes (one row per scene per library per round).
# usage: LIBS="base:ab/lib_x.so" ROUNDS=2 SCENES="volume transformed" bash tools/gpu_ab_scenes.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-abscenes}; mkdir -p $D
CUR=ptsharp_amd/libptsharp_hip.so
cp $CUR $D/.cur.so || exit 1
restore() { cp $D/.cur.so $CUR; rm -f $D/.cur.so; }
IFS=' ' read -ra LS <<< "cur:$D/.cur.so ${LIBS:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in "${LS[@]}"; do
    N=${L%%:*}; P=${L#*:}
    cp $P $CUR || { restore; exit 1; }
    timeout -k 10 300 python -u tools/bench_scenes.py ${SCENES:-volume} > $D/${N}_$r.jsonl 2> $D/${N}_$r.log || { restore; exit 1; }
    python -c "
import json,sys
for l in open('$D/${N}_$r.jsonl'):
    j=json.loads(l); print('$N round $r', j['scene'], j['Mrays_per_s'], j['ms_per_pass'])" >> $D/summary.txt
  done
done
restore
exit 0
