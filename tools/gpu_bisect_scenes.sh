mkdir -p gpurun_out/r05bis
for r in 1 2; do
for c in r04 04a8eb0 5a6106b 2702210; do
  (cd ab/$c && timeout -k 10 200 python -u tools/bench_scenes.py instances transformed > ../../gpurun_out/r05bis/${c}_$r.jsonl 2> ../../gpurun_out/r05bis/${c}_$r.log) || exit 1
done
timeout -k 10 200 python -u tools/bench_scenes.py instances transformed > gpurun_out/r05bis/cur_$r.jsonl 2> gpurun_out/r05bis/cur_$r.log || exit 1
done
