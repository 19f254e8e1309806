# run-to-run variance of the quick bench on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-seconds 0 --no-parity --json-out gpurun_out/var/run$i.json > gpurun_out/var/run$i.log 2>&1 || exit 1
done
