# Counters of compile-time variants (the C4 bench configuration, 16 spp, 2 timed steps): per variant,
# rocprofv3 --pmc passes p4 (residency, VALU), p5 (TA / TCP), p6 (L2 hit, fabric latency), FETCH_SIZE,
# WRITE_SIZE, each its own run, kernel trace only; tools/residency.py and tools/traffic_ab.py summarise.
# usage: gpurun -- 'VARIANTS="a:|b:-DFLAG=1" bash tools/gpu_counters_ab.sh TAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-cab}
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
CTR="--steps 2 --warmup 1 --spp 16 --cpu-seconds 0 --no-parity"
for V in "${VS[@]}"; do
  NAME=${V%%:*}; FLAGS=${V#*:}
  D=gpurun_out/${T}_$NAME; mkdir -p $D
  make -s -C ptsharp_amd/csrc clean >/dev/null && make -s -j16 -C ptsharp_amd/csrc EXTRA="$FLAGS" > $D/build.log 2>&1 || exit 1
  pmc() { P=$1; shift; timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d $D/$P -o p --output-format csv -- python3 bench.py $CTR --json-out $D/bench_$P.json > $D/$P.log 2>&1; }
  pmc p4 SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU && \
  pmc p5 TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_TA_BUSY_sum TCP_PERF_SEL_TOTAL_HIT_LRU_READ_sum TCP_PERF_SEL_TOTAL_MISS_LRU_READ_sum && \
  pmc p6 TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum && \
  pmc fetch FETCH_SIZE && pmc write WRITE_SIZE || exit 1
  python tools/residency.py $D $NAME > $D/residency.txt 2>&1 || exit 1
  python tools/traffic_ab.py $D > $D/traffic.txt 2>&1 || exit 1
done
