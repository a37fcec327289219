#!/bin/bash
# Memory-side PMC passes (each set in a run of its own, --pmc only): DRAM read requests and
# credit stalls, L2 tag stalls and hits, L1->L2 read latency and pending stalls.
# Outputs gpurun_out/pmc_<set>_<cfg>_$TAG/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CFGS:-c1 c2 c3_reasm}; do
  run() { timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/pmc_${SET}_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_${SET}_${c}_$TAG.log 2>&1; }
  SET=tcca run TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum GRBM_GUI_ACTIVE
  SET=tccb run TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE
  SET=tcp run TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE
  echo "pmc $c ok"
done
