#!/bin/bash
# PMC passes of one round (each counter set in a run of its own, --pmc only): FETCH_SIZE and
# WRITE_SIZE per config (the `traffic` figure), and two SQ passes on C2 (VALU / wait / issue).
# Outputs gpurun_out/pmc_{fetch,write}_<cfg>_$TAG/ and gpurun_out/pmc_sq{a,b}_c2_$TAG/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CFGS:-c1 c2 c2slot c2tx c2tx_nw c2nat c2v6 c2eth c2ethmix c3_reasm c3_reasm6}; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_fetch_${c}_$TAG.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_write_${c}_$TAG.log 2>&1
  echo "pmc $c ok"
done
for c in ${SQCFGS:-c2 c2slot}; do
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sqa_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_sqa_${c}_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d $O/pmc_sqb_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_sqb_${c}_$TAG.log 2>&1
echo "sq $c ok"
done
