#!/bin/bash
# PMC passes on the reassembly configs (each counter set in a run of its own, --pmc only), and the
# box's counter list.  Outputs gpurun_out/pmc_<set>_<cfg>_$TAG/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/pmc_avail.txt 2>&1 || true
for c in ${CFGS:-c3_reasm}; do
  run() { timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/pmc_${SET}_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_${SET}_${c}_$TAG.log 2>&1; }
  SET=sqa run SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES
  SET=sqb run SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
  SET=fetch run FETCH_SIZE
  SET=write run WRITE_SIZE
  echo "pmc $c ok"
done
