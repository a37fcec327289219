#!/bin/bash
# SQ / GRBM counters for the sorted kernel on C2 (full, and phases 1+2+4 only), one pass each.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_c2
mkdir -p $O
cd $R
export TMPDIR=/tmp
for ab in 0 1; do
  export PICO_CSUM_ABLATE=$ab
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/a$ab -o p -- python tools/sweep.py --config c2 --rounds 1 --iters 5 --rotate 3 --shapes 2,8,1,64,2 > $O/a$ab.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $O/b$ab -o p -- python tools/sweep.py --config c2 --rounds 1 --iters 5 --rotate 3 --shapes 2,8,1,64,2 > $O/b$ab.log 2>&1
done
echo "pmc ok"
