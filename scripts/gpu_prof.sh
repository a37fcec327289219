#!/bin/bash
# PMC passes over single-shape sweeps: where does the time of each kernel go?
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
PB="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES"
PC="TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
run() { # name config shape
  for pass in A B C; do
    eval P=\$P$pass
    timeout -k 10 240 rocprofv3 --pmc $P -d $O/${1}_$pass -o run --output-format csv -- python3 $R/tools/sweep.py --config $2 --rounds 1 --iters 10 --shapes $3 > $O/${1}_$pass.log 2>&1
  done
}
run u354 u354 4,8,1,32,1
run c2raw_lg c2raw 4,8,1,32,1
run c2raw_flat c2raw 1,4,1,32,1
run c2_flat c2 1,4,1,32,1
echo prof ok
