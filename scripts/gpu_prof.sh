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
PD="FETCH_SIZE"
run() { # name config shape
  for pass in A B C D; do
    eval P=\$P$pass
    timeout -k 10 240 rocprofv3 --pmc $P -d $O/${1}_$pass -o run --output-format csv -- python3 $R/tools/sweep.py --config $2 --rounds 1 --iters 10 --shapes $3 > $O/${1}_$pass.log 2>&1
  done
}
SPECS=${PROF_SPECS:-"c2raw_sorted:c2raw:2,8,0,64,2 c2_sorted:c2:2,8,0,64,2 c1d_sorted:c1d:2,8,0,64,2 c1d_adapt:c1d:3,8,0,16,1 u576d_sorted:u576d:2,8,0,64,2"}
for spec in $SPECS; do
  IFS=: read name cfg shape <<< "$spec"
  run $name $cfg $shape
done
echo prof ok
