#!/bin/bash
# PMC passes on one config for several builds (A="name ..." from ablib/, plus "new" = the
# in-tree library): SQ issue / wait / LDS counters, FETCH_SIZE, DRAM requests and stalls, each set
# in a run of its own (--pmc only).  Outputs gpurun_out/pmcab_<set>_<variant>_$TAG/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
C=${CFG:-c2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${A:-base} new; do
  lib=$R/picotcp_amd/libpicocsum.so
  [ $v != new ] && lib=$R/ablib/libpicocsum_$v.so
  run() { PICO_CSUM_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/pmcab_${SET}_${v}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $C --steps 10 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmcab_${SET}_${v}_$TAG.log 2>&1; }
  SET=sq run SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  SET=sq2 run SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
  SET=fetch run FETCH_SIZE GRBM_GUI_ACTIVE
  SET=tcca run TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE
  echo "pmc $v ok"
done
python3 $R/tools/pmc_summary.py $O > $O/pmcab_$TAG.txt 2>&1 || true
