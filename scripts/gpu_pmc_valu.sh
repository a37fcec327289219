#!/bin/bash
# Instruction counts of the C2 kernel (one --pmc pass per library): the in-tree library against
# the round-3 one (picotcp_amd/ab/libpicocsum_r03.so).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-v}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in new ${VARIANTS:-r03}; do
  lib=$R/picotcp_amd/libpicocsum.so
  [ $v != new ] && lib=$R/picotcp_amd/ab/libpicocsum_$v.so
  for c in ${CFGS:-c2}; do
    PICO_CSUM_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d $O/pmc_valu_${v}_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_valu_${v}_${c}_$TAG.log 2>&1
    echo "pmc $v $c ok"
  done
done
