#!/bin/bash
# Instruction-cache counters of the C2 stream kernel, the in-tree library against the round-3
# per-wave stream (one --pmc pass each).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in new r03; do
  lib=$R/picotcp_amd/libpicocsum.so
  [ $v != new ] && lib=$R/picotcp_amd/ab/libpicocsum_$v.so
  PICO_CSUM_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $O/pmc_icache_$v -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 20 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_icache_$v.log 2>&1
  echo "icache $v ok"
done
