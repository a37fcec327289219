#!/bin/bash
# Bench lines of the reassembly and large-ring configs (not in the session's list).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-more}
mkdir -p $O
cd $R
for c in ${CFGS:-c3_reasm c3_reasm6 c2tx_nw}; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
  echo "bench $c ok"
done
