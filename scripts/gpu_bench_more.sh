#!/bin/bash
# Parity, then the extra bench configs (TX compute mode, reassembly-size datagrams).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
for c in ${CFGS:-c2 c2tx c2v6 c3_frag}; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
  echo "bench $c ok"
done
