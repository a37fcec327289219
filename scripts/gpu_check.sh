#!/bin/bash
# Full GPU parity suite, a sorted-kernel sweep over the descriptor configs, and the
# bench lines of the descriptor configs.  Every GPU step under its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
echo "pytest ok"
for cfg in ${CFGS:-c2raw c2 c2tx c2v6 u64d u576d}; do
  timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 5 --shapes ${SHAPES:-2,8,1,64,2 2,8,4,64,2} | grep -v amdgpu
done > $O/sweep_$TAG.txt 2>&1
echo "sweep ok"
for c in ${BENCH:-c2 c2tx c2v6}; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
done
echo "bench ok"
