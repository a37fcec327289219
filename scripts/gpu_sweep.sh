#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 300 python tools/sweep.py --config c2v6 --rounds 3 --shapes 0,0,0,0,0 1,2,0,16,1 1,4,0,16,1 1,2,0,32,1 > $O/sweep_c2v6.jsonl 2>&1
timeout -k 10 300 python bench.py --config c2v6 --steps 100 --warmup 10 > $O/bench_c2v6.json 2> $O/bench_c2v6.err
echo ok
