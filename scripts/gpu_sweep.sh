#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
for c in c2raw u354d c1d; do
timeout -k 10 300 python tools/sweep.py --config $c --rounds 3 --shapes 0,0,0,0,0 4,8,1,16,1 16,8,1,16,2 > $O/sweep_$c.jsonl 2>&1
done
echo sweeps ok
