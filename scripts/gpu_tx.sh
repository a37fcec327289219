#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
for cfg in c2raw c2 c2tx c2txnw c2v6; do
  timeout -k 10 120 python tools/sweep.py --config $cfg --rounds 3 --shapes 0,0,0,0,0 1,2,0,16,1 > $O/sw_$cfg.jsonl 2>&1
done
