#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
S2="0,0,0,0,0 4,8,1,32,1 1,1,1,64,1 1,2,1,64,1 1,4,1,64,1 1,8,1,64,1 1,4,1,32,1 1,2,1,32,1 1,4,1,64,2 1,2,1,16,1"
timeout -k 10 300 python tools/sweep.py --config c2raw --rounds 3 --shapes $S2 > $O/sweep_c2raw.jsonl 2>&1
echo "sweep c2raw ok"
S2I="0,0,0,0,0 4,8,1,32,1 16,2,1,32,1 1,1,1,64,1 1,2,1,64,1 1,4,1,64,1 1,8,1,64,1 1,4,1,32,1 1,2,1,32,1"
timeout -k 10 300 python tools/sweep.py --config c2 --rounds 3 --shapes $S2I > $O/sweep_c2.jsonl 2>&1
echo "sweep c2 ok"
