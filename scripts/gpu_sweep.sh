#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
S1="0,0,0,0,0 16,8,1,16,2,1 16,8,1,16,2,2 16,8,1,32,2,2 16,8,1,64,2,2 16,8,1,16,1,2 32,4,1,16,2,2 32,4,1,32,2,2 32,4,1,64,2,2 64,2,1,16,2,2 64,2,1,32,2,2 8,8,1,16,2,1 16,8,1,8,2,2"
timeout -k 10 300 python tools/sweep.py --config c1 --rounds 5 --shapes $S1 > $O/sweep_c1.jsonl 2>&1
echo "sweep c1 ok"
SU="0,0,0,0,0 4,8,1,32,1,1 4,8,1,32,1,2 4,8,1,64,1,2 8,4,1,32,1,2 8,4,1,64,1,2 4,8,1,16,1,2"
timeout -k 10 300 python tools/sweep.py --config u354 --rounds 3 --shapes $SU > $O/sweep_u354.jsonl 2>&1
echo "sweep u354 ok"
