#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
S1="0,0,0,0,0 64,2,1,32,1 64,2,2,32,1 64,2,2,16,1 64,2,2,16,2 32,4,2,32,1 32,4,2,32,2 32,4,2,16,1 32,4,2,16,2 32,4,1,16,2 32,2,4,16,2 32,4,2,8,2 32,4,2,64,2 16,8,1,16,2 16,4,2,16,2 64,4,2,16,2"
timeout -k 10 300 python tools/sweep.py --config c1 --rounds 5 --shapes $S1 > $O/sweep_c1.jsonl 2>&1
echo "sweep c1 ok"
S3="0,0,0,0,0 64,4,2,32,2 64,4,2,8,2 64,2,4,8,2 64,8,1,8,2 64,4,2,16,2 32,4,2,16,2"
timeout -k 10 300 python tools/sweep.py --config c3 --rounds 3 --shapes $S3 > $O/sweep_c3.jsonl 2>&1
echo "sweep c3 ok"
S2="0,0,0,0,0 16,4,1,32,1 8,4,2,32,1 8,8,1,32,1 8,4,2,32,2 8,8,1,64,1 4,8,1,32,1 4,4,2,32,1 8,4,2,16,1"
timeout -k 10 300 python tools/sweep.py --config c2raw --rounds 3 --shapes $S2 > $O/sweep_c2raw.jsonl 2>&1
echo "sweep c2raw ok"
