#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
S="4,8,1,16,1,1 8,4,1,16,1,1 16,2,1,16,1,1 32,1,1,16,1,1 16,2,2,16,1,1 32,1,4,16,1,1 16,2,1,16,2,1 32,1,2,32,1,1 8,4,1,16,1,2 16,2,1,16,1,2 32,1,1,32,1,2"
timeout -k 10 300 python tools/sweep.py --config u354 --rounds 3 --shapes $S > $O/sweep_u354.jsonl 2>&1
S="4,8,1,16,1,1 8,8,1,16,1,1 16,4,1,16,1,1 32,2,1,16,1,1 64,1,1,16,1,1 32,2,1,16,1,2 64,1,2,16,1,1"
timeout -k 10 300 python tools/sweep.py --config u576 --rounds 3 --shapes $S > $O/sweep_u576.jsonl 2>&1
echo sweeps ok
