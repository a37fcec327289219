#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for cfg in u40d u64d u576d u1500d c2raw; do
  timeout -k 10 300 python tools/sweep.py --config $cfg --rounds 3 --shapes 0,0,0,0,0 3,8,0,16,1 1,2,0,16,1 > $O/sw_$cfg.jsonl 2>&1
done
for cfg in u64 u576 c1; do
  timeout -k 10 300 python tools/sweep.py --config $cfg --rounds 3 --shapes 0,0,0,0,0 > $O/sw_$cfg.jsonl 2>&1
done
