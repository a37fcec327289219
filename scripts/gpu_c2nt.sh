#!/bin/bash
# Sorted-kernel shapes on the descriptor configs with >= 1 GiB rotation (no MALL help).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for cfg in ${CFGS:-c2raw c2 c2v6 u64d u576d c1d}; do
  timeout -k 10 240 python tools/sweep.py --config $cfg --rounds 5 --shapes ${SHAPES:-2,8,1,64,2 2,8,1,64,1 2,8,4,64,2 2,4,0,64,2 2,4,0,64,1 2,8,1,32,2} | grep -v amdgpu
done > $O/c2nt_sweep.txt 2>&1
echo "sweep ok"
