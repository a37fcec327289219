#!/bin/bash
# Ablations of the sorted-rounds kernel (PICO_SORTED_DBG: 1 skip rounds, 2 skip sort).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
for d in ${DBG_MODES:-0}; do
  for cfg in ${DBG_CFGS:-c2raw c2 u1500d}; do
    PICO_SORTED_DBG=$d timeout -k 10 120 python tools/sweep.py --config $cfg --rounds 3 --shapes ${DBG_SHAPES:-2,8,0,64,2} | grep -v amdgpu | sed "s/^/dbg$d /"
  done
done > $O/dbg.txt 2>&1
