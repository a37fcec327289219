#!/bin/bash
# Parity first, then interleaved launch-shape sweeps on the descriptor configs.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
COMMON="0,0,0,0,0 2,8,0,64,1 2,8,0,64,2 2,4,0,64,1 2,4,0,64,2 2,8,0,48,2"
for cfg in c2raw u354d c1d c2 c2v6; do
  EXTRA=""
  case $cfg in c2|c2v6) ;; *) EXTRA="3,8,0,16,1";; esac
  timeout -k 10 300 python tools/sweep.py --config $cfg --rounds 3 --shapes $COMMON $EXTRA > $O/sweep_$cfg.jsonl 2>&1
  echo "sweep $cfg ok"
done
