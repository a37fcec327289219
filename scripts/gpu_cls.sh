#!/bin/bash
# Round-class A/B for the sorted kernel: CPL 8 vs 16, with / without the 2-lane class,
# interleaved in one process per config; GPU suite first (the new variants are in it).
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
for c in c2 c2tx c2v6 c2eth c2raw; do
  timeout -k 10 240 python tools/sweep.py --config $c --rounds 5 --iters 30 --shapes 2,8,1,64,2 2,8,2,64,2 2,16,1,64,2 2,16,2,64,2 > $O/sweep_$c.txt 2>&1
  cat $O/sweep_$c.txt
done
echo cls ok
