#!/bin/bash
# GPU tests, then the IMIX descriptor configs with the default shape (>= 1 GiB rotation).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
tail -1 $O/gputests.log
for cfg in ${CFGS:-c2 c2tx c2v6 c2raw}; do
  timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 5 --shapes ${SHAPES:-2,8,1,64,2} | grep -v amdgpu
done > $O/c2quick.txt 2>&1
cat $O/c2quick.txt
