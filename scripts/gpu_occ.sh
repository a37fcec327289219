#!/bin/bash
# A/B: sorted kernel at 4 vs 5 waves per SIMD (PICO_CSUM_ABLATE=16) over frames per wave.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
tail -1 $O/gputests.log
for ab in 0 16; do
  for cfg in c2 c2v6 c2raw; do
    echo "ab=$ab"
    PICO_CSUM_ABLATE=$ab timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 5 --shapes 2,8,1,64,2 2,8,1,52,2 2,8,1,44,2 | grep -v amdgpu
  done
done > $O/occ.txt 2>&1
cat $O/occ.txt
