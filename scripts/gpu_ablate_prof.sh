#!/bin/bash
# Kernel durations (rocprofv3 kernel trace) of the sorted kernel with phases ablated.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ablprof
mkdir -p $O
cd $R
export TMPDIR=/tmp
for ab in 0 1 2; do
  for cfg in c2 c2raw; do
    export PICO_CSUM_ABLATE=$ab
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/${cfg}_$ab -o k -- python tools/sweep.py --config $cfg --rounds 2 --iters 20 --shapes 2,8,1,64,2 > $O/${cfg}_$ab.log 2>&1
  done
done
echo "prof ok"
