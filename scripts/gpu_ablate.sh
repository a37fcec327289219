#!/bin/bash
# Phase ablation of the sorted kernel on the IMIX configs (PICO_CSUM_ABLATE: 1 = no rounds,
# 2 = no head-window loads, 3 = neither), >= 1 GiB rotation.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for ab in 0 1 2 3; do
  for cfg in ${CFGS:-c2 c2tx c2raw}; do
    echo "ablate=$ab"
    PICO_CSUM_ABLATE=$ab timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 5 --shapes ${SHAPES:-2,8,1,64,2} | grep -v amdgpu
  done
done > $O/ablate.txt 2>&1
echo "ablate ok"
