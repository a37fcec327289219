#!/bin/bash
# Sorted-rounds kernel variants: parity on the descriptor kernels, then an
# interleaved sweep (one process per config) of the shapes in $SHAPES.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${TESTS:-sorted or desc or ipv4 or ipv6 or fuzz}" > $O/pytest_sorted.log 2>&1
echo "pytest ok"
for cfg in ${CFGS:-c2raw c2 c2tx c2v6 u64d u576d c1d u9000d}; do
  timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 5 --shapes ${SHAPES:-2,8,4,64,2 2,8,1,64,2} \
    | grep -v amdgpu
done > $O/sorted_sweep.txt 2>&1
echo "sweep ok"
