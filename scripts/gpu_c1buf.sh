#!/bin/bash
# Windowed-buffer pipelined uniform kernel: parity, then C1 A/B sweep (buffer window vs global loads).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${TESTS:-uniform or sorted or desc}" > $O/pytest_c1buf.log 2>&1
echo "pytest ok"
for cfg in ${CFGS:-c1 c1_1536 u576}; do
  timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 7 --shapes ${SHAPES:-16,8,1,8,2,2 16,8,1,8,2,3 16,8,1,16,2,2 16,8,1,4,2,2 16,8,1,32,2,2} \
    | grep -v amdgpu
done > $O/c1buf_sweep.txt 2>&1
echo "sweep ok"
