#!/bin/bash
# Stream-kernel A/B on one box: the GPU suite first, then interleaved bench lines of the in-tree
# library against the round-3 per-wave stream (picotcp_amd/ab/libpicocsum_r03.so).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-diag}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
echo "tests ok"
A=${A:-r03} ROUNDS=${ROUNDS:-2} CFGS="${CFGS:-c2 c2tx c2eth c2v6 c2nat c2slot c2ethmix}" bash scripts/gpu_ab.sh ${A:-r03}_$TAG
PICO_CSUM_LIB=$R/picotcp_amd/diag/libpicocsum_stamps.so timeout -k 10 120 python tools/stamps.py --config c2 > $O/stamps_$TAG.txt 2>&1
echo "stamps ok"
