#!/bin/bash
# Stream-kernel check on one box: the GPU suite, instruction counts of the C2 kernel (in-tree and
# round-3 libraries, one --pmc pass each), then interleaved bench lines of the two libraries.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-diag}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
echo "tests ok"
bash scripts/gpu_pmc_valu.sh $TAG
cd $R
A=${A:-r03} ROUNDS=${ROUNDS:-2} CFGS="${CFGS:-c2 c2tx c2eth c2v6 c2nat c2ethmix}" bash scripts/gpu_ab.sh ${A:-r03}_$TAG
