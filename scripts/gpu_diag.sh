#!/bin/bash
# Stream-kernel diagnosis on one box: interleaved A/B of the round-3 per-wave stream
# (picotcp_amd/ab/libpicocsum_r03.so) against the in-tree library, then per-wave stamps of both
# (picotcp_amd/diag/libpicocsum_stamps{,_r03}.so, tools/stamps.py) on C2.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-diag}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
echo "tests ok"
A=r03 ROUNDS=2 CFGS="${CFGS:-c2 c2tx c2eth}" bash scripts/gpu_ab.sh r03_$TAG
for v in stamps stamps_r03; do
  PICO_CSUM_LIB=$R/picotcp_amd/diag/libpicocsum_$v.so timeout -k 10 120 python tools/stamps.py --config c2 > $O/${v}_$TAG.txt 2>&1
  echo "$v ok"
done
