#!/bin/bash
# Round 6: a kernel variant (ablib/libpicocsum_$V.so): its GPU tests, then an interleaved A/B
# against the in-tree library ("new").
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
PICO_CSUM_LIB=$R/ablib/libpicocsum_$V.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  $TESTS > $O/pytest_$V.txt 2>&1 || { tail -30 $O/pytest_$V.txt; exit 1; }
tail -1 $O/pytest_$V.txt
A="$V" CFGS="$CFGS" STEPS=${STEPS:-100} VERIFY="--rotate 0" ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab.sh $V
