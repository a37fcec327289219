#!/bin/bash
# Round 6: the last-arriver flat grid -- its GPU tests, then an interleaved A/B against the round-5
# planner + finish build (ablib/libpicocsum_base.so).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_frag.py tests/test_gpu_scratch.py} > $O/pytest_reasm.txt 2>&1 || { tail -30 $O/pytest_reasm.txt; exit 1; }
tail -3 $O/pytest_reasm.txt
A="${A:-base}" CFGS="${CFGS:-c3_reasm c3_reasm6}" STEPS=100 VERIFY="--rotate 0" ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab.sh ${TAG:-reasm_lastarriver}
