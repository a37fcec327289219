#!/bin/bash
# Reassembly A/B on one box: A=<ablib variant> against the in-tree library on CFGS (verified
# lines) with EXTRA bench flags (e.g. --reasm-flat 1); TESTS=1 runs the frag GPU tests first.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frag.py \
      > gpurun_out/pytest_frag_prod.txt 2>&1 || exit 1
fi
CFGS=${CFGS:-"c3_reasm c3_reasm6"} ROUNDS=${ROUNDS:-2} VERIFY="--steps 100" timeout -k 10 600 bash scripts/gpu_ab.sh ${TAG:-reasm} > /dev/null 2>&1
