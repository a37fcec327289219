#!/bin/bash
# Flat-grid reassembly, product form (per-thread scratch with events): tests, then A/B against one
# workgroup per datagram and the static-scratch build of the same kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frag.py \
    > gpurun_out/pytest_frag_prod.txt 2>&1 || exit 1
for A in noflat quad; do
  A=$A CFGS="c3_reasm c3_reasm6" ROUNDS=2 VERIFY="--steps 100" timeout -k 10 400 bash scripts/gpu_ab.sh reasm6_$A > /dev/null 2>&1 || exit 1
done
