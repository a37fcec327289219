#!/bin/bash
# Round 5 session g: the claimed-chunk uniform stream -- its tests, then an interleaved A/B on C1,
# C4 and C3 against the lane-group kernels and the fixed-range stream.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_uniform_stream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_uni_r05g.log 2>&1
echo "uniform tests ok"
timeout -k 10 900 python tools/ab.py --tag r05g_c1 --configs c1 --rounds 3 --steps 100 \
    --variant "off=:--stream 255,0" --variant "dyn=:--stream 2,0" --variant "dyn32=:--stream 2,32" \
    --variant "stat=:--stream 3,0" --variant "r64=:--stream 1,64"
timeout -k 10 600 python tools/ab.py --tag r05g_big --configs c3,c4,c3_64k --rounds 2 --steps 20 \
    --variant "auto=" --variant "dyn=:--stream 2,0" --variant "stat=:--stream 3,0"
echo "ab ok"
