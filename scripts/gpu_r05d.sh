#!/bin/bash
# Round 5 session d: the continuous uniform-ring stream (tests, GPU suite, A/B on C1 / C4 / C3).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_uniform_stream.py tests/test_gpu_ref_tx.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_new_r05d.log 2>&1
echo "new tests ok"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r05d.log 2>&1
echo "tests ok"
timeout -k 10 900 python tools/ab.py --tag r05d --configs c1,c3,c4 --rounds 2 --steps 50 \
    --variant r04=picotcp_amd/ab/libpicocsum_r04.so --variant new= --variant "r128=:--stream 4,128" \
    --variant "r256=:--stream 4,256" --variant "off=:--stream 255,0"
echo "ab ok"
