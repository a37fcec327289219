#!/bin/bash
# Round 5 session c: persistent stream waves with per-XCD claims (no stealing) or static groups, and
# the uniform-ring stream -- their tests, the GPU suite, an interleaved A/B (tools/ab.py).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_persistent.py tests/test_gpu_uniform_stream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_persist_r05c.log 2>&1
echo "persist ok"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r05c.log 2>&1
echo "tests ok"
timeout -k 10 900 python tools/ab.py --tag r05c --configs c1,c2,c2v6,c2ethmix --rounds 2 \
    --variant r04=picotcp_amd/ab/libpicocsum_r04.so --variant new= --variant "static=:--stream 258,0" \
    --variant "off=:--stream 255,0"
echo "ab ok"
