#!/bin/bash
# Round 5 session b: the persistent stream waves -- their own tests first, the GPU suite, then an
# interleaved A/B against the round-4 library and the classic grid (tools/ab.py).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_persistent.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_persist_r05b.log 2>&1
echo "persist ok"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r05b.log 2>&1
echo "tests ok"
timeout -k 10 900 python tools/ab.py --tag r05b --configs c2,c2v6,c2ethmix --rounds 2 \
    --variant r04=picotcp_amd/ab/libpicocsum_r04.so --variant new= --variant "p2_32=:--stream 2,32" \
    --variant "p4_32=:--stream 4,32" --variant "cls=:--stream 255,0"
echo "ab ok"
