#!/bin/bash
# Round 5 session e: uniform-ring stream frames-per-wave sweep (C3, C3 64 KiB, C4) after the
# persistent fused kernel's removal; tests first.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r05e.log 2>&1
echo "tests ok"
timeout -k 10 500 python tools/ab.py --tag r05e_c3 --configs c3 --rounds 2 --steps 30 \
    --variant r04=picotcp_amd/ab/libpicocsum_r04.so --variant new= --variant "r128=:--stream 1,128" \
    --variant "r512=:--stream 1,512" --variant "off=:--stream 255,0"
timeout -k 10 400 python tools/ab.py --tag r05e_c3_64k --configs c3_64k --rounds 2 --steps 30 \
    --variant new= --variant "r8=:--stream 1,8" --variant "r32=:--stream 1,32" --variant "off=:--stream 255,0"
timeout -k 10 500 python tools/ab.py --tag r05e_c4 --configs c4 --rounds 2 --steps 20 \
    --variant "r128=:--stream 1,128" --variant "r4096=:--stream 1,4096" --variant "r1024=:--stream 1,1024" --variant "off=:--stream 255,0"
echo "ab ok"
