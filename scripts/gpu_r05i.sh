#!/bin/bash
# Round 5 session i: persistent stream waves in static group order (no claim atomics) vs claimed
# groups vs one wave per group, on C2.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pstream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pstream_r05i.log 2>&1
echo "pstream tests ok"
timeout -k 10 500 python tools/ab.py --tag r05i_c2 --configs c2 --rounds 2 --steps 100 \
    --variant "off=" --variant "s1=:--pstream 2,1,64" --variant "s2=:--pstream 2,2,64" --variant "s1g32=:--pstream 2,1,32" \
    --variant "s2g32=:--pstream 2,2,32" --variant "d1=:--pstream 1,1,64"
echo "ab c2 ok"
