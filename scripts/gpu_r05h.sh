#!/bin/bash
# Round 5 session h (re-entry): the persistent stream waves for IPv4 batches (tests, then an
# interleaved A/B on C2), the full GPU suite, and the claimed-chunk uniform stream A/B (C1, C3, C4)
# now that the claims are read a step late (no atomic optimizer in the sorted TU).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pstream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pstream_r05h.log 2>&1
echo "pstream tests ok"
timeout -k 10 400 python tools/ab.py --tag r05h_c2 --configs c2 --rounds 2 --steps 100 \
    --variant "off=" --variant "p1=:--pstream 1,1,64" --variant "p2=:--pstream 1,2,64" --variant "p1g32=:--pstream 1,1,32"
echo "ab c2 ok"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r05h.log 2>&1
echo "gpu suite ok"
timeout -k 10 400 python tools/ab.py --tag r05h_c1 --configs c1 --rounds 2 --steps 100 \
    --variant "off=:--stream 255,0" --variant "dyn=:--stream 2,0" --variant "dyn32=:--stream 2,32" \
    --variant "stat=:--stream 3,0"
timeout -k 10 400 python tools/ab.py --tag r05h_big --configs c3,c4 --rounds 2 --steps 20 \
    --variant "auto=" --variant "dyn=:--stream 2,0" --variant "stat=:--stream 3,0"
echo "ab ok"
