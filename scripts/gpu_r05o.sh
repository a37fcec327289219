#!/bin/bash
# Round 5 session o: waves per datagram of the reassembly kernel at 4K datagrams (1 = product, 2, 4;
# the bare gather ran 5 % faster at four waves per datagram, profiles/r05/gather_ceiling_shapes.txt).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab.py --tag r05o_wpd --configs c3_reasm,c3_reasm6 --rounds 2 --steps 50 --verify \
    --variant "w1=" --variant "w2=ablib/libpicocsum_wpd2.so" --variant "w4=ablib/libpicocsum_wpd4.so"
echo "ab ok"
