#!/bin/bash
# Round 5 session j: the finish's share of the persistent stream (a measurement build without the
# finish), static order at 1 / 2 waves per SIMD, against one wave per group.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 500 python tools/ab.py --tag r05j_c2 --configs c2 --rounds 2 --steps 100 \
    --variant "off=" --variant "s1=:--pstream 2,1,64" --variant "nf1=ablib/libpicocsum_nofin.so:--pstream 2,1,64" \
    --variant "s2=:--pstream 2,2,64" --variant "nf2=ablib/libpicocsum_nofin.so:--pstream 2,2,64"
echo "ab ok"
