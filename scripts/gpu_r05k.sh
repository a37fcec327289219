#!/bin/bash
# Round 5 session k: frames per wave of the stream-order waves on C2 (a second residency round
# refilled by the dispatcher as light waves finish), C2-IPv6 and the Ethernet batch.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 700 python tools/ab.py --tag r05k_fpw --configs c2,c2v6,c2eth --rounds 2 --steps 100 \
    --variant "f64=" --variant "f48=:--shape 2,0,48" --variant "f40=:--shape 2,0,40" \
    --variant "f32=:--shape 2,0,32" --variant "f24=:--shape 2,0,24" --variant "f16=:--shape 2,0,16"
echo "ab ok"
