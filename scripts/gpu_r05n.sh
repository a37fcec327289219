#!/bin/bash
# Round 5 session n: the reassembly kernel against bare gathers of other grid shapes (one wave per
# datagram with 2 / 4 fragments a step, four waves per datagram, one wave per fragment pair).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for v in "" "--v6"; do
  timeout -k 10 300 python tools/gather_ceiling.py $v >> gpurun_out/gather_ceiling_r05n.txt 2> gpurun_out/gather_ceiling_r05n.err
  echo "gather ceiling $v ok"
done
