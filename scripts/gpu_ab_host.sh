#!/bin/bash
# Interleaved A/B of the host-resident C2 burst (tools/host_e2e.py) between
# picotcp_amd/ab/libpicocsum_<A>.so and the in-tree library.  Output: gpurun_out/ab_host_$TAG.txt
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-ab}
A=${A:-base}
mkdir -p $O
cd $R
: > $O/ab_host_$TAG.txt
for r in $(seq ${ROUNDS:-3}); do
  for v in $A new; do
    lib=$R/picotcp_amd/libpicocsum.so
    [ $v != new ] && lib=$R/picotcp_amd/ab/libpicocsum_$v.so
    PICO_CSUM_LIB=$lib timeout -k 10 180 python tools/host_e2e.py --stagings ${STAGINGS:-16 64} --rounds 2 \
        > $O/ab_host_line.txt 2> $O/ab_host_err.txt
    sed "s/^/$v /" $O/ab_host_line.txt >> $O/ab_host_$TAG.txt
  done
done
cat $O/ab_host_$TAG.txt
