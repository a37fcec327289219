#!/bin/bash
# Round 5 session q: chunk size of the in-place host descriptor batch (32K / 128K / 1M descriptors a
# chunk) against the staged path, interleaved processes.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for r in 1 2; do
  for v in cur z131072 z1048576; do
    lib=; [ $v != cur ] && lib=$PWD/ablib/libpicocsum_$v.so
    PICO_CSUM_LIB=$lib timeout -k 10 300 python tools/host_e2e.py --stagings 32 --rounds 2 --mode both > gpurun_out/host_inplace_${v}_$r.txt 2>&1
    echo "host $v $r ok"
  done
done
