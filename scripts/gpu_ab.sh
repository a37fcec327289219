#!/bin/bash
# Interleaved A/B of two builds of the library on one box: ablib/libpicocsum_<A>.so vs
# the in-tree picotcp_amd/libpicocsum.so ("new"), ROUNDS x configs, bench lines without the CPU
# legs.  Output: gpurun_out/ab_$TAG.txt (variant config kernel_avg_us value).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-ab}
A=${A:-base}
mkdir -p $O
cd $R
: > $O/ab_$TAG.txt
for r in $(seq ${ROUNDS:-3}); do
  for v in $A new; do
    lib=$R/picotcp_amd/libpicocsum.so
    [ $v != new ] && lib=$R/ablib/libpicocsum_$v.so
    for c in ${CFGS:-c2 c2v6 c2eth c2tx}; do
      PICO_CSUM_LIB=$lib timeout -k 10 120 python bench.py --config $c --steps ${STEPS:-100} --warmup 10 \
          --no-e2e --no-cpu ${VERIFY:---no-verify} ${EXTRA:-} > $O/ab_line.json 2> $O/ab_err.txt
      python -c "
import json; d=json.load(open('$O/ab_line.json')); r=d['roofline']
print('$v', '$c', r['kernel_avg_us'], d['value'], d.get('verified', {}).get('mismatches', '-'))" >> $O/ab_$TAG.txt
    done
  done
done
cat $O/ab_$TAG.txt
