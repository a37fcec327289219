#!/bin/bash
# Round 6: C1's lane-group kernel shape on the final binary (bench.py --shape G,CPL,FPW,U,NT,PIPE),
# interleaved rounds; prints config kernel_avg_us value.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
: > $O/c1_sweep.txt
for r in 1 2; do
  for sh in ${SHAPES:-16,8,8,1,2,2 16,8,16,1,2,2 16,8,32,1,2,2 16,8,64,1,2,2 16,8,8,1,3,2 16,8,16,1,3,2}; do
    timeout -k 10 120 python bench.py --config c1 --steps 100 --warmup 10 --no-e2e --no-cpu --no-verify --shape $sh > $O/c1s.json 2>/dev/null
    python -c "
import json; d=json.load(open('$O/c1s.json')); print('$sh', d['roofline']['kernel_avg_us'], d['value'])" >> $O/c1_sweep.txt
  done
done
cat $O/c1_sweep.txt
