#!/bin/bash
# Round 6: the reassembly lines (every datagram verified, the hand-written copy ceiling) and the
# bare-gather / copy shapes of tools/gather_ceiling.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
for c in ${CFGS:-c3_reasm c3_reasm6}; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-e2e > $O/bench_$c.json 2> $O/bench_$c.err
done
[ -n "$NOGC" ] || timeout -k 10 300 python -u tools/gather_ceiling.py --reps 30 > $O/gather_ceiling.txt 2>&1
[ -n "$NOGC" ] || timeout -k 10 300 python -u tools/gather_ceiling.py --v6 --reps 30 >> $O/gather_ceiling.txt 2>&1
for c in ${CFGS:-c3_reasm c3_reasm6}; do python -c "
import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']
print('$c', d['value'], r['kernel_avg_us'], r['frac'], d['verified'], json.dumps(r.get('copy_ceiling')))"; done
