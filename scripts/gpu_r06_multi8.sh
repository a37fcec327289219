#!/bin/bash
# Round 6: bench.py --gpus 8 rehearsed on the one GPU of the box -- 8 ranks under torch.distributed.run,
# every rank on cuda:0 (PICO_BENCH_SAME_DEVICE=1), gloo for the barriers / max-time (RCCL needs one GPU
# per rank): the launcher, the shard split and the per-rank verify at the N the driver uses.  The
# ranks share one device's bandwidth, so the value is one GPU's, not eight's.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
port=29511
for c in ${CFGS:-c1 c4}; do
  PICO_BENCH_SAME_DEVICE=1 PICO_BENCH_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 600 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 8 --config $c --steps ${STEPS:-20} --warmup 5 > $O/bench_multi_8_$c.out 2> $O/bench_multi_8_$c.err
  port=$((port + 1))
  grep '^{' $O/bench_multi_8_$c.out > $O/bench_multi_8_$c.json      # (gloo prints its connections to stdout)
  python -c "
import json; d=json.load(open('$O/bench_multi_8_$c.json')); print('$c', d['n_gpus'], d['value'], d['ms_per_step'], json.dumps(d.get('verified'))[:300])"
done
