#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: 2 and 4 ranks on GPU 0, gloo timing collectives.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export PICO_BENCH_SAME_DEVICE=1 PICO_BENCH_DIST_BACKEND=gloo
for n in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 50 --warmup 5 > $O/bench_multi_$n.json 2> $O/bench_multi_$n.err
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c4 --steps 20 --warmup 3 > $O/bench_multi_c4.json 2> $O/bench_multi_c4.err
echo multi ok
