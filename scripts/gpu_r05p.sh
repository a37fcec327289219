#!/bin/bash
# Round 5 session p: host descriptor batches read in place when the burst is device-addressable
# (tests, then the C2 line with the in-place / staged / raw zero-copy host rates), and the
# multi-rank rehearsal on the final binary (2 ranks on the one GPU, gloo timing; C1 and C4).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_inplace.py tests/test_gpu_host_desc.py tests/test_gpu_zerocopy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_host_r05p.log 2>&1
echo "host tests ok"
timeout -k 10 400 python bench.py --config c2 --steps 100 --warmup 10 > gpurun_out/bench_c2_r05p.json 2> gpurun_out/bench_c2_r05p.err
echo "bench c2 ok"
export PICO_BENCH_SAME_DEVICE=1 PICO_BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 --no-e2e > gpurun_out/bench_multi_2_c1_r05p.json 2> gpurun_out/bench_multi_2_c1_r05p.err
echo "multi c1 ok"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c4 --steps 20 --warmup 3 --no-e2e > gpurun_out/bench_multi_2_c4_r05p.json 2> gpurun_out/bench_multi_2_c4_r05p.err
echo "multi c4 ok"
