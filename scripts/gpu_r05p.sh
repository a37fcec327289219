#!/bin/bash
# Round 5 session p: host descriptor batches read in place when the burst is device-addressable and
# in one zero-copy launch when the descriptors and results are too (tests, then the C2 line with the
# staged / in-place / pinned-ring / raw zero-copy host rates).  (The multi-rank rehearsal of this
# session's first run: profiles/r05/bench_multi_2_*.json.)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_inplace.py tests/test_gpu_host_desc.py tests/test_gpu_zerocopy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_host_r05p2.log 2>&1
echo "host tests ok"
timeout -k 10 400 python bench.py --config c2 --steps 100 --warmup 10 > gpurun_out/bench_c2_r05p2.json 2> gpurun_out/bench_c2_r05p2.err
echo "bench c2 ok"
