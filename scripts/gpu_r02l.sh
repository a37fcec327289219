#!/bin/bash
# GPU suite + multi-rank rehearsal of the graph-replay bench on one GPU (gloo timing, 2 ranks) +
# FETCH_SIZE of the raw-descriptor C2 layout (no head window) for the over-fetch breakdown.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
PICO_BENCH_SAME_DEVICE=1 PICO_BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c4 --steps 20 --warmup 3 --no-cpu --no-e2e > $O/bench_multi_c4.json 2> $O/bench_multi_c4.err
tail -c 300 $O/bench_multi_c4.json
PICO_BENCH_SAME_DEVICE=1 PICO_BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c2 --steps 50 --warmup 5 --no-cpu --no-e2e > $O/bench_multi_c2.json 2> $O/bench_multi_c2.err
tail -c 300 $O/bench_multi_c2.json
cd /tmp && export TMPDIR=/tmp
for c in c2raw c2; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$c -o run --output-format csv -- \
    python3 $R/tools/sweep.py --config $c --rounds 1 --iters 20 --shapes 2,8,1,64,2 > $O/pmc_fetch_$c.txt 2>&1
done
cd $R
echo "r02l ok"
