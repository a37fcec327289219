#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace + PMC passes.
# Every GPU step has its own time limit; any failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 400 python bench.py --steps 200 --warmup 20 > $O/bench_c1.json 2> $O/bench_c1.err
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu --no-e2e > $O/prof_c1.log 2>&1
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_c1 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_fetch_c1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_c1 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_write_c1.log 2>&1
echo "pmc ok"
