#!/bin/bash
# One GPU-box session: parity tests, bench (c1 + other configs), rocprofv3
# kernel trace + PMC passes for c1.  Each GPU step has its own time limit;
# any failure ends the script (set -e).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 400 python bench.py > $O/bench_c1_$TAG.json 2> $O/bench_c1_$TAG.err
echo "bench c1 ok"
for c in c2 c2tx c2v6 c3 c3_64k c3_frag; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-cpu --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
done
echo "bench configs ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu --no-e2e > $O/prof_c1_$TAG.log 2>&1
for cfg in c2 c2v6; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${cfg}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e > $O/prof_${cfg}_$TAG.log 2>&1
done
echo "trace ok"
for cfg in c1 c2 c2v6; do
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_${cfg}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_fetch_${cfg}_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_${cfg}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_write_${cfg}_$TAG.log 2>&1
done
echo "pmc ok"
