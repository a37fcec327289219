#!/bin/bash
# Re-verify a rebuilt tree: GPU suite, smoke, default bench line, C2 line.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_c1.json 2> $O/bench_c1.err
tail -c 400 $O/bench_c1.json
for c in c2 c2tx; do
timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 --no-cpu --no-e2e > $O/bench_$c.json 2> $O/bench_$c.err
tail -c 300 $O/bench_$c.json
done
echo verify ok
