#!/bin/bash
# GPU parity suite + smoke + short bench lines (verified) on one box.  Each GPU step has its own
# time limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu_$TAG.log 2>&1
echo "pytest ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1
echo "smoke ok"
for c in ${BENCHES:-c1 c2 c2tx c2v6 c2eth}; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-e2e \
      > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
done
echo "bench ok"
