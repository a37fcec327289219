#!/bin/bash
# Round 6, after r06f: the reassembly configs on the final frag kernels (128-fragment planners, the
# finish's loads in one round trip), C1's stride-1536 variant, traces + PMC of those (tag r06g).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${TAG:-r06g}
CF="${CF:-c1_s1536 c3_reasm c3_reasm6 c3_reasm_il c3_reasm_retx c3_reasm_576}"
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.txt 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.txt 2>&1
for c in $CF; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 5 --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
for c in $CF; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 100 --warmup 5 --no-cpu --no-e2e --no-verify > $O/prof_${c}_$TAG.log 2>&1
  echo "trace $c ok"
done
CFGS="$CF" SQCFGS=" " bash $R/scripts/gpu_pmc_round.sh $TAG
