#!/bin/bash
# Round 6 final measurement, part $1 (tag r06f):
#   a: GPU suite, smoke, every config's bench line (C1 and C2 with their CPU baselines and host-memory
#      rates, the others --no-e2e)
#   b: rocprofv3 kernel traces of every config (the timed kernel's average, to check each line's frac)
#   c: PMC passes (FETCH_SIZE / WRITE_SIZE per config, the SQ passes on C2)
# Every GPU step under its own limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${TAG:-r06f}
ALL="c1 c2 c2slot c2tx c2tx_nw c2nat c2v6 c2eth c2ethmix c3 c3_64k c3_frag c3_reasm c3_reasm6 c3_reasm_il c3_reasm_retx c3_reasm_576 c4"
mkdir -p $O
cd $R
case "$1" in
a)
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.txt 2>&1
  echo "tests ok"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.txt 2>&1
  echo "smoke ok"
  timeout -k 10 400 python bench.py > $O/bench_c1_$TAG.json 2> $O/bench_c1_$TAG.err
  echo "bench c1 ok"
  timeout -k 10 400 python bench.py --config c2 --steps 100 --warmup 10 > $O/bench_c2_$TAG.json 2> $O/bench_c2_$TAG.err
  echo "bench c2 ok"
  for c in c2slot c2tx c2tx_nw c2nat c2v6 c2eth c2ethmix c3 c3_64k c3_frag c3_reasm c3_reasm6 c3_reasm_il c3_reasm_retx c3_reasm_576 c4; do
    st=100; case $c in c3|c3_64k|c3_frag) st=50;; c4) st=20;; esac
    timeout -k 10 300 python bench.py --config $c --steps $st --warmup 5 --no-e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
    echo "bench $c ok"
  done
  ;;
b)
  cd /tmp && export TMPDIR=/tmp
  for c in $ALL; do
    st=100; case $c in c3|c3_64k|c3_frag) st=50;; c4) st=20;; esac
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps $st --warmup 5 --no-cpu --no-e2e --no-verify > $O/prof_${c}_$TAG.log 2>&1
    echo "trace $c ok"
  done
  ;;
c)
  CFGS="${PMCCFGS:-$ALL}" SQCFGS="c2" bash $R/scripts/gpu_pmc_round.sh $TAG
  ;;
esac
