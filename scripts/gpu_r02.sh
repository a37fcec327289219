#!/bin/bash
# Round-2 GPU session: parity suite, bench lines, and for each bench config a rocprofv3
# kernel trace of the SAME process whose JSON line is kept beside it (so the line's
# roofline.frac can be re-derived from profiles/: tools/prof_timed.py), then PMC passes
# (FETCH_SIZE / WRITE_SIZE, separate runs).  Every GPU step has its own time limit and
# any failure ends the script.
#   scripts/gpu_r02.sh TAG [tests|bench|prof|pmc ...]   (default: all four)
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
STEPS=${STEPS:-"tests bench prof pmc"}
[ $# -gt 0 ] && STEPS="$*"
CFGS=${CFGS:-"c1 c2 c2tx c2v6 c4"}
mkdir -p $O
cd $R
for s in $STEPS; do
case $s in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -3 $O/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  echo "tests ok" ;;
bench)
  timeout -k 10 400 python bench.py > $O/bench_c1.json 2> $O/bench_c1.err
  for c in $CFGS; do
    [ $c = c1 ] && continue
    timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 > $O/bench_$c.json 2> $O/bench_$c.err
  done
  echo "bench ok" ;;
prof)
  cd /tmp && export TMPDIR=/tmp
  for c in $CFGS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- \
      python3 $R/bench.py --config $c --steps 200 --warmup 20 --no-cpu --no-e2e > $O/prof_$c.json 2> $O/prof_$c.err
  done
  cd $R
  echo "prof ok" ;;
pmc)
  cd /tmp && export TMPDIR=/tmp
  for c in $CFGS; do
    [ $c = c4 ] && continue
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$c -o run --output-format csv -- \
      python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_fetch_$c.json 2> $O/pmc_fetch_$c.err
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$c -o run --output-format csv -- \
      python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_write_$c.json 2> $O/pmc_write_$c.err
  done
  cd $R
  echo "pmc ok" ;;
esac
done
