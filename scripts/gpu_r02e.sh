#!/bin/bash
# Round-2 measurement session: bench lines + same-process rocprofv3 kernel traces for every
# config, FETCH_SIZE / WRITE_SIZE passes per config, and the FETCH_SIZE calibration for
# partial-line reads (tools/fetch_calib.py).  Each GPU step has its own limit; a failure ends it.
#   scripts/gpu_r02e.sh TAG [bench] [prof] [pmc] [calib]
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
STEPS=${*:-"bench prof pmc calib"}
CFGS=${CFGS:-"c1 c2 c2tx c2v6 c2eth c3_reasm c4"}
mkdir -p $O
cd $R
for s in $STEPS; do
case $s in
bench)
  for c in $CFGS; do
    rc=0
    timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || rc=$?
    # a Python error (1) is reported and the next config runs; any other failure ends the script
    [ $rc -eq 0 ] || { tail -5 $O/bench_$c.err; [ $rc -eq 1 ] || exit $rc; }
    tail -c 400 $O/bench_$c.json
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
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$c -o run --output-format csv -- \
      python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_fetch_$c.json 2> $O/pmc_fetch_$c.err
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$c -o run --output-format csv -- \
      python3 $R/bench.py --config $c --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_write_$c.json 2> $O/pmc_write_$c.err
  done
  cd $R
  echo "pmc ok" ;;
calib)
  cd /tmp && export TMPDIR=/tmp
  for p in "128 128" "64 128" "32 128" "16 128" "64 64" "1500 1500" "80 80" "40 96"; do
    set -- $p
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/calib_len$1_stride$2 -o run --output-format csv -- \
      python3 $R/tools/fetch_calib.py --len $1 --stride $2 > $O/calib_len$1_stride$2.json 2> $O/calib_len$1_stride$2.err
  done
  cd $R
  echo "calib ok" ;;
esac
done
