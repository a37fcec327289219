#!/bin/bash
# One measurement session on the current binary: the library rebuilt from source on the box, the GPU
# suite, smoke, verified bench lines of $BENCHES (host-to-host legs on for $E2E), rocprofv3 kernel
# traces of $TRACES, FETCH_SIZE / WRITE_SIZE passes of $PMCS (each pass a run of its own), then the
# N>1 rehearsal (every rank on GPU 0, gloo timing).  Every GPU step has its own time limit and the
# first failure ends the script.  tools/record_profiles.py <tag> <round> files the outputs.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd $R
if [ -z "$NOBUILD" ]; then
  timeout -k 10 600 make -s -B -j16 -C picotcp_amd/csrc > $O/build_$TAG.log 2>&1
  timeout -k 10 600 python -c "import __graft_entry__ as g; g.build(); print('build ok')" >> $O/build_$TAG.log 2>&1
  echo "build ok"
fi
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
  echo "tests ok"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1
  echo "smoke ok"
fi
for c in $BENCHES; do
  e2e=--no-e2e
  case " $E2E " in *" $c "*) e2e= ;; esac
  st=100; [ $c = c4 ] && st=20
  timeout -k 10 400 python bench.py --config $c --steps $st --warmup 10 $e2e > $O/bench_${c}_$TAG.json 2> $O/bench_${c}_$TAG.err
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
for c in $TRACES; do
  st=100; [ $c = c4 ] && st=20
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps $st --warmup 10 --no-cpu --no-e2e --no-verify > $O/prof_${c}_$TAG.log 2>&1
  echo "trace $c ok"
done
for c in $PMCS; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_fetch_${c}_$TAG.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_${c}_$TAG -o run --output-format csv -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_write_${c}_$TAG.log 2>&1
  echo "pmc $c ok"
done
cd $R
if [ -n "$MULTI" ]; then
  export PICO_BENCH_SAME_DEVICE=1 PICO_BENCH_DIST_BACKEND=gloo
  for spec in $MULTI; do        # <n>:<config>
    n=${spec%%:*}; c=${spec#*:}
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --config $c --steps 20 --warmup 3 > $O/bench_multi_${n}_${c}_$TAG.json 2> $O/bench_multi_${n}_${c}_$TAG.err
    echo "multi $n $c ok"
  done
fi
