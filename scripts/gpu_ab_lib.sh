#!/bin/bash
# A/B of two builds of libpicocsum in separate processes, interleaved (tools/sweep.py, same box):
#   ab/libpicocsum_base.so (the previous commit's build) vs picotcp_amd/libpicocsum.so.
#   scripts/gpu_ab_lib.sh TAG [tests] [ab] [pmc]
# Every GPU step has its own time limit; any failure ends the script.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
STEPS=${*:-"tests ab pmc"}
CFGS=${CFGS:-"c2 c2tx c2v6 c2raw"}
mkdir -p $O
cd $R
for s in $STEPS; do
case $s in
tests)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -1 $O/pytest_gpu.log ;;
ab)
  for rep in 1 2; do
    for lib in ab/libpicocsum_base.so picotcp_amd/libpicocsum.so; do
      for cfg in $CFGS; do
        echo "lib=$lib $(PICO_CSUM_LIB=$lib timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 3 --shapes ${SHAPES:-2,8,1,64,2} 2>&1 | grep -v amdgpu)"
      done
    done
  done > $O/ab.txt 2>&1
  cat $O/ab.txt ;;
pmc)
  cd /tmp && export TMPDIR=/tmp
  for lib in ab/libpicocsum_base.so picotcp_amd/libpicocsum.so; do
    t=$(basename $lib .so)
    PICO_CSUM_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      -d $O/pmc_sq_$t -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 20 --warmup 2 --no-cpu --no-e2e > $O/pmc_sq_$t.json 2> $O/pmc_sq_$t.err
  done
  cd $R
  echo "pmc ok" ;;
esac
done
