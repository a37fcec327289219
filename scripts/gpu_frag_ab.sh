#!/bin/bash
# Reassembly gather A/B: 128-unit steps (product) vs 64-unit steps (picotcp_amd/ab build), both
# software-pipelined; frag GPU tests first; interleaved processes on one box.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_frag.py -x -q --timeout 120 --timeout-method thread > $O/pytest_frag.log 2>&1 || { tail -30 $O/pytest_frag.log; exit 1; }
tail -1 $O/pytest_frag.log
for i in 1 2 3; do
  for v in u2 u1 orig; do
    if [ $v = u2 ]; then unset PICO_CSUM_LIB; else export PICO_CSUM_LIB=$R/picotcp_amd/ab/libpicocsum_$v.so; fi
    timeout -k 10 200 python bench.py --config c3_reasm --steps 50 --warmup 5 --no-cpu --no-e2e > $O/c3r_$v.$i.json 2>$O/err.txt
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_avg_us'], d['value'])" $O/c3r_$v.$i.json $v
  done
done
echo frag ab ok
