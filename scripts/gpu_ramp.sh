#!/bin/bash
# Host-resident descriptor batches: chunk-size ramp vs fixed chunks (PICO_CSUM_NO_RAMP), C2 burst
# host-to-host rate, interleaved processes on one box; then the host-batch GPU tests.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_desc.py -x -q --timeout 120 --timeout-method thread > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
for i in 1 2 3; do
  for m in ramp fixed; do
    if [ $m = fixed ]; then export PICO_CSUM_NO_RAMP=1; else unset PICO_CSUM_NO_RAMP; fi
    timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu > $O/c2_$m.$i.json 2>$O/err.txt
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['e2e_host_to_host']['value'])" $O/c2_$m.$i.json $m
  done
done
echo ramp ok
