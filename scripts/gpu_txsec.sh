#!/bin/bash
# Whole-sector TX crc stores: GPU suite (TX parity), then A/B vs 2-byte stores (PICO_CSUM_ABLATE=16)
# and vs no stores (4), interleaved processes on one box.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in c2tx c2eth_tx; do :; done
for i in 1 2 3; do
  for a in 0 16 4; do
    PICO_CSUM_ABLATE=$a timeout -k 10 200 python bench.py --config c2tx --steps 100 --warmup 10 --no-cpu --no-e2e > $O/c2tx_ab$a.$i.json 2>$O/err.txt
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us'])" $O/c2tx_ab$a.$i.json ablate=$a
  done
done
echo txsec ok
