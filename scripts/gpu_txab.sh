#!/bin/bash
# TX write A/B (measurement only): 2-byte crc stores vs whole 32-byte sectors (PICO_CSUM_ABLATE=8)
# vs no writes (PICO_CSUM_ABLATE=4), interleaved processes on one box.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in 1 2 3; do
  for a in 0 8 4; do
    PICO_CSUM_ABLATE=$a timeout -k 10 200 python bench.py --config c2tx --steps 100 --warmup 10 --no-cpu --no-e2e > $O/c2tx_ab$a.$i.json 2>$O/err.txt
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us'])" $O/c2tx_ab$a.$i.json ablate=$a
  done
done
echo txab ok
