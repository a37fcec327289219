#!/bin/bash
# C2 phase ablation on the final binary (PICO_CSUM_ABLATE: 1 skip the rounds, 2 skip the head
# windows, 3 both), interleaved processes; plus the raw-layout C2 for reference.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in 1 2 3; do
  for a in 0 1 2 3; do
    PICO_CSUM_ABLATE=$a timeout -k 10 200 python bench.py --config c2 --steps 100 --warmup 10 --no-cpu --no-e2e > $O/c2_ab$a.$i.json 2>$O/err.txt
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_avg_us'])" $O/c2_ab$a.$i.json "ablate=$a"
  done
done
echo phase ok
