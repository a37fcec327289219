#!/bin/bash
# 8 waves per workgroup in the sorted kernel (picotcp_amd/ab build) vs the product, interleaved processes.
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in 1 2 3; do
  for v in prod wpb8; do
    for c in c2 c2v6 c2eth c2tx; do
      if [ $v = prod ]; then unset PICO_CSUM_LIB; else export PICO_CSUM_LIB=$R/picotcp_amd/ab/libpicocsum_$v.so; fi
      timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 --no-cpu --no-e2e > $O/${c}_$v.$i.json 2>$O/err.txt
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_avg_us'])" $O/${c}_$v.$i.json "$c $v"
    done
  done
done
echo wpb ok
