#!/bin/bash
# GPU tests, then an in-process A/B of the descriptor configs: PICO_CSUM_ABLATE=0 vs $AB,
# twice, interleaved.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
tail -1 $O/gputests.log
for rep in 1 2; do
  for ab in 0 ${AB:-16}; do
    for cfg in ${CFGS:-c2 c2tx c2v6 c2raw u576d c1d}; do
      echo "ab=$ab $(PICO_CSUM_ABLATE=$ab timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 3 --shapes ${SHAPES:-2,8,1,64,2} 2>&1 | grep -v amdgpu)"
    done
  done
done > $O/ab.txt 2>&1
cat $O/ab.txt
