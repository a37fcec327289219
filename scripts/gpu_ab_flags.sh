#!/bin/bash
# In-binary A/B of an ablation bit (PICO_CSUM_ABLATE) on the descriptor configs, separate
# processes, interleaved, after the GPU tests:  AB=8 CFGS="c2 c2v6" scripts/gpu_ab_flags.sh TAG
set -e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do
  for ab in 0 ${AB:-8}; do
    for cfg in ${CFGS:-c2 c2tx c2v6 c2eth}; do
      echo "ab=$ab $(PICO_CSUM_ABLATE=$ab timeout -k 10 180 python tools/sweep.py --config $cfg --rounds 3 --shapes ${SHAPES:-2,8,1,64,2} 2>&1 | grep -v amdgpu)"
    done
  done
done > $O/ab.txt 2>&1
cat $O/ab.txt
