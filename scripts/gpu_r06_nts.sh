#!/bin/bash
# Round 6: non-temporal stores in the reassembly gather -- the copy ceiling with nt stores, then an
# interleaved A/B of ablib/libpicocsum_{nts,ntsall}.so against the in-tree library.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
timeout -k 10 300 python tools/gather_ceiling.py > $O/gather_ceiling_nts.txt 2>&1
timeout -k 10 300 python tools/gather_ceiling.py --v6 >> $O/gather_ceiling_nts.txt 2>&1
grep '^{' $O/gather_ceiling_nts.txt
A="${A:-nts ntsall}" CFGS="${CFGS:-c3_reasm c3_reasm6}" STEPS=100 VERIFY="--rotate 0" ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab.sh ${TAG:-reasm_nts}
