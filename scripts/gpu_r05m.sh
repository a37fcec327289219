#!/bin/bash
# Round 5 session m: the reassembly kernel priced against the bare gather of its batch and the
# device's sequential copy (tools/gather_ceiling.py), then the final session's PMC passes (part c).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for v in "" "--v6" "--interleave"; do
  timeout -k 10 300 python tools/gather_ceiling.py $v >> gpurun_out/gather_ceiling_r05m.txt 2> gpurun_out/gather_ceiling_r05m.err
  echo "gather ceiling $v ok"
done
bash scripts/gpu_r05_final.sh c
