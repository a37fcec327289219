#!/bin/bash
# Round 6, first probe: is C2's tail the per-wave byte spread?  balance_probe (product library)
# and the stamps of the diagnostic build on both layouts.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
timeout -k 10 240 python -u tools/balance_probe.py --rounds 5 > $O/balance_probe.txt 2>&1
timeout -k 10 120 python -u tools/stamps.py --config c2 > $O/stamps_c2.txt 2>&1
timeout -k 10 120 python -u tools/stamps.py --config c2 --balanced > $O/stamps_c2_balanced.txt 2>&1
cat $O/balance_probe.txt
