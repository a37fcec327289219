#!/bin/bash
# Per-wave stamps (tools/stamps.py) of the diagnostic builds (make -C picotcp_amd/csrc diag; the
# round-3 one built from picotcp_amd/ab/r03): remove ./picotcp_amd/diag from .gpurunignore first,
# so the libraries travel to the box.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in stamps stamps_r03; do
  PICO_CSUM_LIB=$PWD/picotcp_amd/diag/libpicocsum_$v.so timeout -k 10 120 python tools/stamps.py --config c2 > gpurun_out/${v}_x1.txt 2>&1
  echo "$v ok"
done
