#!/bin/bash
# Per-wave stamps (tools/stamps.py) of the diagnostic build (make -C picotcp_amd/csrc diag): remove
# ./picotcp_amd/diag from .gpurunignore first, so the library travels to the box.
#   scripts/gpu_stamps.sh [config ...]      (default: c2; c1stream / c4stream: the uniform rings'
#                                            stream waves, profiles/r05/stamps_c*stream.txt)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for c in ${@:-c2}; do
  PICO_CSUM_LIB=$PWD/picotcp_amd/diag/libpicocsum_stamps.so timeout -k 10 120 python -u tools/stamps.py --config $c > gpurun_out/stamps_$c.txt 2>&1
  echo "$c ok"
done
