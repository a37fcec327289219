#!/bin/bash
# Stamps of the uniform stream kernel (diag build) on C1- and C4-sized rings: per-XCD start / end spread.
set -o pipefail
mkdir -p gpurun_out
export PICO_CSUM_LIB=picotcp_amd/diag/libpicocsum_stamps.so
timeout -k 10 120 python -u tools/stamps.py --config c1stream > gpurun_out/stamps_c1stream.txt 2>&1 &&
timeout -k 10 120 python -u tools/stamps.py --config c4stream > gpurun_out/stamps_c4stream.txt 2>&1
