#!/bin/bash
# Round 5 session l: the reassembly prologue variants (header copy from the parse's own loads; and
# the completeness check after the gather for one-wave datagrams) -- their GPU tests on the variant
# library, an interleaved A/B against the in-tree library -- then the final session's traces (part b).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
PICO_CSUM_LIB=$PWD/ablib/libpicocsum_h0c.so timeout -k 10 400 python -u -m pytest tests/test_gpu_frag.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_frag_h0c.log 2>&1
echo "frag tests (h0c) ok"
timeout -k 10 600 python tools/ab.py --tag r05l_reasm --configs c3_reasm,c3_reasm6 --rounds 2 --steps 50 \
    --variant "cur=" --variant "h0=ablib/libpicocsum_h0.so" --variant "h0c=ablib/libpicocsum_h0c.so"
echo "ab ok"
bash scripts/gpu_r05_final.sh b
