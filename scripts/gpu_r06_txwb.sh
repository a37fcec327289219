#!/bin/bash
# Round 6: in-place TX as whole 16-byte head-window chunks (ablib/libpicocsum_txwb.so, -DPICO_TX_CHUNK_WB)
# against the product's 2-byte field stores: the TX tests on the variant, an interleaved A/B, and
# WRITE_SIZE / FETCH_SIZE passes of c2tx for both.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
PICO_CSUM_LIB=$R/ablib/libpicocsum_txwb.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ref_tx.py tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_nat.py > $O/pytest_txwb.txt 2>&1 || { tail -30 $O/pytest_txwb.txt; exit 1; }
tail -2 $O/pytest_txwb.txt
A="txwb" CFGS="c2tx c2tx_nw" STEPS=100 VERIFY="--rotate 0" ROUNDS=3 bash scripts/gpu_ab.sh txwb
cd /tmp && export TMPDIR=/tmp
for v in txwb new; do
  lib=$R/picotcp_amd/libpicocsum.so
  [ $v != new ] && lib=$R/ablib/libpicocsum_$v.so
  for set in "WRITE_SIZE GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE"; do
    n=$(echo $set | cut -d' ' -f1)
    PICO_CSUM_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $set -d $O/pmc_txwb_${n}_$v -o run --output-format csv -- python3 $R/bench.py --config c2tx --steps 10 --warmup 2 --no-cpu --no-e2e --no-verify > $O/pmc_txwb_${n}_$v.log 2>&1
  done
done
echo pmc ok
