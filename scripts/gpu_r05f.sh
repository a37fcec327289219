#!/bin/bash
# Round 5 session f: the uniform-stream rule on its bench lines, the reassembly locality experiment
# (datagram-major vs interleaved arrival), the host-resident C2 path (3 staging slots vs round 4),
# the C2 line with the reference-callers CPU baseline and both host legs.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_uniform_stream.py tests/test_gpu_host_desc.py tests/test_gpu_zerocopy.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_f_r05f.log 2>&1
echo "tests ok"
for c in c3 c3_64k c4 c1; do
  st=50; [ $c = c4 ] && st=20
  timeout -k 10 400 python bench.py --config $c --steps $st --warmup 5 --no-e2e > gpurun_out/bench_${c}_r05f.json 2> gpurun_out/bench_${c}_r05f.err
  echo "bench $c ok"
done
timeout -k 10 400 python bench.py --config c2 --steps 100 --warmup 10 > gpurun_out/bench_c2_r05f.json 2> gpurun_out/bench_c2_r05f.err
echo "bench c2 ok"
timeout -k 10 500 python tools/ab.py --tag r05f_il --configs c3_reasm,c3_reasm_il --rounds 2 --steps 30 --variant new=
echo "ab il ok"
for v in new r04; do
  lib=; [ $v = r04 ] && lib=picotcp_amd/ab/libpicocsum_r04.so
  PICO_CSUM_LIB=${lib:+$PWD/$lib} timeout -k 10 300 python tools/host_e2e.py --stagings 16 32 64 --rounds 2 > gpurun_out/host_e2e_${v}_r05f.txt 2>&1
  echo "host $v ok"
done
