# one GPU session: the GPU suite, interleaved A/Bs against the in-tree library of the round-3 stream
# kernels (picotcp_amd/ab/libpicocsum_r03.so) and of 8-wave workgroups (libpicocsum_wpb8.so)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r04a.log 2>&1
echo "tests ok"
A=r03 ROUNDS=2 CFGS="c2 c2slot c2v6 c2eth c2ethmix c2nat" bash scripts/gpu_ab.sh wg_r04a
echo "ab r03 ok"
A=wpb8 ROUNDS=2 CFGS="c2 c2slot" bash scripts/gpu_ab.sh wpb8_r04a
echo "ab wpb8 ok"
