# one GPU session: the GPU suite, an interleaved A/B of the round-3 stream kernels (picotcp_amd/ab/
# libpicocsum_r03.so) against the in-tree library, the C1 roofline reproducibility runs
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r04a.log 2>&1
echo "tests ok"
A=r03 ROUNDS=3 CFGS="c2 c2slot c2v6 c2eth c2nat c2tx" bash scripts/gpu_ab.sh wg_r04a
echo "ab ok"
bash scripts/gpu_c1_repro.sh r04a
