set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_forward.py tests/test_gpu_ref_rx.py tests/test_gpu_far.py tests/test_abi.py tests/test_burst_driver.py tests/test_gpu_host_desc.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t_r04a.log 2>&1
echo "tests ok"
bash scripts/gpu_c1_repro.sh r04a
