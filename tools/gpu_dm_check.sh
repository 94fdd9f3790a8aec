# DFT-kernel parity (dft / dftx / dftp / GLU / native ops) and the fp32 headline timings of the product library
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/clean || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_dftp.py tests/test_gpu_0_north_star.py tests/test_gpu_glu.py tests/test_gpu_native_op.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/clean/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/time_algos.py dftx dft dftp --fp32n > gpurun_out/clean/time.log 2>&1
