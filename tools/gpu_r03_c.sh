set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_0_north_star.py tests/test_gpu_dmg.py -x -v --timeout 200 --timeout-method thread -s > gpurun_out/r03_c_pytest_new.log 2>&1
rc=$?; tail -3 gpurun_out/r03_c_pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_c_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r03_c_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r03_c_bench.log 2>&1 || exit 1
BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/libbcfft_exp_nodmg.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 > gpurun_out/r03_c_bench_nodmg.log 2>&1
