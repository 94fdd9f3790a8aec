# precise-engine session: its GPU tests, then the bench line under BCFFT_ALGO=dftp and dftx
set -o pipefail
TAG=${1:-dftp}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_op.py tests/test_gpu_dftp.py tests/test_gpu_dft.py "tests/test_gpu_0_north_star.py" -m gpu -x -v --timeout 150 --timeout-method thread -s > gpurun_out/$TAG/pytest_gpu.log 2>&1 &&
BCFFT_ALGO=dftp timeout -k 10 300 python -u bench.py --variants 0 --cpu-budget 0 > gpurun_out/$TAG/bench_dftp.json 2> gpurun_out/$TAG/bench_dftp.err &&
BCFFT_ALGO=dftx timeout -k 10 300 python -u bench.py --variants 0 --cpu-budget 0 > gpurun_out/$TAG/bench_dftx.json 2> gpurun_out/$TAG/bench_dftx.err &&
BCFFT_ALGO=dftx timeout -k 10 300 python -u bench.py --variants 0 --cpu-budget 0 --bias 1 > gpurun_out/$TAG/bench_dftx_bias.json 2> gpurun_out/$TAG/bench_dftx_bias.err &&
for a in dftx dftp; do TIMELINE_ALGO=$a timeout -k 10 120 python -u tools/timeline_dm.py 4096 fp32 8192 > gpurun_out/$TAG/timeline_$a.txt 2>&1 || exit 1; done &&
bash tools/ab_fp32.sh lw_$TAG "dftx dftp" "" libbcfft_exp_lw0.so libbcfft_exp_ex0.so > /dev/null
