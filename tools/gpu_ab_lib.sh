set -o pipefail
TAG=$1; LIB=$2   # usage: bash tools/gpu_ab_lib.sh TAG libbcfft_exp_<name>.so: DFT parity on that library, then the fp32 A/B vs the product
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/${TAG} || exit 1
BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/$LIB timeout -k 10 400 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_0_north_star.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}/pytest_gpu.log 2>&1 &&
bash tools/ab_fp32.sh ${TAG} "dftx dft" "" $LIB > /dev/null
