# (the bcfft_dm.hip switch this script measured was removed after its A/B; commit f61fd28 has it)
# The symmetric P1 schedule (BCFFT_DM_SYM=1, libbcfft_exp_sym.so): DFT-kernel parity on that
# library, then the interleaved fp32 headline A/B against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/sym || exit 1
BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/libbcfft_exp_sym.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_0_north_star.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/sym/pytest_gpu.log 2>&1 &&
bash tools/ab_fp32.sh sym "dftx dft" "" libbcfft_exp_sym.so > /dev/null
