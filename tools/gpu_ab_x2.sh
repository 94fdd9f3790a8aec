# (the bcfft_dm.hip switch this script measured was removed after its A/B; commit f61fd28 has it)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/x2 || exit 1
for L in libbcfft_exp_x21.so libbcfft_exp_x22.so; do
BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/$L timeout -k 10 400 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_0_north_star.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/x2/pytest_$L.log 2>&1 || exit 1
done
bash tools/ab_fp32.sh x2 "dftx dft" "" libbcfft_exp_x21.so libbcfft_exp_x22.so > /dev/null
