# precise-engine experiment libraries (lib/libbcfft_exp_<name>.so) through tools/check_dftp.py
mkdir -p gpurun_out/p3
for v in "$@"; do
  QUICK=1 BCFFT_LIB_PATH=$GRAFT_REPO_ROOT/llama-fft_amd/lib/libbcfft_exp_$v.so timeout -k 10 120 python -u tools/check_dftp.py > gpurun_out/p3/$v.txt 2>&1 || exit 1
done
