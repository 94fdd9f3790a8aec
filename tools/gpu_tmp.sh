cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r05n || exit 1
BCFFT_LIB_PATH=llama-fft_amd/lib/libbcfft_exp_st_dm8.so timeout -k 10 120 python3 -u tools/timeline_dm8.py 8192 2>&1 | grep -v amdgpu.ids > gpurun_out/r05n/timeline_dm8.txt || exit 1
cat gpurun_out/r05n/timeline_dm8.txt
