# Round-6 checkpoint: the GPU tests touched by this round's changes, then the precise-engine A/B
# (tools/precise_probe.py over the experiment libraries). One timeout per step; stop at a failure.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06a || exit 1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_0_north_star.py tests/test_gpu_dftp.py tests/test_gpu_dm256.py tests/test_gpu_dmk.py \
  tests/test_gpu_native_op.py tests/test_gpu_sn.py tests/test_gpu_rccl.py tests/test_gpu_model_dist.py \
  > gpurun_out/r06a/pytest.log 2>&1 || exit 1
for lib in libbcfft.so libbcfft_exp_x8fep2.so libbcfft_exp_x8fr8.so libbcfft_exp_x8fep2r8.so; do
  BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 150 python3 -u tools/precise_probe.py dftx dftp >> gpurun_out/r06a/probe.txt 2>&1 || exit 1
done
