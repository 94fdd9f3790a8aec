# A/B of the precise engine's residual terms (EP) and the dmk late-DMA reproduction (analysis builds;
# DESIGN.md sections 6b / 6c). Every step under its own timeout; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ep || exit 1
for lib in libbcfft_exp_late1.so libbcfft_exp_late2.so libbcfft.so; do
  echo "== $lib" >> gpurun_out/ep/late.txt
  BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 180 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    "tests/test_gpu_dmk.py::test_dmk_per_token_chunk_scales" >> gpurun_out/ep/late.txt 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/ep/late.txt
  [ $rc -ge 124 ] && exit $rc
done
for lib in libbcfft.so libbcfft_exp_ep2.so libbcfft_exp_ep6.so libbcfft_exp_ep2nsb.so; do
  BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 150 python3 -u tools/precise_probe.py dftx dftp >> gpurun_out/ep/probe.txt 2>&1 || exit 1
done
