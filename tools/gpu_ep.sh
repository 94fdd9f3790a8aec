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
for lib in libbcfft_exp_late1.so libbcfft.so; do
  BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 120 python3 -u tools/dbg_dmk_late.py run >> gpurun_out/ep/late.txt 2>&1 || exit 1
done
for lib in libbcfft.so libbcfft_exp_ep2.so libbcfft_exp_ep6.so libbcfft_exp_ep2nsb.so libbcfft_exp_x8.so libbcfft_exp_x8ep2.so; do
  BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 150 python3 -u tools/precise_probe.py dftx dftp >> gpurun_out/ep/probe.txt 2>&1 || exit 1
done
for a in dftx dftp; do
  TIMELINE_LIB=libbcfft_exp_stdm.so TIMELINE_ALGO=$a timeout -k 10 120 python3 -u tools/timeline_dm.py 4096 fp32 8192 > gpurun_out/ep/timeline_$a.txt 2>&1 || exit 1
done
timeout -k 10 30 tools/probe/cvt_fp8 > gpurun_out/ep/cvt_fp8.txt 2>&1 || exit 1
