# dm8 A/B: parity of a library build (the bf16 DFT / GLU tests and the bf16 north star), then an
# interleaved timing of the bf16 K = 4096 DFT kernels against the product library.
# usage: bash tools/gpu_ab_dm8.sh TAG lib
TAG=$1; LIB=$2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
BCFFT_LIB_PATH=llama-fft_amd/lib/${TESTLIB:-$LIB} timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dft.py tests/test_gpu_glu.py tests/test_gpu_0_north_star.py -k "bf16 or dft8 or glu or dft64 or dm64" -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
for rep in 1 2 3; do
  for lib in libbcfft.so $LIB; do
    echo "== $lib (pass $rep)"
    BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 120 python3 -u tools/time_algos.py dft --pipe 2>&1 | grep -v amdgpu.ids || exit 1
  done
done | tee gpurun_out/$TAG/ab.log
