# bf16 DFT kernels: their GPU parity tests, then an interleaved A/B of library builds over the
# sweep's bf16 shapes (N = 8192). usage: bash tools/gpu_ab_bf16.sh TAG lib1 lib2 ...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_dmg.py tests/test_gpu_dm64g.py tests/test_gpu_dm64k.py tests/test_gpu_dmk.py tests/test_gpu_dm256.py tests/test_gpu_glu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "$@"; do
    echo "== $lib (pass $rep)"
    BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 200 python3 -u tools/time_algos.py dft --bf16all 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/$TAG/ab.log
tail -2 gpurun_out/$TAG/pytest.log; cat gpurun_out/$TAG/ab.log
