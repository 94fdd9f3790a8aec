# fp32 headline engines (dftx, dft) and the 1024-token shard, interleaved A/B of library builds,
# after the headline parity tests. usage: bash tools/gpu_ab_fp32.sh TAG lib1 lib2 ...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_0_north_star.py tests/test_gpu_dft.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
for rep in 1 2 3; do
  for lib in "$@"; do
    echo "== $lib (pass $rep)"
    BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 120 python3 -u tools/time_algos.py dftx dft --fp32n 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/$TAG/ab.log
tail -3 gpurun_out/$TAG/pytest.log; cat gpurun_out/$TAG/ab.log
