# dm64k: parity tests, then an interleaved A/B of library builds at 11008 -> 4096, b = 64 (N = 1700,
# 8192), then the stamps timeline of any lib named st_*. usage: bash tools/gpu_ab_dm64k.sh TAG lib1 lib2 ...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dm64k.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_dm64k.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_dm64k.log; exit 1; }
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "$@"; do
    case $lib in *st_*) continue;; esac
    echo "== $lib (pass $rep)"
    BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 120 python3 -u tools/time_algos.py dft --b64down 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/$TAG/ab.log
for lib in "$@"; do
  case $lib in *st_*) ;; *) continue;; esac
  echo "== $lib"
  BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 120 python3 -u tools/timeline_dm64k.py 8192 2>&1 | grep -v amdgpu.ids | grep -v "chunk [0245]" || exit 1
done > gpurun_out/$TAG/timeline.txt
cat gpurun_out/$TAG/ab.log gpurun_out/$TAG/timeline.txt
