# interleaved A/B of library builds with tools/ab_stream.py. usage: bash tools/ab_stream.sh TAG lib1 lib2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=$1; shift
for round in 1 2; do
  for L in "$@"; do
    echo "== ${L:-product} round $round" >> gpurun_out/abs_$TAG.log
    BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/${L:-libbcfft.so} timeout -k 10 240 python3 -u tools/ab_stream.py >> gpurun_out/abs_$TAG.log 2>&1 || exit 1
  done
done
