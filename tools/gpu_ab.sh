# correctness of the DFT kernels, then an interleaved A/B of library builds at the fp32 headline
# and its 1024-token shard. usage: bash tools/gpu_ab.sh TAG "algos" lib1 lib2 ...
set -o pipefail
TAG=$1; ALGOS=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dft.py tests/test_gpu_dftp.py tests/test_gpu_glu.py tests/test_gpu_0_north_star.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 &&
bash tools/ab_fp32.sh ab_$TAG "$ALGOS" "$@" > /dev/null
