# the whole GPU suite (one process), then optional extra commands. usage: bash tools/gpu_full.sh TAG
TAG=$1
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/$TAG/pytest_gpu.log
exit $rc
