set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/dmk
timeout -k 10 400 python -u -m pytest tests/test_gpu_dmk.py tests/test_gpu_dm64k.py tests/test_gpu_mlp.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/dmk/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/time_algos.py auto --downsmall > gpurun_out/dmk/downsmall.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_stream.py > gpurun_out/dmk/ab.log 2>&1
