#!/bin/bash
# round 3: fused BC-MLP parity + timing (tests/test_gpu_mlp.py, tools/time_mlp.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03_mlp_pytest.log 2>&1 || { tail -40 gpurun_out/r03_mlp_pytest.log; exit 1; }
tail -5 gpurun_out/r03_mlp_pytest.log
timeout -k 10 180 python -u tools/time_mlp.py 1 20 256 1700 4096 8192 > gpurun_out/r03_mlp_time.log 2>&1 \
  || { cat gpurun_out/r03_mlp_time.log; exit 1; }
cat gpurun_out/r03_mlp_time.log
