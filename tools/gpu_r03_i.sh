#!/bin/bash
# round 3, session 2: the multi-group switch (dmg rule in the product lib) re-checked, the b = 64 /
# b = 256 multi-group crossover, and the MLP tests on the switched AUTO paths
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_glu.py tests/test_gpu_dmg.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03i_pytest.log 2>&1 || { tail -40 gpurun_out/r03i_pytest.log; exit 1; }
tail -2 gpurun_out/r03i_pytest.log
NS="1 20 128 256 512 768 1024 1536 2048 3072"
timeout -k 10 200 python -u tools/time_dmg_switch.py rule $NS > gpurun_out/r03i_dmg_rule.log 2>&1 || { cat gpurun_out/r03i_dmg_rule.log; exit 1; }
grep N gpurun_out/r03i_dmg_rule.log
timeout -k 10 200 python -u tools/time_mg_switch.py mg $NS > gpurun_out/r03i_mg_switch.log 2>&1 &&
BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/libbcfft_exp_nomg.so timeout -k 10 200 python -u tools/time_mg_switch.py nomg $NS \
  >> gpurun_out/r03i_mg_switch.log 2>&1 || { cat gpurun_out/r03i_mg_switch.log; exit 1; }
grep N gpurun_out/r03i_mg_switch.log
