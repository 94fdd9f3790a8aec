#!/bin/bash
# round 3, session 2: fused-MLP parity (with the deferred stage 3), smoke(), the multi-group vs
# per-group crossover (product lib vs a BCFFT_NO_DMG experiment build), MLP timing, MLP PMC traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03h_mlp_pytest.log 2>&1 || { tail -40 gpurun_out/r03h_mlp_pytest.log; exit 1; }
tail -3 gpurun_out/r03h_mlp_pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03h_smoke.log 2>&1 \
  || { cat gpurun_out/r03h_smoke.log; exit 1; }
cat gpurun_out/r03h_smoke.log | grep -v amdgpu.ids
timeout -k 10 180 python -u tools/time_mlp.py 1 20 256 1700 4096 8192 > gpurun_out/r03h_mlp_time.log 2>&1 \
  || { cat gpurun_out/r03h_mlp_time.log; exit 1; }
grep N gpurun_out/r03h_mlp_time.log
NS="1 8 20 64 128 256 512 768 1024 1536 2048 3072"
timeout -k 10 200 python -u tools/time_dmg_switch.py dmg $NS > gpurun_out/r03h_dmg_switch.log 2>&1 &&
BCFFT_LIB_PATH=$PWD/llama-fft_amd/lib/libbcfft_exp_nodmg.so timeout -k 10 200 python -u tools/time_dmg_switch.py nodmg $NS \
  >> gpurun_out/r03h_dmg_switch.log 2>&1 || { cat gpurun_out/r03h_dmg_switch.log; exit 1; }
grep N gpurun_out/r03h_dmg_switch.log
bash tools/pmc_mlp.sh
