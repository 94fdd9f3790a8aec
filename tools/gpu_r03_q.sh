#!/bin/bash
# Round-3 evidence on one GPU: every -m gpu test, smoke(), the bench line, and the rocprofv3
# kernel-trace summary (CSV) of the same bench command, under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03q_final_pytest_gpu.log 2>&1 &&
tail -2 gpurun_out/r03q_final_pytest_gpu.log &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03q_final_smoke.log 2>&1 &&
tail -1 gpurun_out/r03q_final_smoke.log &&
timeout -k 10 400 python -u bench.py > gpurun_out/r03q_final_bench.log 2>&1 &&
tail -1 gpurun_out/r03q_final_bench.log | cut -c1-400 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r03q_final" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/r03q_final_bench_under_rocprof.log" 2>&1 &&
echo rocprof ok
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 600 python -u tools/model_bench.py > gpurun_out/r03q_model_bench.log 2>&1 &&
timeout -k 10 200 python -u tools/time_layer_projections.py > gpurun_out/r03q_layer.log 2>&1 &&
echo model ok
