#!/bin/bash
# Round-end evidence on one GPU: every -m gpu test, smoke(), the bench line, and rocprofv3
# kernel-trace summaries (CSV) of bench.py and of tools/time_grad_prep.py under gpurun_out/,
# and the model-level line of tools/model_bench.py (BASELINE configs 3/5).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python -u tools/model_bench.py > gpurun_out/model_bench_1gpu.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/bench_under_rocprof.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_grad" -o run -- python3 "$GRAFT_REPO_ROOT/tools/time_grad_prep.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_grad.log" 2>&1
