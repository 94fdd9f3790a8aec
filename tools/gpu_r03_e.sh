set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_e_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r03_e_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r03_e_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r03_e_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); [print(v) for v in d.get("variants",[])]; print(d["value"], d["ms_per_step"], d["roofline"]["frac"])'
