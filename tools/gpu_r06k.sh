# precise engine after the cross-opcode SrcC fix: its parity tests (16-bit x and 16-bit bias forms
# included), the north-star dftp / precise cases, the round-5 16-bit-x failure case, and its time.
TAG=${1:-r06k}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dftp.py tests/test_gpu_0_north_star.py -k "dftp or precise" -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
timeout -k 10 120 python3 -u tools/dbg_ep9b.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$TAG/dbg_ep9b.txt || exit 1
timeout -k 10 150 python3 -u tools/precise_probe.py dftx dftp 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$TAG/probe.txt || exit 1
