"""The RCCL path on the GPU: a fresh child process under torch.distributed.run
creates the "nccl" (= RCCL) process group with device_id before touching the GPU, runs the
token-sharded forward with the device all-gather and bench.py's timed core, and checks the result
against the oracle (tests/rccl_child.py). One GPU, one rank: the multi-rank curve is the driver's
8-GPU run; this proves the code it executes (init, barrier, all_reduce, all_gather_into_tensor)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_rccl_sharded_forward_and_bench_core():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tests", "rccl_child.py")]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-4000:])
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("RCCL_OK ")]
    assert len(lines) == 1, out.stdout[-2000:]
    print(lines[0])
