"""Config 5's distributed branch of tools/model_bench.py on the GPU (BASELINE config 5, SURVEY.md
§8e; reference src/bench_all_in_one.py:348-389): a fresh `torch.distributed.run --nproc-per-node 1`
child creates the RCCL ("nccl") group with device_id before it touches the GPU, runs the prompt
shard, the patched prefill and the single all-gather of the last-token logits; its gathered logits
must equal a plain single-process run of the same harness bit for bit (one rank holds every
prompt, and the BC kernels are deterministic). The 8-rank run itself is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

ARGS = ["--layers", "2", "--prompts", "7", "--max-len", "40", "--batch-size", "3", "--runs", "1", "--warmup", "0",
        "--new-tokens", "0", "--dense", "0", "--block-sizes", "128", "--config-overrides",
        '{"hidden_size": 1024, "intermediate_size": 2816, "num_attention_heads": 8, '
        '"num_key_value_heads": 8, "vocab_size": 512}']


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_model_bench_distributed_branch_matches_single_process(tmp_path):
    pytest.importorskip("transformers")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    script = os.path.join(ROOT, "tools", "model_bench.py")
    single = tmp_path / "single.pt"
    out1 = subprocess.run([sys.executable, script, *ARGS, "--dump-logits", str(single)],
                          capture_output=True, text=True, timeout=300, env=env)
    assert out1.returncode == 0, (out1.stdout[-2000:], out1.stderr[-4000:])
    l1 = _line(out1.stdout)
    assert "allgather_logits_ms" not in l1                     # no launcher: no process group
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist_pt = tmp_path / "dist.pt"
    out2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                           "--master-addr=127.0.0.1", f"--master-port={port}", script, *ARGS,
                           "--dump-logits", str(dist_pt)],
                          capture_output=True, text=True, timeout=300, env=env)
    assert out2.returncode == 0, (out2.stdout[-2000:], out2.stderr[-4000:])
    l2 = _line(out2.stdout)
    assert l2["n_gpus"] == 1 and l2["allgather_logits_ms"] > 0 and l2["value_with_allgather"] > 0
    assert l2["config"]["tokens"] == l1["config"]["tokens"]
    a = torch.load(single, weights_only=True)
    b = torch.load(dist_pt, weights_only=True)
    assert b["world"] == 1 and b["student_last"].shape == (7, 512)
    assert torch.equal(a["student_last"], b["student_last"])   # the gathered logits, prompt order
    assert torch.equal(a["teacher_last_local"], b["teacher_last_local"])


def test_model_bench_two_ranks_one_gpu_match_single_process(tmp_path):
    """Config 5 at world size 2 through the real BC kernels (verdict r5 item 6): a fresh
    `torch.distributed.run --nproc-per-node 2` child, both ranks on cuda:0 (RCCL refuses two ranks
    on one device, so the group is gloo and the last-token logits are gathered from host copies),
    each rank prefilling its contiguous prompt shard through the patched model. 8 prompts in
    batches of 2 give both runs the same batches, so the gathered logits must equal the
    single-process run bit for bit (deterministic kernels on identical launches)."""
    pytest.importorskip("transformers")
    args = [a for a in ARGS]
    args[args.index("--prompts") + 1] = "8"
    args[args.index("--batch-size") + 1] = "2"
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    script = os.path.join(ROOT, "tools", "model_bench.py")
    single = tmp_path / "single.pt"
    out1 = subprocess.run([sys.executable, script, *args, "--dump-logits", str(single)],
                          capture_output=True, text=True, timeout=300, env=env)
    assert out1.returncode == 0, (out1.stdout[-2000:], out1.stderr[-4000:])
    l1 = _line(out1.stdout)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist_pt = tmp_path / "dist2.pt"
    out2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                           "--master-addr=127.0.0.1", f"--master-port={port}", script, *args,
                           "--backend", "gloo", "--dump-logits", str(dist_pt)],
                          capture_output=True, text=True, timeout=300, env=env)
    assert out2.returncode == 0, (out2.stdout[-2000:], out2.stderr[-4000:])
    l2 = _line(out2.stdout)
    assert l2["n_gpus"] == 2 and l2["allgather_logits_ms"] > 0
    assert l2["config"]["tokens"] == l1["config"]["tokens"]      # the shards cover every prompt once
    a = torch.load(single, weights_only=True)
    b = torch.load(dist_pt, weights_only=True)
    assert b["world"] == 2 and b["student_last"].shape == (8, 512)
    assert torch.equal(a["student_last"], b["student_last"])     # gathered in prompt order, bit-equal
