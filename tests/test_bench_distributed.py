"""bench.py's multi-GPU path without a GPU: `--gpus 2` re-launches the script under
torch.distributed.run, and the two gloo ranks run the same partition / timing / all-gather core
(run_partitioned) as the RCCL ranks, on a CPU stand-in layer (tests/bench_stub.py)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import bench  # noqa: E402

ARGS = ["--stub", "bench_stub:cpu_forward", "--tokens", "200", "--in-features", "512", "--out-features", "256",
        "--block-size", "64", "--steps", "3", "--warmup", "1", "--variants", "0", "--cpu-budget", "0"]


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), env.get("PYTHONPATH", "")])
    env["OMP_NUM_THREADS"] = "1"
    return env


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("partition,per_rank,total,scaling", [(None, 100, 200, "strong"),
                                                              ("global", 100, 200, "strong"),
                                                              ("per-rank", 200, 400, "weak")])
def test_gpus2_launches_two_ranks(partition, per_rank, total, scaling):
    """partition None: the default, which must be SURVEY.md §8e's global split (strong scaling), with
    the per-rank (weak) reading beside it under `weak`."""
    part = [] if partition is None else ["--partition", partition]
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *part,
                          *ARGS], capture_output=True, text=True, timeout=300, env=_env())
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == scaling
    assert d["config"]["partition"] == (partition or "global")
    assert d["config"]["tokens_per_rank"] == per_rank and d["config"]["global_tokens"] == total
    assert d["value"] > 0 and d["ms_per_step"] > 0
    g = d["with_allgather"]
    assert g["ms_per_step"] >= d["ms_per_step"] * 0.5 and g["value"] > 0
    if scaling == "strong":
        w = d["weak"]
        assert w["scaling"] == "weak" and w["tokens_per_rank"] == 200 and w["value"] > 0
    else:
        assert "weak" not in d


def test_gpus4_global_partition():
    """Four gloo ranks, as the driver's N=4 scaling run: the global batch splits 4 ways."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--partition", "global",
                          *ARGS], capture_output=True, text=True, timeout=300, env=_env())
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out.stdout)
    assert d["n_gpus"] == 4 and d["scaling"] == "strong"
    assert d["config"]["tokens_per_rank"] == 50 and d["config"]["global_tokens"] == 200
    assert d["value"] > 0 and d["with_allgather"]["value"] > 0


def test_gpus1_single_process():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *ARGS],
                         capture_output=True, text=True, timeout=300, env=_env())
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out.stdout)
    assert d["n_gpus"] == 1 and "with_allgather" not in d and d["config"]["tokens_per_rank"] == 200


def test_world_size_must_match_gpus():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *ARGS],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr


def test_partition_and_spawn_command():
    assert bench.partition(8192, 8, 7, "global") == (1024, (7168, 8192), 8192)
    assert bench.partition(8192, 8, 7, "per-rank") == (8192, (7 * 8192, 8 * 8192), 65536)
    assert bench.partition(8191, 2, 1, "global") == (4095, (4096, 8191), 8191)
    cmd = bench.spawn_cmd(4, ["--gpus", "4"], 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-2:] == ["--gpus", "4"]
