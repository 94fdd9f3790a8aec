"""Multi-process (gloo, world_size 2, CPU) coverage of the token-sharded path.

The per-shard compute here is the oracle (the checker; the HIP forward itself is covered by the
-m gpu parity tests): these tests pin the sharding and the gather — contiguous shards, ragged
tails, rank order — that bench.py and multi-GPU callers use.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
sys.path.insert(0, ROOT)

from bcfft.shard import shard_bounds  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, k, m, b, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bcfft.shard import sharded_forward
        from oracle.bc_oracle import bc_forward
        rng = np.random.default_rng(7)                      # same x and c on every rank
        x = torch.from_numpy(rng.standard_normal((n, k)).astype(np.float32))
        c = rng.standard_normal((m // b, k // b, b)).astype(np.float32) * 0.01
        fn = lambda xs: torch.from_numpy(np.ascontiguousarray(bc_forward(xs.numpy(), c, None)))  # noqa: E731
        y = sharded_forward(fn, x)
        y_local = sharded_forward(fn, x, gather=False)
        q.put((rank, y.numpy(), y_local.shape[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [64, 37, 1])
def test_sharded_forward_gloo_world2(n):
    world, k, m, b = 2, 256, 128, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, k, m, b, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.bc_oracle import bc_forward
    rng = np.random.default_rng(7)
    x = rng.standard_normal((n, k)).astype(np.float32)
    c = rng.standard_normal((m // b, k // b, b)).astype(np.float32) * 0.01
    ref = bc_forward(x, c, None)
    for rank, y, n_local in sorted(res, key=lambda r: r[0]):
        lo, hi = shard_bounds(n, world, rank)
        assert n_local == hi - lo
        assert y.shape == (n, m)
        np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-6)


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 8192, 8193):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, bnd), (c2, _) in zip(spans, spans[1:]):
                assert bnd == c2 and a <= bnd
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _logits_worker(rank, world, port, n_prompts, vocab, q):
    """model_bench's config-5 collective on gloo: each rank holds the last-token logits of its
    prompt slice (bc_eval.prompt_shard), gather_prompt_logits reassembles them in prompt order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bc_eval as E
        import model_bench as MB
        prompts = list(range(n_prompts))                    # stand-ins: prompt i's logits row is i
        mine = E.prompt_shard(prompts, world, rank)
        last = torch.stack([torch.full((vocab,), float(p)) for p in mine]) if mine else torch.zeros(0, vocab)
        q.put((rank, MB.gather_prompt_logits(last, n_prompts).numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_prompts", [100, 7])
def test_model_bench_logits_gather_gloo_world2(n_prompts):
    """tools/model_bench.py's distributed branch (BASELINE config 5: prompt replicas + ONE all-gather
    of last-token logits, bench_all_in_one.py:348-389) with two gloo ranks on the CPU."""
    world, vocab = 2, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_logits_worker, args=(r, world, port, n_prompts, vocab, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.repeat(np.arange(n_prompts, dtype=np.float32)[:, None], vocab, 1)
    for _, rows in res:
        np.testing.assert_array_equal(rows, want)
