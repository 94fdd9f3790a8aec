"""Token-sharded multi-GPU execution of the BC forward.

The forward is a per-token map (patch_llama_fft.py:226-275 treats every row independently), so
ranks split the token axis into contiguous shards and compute without any exchange; the only
collective is the optional all-gather of the output shards at the end (the north star's single
RCCL all-gather over xGMI; backend "nccl" is RCCL on ROCm). Spectra are replicated per rank.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n rows for rank: ceil-sized shards, the tail rank shorter."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    per = -(-n // world)
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def gather_rows(y_local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather row shards (rank order) into the full (n_total, ...) tensor on every rank.

    Shards are padded to the common ceil size so one all_gather_into_tensor moves everything."""
    world = dist.get_world_size(group)
    per = -(-n_total // world)
    if y_local.shape[0] < per:
        pad = y_local.new_zeros((per - y_local.shape[0],) + tuple(y_local.shape[1:]))
        y_local = torch.cat([y_local, pad], 0)
    out = y_local.new_empty((per * world,) + tuple(y_local.shape[1:]))
    if dist.get_backend(group) == "gloo":        # host-side tests: gloo has list all_gather
        dist.all_gather(list(out.chunk(world, 0)), y_local.contiguous(), group=group)
    else:
        dist.all_gather_into_tensor(out, y_local.contiguous(), group=group)
    return out[:n_total]


def sharded_forward(fn, x: torch.Tensor, group=None, gather: bool = True) -> torch.Tensor:
    """y = fn(x) computed token-sharded: this rank runs fn on its contiguous row shard of the
    (N, K) input; with gather=True every rank returns the full (N, M) output."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_bounds(x.shape[0], world, rank)
    y_local = fn(x[lo:hi])
    if not gather:
        return y_local
    return gather_rows(y_local, x.shape[0], group)
