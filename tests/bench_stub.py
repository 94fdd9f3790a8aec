"""CPU stand-in for the BC layer in the gloo runs of bench.py's launcher and distributed timing
core (tests/test_bench_distributed.py): the oracle's torch-CPU restatement of the cached forward
(bench_all_in_one.py:179-231). Test infrastructure only; bench.py loads it only via --stub."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cpu_forward(k, m, b):
    from oracle.bc_oracle import torch_cpu_forward_cached
    g = torch.Generator().manual_seed(1)
    c = torch.randn(m // b, k // b, b, generator=g) * 0.01
    cf = torch.fft.rfft(c, dim=-1)
    return lambda x: torch_cpu_forward_cached(x, cf, None, b)
