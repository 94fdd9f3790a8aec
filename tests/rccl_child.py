"""Child process of tests/test_gpu_rccl.py (not a test module): run under
`python -m torch.distributed.run --nproc-per-node 1`, so the RCCL process group is created in a
fresh process before anything touches the GPU, exactly as bench.py's ranks and the driver's
scaling run create theirs:

  * dist.init_process_group("nccl", device_id=...) (backend "nccl" is RCCL on ROCm),
    dist.barrier(device_ids=[local]);
  * bcfft.shard.sharded_forward with the HIP engine + gather_rows (device all_gather_into_tensor),
    checked against the oracle, on a ragged token count;
  * bench.run_partitioned with allgather=1 (the timed core of every bench rank: barriers,
    all_reduce MAX of the timings, the gather-inclusive loop).

Prints one line `RCCL_OK {json}` on success; any failure raises (non-zero exit)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "llama-fft_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    local = int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl"
    barrier = lambda: dist.barrier(device_ids=[local])  # noqa: E731
    barrier()

    import bench
    from bcfft.shard import gather_rows, sharded_forward
    from oracle import bc_oracle as O
    from patch_llama_fft import BlockCirculantLinear

    rng = np.random.default_rng(7)
    n, k = 1003, 4096                                   # ragged: not a multiple of any tile
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(k) * 0.1).astype(np.float32)
    x = rng.standard_normal((n, k)).astype(np.float32)
    layer = BlockCirculantLinear(k, k, block_size=128, bias=True)
    with torch.no_grad():
        layer.c.copy_(torch.from_numpy(c))
        layer.bias.copy_(torch.from_numpy(bv))
    layer = layer.to(dev).eval()
    xd = torch.from_numpy(x).to(dev)
    with torch.inference_mode():
        y = sharded_forward(layer, xd)                   # shard + RCCL all_gather_into_tensor
        # a second gather of another size; 600 tokens keep AUTO on the engine of the 1003-token
        # call (bit-equal rows) ...
        y2 = gather_rows(layer(xd[:600]), 600)
        # ... and a sub-threshold shard (500 tokens: AUTO takes the short-N kernel while its grid
        # fits one round of CUs, whose roundings differ from dftx's): AUTO results are not
        # batch-size invariant, so this gather is compared with the engines'
        # mutual tolerance, not bit for bit
        y3 = gather_rows(layer(xd[:500]), 500)
    torch.cuda.synchronize()
    ref = O.bc_forward(x, c, bv)
    g = y.cpu().numpy()
    err = float(np.linalg.norm(g - ref) / np.linalg.norm(ref))
    assert y.shape == (n, k) and err < 6e-4, err
    assert torch.equal(y2, y[:600])
    d3 = float(torch.linalg.norm(y3 - y[:500]) / torch.linalg.norm(y[:500]))
    assert y3.shape == (500, k) and d3 < 2e-5, d3

    r = bench.run_partitioned(layer, xd, n, 3, 1, 1, barrier, dev, settle_ms=0.0, allgather=True, repeats=2)
    assert r["gather_wall"] is not None and r["gather_wall"] > 0 and r["wall"] > 0, r
    print("RCCL_OK " + json.dumps({"backend": dist.get_backend(), "rel_err": err, "sub_threshold_rel": d3, "world": dist.get_world_size(),
                                   "wall_ms": r["wall"], "gather_wall_ms": r["gather_wall"],
                                   "rccl_version": ".".join(map(str, torch.cuda.nccl.version()))
                                   if hasattr(torch.cuda, "nccl") else None}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
