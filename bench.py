#!/usr/bin/env python3
"""Benchmark of the MI355X block-circulant (BC) linear forward — BASELINE.json's metric.

Workload (north star / metric): one BlockCirculantLinear forward, 4096 -> 4096, b = 128,
N = batch*seq = 8192 tokens per GPU, fp32 I/O (the reference's fp32 path), weight spectra
precomputed outside the timed region (the reference's cache_cfft=1 perf convention,
bench_all_in_one.py:484). A "step" = one forward over the rank's 8192-token shard.

Multi-GPU: one process per GPU (torch.distributed.run); tokens are sharded, each rank runs
its own 8192-token shard (weak scaling) with no collective in the data path. With
--allgather the single RCCL all-gather of the output shards (north star) is timed in a
second loop and reported as `with_allgather`.

Prints ONE JSON line on rank 0. `roofline.achieved` = algorithmic bytes per launch
(N*K*s_x + N*M*s_y + nO*nI*(b/2+1)*8 [+ M*s_bias]) / the kernel's average
duration measured with HIP events on the launch stream. `roofline.traffic` = HBM bytes per
launch from rocprofv3 PMC counters (profiles/pmc_traffic_*.json, written by
tools/pmc_traffic.py) or null. `cpu_baseline` times the oracle's torch-CPU restatement
(oracle/bc_oracle.py) on a bounded token sample on the host cores.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP32_VALU_TFLOPS = 157.3     # beside it: the FP32 vector ceiling (intensity straddles the ridge)
METRIC = "BC-linear GTok-elem/s + GB/s vs roofline, b=128 4096→4096, 1/2/4/8 GPU"
DT = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}
SZ = {"fp32": 4, "bf16": 2, "fp16": 2}


def algo_bytes(n, k, m, b, io, bias):
    n_out, n_in = m // b, k // b
    return n * k * SZ[io] + n * m * SZ[io] + n_out * n_in * (b // 2 + 1) * 8 + (m * SZ[io] if bias else 0)


def resolved_kernel(algo, k, b, io="fp32"):
    """(algorithm, kernel symbol, MAC arithmetic) that BCFFT_ALGO=algo runs for this geometry and
    I/O dtype; mirrors bcfft_forward_algo's AUTO rule (csrc/bcfft_kernels.hip)."""
    n_in = k // b
    stat_ok = (b == 128 and n_in == 32) or (b == 64 and n_in in (32, 64))
    dft_ok = b == 128 and n_in == 32
    if io == "bf16" and algo in ("dft", "auto") and b == 64 and n_in == 64:
        return ("dft", "bc_forward_dm64_kernel",
                "MFMA fp16 throughout, b=64, 8 tokens per tile, one-term spectra (bf16 I/O)")
    if io == "bf16" and algo in ("dft", "auto") and dft_ok:
        return ("dft", "bc_forward_dm8_kernel",
                "MFMA fp16 throughout, 8 tokens per tile, one-term spectra (bf16 I/O)")
    if io == "bf16" and algo in ("dft", "auto") and b == 128 and 32 < n_in <= 127:   # N >= 32 (bench: 8192)
        return ("dft", "bc_forward_dmk_kernel",
                "MFMA fp16 throughout, 16-block K-chunks with weight fragments streamed from L2 (bf16 I/O)")
    if algo == "dftx":
        return ("dftx", "bc_forward_dm_kernel",
                "MFMA fp16 throughout: block DFT (even/odd split, x hi+lo) x 2^-7 table, stationary "
                "conj(C)*s_C MAC (X hi+lo), inverse DFT of Y hi+lo; f32 accumulate")
    if algo == "dft" or (algo == "auto" and dft_ok):
        return ("dft", "bc_forward_dm_kernel",
                "MFMA fp16 throughout: block DFT (even/odd split, x hi+lo) x 2^-7 table, stationary "
                "conj(C)*s_C MAC (X hi+lo), inverse DFT (Y one fp16 term); f32 accumulate")
    if algo == "stationary" or (algo == "auto" and stat_ok):
        return ("stationary", "bc_forward_stat_kernel",
                "MFMA fp16: conj(C)*s_C (VGPR-resident) x per-token-scaled X split hi+lo, f32 accumulate")
    if algo == "mfma" or (algo == "auto" and b <= 128):
        return ("mfma", "bc_forward_mfma_kernel",
                "MFMA bf16 hi/lo split (Xhi+Xlo)(Chi+Clo), f32 accumulate")
    return ("valu", "bc_forward_valu_kernel", "VALU fp32 FMA")


def algo_flops(n, k, m, b):
    import math
    n_out, n_in = m // b, k // b
    return n * (8 * n_out * n_in * (b // 2 + 1) + (n_in + n_out) * 2.5 * b * math.log2(b))


def make_layer(k, m, b, io, bias, dev, seed=1):
    from patch_llama_fft import BlockCirculantLinear
    torch.manual_seed(seed)                                   # c ~ 0.01 N(0,1), seed 1 (§8d)
    layer = BlockCirculantLinear(k, m, block_size=b, bias=bias)
    if bias:
        with torch.no_grad():
            layer.bias.normal_(0.0, 0.1)
    return layer.to(dev).to(DT[io]).eval()


def settle(layer, x, ms):
    """Run the forward back to back for at least `ms` milliseconds of wall time (untimed)."""
    t0 = time.perf_counter()
    with torch.inference_mode():
        while (time.perf_counter() - t0) * 1e3 < ms:
            for _ in range(20):
                layer(x)
            torch.cuda.synchronize()


def time_layer(layer, x, steps, warmup, barrier=None):
    """Returns (wall ms per step over the bracketed region, mean kernel ms per launch from HIP
    events). One event pair brackets all K back-to-back launches on the launch stream: a pair
    around EACH launch adds its own marker latency (~6 us per step measured on MI355X, see
    tools/event_timing.py), while K launches back to back give the launch duration plus the
    inter-kernel gap, within ~2-3 % of rocprofv3's per-kernel average."""
    stream = torch.cuda.current_stream()
    with torch.inference_mode():
        layer._spectra(layer.c)                                # spectra outside timing
        for _ in range(warmup):
            layer(x)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if barrier:
            barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.record(stream)
        for _ in range(steps):
            layer(x)
        e.record(stream)
        torch.cuda.synchronize()
        if barrier:
            barrier()
        wall = (time.perf_counter() - t0) * 1e3 / steps
    kern = s.elapsed_time(e) / steps
    return wall, kern


def time_spectra(layer, iters=20):
    """Spectra precompute (rfft(c) + the engines' operand images), ms per call: reported
    separately, outside the forward's timed region (the cache_cfft=1 convention)."""
    from bcfft import ops
    with torch.inference_mode():
        ops.spectra(layer.c)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            ops.spectra(layer.c)
        e.record()
        torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def time_glu(dev, steps, k=4096, m=11008, b=128, n=8192, io="bf16"):
    """Config 2's gate/up pair of a BC LLaMA MLP: h = silu(gate(x)) * up(x) as ONE fused launch
    (bcfft_forward_glu) vs the unfused sequence (two BC forwards + torch SiLU and product)."""
    from bcfft import ops
    torch.manual_seed(2)
    cg = (torch.randn(m // b, k // b, b, device=dev) * 0.01).to(DT[io])
    cu = (torch.randn(m // b, k // b, b, device=dev) * 0.01).to(DT[io])
    x = torch.randn(n, k, device=dev).to(DT[io])
    sgu, sg, su = ops.spectra(ops.glu_weights(cg, cu)), ops.spectra(cg), ops.spectra(cu)

    def run(fn):
        for _ in range(5):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(steps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / steps

    with torch.inference_mode():
        fused = run(lambda: ops.forward_glu(x, sgu, b, m, algo="auto"))
        fused_stat = run(lambda: ops.forward_glu(x, sgu, b, m, algo="stationary"))
        unfused = run(lambda: torch.nn.functional.silu(ops.forward(x, sg, None, b, m)) * ops.forward(x, su, None, b, m))
    nbytes = n * k * SZ[io] + n * m * SZ[io] + 2 * (m // b) * (k // b) * (b // 2 + 1) * 8
    engine = "dft-glu" if resolved_kernel("auto", k, b)[0] == "dft" else "stationary-glu"
    return {"workload": f"gate/up {k}->{m} b={b} N={n} {io}-io + SwiGLU", "engine": engine,
            "ms": round(fused, 4), "stationary_glu_ms": round(fused_stat, 4), "unfused_ms": round(unfused, 4),
            "GB_s": round(nbytes / (fused * 1e-3) / 1e9, 1),
            "frac": round(nbytes / (fused * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def load_traffic(tag, kernel):
    """Per-launch HBM bytes of this kernel on this workload from the newest
    profiles/pmc_traffic_*.json that measured that pair (None if none did)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if tag in d and d[tag].get("kernel") == kernel:
            return d[tag].get("hbm_bytes_per_launch")
    return None


def cpu_baseline(k, m, b, io, bias, budget_s):
    """Oracle's torch-CPU restatement of the cached forward (bench_all_in_one.py:179-231),
    fp32, on a bounded token sample; GTok-elem/s."""
    sys.path.insert(0, ROOT)
    from oracle.bc_oracle import torch_cpu_forward_cached
    threads = int(os.environ.get("BENCH_CPU_THREADS", min(os.cpu_count() or 1, 16)))
    torch.set_num_threads(threads)
    n = 1024
    g = torch.Generator().manual_seed(0)
    x = torch.randn(n, k, generator=g)
    c = torch.randn(m // b, k // b, b, generator=g) * 0.01
    cf = torch.fft.rfft(c, dim=-1)
    bv = torch.randn(m, generator=g) * 0.1 if bias else None
    torch_cpu_forward_cached(x, cf, bv, b)                     # warmup
    it, t0 = 0, time.perf_counter()
    while True:
        torch_cpu_forward_cached(x, cf, bv, b)
        it += 1
        el = time.perf_counter() - t0
        if el >= budget_s or it >= 10000:
            break
    return {"value": round(n * m * it / el / 1e9, 5), "unit": "GTok-elem/s", "cores": threads,
            "kind": "port",
            "sample": f"{it} x forward of {n} tokens, {k}->{m} b={b} fp32 (torch CPU rfft/einsum/"
                      f"irfft, cached spectra), {el:.1f} s on {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--tokens", type=int, default=8192, help="tokens per rank (batch*seq)")
    ap.add_argument("--in-features", type=int, default=4096)
    ap.add_argument("--out-features", type=int, default=4096)
    ap.add_argument("--block-size", type=int, default=128)
    ap.add_argument("--io", default="fp32", choices=list(DT))
    ap.add_argument("--bias", type=int, default=0)
    ap.add_argument("--allgather", type=int, default=1, help="also time the RCCL all-gather (N>1)")
    ap.add_argument("--variants", type=int, default=1, help="also time bf16-I/O and config-2 shapes")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU baseline work")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed clock-settle phase of the hot path on every rank before the W warmup steps")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        barrier = lambda: dist.barrier(device_ids=[local])  # noqa: E731
    else:
        barrier = None

    n, k, m, b, io = args.tokens, args.in_features, args.out_features, args.block_size, args.io
    algo = os.environ.setdefault("BCFFT_ALGO", "auto")
    layer = make_layer(k, m, b, io, bool(args.bias), dev)
    torch.manual_seed(1000 + rank)                           # x ~ N(0,1) per rank shard
    x = torch.randn(n, k, device=dev).to(DT[io])

    # the variant sweep (rank 0, N=1) runs first: real work, timed per variant
    variants = []
    if args.variants and rank == 0 and world == 1:
        # config 1 (4096², b=64, N=128 fp32), config 2 (4096->11008 b=128 bf16),
        # the north star in bf16 and on the other engines, and the config-4 sweep b x shape (bf16)
        vlist = [(4096, 4096, 64, "fp32", 128, "auto"),
                 (4096, 4096, 128, "bf16", 8192, "auto"),
                 (4096, 4096, 128, "fp32", 8192, "dftx"),
                 (4096, 4096, 128, "fp32", 8192, "stationary"),
                 (4096, 4096, 128, "bf16", 8192, "stationary"),
                 (4096, 4096, 128, "fp32", 8192, "mfma"),
                 (4096, 4096, 128, "fp32", 8192, "valu")]
        for vb in (64, 128, 256):
            for (vk, vm) in ((4096, 4096), (4096, 11008), (11008, 4096)):
                if not (vb == 128 and (vk, vm) == (4096, 4096)):
                    vlist.append((vk, vm, vb, "bf16", 8192, "auto"))
        for (vk, vm, vb, vio, vn, va) in vlist:
            os.environ["BCFFT_ALGO"] = va
            vl = make_layer(vk, vm, vb, vio, False, dev)
            vx = torch.randn(vn, vk, device=dev).to(DT[vio])
            vw, vkern = time_layer(vl, vx, max(10, args.steps // 2), 5)
            os.environ["BCFFT_ALGO"] = algo
            vbytes = algo_bytes(vn, vk, vm, vb, vio, False)
            variants.append({"workload": f"{vk}->{vm} b={vb} N={vn} {vio}-io algo={va}",
                             "engine": resolved_kernel(va, vk, vb, vio)[1].replace("bc_forward_", "").replace("_kernel", ""),
                             "ms": round(vkern, 4),
                             "GTok_elem_s": round(vn * vm / (vkern * 1e-3) / 1e9, 3),
                             "GB_s": round(vbytes / (vkern * 1e-3) / 1e9, 1),
                             "frac": round(vbytes / (vkern * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
            del vl, vx
        variants.append(time_glu(dev, max(10, args.steps // 2)))
    # Clock settle, untimed, on every rank: the same forward back to back for --settle-ms of wall
    # time. Right after a cold start the first launches run ~15 % slow while the clock ramps
    # (measured: 60 us vs 51.5 us per launch, 50 warmup steps and no other GPU work before). N > 1
    # ranks skip the variant sweep, so without this their windows would time the ramp. The W
    # warmup steps and the K timed steps that follow are exactly the contract's.
    settle(layer, x, args.settle_ms)
    wall, kern = time_layer(layer, x, args.steps, args.warmup, barrier)
    t = torch.tensor([wall, kern], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, kern = float(t[0]), float(t[1])

    # SURVEY.md §8d extras beside the contract's single K-step region: 5 more repeats of K steps
    # (median and spread of the per-launch kernel time) and the spectra precompute time
    reps = []
    for _ in range(5):
        reps.append(time_layer(layer, x, args.steps, 2, barrier)[1])
    reps_t = torch.tensor(reps, device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(reps_t, op=dist.ReduceOp.MAX)
    reps = sorted(float(v) for v in reps_t)
    spectra_ms = time_spectra(layer)

    nbytes = algo_bytes(n, k, m, b, io, bool(args.bias))
    gbs = nbytes / (kern * 1e-3) / 1e9
    total_elems = n * m * world
    value = total_elems / (wall * 1e-3) / 1e9

    gather = None
    if world > 1 and args.allgather:
        from bcfft.shard import gather_rows
        with torch.inference_mode():
            for _ in range(3):
                gather_rows(layer(x), world * n)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                gather_rows(layer(x), world * n)
            torch.cuda.synchronize()
            barrier()
            g_ms = (time.perf_counter() - t0) * 1e3 / args.steps
        tg = torch.tensor([g_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(tg, op=dist.ReduceOp.MAX)
        gather = {"ms_per_step": round(float(tg[0]), 4),
                  "value": round(total_elems / (float(tg[0]) * 1e-3) / 1e9, 3),
                  "note": "forward + RCCL all_gather_into_tensor of all y shards to every rank"}


    tag = f"{k}x{m}_b{b}_n{n}_{io}"
    kname = resolved_kernel(algo, k, b, io if not args.bias else "fp32")
    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        cpu = cpu_baseline(k, m, b, io, bool(args.bias), args.cpu_budget)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "GTok-elem/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (x~N(0,1) seed 1000+rank, c~0.01 N(0,1) seed 1)",
            "config": {"workload": f"BlockCirculantLinear.forward {k}->{m} b={b}, {n} tokens/rank, "
                                   f"{io} I/O, spectra cached",
                       "in_features": k, "out_features": m, "block_size": b,
                       "tokens_per_rank": n, "global_tokens": n * world, "io_dtype": io,
                       "bias": bool(args.bias), "parallelism": f"token-shard x{world}",
                       "algo": algo, "algo_resolved": kname[0], "mac": kname[2]},
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(tag, kname[1]),
                         "kernel": kname[1], "kernel_ms": round(kern, 5),
                         "algorithmic_bytes_per_launch": nbytes,
                         "fp32_tflops": round(algo_flops(n, k, m, b) / (kern * 1e-3) / 1e12, 2),
                         "fp32_valu_peak_tflops": FP32_VALU_TFLOPS,
                         "kernel_ms_repeats": {"n": len(reps), "steps_each": args.steps,
                                               "median": round(reps[len(reps) // 2], 5),
                                               "min": round(reps[0], 5), "max": round(reps[-1], 5)}},
            "spectra_precompute_ms": round(spectra_ms, 4),
            "cpu_baseline": cpu,
        }
        if gather:
            line["with_allgather"] = gather
        if variants:
            line["variants"] = variants
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
