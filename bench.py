#!/usr/bin/env python3
"""Benchmark of the MI355X block-circulant (BC) linear forward — BASELINE.json's metric.

Workload (north star / metric): one BlockCirculantLinear forward, 4096 -> 4096, b = 128,
N = batch*seq = 8192 tokens, fp32 I/O (the reference's fp32 path), weight spectra precomputed
outside the timed region (the reference's cache_cfft=1 perf convention,
bench_all_in_one.py:484). A "step" = one forward over the rank's token shard.

Multi-GPU: one process per GPU. `--gpus N` without a torch.distributed
environment re-launches this script under `torch.distributed.run` with N ranks before any GPU
call; with one (the driver's launch) WORLD_SIZE must equal --gpus. `--partition global` (the
default, SURVEY.md §8e's contract): ONE batch*seq = 8192-token batch is split into contiguous
ceil(8192 / N)-row shards (1024 per rank at N = 8; "scaling": "strong"), no collective in the data
path, and `value` = 8192 x M / the slowest rank's time. At N > 1 the line also carries `weak`: the
same ranks each running their own 8192-token batch (the per-rank reading, value = N x 8192 x M /
the slowest rank's time); `--partition per-rank` makes that reading the headline instead. With
--allgather the single RCCL all-gather of the output shards (north star) is timed in a second loop:
forward + all_gather_into_tensor, reported as `with_allgather` (gather-inclusive throughput) beside
the sharded-compute `value`.

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


MAC = {
    "bc_forward_dm_kernel": "MFMA fp16 throughout: block DFT (even/odd split, x hi+lo) x 2^-7 table, stationary "
                            "conj(C)*s_o MAC (X hi+lo; s_o per output block), inverse DFT; f32 accumulate",
    "bc_forward_dm8_kernel": "MFMA fp16 throughout, 8 tokens per tile, one-term spectra (bf16 I/O)",
    "bc_forward_dmg_kernel": "MFMA fp16 throughout, 8 tokens per tile, stage 1 once per tile, every output group's "
                             "weight fragments streamed from L2 (bf16 I/O)",
    "bc_forward_dmk_kernel": "MFMA fp16 throughout, 16-block K-chunks with weight fragments streamed from L2 (bf16 I/O)",
    "bc_forward_dm64_kernel": "MFMA fp16 throughout, b=64, 8 tokens per tile, one-term spectra (bf16 I/O)",
    "bc_forward_dm64g_kernel": "MFMA fp16 throughout, b=64, 8 tokens per tile, stage 1 once per tile, every output "
                               "group's weight fragments streamed from L2 (bf16 I/O)",
    "bc_forward_dm64k_kernel": "MFMA fp16 throughout, b=64, 16 tokens per tile, 32-block K-chunks with weight "
                               "fragments streamed from L2 (bf16 I/O)",
    "bc_forward_dm256_kernel": "MFMA fp16 throughout, b=256 as three 128-point virtual rows, 8 tokens per tile, "
                               "16 output blocks per workgroup (bf16 I/O)",
    "bc_forward_dm256g_kernel": "MFMA fp16 throughout, b=256 as three 128-point virtual rows, stage 1 once per "
                                "8-token tile, every output group's weight fragments streamed from L2 (bf16 I/O)",
    "bc_forward_dm256k_kernel": "MFMA fp16 throughout, b=256 as three 128-point virtual rows, 16-block K-chunks with "
                                "weight fragments streamed from L2 (bf16 I/O)",
    "bc_forward_stat_kernel": "MFMA fp16: conj(C)*s_o (VGPR-resident) x per-token-scaled X split hi+lo, f32 accumulate",
    "bc_forward_sn_kernel": "MFMA fp16 throughout (short-N: one workgroup per 4-token tile and 16 output blocks), "
                            "a/d, X and Y hi+lo, f32 accumulate",
    "bc_forward_mfma_kernel": "MFMA bf16 hi/lo split (Xhi+Xlo)(Chi+Clo), f32 accumulate",
    "bc_forward_valu_kernel": "VALU fp32 FMA",
}
ALGO_NAMES = {0: "auto", 1: "mfma", 2: "valu", 3: "stationary", 4: "dft", 5: "dftx", 6: "dftp", 7: "short"}


def resolved_kernel(algo, k, b, io="fp32", m=4096, n=8192):
    """(algorithm, kernel symbol, MAC arithmetic) that BCFFT_ALGO=algo runs for this geometry, token
    count and I/O dtype (the output has the I/O dtype): asked of the library itself
    (bcfft_forward_resolve / bcfft_forward_kernel_name, include/bcfft.h), which follows the
    launchers' own choices (per-group / multi-group / K-split forms by token count and CUs)."""
    from bcfft import _lib
    lib = _lib.load()
    code = _lib.dtype_code(DT[io])
    a = lib.bcfft_forward_resolve(n, k, m, b, _lib.ALGOS[algo], code, code)
    name = lib.bcfft_forward_kernel_name(n, k, m, b, _lib.ALGOS[algo], code, code).decode()
    if a < 0:
        raise ValueError(f"BCFFT_ALGO={algo} does not serve {k}->{m} b={b} {io}")
    mac = MAC.get(name, "")
    if name == "bc_forward_dm_kernel":
        mac += {"dftx": "; Y hi+lo", "dftp": "; Y hi+lo, and every single fp16 term's rounding residual "
                "(table, weight spectra) added back by fp8 MFMAs (e4m3 residual x bf8 operand)"}.get(
                    ALGO_NAMES[a], "; Y one fp16 term")
    return ALGO_NAMES[a], name, mac


def algo_flops(n, k, m, b):
    import math
    n_out, n_in = m // b, k // b
    return n * (8 * n_out * n_in * (b // 2 + 1) + (n_in + n_out) * 2.5 * b * math.log2(b))


MFMA_PEAK_TFLOPS = 2500.0                           # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)


def dft_mfma_flops(n, k, m, b):
    """Matrix-core flops of the DFT-on-MFMA formulation at b = 128 (one fp16 term per operand):
    per token, stage 1 (n_in blocks x 64 t x 128 bin reals), stage 2 (n_in x n_out x 64 packed
    bins x 4 real products) and stage 3 (n_out blocks x 128 t x 64 bin reals), 2 flops a MAC."""
    n_in, n_out = k // b, m // b
    h = b // 2
    return 2.0 * n * (n_in * h * b + 4 * n_in * n_out * h + n_out * b * h)


def make_layer(k, m, b, io, bias, dev, seed=1):
    from patch_llama_fft import BlockCirculantLinear
    torch.manual_seed(seed)                                   # c ~ 0.01 N(0,1), seed 1 (§8d)
    layer = BlockCirculantLinear(k, m, block_size=b, bias=bias)
    if bias:
        with torch.no_grad():
            layer.bias.normal_(0.0, 0.1)
    return layer.to(dev).to(DT[io]).eval()


def settle(fn, ms, dev):
    """Run fn back to back for at least `ms` milliseconds of wall time (untimed)."""
    t0 = time.perf_counter()
    with torch.inference_mode():
        while (time.perf_counter() - t0) * 1e3 < ms:
            for _ in range(20):
                fn()
            if dev.type == "cuda":
                torch.cuda.synchronize()


def time_fn(fn, steps, warmup, barrier=None, dev=None):
    """Returns (wall ms per step over the bracketed region, mean ms per launch). On a GPU the
    second figure comes from ONE HIP-event pair around the K back-to-back launches on the launch
    stream: a pair around EACH launch adds its own marker latency (~6 us per step measured on
    MI355X, see tools/event_timing.py), while K launches back to back give the launch duration
    plus the inter-kernel gap, within ~2-3 % of rocprofv3's per-kernel average. On the CPU (the
    gloo test of the distributed path) both are the wall time."""
    cuda = dev is not None and dev.type == "cuda"
    with torch.inference_mode():
        for _ in range(warmup):
            fn()
        if cuda:
            stream = torch.cuda.current_stream()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if barrier:
            barrier()
        if cuda:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        if cuda:
            s.record(stream)
        for _ in range(steps):
            fn()
        if cuda:
            e.record(stream)
            torch.cuda.synchronize()
        if barrier:
            barrier()
        wall = (time.perf_counter() - t0) * 1e3 / steps
    kern = s.elapsed_time(e) / steps if cuda else wall
    return wall, kern


def time_layer(layer, x, steps, warmup, barrier=None):
    """time_fn of one BC layer on x, spectra computed outside the timed region."""
    with torch.inference_mode():
        layer._spectra(layer.c)
    return time_fn(lambda: layer(x), steps, warmup, barrier, x.device)


def reduce_max(vals, dev, world):
    """Elementwise max over ranks (the slowest rank sets every timed figure); through the process
    group whenever one exists (the RCCL test runs it at world size 1 too)."""
    t = torch.tensor([float(v) for v in vals], device=dev, dtype=torch.float64)
    if world > 1 or dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def partition(n, world, rank, mode):
    """(tokens this rank runs, its row range in the global batch, global tokens). 'global': the
    global n tokens in contiguous ceil(n / world) shards; 'per-rank': n each."""
    if mode == "global":
        from bcfft.shard import shard_bounds
        lo, hi = shard_bounds(n, world, rank)
        return hi - lo, (lo, hi), n
    return n, (rank * n, (rank + 1) * n), n * world


def run_partitioned(fwd, x_local, n_total, steps, warmup, world, barrier, dev, settle_ms=0.0,
                    allgather=True, repeats=5):
    """The timed core every rank runs (GPU ranks over RCCL, and the gloo test on CPU stubs):
    settle, then W warmup + K timed steps of fwd on the rank's shard between barriers, the max
    over ranks; `repeats` more K-step windows; with a process group (N > 1, or the RCCL test's
    single rank) and allgather, forward + the single all-gather of the y shards
    (bcfft.shard.gather_rows) timed the same way. Returns {wall, kern, reps (sorted), gather_wall
    or None}."""
    from bcfft.shard import gather_rows
    step = lambda: fwd(x_local)  # noqa: E731
    settle(step, settle_ms, dev)
    wall, kern = reduce_max(time_fn(step, steps, warmup, barrier, dev), dev, world)
    reps = sorted(reduce_max([time_fn(step, steps, 2, barrier, dev)[1] for _ in range(repeats)], dev, world))
    gather = None
    if (world > 1 or dist.is_initialized()) and allgather:
        g = time_fn(lambda: gather_rows(fwd(x_local), n_total), steps, 3, barrier, dev)[0]
        gather = reduce_max([g], dev, world)[0]
    return {"wall": wall, "kern": kern, "reps": reps, "gather_wall": gather}


def spawn_cmd(gpus, argv, port):
    """The torch.distributed.run command that re-launches this script with one rank per GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def spawn_ranks(gpus, argv):
    """`bench.py --gpus N` outside torch.distributed: start N fresh rank processes (nothing here
    has touched the GPU yet) and return their launcher's exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(spawn_cmd(gpus, argv, port), env=env)


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
        fused_stat = run(lambda: ops.forward_glu(x, sgu, b, m, algo="stationary")) if b <= 128 else None
        unfused = run(lambda: torch.nn.functional.silu(ops.forward(x, sg, None, b, m)) * ops.forward(x, su, None, b, m))
    nbytes = n * k * SZ[io] + n * m * SZ[io] + 2 * (m // b) * (k // b) * (b // 2 + 1) * 8
    engine = "dft-glu" if resolved_kernel("auto", k, b, io, k, n)[0] in ("dft", "dftx") else "stationary-glu"
    return {"workload": f"gate/up {k}->{m} b={b} N={n} {io}-io + SwiGLU", "engine": engine,
            "ms": round(fused, 4), "stationary_glu_ms": None if fused_stat is None else round(fused_stat, 4),
            "unfused_ms": round(unfused, 4),
            "GB_s": round(nbytes / (fused * 1e-3) / 1e9, 1),
            "frac": round(nbytes / (fused * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def time_mlp(dev, steps, k=4096, m=11008, b=128, n=8192):
    """The whole BC-MLP down(silu(gate(x)) * up(x)) (microbench_dense_vs_bc.py:183-188, the
    reference's --bench_mlp unit): ONE launch (bcfft_forward_mlp FUSED, h never
    written) vs the split form (gate/up + SwiGLU launch, h in HBM, down launch). bf16."""
    from bcfft import ops
    torch.manual_seed(4)
    cg = torch.randn(m // b, k // b, b, device=dev) * 0.01
    cu = torch.randn(m // b, k // b, b, device=dev) * 0.01
    cd = torch.randn(k // b, m // b, b, device=dev) * 0.01
    x = torch.randn(n, k, device=dev).to(torch.bfloat16)
    sgu, sd = ops.spectra(ops.glu_weights(cg, cu)), ops.spectra(cd)

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
        fused = run(lambda: ops.forward_mlp(x, sgu, sd, b, m, mode="fused"))
        split = run(lambda: ops.forward_mlp(x, sgu, sd, b, m, mode="split"))
    nbytes = 2 * n * k * 2                          # x + y (the weights stream from L2)
    # the launch's matrix-core work: gate + up (k -> 2m) and down (m -> k) in the DFT formulation
    flops = dft_mfma_flops(n, k, 2 * m, b) + dft_mfma_flops(n, m, k, b)
    traffic, src = load_traffic("mlp_fused", "bc_mlp_dmm_kernel")
    return {"workload": f"MLP {k}->{m}->{k} b={b} N={n} bf16-io (gate/up + SwiGLU + down)",
            "engine": "mlp_dmm (one launch)", "ms": round(fused, 4), "split_ms": round(split, 4),
            "GTok_s": round(n / (fused * 1e-3) / 1e9, 4),
            "xy_GB_s": round(nbytes / (fused * 1e-3) / 1e9, 1),
            "mfma_roofline": {"bound": "mfma", "flops_per_launch": flops,
                              "achieved": round(flops / (fused * 1e-3) / 1e12, 1), "peak": MFMA_PEAK_TFLOPS,
                              "unit": "TFLOP/s", "frac": round(flops / (fused * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS, 4)},
            "hbm": {"algorithmic_bytes": nbytes, "traffic_bytes": traffic, "traffic_src": src,
                    "traffic_over_algorithmic": round(traffic / nbytes, 3) if traffic else None}}


def load_traffic(tag, kernel, algo=None):
    """Per-launch HBM bytes of this kernel and engine on this workload from the newest
    profiles/pmc_traffic_*.json that measured that triple (None if none did; tools/pmc_traffic.py
    writes them from rocprofv3 PMC passes: FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        e = d.get(tag)
        if e and e.get("kernel") == kernel and (algo is None or e.get("algo", algo) == algo):
            return e.get("hbm_bytes_per_launch"), os.path.relpath(f, ROOT)
    return None, None


def run_variants(dev, algo, steps):
    """SURVEY.md §8d beside the headline: config 1 (4096², b=64, N=128 fp32), config 2
    (4096->11008 b=128 bf16), the north star in bf16 and on the other engines, the config-4 sweep
    b x shape (bf16), and config 2's fused gate/up + SwiGLU."""
    vlist = [(4096, 4096, 64, "fp32", 128, "auto"),
             (4096, 4096, 128, "bf16", 8192, "auto"),
             (4096, 4096, 128, "fp32", 8192, "dftp"),     # the precise engine (BCFFT_PRECISE=1's AUTO)
             (4096, 4096, 128, "fp32", 8192, "dft"),
             (4096, 4096, 128, "fp32", 8192, "stationary"),
             (4096, 4096, 128, "bf16", 8192, "stationary"),
             (4096, 4096, 128, "fp32", 8192, "mfma"),
             (4096, 4096, 128, "fp32", 8192, "valu")]
    for vb in (64, 128, 256):
        for (vk, vm) in ((4096, 4096), (4096, 11008), (11008, 4096)):
            if not (vb == 128 and (vk, vm) == (4096, 4096)):
                vlist.append((vk, vm, vb, "bf16", 8192, "auto"))
    variants = []
    for (vk, vm, vb, vio, vn, va) in vlist:
        os.environ["BCFFT_ALGO"] = va
        vl = make_layer(vk, vm, vb, vio, False, dev)
        vx = torch.randn(vn, vk, device=dev).to(DT[vio])
        vw, vkern = time_layer(vl, vx, max(10, steps // 2), 5)
        # the same forward replayed from a HIP graph (bcfft.graph), 10 forwards per graph: the
        # GPU's time per launch whatever the host's per-call cost (eager back-to-back launches of
        # a ~40 us kernel become host-bound on a busy host); this is the figure frac uses
        from bcfft.graph import GraphedCall
        g = GraphedCall(lambda t: vl(t), [vx], repeat=10)
        os.environ["BCFFT_ALGO"] = algo
        gk = time_fn(g.replay, max(10, steps // 2), 3, None, dev)[1] / 10
        del g
        vbytes = algo_bytes(vn, vk, vm, vb, vio, False)
        variants.append({"workload": f"{vk}->{vm} b={vb} N={vn} {vio}-io algo={va}",
                         "engine": resolved_kernel(va, vk, vb, vio, vm, vn)[1].replace("bc_forward_", "").replace("_kernel", ""),
                         "ms": round(gk, 4),
                         "eager_ms": round(vkern, 4),
                         "GTok_elem_s": round(vn * vm / (gk * 1e-3) / 1e9, 3),
                         "GB_s": round(vbytes / (gk * 1e-3) / 1e9, 1),
                         "frac": round(vbytes / (gk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
        del vl, vx
    for gb in (128, 64, 256):                       # the fused gate/up at every block size of the sweep
        variants.append(time_glu(dev, max(10, steps // 2), b=gb))
    variants.append(time_mlp(dev, max(10, steps // 2)))
    return variants


def host_cores():
    """Host cores this process may run on: the affinity mask, capped by a cgroup CPU quota where
    one is set (a GPU box's share of a many-core host shows all of the host's CPUs in
    os.cpu_count())."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    """The host CPU's model name and thread count (lscpu's "Model name" / "CPU(s)"), for the
    cpu_baseline record: the CPU figure depends on which host the box landed on."""
    name, threads = None, os.cpu_count()
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            key, _, val = ln.partition(":")
            if key.strip() == "Model name" and name is None:
                name = val.strip()
            elif key.strip() == "CPU(s)":
                threads = int(val.strip())
    except (OSError, ValueError, Exception):
        pass
    if name is None:
        try:
            for ln in open("/proc/cpuinfo"):
                if ln.startswith("model name"):
                    name = ln.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
    return name, threads


def cpu_baseline(k, m, b, io, bias, budget_s):
    """Oracle's torch-CPU restatement of the cached forward (bench_all_in_one.py:179-231),
    fp32, on a bounded token sample, on all the host cores this process may use; GTok-elem/s."""
    sys.path.insert(0, ROOT)
    from oracle.bc_oracle import torch_cpu_forward_cached
    threads = int(os.environ.get("BENCH_CPU_THREADS", host_cores()))
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
    model, host_threads = cpu_model()
    return {"value": round(n * m * it / el / 1e9, 5), "unit": "GTok-elem/s", "cores": threads,
            "kind": "port", "cpu_model": model, "host_threads": host_threads,
            "sample": f"{it} x forward of {n} tokens, {k}->{m} b={b} fp32 (torch CPU rfft/einsum/"
                      f"irfft, cached spectra), {el:.1f} s on {threads} of the host's {host_threads} "
                      f"threads ({model}); the box's CPU share (affinity / cgroup quota) sets `cores`"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--tokens", type=int, default=8192,
                    help="batch*seq: global tokens (--partition global) or tokens per rank (per-rank)")
    ap.add_argument("--partition", default="global", choices=("global", "per-rank"),
                    help="global (default): shard the global tokens over the ranks (SURVEY.md §8e, strong "
                         "scaling); per-rank: every rank runs --tokens (weak scaling; reported as `weak` "
                         "beside a global headline at N > 1)")
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
    ap.add_argument("--stub", default="",
                    help="tests only: module:function returning a CPU forward(k, m, b) for a gloo run of the "
                         "launcher and the distributed timing core without a GPU")
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:          # before anything touches the GPU
        sys.exit(spawn_ranks(args.gpus, argv))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; run one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop WORLD_SIZE")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    stub = None
    if args.stub:
        import importlib
        mod, fn = args.stub.split(":")
        stub = getattr(importlib.import_module(mod), fn)
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)
    if world > 1:
        barrier = (lambda: dist.barrier()) if stub else (lambda: dist.barrier(device_ids=[local]))
    else:
        barrier = None

    k, m, b, io = args.in_features, args.out_features, args.block_size, args.io
    n_local, (lo, hi), n_total = partition(args.tokens, world, rank, args.partition)
    algo = os.environ.setdefault("BCFFT_ALGO", "auto")
    if stub:
        fwd = stub(k, m, b)
        layer = None
    else:
        layer = make_layer(k, m, b, io, bool(args.bias), dev)
        fwd = layer
    if args.partition == "global":                   # one global batch, the rank's contiguous rows
        torch.manual_seed(0)                          # x ~ N(0,1), seed 0
        x = torch.randn(n_total, k, device=dev)[lo:hi].to(DT[io]).contiguous()
    else:
        torch.manual_seed(rank)
        x = torch.randn(n_local, k, device=dev).to(DT[io])

    # the variant sweep (rank 0, N=1) runs first: real work, timed per variant
    variants = []
    if args.variants and rank == 0 and world == 1 and not stub:
        variants = run_variants(dev, algo, args.steps)
    # Clock settle, untimed, on every rank: the same forward back to back for --settle-ms of wall
    # time. Right after a cold start the first launches run ~15 % slow while the clock ramps
    # (measured: 60 us vs 51.5 us per launch, 50 warmup steps and no other GPU work before). N > 1
    # ranks skip the variant sweep, so without this their windows would time the ramp. The W
    # warmup steps and the K timed steps that follow are exactly the contract's.
    if layer is not None:
        with torch.inference_mode():
            layer._spectra(layer.c)                   # spectra outside the timed region
    r = run_partitioned(fwd, x, n_total, args.steps, args.warmup, world, barrier, dev,
                        settle_ms=0.0 if stub else args.settle_ms, allgather=bool(args.allgather))
    wall, kern, reps = r["wall"], r["kern"], r["reps"]
    weak = None
    if world > 1 and args.partition == "global":     # the per-rank (weak-scaling) reading, same ranks
        torch.manual_seed(rank)
        xw = torch.randn(args.tokens, k, device=dev).to(DT[io])
        rw = run_partitioned(fwd, xw, args.tokens * world, args.steps, args.warmup, world, barrier, dev,
                             settle_ms=0.0, allgather=False, repeats=1)
        weak = {"value": round(args.tokens * world * m / (rw["wall"] * 1e-3) / 1e9, 4),
                "ms_per_step": round(rw["wall"], 5), "kernel_ms": round(rw["kern"], 5),
                "tokens_per_rank": args.tokens, "scaling": "weak",
                "note": "every rank runs its own batch*seq-token batch (no collective); value = all ranks' "
                        "tokens x M / the slowest rank's time"}
        del xw
    io16 = None
    if world > 1 and layer is not None and io == "fp32":
        # BASELINE.md's config-5 row names bf16: the same shard through the bf16-I/O layer (the
        # 8-token kernel), timed by the same core; beside the fp32 headline, not instead of it
        l16 = make_layer(k, m, b, "bf16", bool(args.bias), dev)
        with torch.inference_mode():
            l16._spectra(l16.c)
        r16 = run_partitioned(l16, x.to(torch.bfloat16), n_total, args.steps, args.warmup, world, barrier, dev,
                              settle_ms=0.0, allgather=bool(args.allgather), repeats=1)
        io16 = {"value": round(n_total * m / (r16["wall"] * 1e-3) / 1e9, 4), "ms_per_step": round(r16["wall"], 5),
                "kernel_ms": round(r16["kern"], 5), "io_dtype": "bf16",
                "kernel": resolved_kernel(algo, k, b, "bf16", m, n_local)[1],
                "with_allgather_ms": None if r16["gather_wall"] is None else round(r16["gather_wall"], 4),
                "note": "the same partition with bf16 x / y (BASELINE.md config 5); value = global tokens x M / "
                        "the slowest rank's time"}
        del l16
    shards = None
    if world == 1 and layer is not None and args.partition == "global" and n_local >= 2048:
        # the strong-scaling ceiling before an 8-GPU node exists: the kernel time of
        # the 1/2/4/8-GPU shard of this batch on this GPU (HIP events, back-to-back launches)
        shards = []
        for g in (2, 4, 8):
            ns = -(-n_local // g)
            ks = time_fn(lambda: layer(x[:ns]), args.steps, args.warmup, None, dev)[1]
            shards.append({"gpus": g, "tokens_per_rank": ns, "kernel_ms": round(ks, 5),
                           "speedup_ceiling": round(kern / ks, 3)})
    value = n_total * m / (wall * 1e-3) / 1e9
    nbytes = algo_bytes(n_local, k, m, b, io, bool(args.bias))
    gather = None
    if r["gather_wall"] is not None:
        gather = {"ms_per_step": round(r["gather_wall"], 4),
                  "value": round(n_total * m / (r["gather_wall"] * 1e-3) / 1e9, 3),
                  "note": "gather-inclusive: forward of the rank's shard + the single RCCL "
                          "all_gather_into_tensor of all y shards to every rank (slowest rank)"}

    spectra_ms = time_spectra(layer) if layer is not None else None
    tag = f"{k}x{m}_b{b}_n{n_local}_{io}"
    kname = resolved_kernel(algo, k, b, io, m, n_local) if not stub else ("stub", "stub", "CPU stub")
    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0 and not stub:
        cpu = cpu_baseline(k, m, b, io, bool(args.bias), args.cpu_budget)

    if rank == 0:
        roofline = None
        if not stub:
            # PMC-measured HBM bytes of this kernel on this workload, from the committed rocprofv3
            # passes (FETCH_SIZE x 2 + WRITE_SIZE); the source file is reported beside the number
            traffic, traffic_src = load_traffic(tag, kname[1], kname[0])
            gbs = nbytes / (kern * 1e-3) / 1e9
            roofline = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "traffic": traffic,
                        "traffic_source": traffic_src,
                        "kernel": kname[1], "kernel_ms": round(kern, 5),
                        "algorithmic_bytes_per_launch": nbytes,
                        "fp32_tflops": round(algo_flops(n_local, k, m, b) / (kern * 1e-3) / 1e12, 2),
                        "fp32_valu_peak_tflops": FP32_VALU_TFLOPS,
                        "kernel_ms_repeats": {"n": len(reps), "steps_each": args.steps,
                                              "median": round(reps[len(reps) // 2], 5),
                                              "min": round(reps[0], 5), "max": round(reps[-1], 5)}}
        line = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "GTok-elem/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall, 5),
            "higher_is_better": True,
            "scaling": "strong" if args.partition == "global" else "weak",
            "vs_baseline": None,
            "dtype": "f32" if io == "fp32" else io,
            "data": (f"synthetic (x~N(0,1) seed {0 if args.partition == 'global' else 'rank'}, "
                     "c~0.01 N(0,1) seed 1)"),
            "config": {"workload": f"BlockCirculantLinear.forward {k}->{m} b={b}, {n_total} tokens "
                                   f"({args.partition} partition: {n_local} per rank), {io} I/O, spectra cached",
                       "in_features": k, "out_features": m, "block_size": b,
                       "tokens_per_rank": n_local, "global_tokens": n_total, "io_dtype": io,
                       "bias": bool(args.bias), "partition": args.partition,
                       "parallelism": f"token-shard x{world}",
                       "algo": algo, "algo_resolved": kname[0], "mac": kname[2]},
            "roofline": roofline,
            "spectra_precompute_ms": None if spectra_ms is None else round(spectra_ms, 4),
            "cpu_baseline": cpu,
        }
        if stub:
            line["stub"] = args.stub
        if world > 1 and args.partition == "global":
            line["scaling_note"] = ("strong scaling: the global 8192 tokens split over the ranks; every rank's "
                                    "shard runs the same kernel as N=1 on fewer tokens (1024 at N=8)")
        if gather:
            line["with_allgather"] = gather
        if weak:
            line["weak"] = weak
        if io16:
            line["bf16_io"] = io16
        if shards:
            line["strong_scaling_shards"] = {
                "note": "kernel time of each rank's shard of this batch at N GPUs, measured here on one GPU; "
                        "speedup_ceiling = this line's kernel_ms / the shard's (the compute-only bound of the "
                        "driver's 1/2/4/8 curve, before launch gaps and the all-gather)",
                "shards": shards}
        if variants:
            line["variants"] = variants
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
