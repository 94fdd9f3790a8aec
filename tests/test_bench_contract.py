"""bench.py keeps the driver's contract: the SURVEY.md §8d byte figures, the engine each BCFFT_ALGO
resolves to, and (GPU) one JSON line with the required keys, roofline and cpu_baseline."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_algorithmic_bytes_match_survey():
    assert bench.algo_bytes(8192, 4096, 4096, 128, "fp32", False) == 268_967_936
    assert bench.algo_bytes(8192, 4096, 4096, 128, "bf16", False) == 134_750_208


def test_engine_resolution_mirrors_auto_rule(built_lib):
    """bench.py names the kernel the library itself resolves (bcfft_forward_kernel_name): the AUTO
    rule and each launcher's per-group / multi-group choice by token count (no GPU: 256 CUs)."""
    assert bench.resolved_kernel("auto", 4096, 128)[:2] == ("dftx", "bc_forward_dm_kernel")   # fp32 out
    assert bench.resolved_kernel("auto", 4096, 128, "fp16")[:2] == ("dft", "bc_forward_dm_kernel")
    assert bench.resolved_kernel("dft", 4096, 128)[:2] == ("dft", "bc_forward_dm_kernel")
    assert bench.resolved_kernel("stationary", 4096, 128)[1] == "bc_forward_stat_kernel"
    assert bench.resolved_kernel("auto", 4096, 64)[1] == "bc_forward_stat_kernel"
    assert bench.resolved_kernel("auto", 2048, 64)[1] == "bc_forward_stat_kernel"
    assert bench.resolved_kernel("auto", 11008, 128)[1] == "bc_forward_mfma_kernel"
    assert bench.resolved_kernel("auto", 4096, 256)[1] == "bc_forward_valu_kernel"
    assert bench.resolved_kernel("auto", 4096, 128, "bf16")[1] == "bc_forward_dm8_kernel"
    assert bench.resolved_kernel("auto", 4096, 64, "bf16")[1] == "bc_forward_dm64_kernel"    # 2 output groups
    assert bench.resolved_kernel("auto", 4096, 64, "bf16", 11008)[1] == "bc_forward_dm64g_kernel"
    assert bench.resolved_kernel("auto", 2048, 64, "bf16")[1] == "bc_forward_stat_kernel"
    assert bench.resolved_kernel("valu", 4096, 128)[1] == "bc_forward_valu_kernel"
    assert bench.resolved_kernel("auto", 4096, 128, "bf16", 11008, 8192)[1] == "bc_forward_dmg_kernel"
    # short token counts on the STAT geometries: the short-N kernel (bcfft_sn.hip), e.g. a decode step
    # and BASELINE config 1; the persistent engines once the short grid exceeds the CUs (sn_pays)
    assert bench.resolved_kernel("auto", 4096, 128, "bf16", 11008, 20)[:2] == ("short", "bc_forward_sn_kernel")
    assert bench.resolved_kernel("auto", 4096, 64, "fp32", 4096, 128)[:2] == ("short", "bc_forward_sn_kernel")
    assert bench.resolved_kernel("auto", 4096, 128, "fp32", 4096, 1)[1] == "bc_forward_sn_kernel"
    assert bench.resolved_kernel("auto", 4096, 128, "fp32", 4096, 8192)[1] == "bc_forward_dm_kernel"
    assert bench.resolved_kernel("short", 4096, 128, "fp32", 4096, 8192)[1] == "bc_forward_sn_kernel"
    with pytest.raises(ValueError):
        bench.resolved_kernel("short", 11008, 128, "bf16")   # not a STAT geometry
    assert bench.resolved_kernel("auto", 11008, 128, "bf16", 4096, 8192)[1] == "bc_forward_dmk_kernel"
    assert bench.resolved_kernel("auto", 11008, 64, "bf16", 4096, 8192)[1] == "bc_forward_dm64k_kernel"
    assert bench.resolved_kernel("auto", 11008, 64, "bf16", 4096, 64)[1] == "bc_forward_mfma_kernel"  # < 128 tokens
    assert bench.resolved_kernel("auto", 4096, 256, "bf16", 11008, 8192)[1] == "bc_forward_dm256g_kernel"
    assert bench.resolved_kernel("auto", 4096, 256, "bf16", 11008, 20)[1] == "bc_forward_dm256_kernel"
    assert bench.resolved_kernel("auto", 11008, 256, "bf16", 4096, 8192)[1] == "bc_forward_dm256k_kernel"
    with pytest.raises(ValueError):
        bench.resolved_kernel("dftx", 4096, 64)


@pytest.mark.gpu
def test_bench_prints_one_contract_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2",
                          "--variants", "0", "--cpu-budget", "0"], capture_output=True, text=True,
                         timeout=300, check=True).stdout
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["warmup"] == 2
    assert d["value"] > 0 and d["ms_per_step"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["kernel"] == "bc_forward_dm_kernel"
