"""Host-side rules that must agree with the library (no GPU: these calls launch nothing).

* bcfft.ops.glu_eligible mirrors bcfft_forward_glu_algo's refusals for every engine, so the patched
  LLaMA MLP (BCFusedGateUp) falls back to two launches instead of raising (b = 256 with
  BCFFT_ALGO=stationary / dftx, dftx at b = 64).
* the b = 256 fused gate/up kernel's group limit (2 ceil(gate_blocks / 16) <= 64) is refused,
  not run past its LDS array.
"""
import itertools

import pytest
import torch


@pytest.fixture(scope="module")
def lib(built_lib):
    from bcfft import _lib
    return _lib.load()


GEOMS = [(4096, 128, 11008), (4096, 64, 11008), (2048, 64, 5504), (4096, 256, 11008), (4096, 256, 16384 * 8),
         (4096, 256, 131072 + 256 * 16), (11008, 128, 4096), (4096, 32, 4096), (8192, 128, 4096)]


@pytest.mark.parametrize("algo,dt", list(itertools.product(["auto", "stationary", "dft", "dftx", "mfma", "valu"],
                                                            [torch.float32, torch.float16, torch.bfloat16])))
def test_glu_eligible_mirrors_library(lib, algo, dt):
    from bcfft import _lib, ops
    for k, b, g in GEOMS:
        want = ops.glu_eligible(k, b, dt, algo, g)
        if algo in ("mfma", "valu"):
            assert not want
            continue
        # n_tokens = 0: the library returns BCFFT_OK after its refusal checks, before any launch
        st = lib.bcfft_forward_glu_algo(None, _lib.dtype_code(dt), 0, k, g, b, None, None, _lib.ALGOS[algo], None)
        assert st in (0, 2), (k, b, g, algo, dt, st)
        assert (st == 0) == want, (k, b, g, algo, dt, st)


def test_b256_glu_group_limit(lib):
    from bcfft import _lib
    BF16 = _lib.BCFFT_BF16
    ok = lib.bcfft_forward_glu_algo(None, BF16, 0, 4096, 512 * 256, 256, None, None, 0, None)
    over = lib.bcfft_forward_glu_algo(None, BF16, 0, 4096, 513 * 256, 256, None, None, 0, None)
    assert ok == 0 and over == 2


def test_fused_gate_up_falls_back_under_other_engines(monkeypatch):
    """BCFusedGateUp._fused_ok follows the engine: no fused launch is attempted where the library
    would refuse it (the module then runs gate and up as two forwards)."""
    from bcfft import ops
    monkeypatch.setenv("BCFFT_ALGO", "stationary")
    assert not ops.glu_eligible(4096, 256, torch.bfloat16, gate_features=11008)
    monkeypatch.setenv("BCFFT_ALGO", "dftx")
    assert not ops.glu_eligible(4096, 64, torch.bfloat16, gate_features=11008)
    assert ops.glu_eligible(4096, 128, torch.bfloat16, gate_features=11008)
    monkeypatch.setenv("BCFFT_ALGO", "auto")
    assert ops.glu_eligible(4096, 256, torch.bfloat16, gate_features=11008)


def test_precise_mode_resolution(monkeypatch):
    """BCFFT_PRECISE=1 makes AUTO pick the fp32-faithful engines for fp32 activations: dftp at
    b = 128 with K = 4096, the split-bf16 MFMA kernel at other b <= 128, fp32 VALU above; 16-bit
    activations and explicit engines are unaffected, and the fused gate/up falls back to two
    launches where no precise fused form exists."""
    import torch
    from bcfft import ops
    monkeypatch.delenv("BCFFT_ALGO", raising=False)
    monkeypatch.setenv("BCFFT_PRECISE", "1")
    assert ops.resolve_algo(None, torch.float32, 128, 4096) == "dftp"
    assert ops.resolve_algo(None, torch.float32, 64, 4096) == "mfma"
    assert ops.resolve_algo(None, torch.float32, 256, 4096) == "valu"
    assert ops.resolve_algo(None, torch.bfloat16, 128, 4096) == "auto"
    assert ops.resolve_algo("dftx", torch.float32, 128, 4096) == "dftx"
    assert ops.glu_eligible(4096, 128, torch.float32, ops.resolve_algo(None, torch.float32, 128, 4096))
    assert not ops.glu_eligible(4096, 64, torch.float32, ops.resolve_algo(None, torch.float32, 64, 4096))
    monkeypatch.setenv("BCFFT_PRECISE", "0")
    assert ops.resolve_algo(None, torch.float32, 128, 4096) == "auto"


def test_operand_device_and_layout_checks():
    """bcfft.ops refuses a spectra buffer or bias that is not on x's device, and a strided spectra
    view, before any launch (the C ABI reads them by raw device pointer; csrc/bcfft_torch.cpp
    repeats the check for the C++ operators)."""
    import torch
    from bcfft import ops
    dev = torch.device("cuda", 0)                 # x's device; the operands below live on the host
    spec = torch.zeros(64)
    with pytest.raises(ValueError, match="spectra is on cpu but x is on cuda:0"):
        ops._check_operand(spec, dev, "bcfft.forward", "spectra")
    with pytest.raises(ValueError, match="bias is on cpu"):
        ops._check_operand(torch.zeros(8), dev, "bcfft.forward", "bias")
    with pytest.raises(ValueError, match="contiguous"):
        ops._check_operand(torch.zeros(128)[::2], torch.device("cpu"), "bcfft.forward", "spectra")
    ops._check_operand(spec, torch.device("cpu"), "bcfft.forward", "spectra")
    ops._check_operand(torch.zeros(16)[::2], torch.device("cpu"), "bcfft.forward", "bias")   # bias views are copied
