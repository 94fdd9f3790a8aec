"""GPU parity of the fused BC-MLP (bcfft_forward_mlp): y = down(silu(gate(x)) *
up(x)) in one launch (bcfft_dmm.hip), the unit the reference times with `--bench_mlp`
(src/microbench_dense_vs_bc.py:183-188) and the MLP of patch_mlp_with_block_circulant
(patch_llama_fft.py:343-394).

* Against the split form (the gate/up + SwiGLU launch, h in HBM, then the down launch): every
  rounding is the same, so the outputs must be BIT-IDENTICAL (torch.equal). That covers ragged
  token counts, partial last gate/up groups (the down projection's partial last K-chunk), chunks
  of very different magnitude (the down kernel's reference-exponent rescale), zero tokens, and
  the full 8192-token LLaMA-7B shape.
* Against the CPU oracle (oracle/bc_oracle.py: the reference's fp32 FFT forward per projection,
  bf16 roundings where torch rounds): 16-bit output bounds as the GLU tests use."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from oracle import bc_oracle as O

pytestmark = pytest.mark.gpu

B = 128
HID = 4096


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


def _weights(dev, n_h, seed, chunk_gain=None):
    g = torch.Generator(device="cpu").manual_seed(seed)
    cg = torch.randn(n_h, HID // B, B, generator=g) * 0.01
    cu = torch.randn(n_h, HID // B, B, generator=g) * 0.01
    cd = torch.randn(HID // B, n_h, B, generator=g) * 0.01
    if chunk_gain is not None:                       # h chunk k (16 blocks) scaled by chunk_gain[k]
        for k, s in enumerate(chunk_gain):
            cu[16 * k:16 * k + 16] *= s
    return cg.to(dev), cu.to(dev), cd.to(dev)


def _run(dev, x, cg, cu, cd, mode):
    from bcfft import ops
    n_h = cg.shape[0]
    sgu = ops.spectra(ops.glu_weights(cg, cu))
    sd = ops.spectra(cd)
    y = ops.forward_mlp(x, sgu, sd, B, n_h * B, mode=mode)
    torch.cuda.synchronize()
    return y


def _silu(a):
    """a * sigmoid(a) in fp64 without overflow: exp of a non-positive argument only."""
    a = a.astype(np.float64)
    e = np.exp(-np.abs(a))
    return a * np.where(a >= 0, 1.0 / (1.0 + e), e / (1.0 + e))


def oracle_mlp(x, cg, cu, cd, dt=O.BF16):
    xr = O.round_to(x, dt)
    gt = O.bc_forward(xr, cg, x_dtype=dt)
    ut = O.bc_forward(xr, cu, x_dtype=dt)
    s = O.round_to(_silu(gt).astype(np.float32), dt)
    h = O.round_to((s.astype(np.float64) * ut).astype(np.float32), dt)
    return O.bc_forward(h, cd, x_dtype=dt)


@pytest.mark.parametrize("n,n_h", [(1, 86), (5, 86), (8, 86), (9, 86), (37, 86), (300, 86),
                                   (16, 96), (23, 33), (19, 127), (2048, 86)])
def test_fused_equals_split(dev, n, n_h):
    torch.manual_seed(n + n_h)
    cg, cu, cd = _weights(dev, n_h, seed=n_h)
    x = torch.randn(n, HID, device=dev).to(torch.bfloat16)
    yf = _run(dev, x, cg, cu, cd, "fused")
    ys = _run(dev, x, cg, cu, cd, "split")
    assert yf.shape == (n, HID) and yf.dtype == torch.bfloat16
    assert torch.isfinite(yf.float()).all()
    diff = (yf.float() - ys.float()).abs().max().item()
    assert torch.equal(yf, ys), f"fused != split (max |diff| {diff:.3e})"


def test_fused_equals_split_loud_quiet_chunks_and_zero_tokens(dev):
    """h chunks 1e3 louder / 1e-3 quieter than the first (the down kernel lowers a token's
    reference exponent and rescales its accumulators), plus all-zero and tiny tokens."""
    gains = [1.0, 1e3, 1e-3, 1.0, 30.0, 1e-2]
    cg, cu, cd = _weights(dev, 86, seed=5, chunk_gain=gains)
    torch.manual_seed(5)
    x = torch.randn(45, HID, device=dev)
    x[3] = 0
    x[10] *= 1e-6
    x[20, :2048] = 0
    x = x.to(torch.bfloat16)
    yf = _run(dev, x, cg, cu, cd, "fused")
    ys = _run(dev, x, cg, cu, cd, "split")
    assert torch.equal(yf, ys)
    assert (yf[3] == 0).all()


def test_fused_vs_oracle(dev):
    n, n_h = 37, 86
    cg, cu, cd = _weights(dev, n_h, seed=11)
    torch.manual_seed(11)
    x = torch.randn(n, HID, device=dev).to(torch.bfloat16)
    y = _run(dev, x, cg, cu, cd, "fused").float().cpu().numpy()
    ref = oracle_mlp(x.float().cpu().numpy(), cg.cpu().numpy(), cu.cpu().numpy(), cd.cpu().numpy())
    e = rel_err(y, ref)
    # bf16 output (2^-8 relative rounding), the fp16 weight spectra of both BC stages (~4e-4 each)
    # carried through SiLU, and the bf16 rounding of h feeding the down projection
    assert e < 4e-3, f"rel err {e:.3e}"
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    assert np.max(np.abs(y - ref)) < 8 * 2.0 ** -7 * rms + 2 * 2.0 ** -7 * np.max(np.abs(ref))


def test_fused_full_size_llama7b(dev):
    """8192 tokens, 4096 -> 11008 -> 4096 (the reference's --bench_mlp shape at batch 4 x seq 2048):
    against the split form bit for bit (the split form's down launch takes 16-token tiles here),
    and every token against the oracle (Frobenius 4e-3 as test_fused_vs_oracle; per token 8e-3:
    bf16 h and y roundings over 8192 tokens' tails)."""
    n, n_h = 8192, 86
    cg, cu, cd = _weights(dev, n_h, seed=21)
    torch.manual_seed(21)
    x = torch.randn(n, HID, device=dev).to(torch.bfloat16)
    yf = _run(dev, x, cg, cu, cd, "fused")
    ys = _run(dev, x, cg, cu, cd, "split")
    assert torch.isfinite(yf.float()).all()
    d = (yf.float() - ys.float())
    assert torch.equal(yf, ys), (f"max |diff| {d.abs().max().item():.3e}, rel "
                                 f"{(d.norm() / ys.float().norm()).item():.3e}")
    ref = oracle_mlp(x.float().cpu().numpy(), cg.cpu().numpy(), cu.cpu().numpy(), cd.cpu().numpy())
    g = yf.float().cpu().numpy()
    e = rel_err(g, ref)
    tok = np.sqrt(((g.astype(np.float64) - ref) ** 2).sum(1) / (ref.astype(np.float64) ** 2).sum(1))
    print(f"fused MLP full size vs oracle: Frobenius {e:.3e}, worst token {tok.max():.3e}")
    assert e < 4e-3, e
    assert tok.max() < 8e-3, (int(tok.argmax()), tok.max())


def test_auto_and_ineligible(dev):
    """AUTO: one launch on the fused geometry; fp32 x and b = 64 run the split form; a forced
    fused launch on them raises with the reason."""
    from bcfft import ops
    cg, cu, cd = _weights(dev, 86, seed=3)
    x = torch.randn(11, HID, device=dev)
    ya = _run(dev, x.to(torch.bfloat16), cg, cu, cd, "auto")
    yf = _run(dev, x.to(torch.bfloat16), cg, cu, cd, "fused")
    assert torch.equal(ya, _run(dev, x.to(torch.bfloat16), cg, cu, cd, "fused_splitk"))   # AUTO at 11 tokens
    assert ((ya.float() - yf.float()).norm() / yf.float().norm()).item() < 3e-3
    y32 = _run(dev, x, cg, cu, cd, "auto")
    assert y32.dtype == torch.float32
    ref = oracle_mlp(x.cpu().numpy(), cg.cpu().numpy(), cu.cpu().numpy(), cd.cpu().numpy(), O.F32)
    assert rel_err(y32.cpu().numpy(), ref) < 1e-3
    with pytest.raises(RuntimeError, match="intermediate 11008"):
        _run(dev, x, cg, cu, cd, "fused")
    c64g = torch.randn(44, 32, 64, device=dev) * 0.01
    c64d = torch.randn(32, 44, 64, device=dev) * 0.01
    x64 = torch.randn(6, 2048, device=dev).to(torch.bfloat16)
    y64 = ops.forward_mlp(x64, ops.spectra(ops.glu_weights(c64g, c64g)), ops.spectra(c64d), 64, 44 * 64)
    h = ops.forward_glu(x64, ops.spectra(ops.glu_weights(c64g, c64g)), 64, 44 * 64)
    y64r = ops.forward(h, ops.spectra(c64d), None, 64, 2048)
    # the C ABI's split form runs the down launch unsplit; ops.forward may split K at this size
    assert ((y64.float() - y64r.float()).norm() / y64r.float().norm()).item() < 2e-3


def test_llama_mlp_module_runs_one_launch(dev):
    """fuse_mlp_gate_up on a one-layer LLaMA-7B-width model (hidden 4096, intermediate 11008,
    every projection BC at b = 128, bf16): the MLP forward is the one-launch kernel, equal to its
    own two-launch composition bit for bit, and the logits match the unfused model."""
    transformers = pytest.importorskip("transformers")
    import patch_llama_fft as P
    torch.manual_seed(0)
    cfg = transformers.LlamaConfig(hidden_size=4096, intermediate_size=11008, num_hidden_layers=1,
                                   num_attention_heads=32, num_key_value_heads=32, vocab_size=256,
                                   max_position_embeddings=64)
    model = transformers.LlamaForCausalLM(cfg).to(dev).to(torch.bfloat16).eval()
    P.patch_linear_with_block_circulant(model, num_layers_to_patch=1, block_size=128)   # c stays fp32
    ids = torch.randint(0, 256, (2, 16), device=dev)
    mlp = model.model.layers[0].mlp
    x = torch.randn(2, 1024, 4096, device=dev).to(torch.bfloat16)    # 2048 tokens: AUTO is one launch
    xs = x[:, :16]                                                    # 32 tokens: the two launches
    from bcfft import ops
    with torch.no_grad():
        ref = model(input_ids=ids).logits.float()
        assert P.fuse_mlp_gate_up(model) == 1
        assert P._mlp_fused_ok(mlp, x) and ops.mlp_auto_is_fused(2048, 4096, 11008, 128, torch.bfloat16)
        assert ops.mlp_auto_is_fused(32, 4096, 11008, 128, torch.bfloat16)          # the group split
        assert not ops.mlp_auto_is_fused(2380, 4096, 11008, 128, torch.bfloat16)    # two launches
        y1 = mlp(x)
        sgu, sd = mlp._bc_gate_up._spectra(), mlp.down_proj._spectra(mlp.down_proj.c)
        y2 = ops.forward_mlp(x.reshape(-1, 4096), sgu, sd, 128, 11008, mode="split").view_as(y1)
        ys = mlp(xs)
        ys2 = ops.forward_mlp(xs.reshape(-1, 4096), sgu, sd, 128, 11008, mode="split").view_as(ys)
        out = model(input_ids=ids).logits.float()
    assert torch.equal(y1, y2)                      # one launch == the two-launch form, bit for bit
    assert ((ys.float() - ys2.float()).norm() / ys2.float().norm()).item() < 3e-3   # the group split
    assert ((out - ref).norm() / ref.norm()).item() < 2e-2


def test_torch_op_forward_mlp(dev):
    import bcfft.torch_ops  # noqa: F401
    from bcfft import ops
    cg, cu, cd = _weights(dev, 86, seed=8)
    x = torch.randn(13, HID, device=dev).to(torch.bfloat16)
    sgu, sd = ops.spectra(ops.glu_weights(cg, cu)), ops.spectra(cd)
    y = torch.ops.bcfft.forward_mlp(x, sgu, sd, B, 86 * B, "auto")
    assert torch.equal(y, ops.forward_mlp(x, sgu, sd, B, 86 * B))
    torch.library.opcheck(torch.ops.bcfft.forward_mlp.default, (x, sgu, sd, B, 86 * B, "fused"),
                          test_utils=("test_schema", "test_faketensor"))


@pytest.mark.parametrize("n,n_h", [(1, 86), (9, 86), (37, 86), (300, 86), (760, 86), (20, 33), (19, 127)])
def test_fused_splitk_short_grids(dev, n, n_h):
    """Decode / short-prefill sizes: the fused kernel with its gate/up groups (the down projection's
    K-chunks) split over kz workgroups per tile, fp32 partials summed in a fixed order and rounded
    once (BCFFT_MLP_FUSED_SPLITK, AUTO's choice here). Against the one-launch kernel (same
    numerics up to the slices' own down-projection reference exponents), the oracle, and
    itself (deterministic)."""
    from bcfft import _lib
    lib = _lib.load()
    assert lib.bcfft_forward_mlp_mode(n, HID, n_h * B, B, _lib.BCFFT_BF16, 0) == _lib.MLP_MODES["fused_splitk"]
    cg, cu, cd = _weights(dev, n_h, seed=40 + n)
    torch.manual_seed(n)
    x = torch.randn(n, HID, device=dev)
    if n >= 9:
        x[3] = 0
        x[5, :2048] *= 1e3
    x = x.to(torch.bfloat16)
    ys = _run(dev, x, cg, cu, cd, "fused_splitk")
    yf = _run(dev, x, cg, cu, cd, "fused")
    assert torch.isfinite(ys.float()).all()
    rms = yf.float().pow(2).mean().sqrt().item()
    d = (ys.float() - yf.float()).abs()
    assert (d <= 2.0 ** -7 * (yf.float().abs() + rms)).float().mean().item() > 0.999
    assert ((ys.float() - yf.float()).norm() / yf.float().norm()).item() < 3e-3
    assert torch.equal(ys, _run(dev, x, cg, cu, cd, "auto"))
    if n >= 9:
        assert (ys[3] == 0).all()
    if n <= 37:
        ref = oracle_mlp(x.float().cpu().numpy(), cg.cpu().numpy(), cu.cpu().numpy(), cd.cpu().numpy())
        assert rel_err(ys.float().cpu().numpy(), ref) < 4e-3
