"""GPU parity of the fused gate/up + SwiGLU launch (bcfft_forward_glu)
against the CPU oracle: h = silu(BC_gate(x)) * BC_up(x), the LLaMA MLP's inner product of
patch_mlp_with_block_circulant's gate/up projections (patch_llama_fft.py:343-394).

The oracle follows torch on the reference's tensors: gate(x) and up(x) rounded to x's dtype
(the BC forward's .to(x.dtype), patch_llama_fft.py:266), SiLU computed in fp32 and rounded,
the product rounded. The weights are fp16 in both engines (stationary ~3e-4 per output, DFT
~4e-4, `dftx` ~3e-4), and SiLU and the product carry that error along, so fp32 outputs are checked at 1e-3 relative Frobenius
and 16-bit outputs within ~2 output ulp plus 2e-3 (the weight error SiLU can amplify) per
element, plus the norm bound."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from oracle import bc_oracle as O

pytestmark = pytest.mark.gpu

TDT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}
ODT = {"float32": O.F32, "float16": O.F16, "bfloat16": O.BF16}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


def _silu(a):
    return a / (1.0 + np.exp(-a.astype(np.float64)))


def oracle_glu(x, cg, cu, xdt):
    xr = O.round_to(x, ODT[xdt])
    g = O.bc_forward(xr, cg, x_dtype=ODT[xdt])         # rounded to x dtype (:266)
    u = O.bc_forward(xr, cu, x_dtype=ODT[xdt])
    s = O.round_to(_silu(g).astype(np.float32), ODT[xdt])
    return O.round_to((s.astype(np.float64) * u).astype(np.float32), ODT[xdt])


def _check(h, ref, xdt):
    g = h.detach().float().cpu().numpy()
    assert g.shape == ref.shape and np.isfinite(g).all()
    e = rel_err(g, ref)
    if xdt == "float32":
        assert e < 1e-3, f"rel err {e:.3e}"
    else:
        ulp = 2.0 ** -7 if xdt == "bfloat16" else 2.0 ** -10
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        # 2 output ulp of rounding plus the weights' ~3-4e-4 carried through SiLU, whose relative
        # sensitivity |1 + g (1 - sigmoid(g))| reaches ~|g| for negative g: 2e-3 per element, and
        # an absolute 4 ulp of the rms (the weight error of large |u| * |g| products: measured
        # worst 3.1 with the DFT engine, fp16, 262k elements)
        bad = np.abs(g - ref) > (2 * ulp + 2e-3) * np.abs(ref) + 4 * ulp * rms
        worst = float(np.max(np.abs(g - ref) / ((2 * ulp + 2e-3) * np.abs(ref) + ulp * rms)))
        assert not bad.any(), f"{int(bad.sum())} elements beyond ~2 ulp (worst {worst:.2f} ulp of rms)"
        assert e < 4e-3, e
    return e


CASES = [
    # (K, M_gate, b, N, dtype)
    (4096, 11008, 128, 37, "bfloat16"),   # LLaMA-7B gate/up shape: 86 blocks -> 6 groups, last partial
    (4096, 4096, 128, 9, "float32"),
    (4096, 4096, 128, 64, "float16"),
    (4096, 11008, 64, 23, "bfloat16"),    # b = 64, 4 K-steps, 172 blocks -> 11 groups
    (2048, 5632, 64, 5, "float32"),       # b = 64, 2 K-steps, 88 blocks
    (4096, 2048, 128, 1, "float32"),      # one token, one group
]


@pytest.mark.parametrize("algo", ["auto", "stationary", "dftx"])
@pytest.mark.parametrize("k,m,b,n,xdt", CASES)
def test_glu_vs_oracle(dev, k, m, b, n, xdt, algo):
    if b != 128 and algo == "dftx":
        pytest.skip("the DFT kernel serves b = 128 with K = 4096")
    from bcfft import ops
    rng = np.random.default_rng(k + m + b + n)
    cg = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    cu = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    x = rng.standard_normal((n, k)).astype(np.float32)
    spec = ops.spectra(ops.glu_weights(torch.from_numpy(cg).to(dev), torch.from_numpy(cu).to(dev)))
    h = ops.forward_glu(torch.from_numpy(x).to(dev).to(TDT[xdt]), spec, b, m, algo=algo)
    torch.cuda.synchronize()
    assert h.dtype == TDT[xdt] and h.shape == (n, m)
    _check(h, oracle_glu(x, cg, cu, xdt), xdt)


@pytest.mark.parametrize("algo", ["stationary", "dft"])
def test_glu_equals_unfused_composition(dev, algo):
    """The fused launch against the same engine's two separate launches + torch SiLU and product
    (the fused weights share one fp16 scale, so roundings differ slightly)."""
    from bcfft import ops
    torch.manual_seed(3)
    k, m, b = 4096, 11008, 128
    cg = torch.randn(m // b, k // b, b, device=dev) * 0.01
    cu = torch.randn(m // b, k // b, b, device=dev) * 0.01
    x = torch.randn(301, k, device=dev).to(torch.bfloat16)
    h = ops.forward_glu(x, ops.spectra(ops.glu_weights(cg, cu)), b, m, algo=algo)
    ref = (torch.nn.functional.silu(ops.forward(x, ops.spectra(cg), None, b, m, algo=algo))
           * ops.forward(x, ops.spectra(cu), None, b, m, algo=algo))
    d = (h.float() - ref.float()).abs()
    assert (d <= 2 * 2.0 ** -7 * ref.float().abs() + 1e-6).float().mean().item() > 0.999
    assert ((h.float() - ref.float()).norm() / ref.float().norm()).item() < 4e-3


def test_glu_rejects_ineligible_geometry(dev):
    from bcfft import ops
    cg = torch.zeros(4, 4, 128, device=dev)
    spec = ops.spectra(ops.glu_weights(cg, cg))
    with pytest.raises(RuntimeError, match="block_size"):
        ops.forward_glu(torch.zeros(3, 512, device=dev), spec, 128, 512)
    c64 = torch.zeros(8, 32, 64, device=dev)                  # stationary geometry, not the DFT one
    spec64 = ops.spectra(ops.glu_weights(c64, c64))
    with pytest.raises(RuntimeError, match="block_size"):
        ops.forward_glu(torch.zeros(3, 2048, device=dev), spec64, 64, 512, algo="dft")


def test_fused_mlp_module_matches_unfused(dev):
    """BCFusedGateUp / fuse_mlp_gate_up on a one-layer LLaMA patched with b = 64 blocks."""
    transformers = pytest.importorskip("transformers")
    import patch_llama_fft as P
    torch.manual_seed(0)
    cfg = transformers.LlamaConfig(hidden_size=2048, intermediate_size=5632, num_hidden_layers=1,
                                   num_attention_heads=16, num_key_value_heads=16, vocab_size=256,
                                   max_position_embeddings=64)
    model = transformers.LlamaForCausalLM(cfg).eval()
    P.patch_mlp_with_block_circulant(model, num_layers_to_patch=1, block_size=64)
    model = model.to(dev)
    ids = torch.randint(0, 256, (2, 16), device=dev)
    with torch.no_grad():
        ref = model(input_ids=ids).logits.float()
        assert P.fuse_mlp_gate_up(model) == 1
        out = model(input_ids=ids).logits.float()
    assert ((out - ref).norm() / ref.norm()).item() < 1e-3


def test_fused_qkv_matches_unfused(dev):
    """fuse_attention_qkv: q/k/v of a GQA LLaMA layer (k/v narrower than q) in one launch over the
    concatenated weights, against the three separate launches (bit-identical per output block),
    then a whole one-layer LLaMA's logits."""
    transformers = pytest.importorskip("transformers")
    import patch_llama_fft as P
    torch.manual_seed(1)
    cfg = transformers.LlamaConfig(hidden_size=2048, intermediate_size=5632, num_hidden_layers=1,
                                   num_attention_heads=16, num_key_value_heads=4, vocab_size=256,
                                   max_position_embeddings=64)
    model = transformers.LlamaForCausalLM(cfg).eval()
    P.patch_linear_with_block_circulant(model, num_layers_to_patch=1, block_size=128)
    model = model.to(dev)
    attn = model.model.layers[0].self_attn
    x = torch.randn(3, 17, 2048, device=dev)
    ids = torch.randint(0, 256, (2, 16), device=dev)
    with torch.no_grad():
        sep = [attn.q_proj(x), attn.k_proj(x), attn.v_proj(x)]
        ref = model(input_ids=ids).logits.float()
        assert P.fuse_attention_qkv(model) == 1
        fused = [attn.q_proj(x), attn.k_proj(x), attn.v_proj(x)]
        out = model(input_ids=ids).logits.float()
    for a, b in zip(sep, fused):
        assert a.shape == b.shape and torch.equal(a, b)
    assert ((out - ref).norm() / ref.norm()).item() < 1e-6



def test_fused_routes_check_width_and_see_bias_updates(dev):
    """The fused q/k/v and gate/up routes raise the module's errors for a wrong-width input, and
    a bias-only update reaches the fused q/k/v launch."""
    import patch_llama_fft as P
    torch.manual_seed(3)
    mods = [P.BlockCirculantLinear(4096, m, block_size=128, bias=True).to(dev).eval() for m in (4096, 1024, 1024)]
    fused = P.BCFusedProjections(mods)
    x = torch.randn(2, 5, 4096, device=dev)
    with torch.no_grad():
        y0 = fused.output(0, x).clone()
        for i in (1, 2):
            fused.output(i, x)
        with pytest.raises(AssertionError):
            fused.output(0, torch.randn(2, 5, 2048, device=dev))
        with pytest.raises(RuntimeError):
            fused.output(0, torch.randn(10, 2048, device=dev))
        mods[0].bias.add_(1.0)                      # bias-only update
        y1 = fused.output(0, x)
        assert torch.allclose(y1, y0 + 1.0, rtol=1e-5, atol=1e-4)
        g = P.BlockCirculantLinear(4096, 4096, block_size=128, bias=False).to(dev).eval()
        u = P.BlockCirculantLinear(4096, 4096, block_size=128, bias=False).to(dev).eval()
        with pytest.raises(AssertionError):
            P.BCFusedGateUp(g, u)(torch.randn(1, 3, 2048, device=dev))
