"""The drop-in module surface (patch_llama_fft / fft_utils) on the CPU: constructor contract,
weight preparation (from_linear) against the reference's golden vectors, param I/O format and
the model patcher on a tiny locally-built LLaMA. No kernel runs here."""
import os

import numpy as np
import pytest
import torch

from golden_io import load, names, rel_err


@pytest.fixture(scope="module")
def plf(built_lib):
    import patch_llama_fft
    return patch_llama_fft


def test_constructor_contract(plf):
    m = plf.BlockCirculantLinear(512, 256, block_size=128)
    assert (m.in_features, m.out_features, m.block_size) == (512, 256, 128)
    assert (m.in_blocks, m.out_blocks) == (4, 2)
    assert m.c.shape == (2, 4, 128) and m.c.dtype == torch.float32
    assert m.bias.shape == (256,) and torch.all(m.bias == 0)
    assert 0.005 < m.c.std().item() < 0.02                       # randn * 0.01 (:171-173)
    assert set(m.state_dict()) == {"c", "bias"}
    assert plf.BlockCirculantLinear(256, 256, block_size=64, bias=False).bias is None
    with pytest.raises(AssertionError, match="in_features must be divisible"):
        plf.BlockCirculantLinear(100, 256, block_size=64)
    with pytest.raises(AssertionError, match="out_features must be divisible"):
        plf.BlockCirculantLinear(256, 100, block_size=64)
    assert plf.BLOCK_SIZE == 256 and plf.NUM_LAYERS_TO_PATCH == 1


def test_default_block_size(plf):
    assert plf.BlockCirculantLinear(512, 512).block_size == 256


@pytest.mark.parametrize("name", names("from_linear_"))
def test_from_linear_vs_reference_golden(plf, name):
    g = load(name)
    dt = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[g["w__dt"]]
    m, k = g["w"].shape
    lin = torch.nn.Linear(k, m, bias="lin_bias" in g).to(dt)
    with torch.no_grad():
        lin.weight.copy_(torch.from_numpy(g["w"]))
        if "lin_bias" in g:
            lin.bias.copy_(torch.from_numpy(g["lin_bias"]))
    bc = plf.BlockCirculantLinear.from_linear(lin, block_size=int(g["block_size"]))
    assert bc.c.dtype == torch.float32                            # c stays fp32 (:192-198)
    tol = 1e-6 if dt == torch.float32 else 1e-3
    assert rel_err(bc.c.detach().numpy(), g["c"]) < tol
    if "bias" in g:
        assert np.array_equal(bc.bias.detach().numpy(), g["bias"])


def test_projection_helpers(plf):
    g = load("project_t2_exact")
    c = plf.dense_block_to_circulant_column_loss_aware(torch.from_numpy(g["w"]))
    assert torch.allclose(c, torch.from_numpy(g["c"]), rtol=1e-6, atol=1e-6)
    c0 = torch.randn(16)
    C = plf.circulant_from_first_col(c0)
    idx = torch.arange(16)
    assert torch.equal(C, c0[(idx[:, None] - idx[None, :]) % 16])
    assert torch.allclose(plf.dense_block_to_circulant_column(C.T.contiguous()), c0, atol=1e-6)
    with pytest.raises(ValueError):
        plf.dense_block_to_circulant_column(C, convention="bogus")


def test_save_load_roundtrip(plf, tmp_path):
    net = torch.nn.Sequential(plf.BlockCirculantLinear(256, 128, block_size=64),
                              plf.BlockCirculantLinear(128, 256, block_size=64, bias=False))
    p = os.path.join(tmp_path, "sub", "bc.pt")
    plf.save_bc_params(net, p)
    state = torch.load(p, weights_only=True)
    assert set(state) == {"0.c", "0.bias", "1.c"}
    net2 = torch.nn.Sequential(plf.BlockCirculantLinear(256, 128, block_size=64),
                               plf.BlockCirculantLinear(128, 256, block_size=64, bias=False))
    plf.load_bc_params(net2, p)
    assert torch.equal(net2[0].c, net[0].c) and torch.equal(net2[1].c, net[1].c)
    # mismatched shape is skipped under strict_shapes
    net3 = torch.nn.Sequential(plf.BlockCirculantLinear(256, 128, block_size=32))
    plf.load_bc_params(net3, p)
    assert not torch.equal(net3[0].c.flatten()[:10], net[0].c.flatten()[:10])


def test_load_skips_like_the_reference(plf, tmp_path, capsys):
    """load_bc_params (patch_llama_fft.py:303-340): entries that are not .c / .bias, name no
    module or attribute, or mismatch in shape are skipped and counted; the rest are copied in
    the parameter's dtype."""
    net = torch.nn.Sequential(plf.BlockCirculantLinear(128, 128, block_size=64))
    p = os.path.join(tmp_path, "bc.pt")
    state = {"0.c": torch.randn(2, 2, 64, dtype=torch.float64), "0.bias": torch.randn(128),
             "0.weight": torch.randn(3), "7.c": torch.randn(2, 2, 64), "0.zz.c": torch.randn(1),
             "0.c.bias": torch.randn(1)}
    torch.save(state, p)
    plf.load_bc_params(net, p)
    out = capsys.readouterr().out
    assert "loaded=2, skipped=4" in out, out
    assert net[0].c.dtype == torch.float32 and torch.equal(net[0].c, state["0.c"].float())
    assert torch.equal(net[0].bias, state["0.bias"])
    torch.save({"0.c": torch.randn(1, 2, 64)}, p)
    plf.load_bc_params(net, p, strict_shapes=False)       # non-strict: copy_ broadcasts or raises
    assert "loaded=1, skipped=0" in capsys.readouterr().out


def _tiny_llama():
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=64, hidden_size=256, intermediate_size=512, num_hidden_layers=3,
                      num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=64)
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg).eval()


def test_patch_mlp_first_last(plf):
    model = _tiny_llama()
    plf.patch_mlp_with_block_circulant(model, num_layers_to_patch=2, block_size=128, patch_position="last")
    kinds = [type(l.mlp.up_proj).__name__ for l in model.model.layers]
    assert kinds == ["Linear", "BlockCirculantLinear", "BlockCirculantLinear"]
    assert type(model.model.layers[2].self_attn.q_proj).__name__ == "Linear"
    with pytest.raises(ValueError):
        plf.patch_mlp_with_block_circulant(model, num_layers_to_patch=-1)
    with pytest.raises(ValueError):
        plf.patch_mlp_with_block_circulant(model, patch_position="middle")


def test_patch_all_linear(plf):
    model = _tiny_llama()
    plf.patch_linear_with_block_circulant(model, num_layers_to_patch=1, block_size=64)
    l0 = model.model.layers[0]
    for name in ("q_proj", "k_proj", "v_proj", "o_proj"):
        assert isinstance(getattr(l0.self_attn, name), plf.BlockCirculantLinear)
    assert isinstance(l0.mlp.down_proj, plf.BlockCirculantLinear)
    assert l0.mlp.down_proj.bias is None                           # LLaMA: mlp_bias=False


def test_forward_refuses_cpu(plf):
    m = plf.BlockCirculantLinear(128, 128, block_size=64)
    with pytest.raises(RuntimeError, match="ROCm device"):
        m(torch.zeros(2, 128))
    with pytest.raises(ValueError, match="Unsupported input dim"):
        m(torch.zeros(128))


def test_glu_weights_interleave_groups():
    """bcfft_forward_glu's weight layout: group g = gate blocks [16g, 16g+16), up blocks."""
    from bcfft import ops
    g = torch.randn(40, 3, 8)
    u = torch.randn(40, 3, 8)
    w = ops.glu_weights(g, u)
    assert w.shape == (96, 3, 8)
    for grp in range(3):
        n = min(16, 40 - 16 * grp)
        assert torch.equal(w[32 * grp:32 * grp + n], g[16 * grp:16 * grp + n])
        assert torch.equal(w[32 * grp + 16:32 * grp + 16 + n], u[16 * grp:16 * grp + n])
        assert (w[32 * grp + n:32 * grp + 16] == 0).all() and (w[32 * grp + 16 + n:32 * grp + 32] == 0).all()


def test_fuse_mlp_gate_up_rewires_without_new_parameters():
    transformers = pytest.importorskip("transformers")
    import patch_llama_fft as P
    cfg = transformers.LlamaConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=4, vocab_size=64)
    model = transformers.LlamaForCausalLM(cfg)
    P.patch_mlp_with_block_circulant(model, num_layers_to_patch=1, block_size=64)
    keys = sorted(model.state_dict().keys())
    assert P.fuse_mlp_gate_up(model) == 1           # only the patched layer qualifies
    assert sorted(model.state_dict().keys()) == keys
    assert isinstance(model.model.layers[0].mlp._bc_gate_up, P.BCFusedGateUp)


def test_fuse_attention_qkv_rewires_without_new_parameters():
    transformers = pytest.importorskip("transformers")
    import patch_llama_fft as P
    cfg = transformers.LlamaConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, vocab_size=64)
    model = transformers.LlamaForCausalLM(cfg)
    P.patch_linear_with_block_circulant(model, num_layers_to_patch=1, block_size=64)
    keys = sorted(model.state_dict().keys())
    assert P.fuse_attention_qkv(model) == 1         # only the patched layer qualifies
    assert sorted(model.state_dict().keys()) == keys
    fused = model.model.layers[0].self_attn._bc_qkv
    assert fused.splits == [256, 128, 128]          # GQA: k/v have num_key_value_heads * head_dim
    with pytest.raises(RuntimeError, match="ROCm device"):   # no CPU path behind the fused route
        model.model.layers[0].self_attn.q_proj(torch.zeros(2, 256))



def test_flatten_reference_errors(plf):
    """The module's (and the fused routes') input checks raise the reference's exceptions:
    AssertionError for a 3D input of the wrong width (:230), the reshape's RuntimeError for a 2D
    one (:246), ValueError for other ranks (:239)."""
    m = plf.BlockCirculantLinear(256, 128, block_size=64)
    assert m._flatten(torch.zeros(2, 3, 256)).shape == (6, 256)
    with pytest.raises(AssertionError):
        m._flatten(torch.zeros(2, 3, 192))
    with pytest.raises(RuntimeError):
        m._flatten(torch.zeros(5, 192))
    with pytest.raises(ValueError, match="Unsupported input dim"):
        m._flatten(torch.zeros(1, 2, 3, 256))


def test_spectra_buffer_size_is_checked():
    """ops.forward / forward_glu refuse a spectra buffer built for a smaller operator before
    anything reaches the library (which cannot see the buffer's size)."""
    from bcfft import ops
    ok = torch.empty(ops.spectra_numel(32, 32, 128), dtype=torch.float32)
    ops._check_spectra(ok, 32, 32, 128, "t")
    with pytest.raises(ValueError, match="does not hold"):
        ops._check_spectra(ok, 86, 32, 128, "t")
    with pytest.raises(ValueError, match="does not hold"):
        ops._check_spectra(ok.to(torch.float16), 32, 32, 128, "t")
