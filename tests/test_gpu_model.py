"""Model-level GPU check of tools/model_bench.py on a small LLaMA (2 layers, hidden 1024,
MLP 2816): every linear projection BC at b = 128, q/k/v and gate/up fused; each projection's
output on the model's own activations vs the fp32 checker, and the harness's JSON line."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu


def test_inference_mode_patched_llama():
    """torch.inference_mode (the reference harnesses' decorator, and model.generate): patching,
    fused q/k/v and fused gate/up all run on inference tensors, which carry no version counter,
    and give the logits of the same model under no_grad."""
    transformers = pytest.importorskip("transformers")
    import patch_llama_fft as P
    torch.manual_seed(3)
    cfg = transformers.LlamaConfig(hidden_size=1024, intermediate_size=2816, num_hidden_layers=2,
                                   num_attention_heads=8, num_key_value_heads=8, vocab_size=256,
                                   max_position_embeddings=64)
    model = transformers.LlamaForCausalLM(cfg).eval().cuda()
    with torch.inference_mode():
        P.patch_linear_with_block_circulant(model, num_layers_to_patch=2, block_size=128)
    assert P.fuse_attention_qkv(model) == 2 and P.fuse_mlp_gate_up(model) == 2
    ids = torch.randint(0, 256, (2, 12), device="cuda")
    with torch.no_grad():
        ref = model(input_ids=ids).logits.float()
    with torch.inference_mode():
        out = model(input_ids=ids).logits.float()
        gen = model.generate(input_ids=ids, max_new_tokens=3, min_new_tokens=3, do_sample=False,
                             pad_token_id=0)
    assert torch.equal(out, ref)
    assert gen.shape == (2, 15)


@pytest.mark.parametrize("targets", ["all", "mlp"])
def test_model_bench_small_llama(targets):
    pytest.importorskip("transformers")
    assert torch.cuda.is_available()
    import model_bench as MB
    line = MB.main(["--layers", "2", "--prompts", "6", "--max-len", "40", "--batch-size", "3",
                    "--runs", "1", "--warmup", "1", "--new-tokens", "4", "--targets", targets,
                    "--block-sizes", "64,128",
                    "--config-overrides",
                    '{"hidden_size": 1024, "intermediate_size": 2816, "num_attention_heads": 8, '
                    '"num_key_value_heads": 8, "vocab_size": 512}'])
    cfg = line["config"]
    assert cfg["block_size"] == 128 and cfg["patched_layers"] == 2
    assert cfg["fused_qkv_layers"] == (2 if targets == "all" else 0) and cfg["fused_gate_up_layers"] == 2
    assert line["value"] > 0 and line["decode_new_tokens_per_s"] > 0
    par = line["projection_parity_first_patched_layer"]
    want = {"mlp.down_proj", "mlp.gate_up_swiglu(fused)"}
    if targets == "all":
        want |= {"self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj", "self_attn.o_proj"}
    assert want <= set(par), par
    for name, r in par.items():
        # bf16 outputs: one rounding alone is ~1e-3 rms relative vs fp32 (the fused SwiGLU has
        # four: gate, up, silu, product), so the 1e-3 bar is on the rounded checker
        assert r["rel_err_vs_rounded"] < 1e-3, (name, r)
        assert r["rel_err"] < 5e-3, (name, r)
    for k in ("last_kl", "last_cos", "last_top1_acc", "last_topk_overlap"):
        assert k in line["teacher_student"]


def test_model_bench_last_k_layers():
    """--num-layers / --patch-position (the reference patcher's first/last k): the last layer only."""
    pytest.importorskip("transformers")
    import model_bench as MB
    line = MB.main(["--layers", "3", "--prompts", "4", "--max-len", "24", "--batch-size", "2",
                    "--runs", "1", "--warmup", "0", "--new-tokens", "0", "--num-layers", "1",
                    "--patch-position", "last", "--config-overrides",
                    '{"hidden_size": 1024, "intermediate_size": 2816, "num_attention_heads": 8, '
                    '"num_key_value_heads": 8, "vocab_size": 512}'])
    cfg = line["config"]
    assert cfg["patched_layers"] == 1 and cfg["fused_qkv_layers"] == 1 and cfg["fused_gate_up_layers"] == 1
    for name, r in line["projection_parity_first_patched_layer"].items():
        assert r["rel_err_vs_rounded"] < 1e-3, (name, r)
