"""Model-level harness helpers (llama-fft_amd/bc_eval.py) against per-row restatements of the
reference's formulas (src/bench_all_in_one.py:79-120, 295-345). CPU only: no kernel calls."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bc_eval as E  # noqa: E402


def _ref_metrics(s_rows, t_rows, temperature, topk):
    """The reference's one-prompt-at-a-time loop (bench_all_in_one.py:305-345)."""
    acc = dict(mse=0.0, kl=0.0, cos=0.0, top1=0, topk_in=0, ov=0.0)
    for s, t in zip(s_rows, t_rows):
        p = torch.softmax(t / temperature, -1)
        kl = (p * (torch.log_softmax(t / temperature, -1) - torch.log_softmax(s / temperature, -1))).sum()
        acc["mse"] += (s - t).pow(2).mean().item()
        acc["kl"] += kl.item()
        acc["cos"] += torch.nn.functional.cosine_similarity(s[None], t[None]).item()
        t1 = int(t.argmax())
        acc["top1"] += int(t1 == int(s.argmax()))
        sk = torch.topk(s, topk).indices.tolist()
        tk = torch.topk(t, topk).indices.tolist()
        acc["topk_in"] += int(t1 in sk)
        acc["ov"] += len(set(sk) & set(tk)) / topk
    n = len(s_rows)
    return {"last_mse": acc["mse"] / n, "last_kl": acc["kl"] / n, "last_cos": acc["cos"] / n,
            "last_top1_acc": acc["top1"] / n, "last_top1_in_student_topk": acc["topk_in"] / n,
            "last_topk_overlap": acc["ov"] / n}


@pytest.mark.parametrize("temperature,topk", [(1.0, 5), (2.0, 3)])
def test_last_token_metrics_match_reference_loop(temperature, topk):
    g = torch.Generator().manual_seed(0)
    t = torch.randn(7, 97, generator=g)
    s = t + 0.7 * torch.randn(7, 97, generator=g)
    got = E.last_token_metrics(s, t, temperature, topk)
    ref = _ref_metrics(s, t, temperature, topk)
    assert got.keys() == ref.keys()
    for k in ref:
        assert got[k] == pytest.approx(ref[k], rel=1e-5, abs=1e-6), k


def test_metrics_identity_and_shape_errors():
    t = torch.randn(3, 50)
    m = E.last_token_metrics(t.clone(), t)
    assert m["last_kl"] == pytest.approx(0.0, abs=1e-6) and m["last_mse"] == 0.0
    assert m["last_cos"] == pytest.approx(1.0) and m["last_top1_acc"] == 1.0
    assert m["last_topk_overlap"] == 1.0 and m["last_top1_in_student_topk"] == 1.0
    with pytest.raises(ValueError):
        E.last_token_metrics(t, t[:2])


def test_synthetic_prompts_seeded_and_bounded():
    a = E.synthetic_prompts(10, 32, 100, seed=3)
    b = E.synthetic_prompts(10, 32, 100, seed=3)
    assert all(torch.equal(x[0], y[0]) for x, y in zip(a, b))
    assert all(8 <= p[0].numel() <= 32 and p[0].min() >= 1 and p[0].max() < 100 for p in a)
    assert all(torch.equal(p[1], torch.ones_like(p[0])) for p in a)
    assert E.synthetic_prompts(0, 8, 10) == []


def test_pad_batch_and_gather_last():
    items = [(torch.tensor([5, 6, 7]), torch.ones(3, dtype=torch.long)),
             (torch.tensor([9]), torch.ones(1, dtype=torch.long))]
    ids, mask, last = E.pad_batch(items, pad_id=0)
    assert ids.tolist() == [[5, 6, 7], [9, 0, 0]]
    assert mask.tolist() == [[1, 1, 1], [1, 0, 0]]
    assert last.tolist() == [2, 0]
    logits = torch.arange(2 * 3 * 4, dtype=torch.float32).view(2, 3, 4)
    assert torch.equal(E.gather_last_logits(logits, last), torch.stack([logits[0, 2], logits[1, 0]]))
    batches = list(E.iter_batches(items * 3, 4, 0))
    assert [b[0].shape[0] for b in batches] == [4, 2]
    with pytest.raises(ValueError):
        E.pad_batch([], 0)


@pytest.mark.parametrize("n,world", [(100, 8), (99, 8), (5, 2), (3, 4)])
def test_prompt_shards_partition_in_order(n, world):
    items = E.synthetic_prompts(n, 16, 50, seed=1)
    shards = [E.prompt_shard(items, world, r) for r in range(world)]
    flat = [p for s in shards for p in s]
    assert len(flat) == n and all(a is b for a, b in zip(flat, items))


def test_llama2_7b_config_dims():
    pytest.importorskip("transformers")
    cfg = E.llama2_7b_config()
    assert (cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers) == (4096, 11008, 32)
    assert (cfg.num_attention_heads, cfg.num_key_value_heads, cfg.vocab_size) == (32, 32, 32000)
    # every projection is a BC geometry at b = 128
    assert cfg.hidden_size % 128 == 0 and cfg.intermediate_size % 128 == 0


def test_reference_checker_matches_explicit_dense():
    """model_bench's fp32 checker vs the explicit block-circulant matrix (C[r,s] = c[(r-s)%b])."""
    import model_bench as MB
    g = torch.Generator().manual_seed(2)
    n_out, n_in, b = 3, 2, 8
    c = torch.randn(n_out, n_in, b, generator=g, dtype=torch.float64)
    x = torch.randn(5, n_in * b, generator=g, dtype=torch.float64)
    idx = torch.arange(b)
    W = torch.cat([torch.cat([c[j, i][(idx[:, None] - idx[None, :]) % b] for i in range(n_in)], 1)
                   for j in range(n_out)], 0)
    got = MB.reference_bc_fp32(x, c, None).double()
    assert torch.allclose(got, x @ W.T, rtol=1e-5, atol=1e-5)
