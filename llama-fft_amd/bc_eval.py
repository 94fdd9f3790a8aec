"""Model-level evaluation helpers for a BC-patched LLaMA (BASELINE configs 3/5).

The teacher/student metrics and batching of src/bench_all_in_one.py, restated over batches:
  * pad_batch / iter_batches      bench_all_in_one.py:79-101 (right padding, last real index)
  * gather_last_logits            bench_all_in_one.py:103-110
  * softmax_kl                    bench_all_in_one.py:112-120 (KL(teacher || student), per row)
  * last_token_metrics            bench_all_in_one.py:295-345 (same keys; the reference loops
                                  one prompt at a time, here a batch of rows is scored at once
                                  with the same per-row formulas and averaged the same way)
  * prompt shards                 SURVEY.md §8e, config 5: prompt-level replicas, each rank takes
                                  a contiguous slice of the prompt list
No tokenizer or LLaMA weights exist offline, so prompts are synthetic token ids with seeded
lengths (synthetic_prompts) and models are random-init; tools/model_bench.py says so in its output.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Sequence, Tuple

import torch
import torch.nn.functional as F

Prompt = Tuple[torch.Tensor, torch.Tensor]          # (input_ids 1-D long, attention_mask 1-D long)


def synthetic_prompts(n: int, max_len: int, vocab: int, seed: int = 0,
                      min_len: int | None = None) -> List[Prompt]:
    """n prompts of seeded lengths in [min_len, max_len] (default max_len // 4) and uniform ids
    in [1, vocab) (0 is left for padding); all-ones masks, as tokenize_prompts gives
    (bench_all_in_one.py:65-77 with truncation to max_len)."""
    if n < 0 or max_len < 1 or vocab < 2:
        raise ValueError("need n >= 0, max_len >= 1, vocab >= 2")
    lo = max(1, max_len // 4) if min_len is None else max(1, min(min_len, max_len))
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(lo, max_len + 1, (n,), generator=g).tolist()
    out = []
    for ln in lens:
        ids = torch.randint(1, vocab, (ln,), generator=g, dtype=torch.long)
        out.append((ids, torch.ones(ln, dtype=torch.long)))
    return out


def pad_batch(items: Sequence[Prompt], pad_id: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Right-pad to the longest prompt: input_ids (B,T), attention_mask (B,T), last_idx (B,)."""
    if not items:
        raise ValueError("empty batch")
    t = max(int(ids.numel()) for ids, _ in items)
    input_ids = torch.full((len(items), t), pad_id, dtype=torch.long)
    mask = torch.zeros((len(items), t), dtype=torch.long)
    last = torch.empty(len(items), dtype=torch.long)
    for i, (ids, attn) in enumerate(items):
        input_ids[i, :ids.numel()] = ids
        mask[i, :attn.numel()] = attn
        last[i] = int(attn.sum()) - 1
    return input_ids, mask, last


def iter_batches(items: Sequence[Prompt], batch_size: int, pad_id: int) -> Iterator[Tuple[torch.Tensor, ...]]:
    if batch_size < 1:
        raise ValueError("batch_size must be >= 1")
    for i in range(0, len(items), batch_size):
        yield pad_batch(items[i:i + batch_size], pad_id)


def gather_last_logits(logits: torch.Tensor, last_idx: torch.Tensor) -> torch.Tensor:
    """(B,T,V) logits at each row's last real position -> (B,V)."""
    return logits[torch.arange(logits.shape[0], device=logits.device), last_idx.to(logits.device)]


def softmax_kl(student: torch.Tensor, teacher: torch.Tensor, temperature: float = 1.0) -> torch.Tensor:
    """KL(teacher || student) over the last dim at temperature T, per row."""
    t = float(temperature)
    log_p = torch.log_softmax(teacher / t, dim=-1)
    log_q = torch.log_softmax(student / t, dim=-1)
    return (log_p.exp() * (log_p - log_q)).sum(dim=-1)


def last_token_metrics(student: torch.Tensor, teacher: torch.Tensor, temperature: float = 1.0,
                       topk: int = 5) -> Dict[str, float]:
    """Mean over rows of the reference's last-token metrics (both (B,V), scored in fp32)."""
    if student.shape != teacher.shape or student.dim() != 2:
        raise ValueError("student and teacher last-token logits must both be (B, V)")
    s, t = student.float(), teacher.float()
    n = max(s.shape[0], 1)
    s_top1, t_top1 = s.argmax(-1), t.argmax(-1)
    s_topk = torch.topk(s, topk, dim=-1).indices
    t_topk = torch.topk(t, topk, dim=-1).indices
    in_topk = (s_topk == t_top1[:, None]).any(-1)
    overlap = (s_topk[:, :, None] == t_topk[:, None, :]).any(-1).sum(-1).float() / topk
    return {
        "last_mse": float((s - t).pow(2).mean(-1).sum()) / n,
        "last_kl": float(softmax_kl(s, t, temperature).sum()) / n,
        "last_cos": float(F.cosine_similarity(s, t, dim=-1).sum()) / n,
        "last_top1_acc": float((s_top1 == t_top1).sum()) / n,
        "last_top1_in_student_topk": float(in_topk.sum()) / n,
        "last_topk_overlap": float(overlap.sum()) / n,
    }


def prompt_shard(items: Sequence[Prompt], world: int, rank: int) -> List[Prompt]:
    """Rank's contiguous slice of the prompt list (ceil-sized, the tail rank shorter)."""
    from bcfft.shard import shard_bounds
    lo, hi = shard_bounds(len(items), world, rank)
    return list(items[lo:hi])


def llama2_7b_config(num_layers: int = 32, **overrides):
    """LLaMA-2-7B architecture (hidden 4096, MLP 11008, 32 heads, 32 KV heads, vocab 32000), built
    locally: no model-name fetch (the reference reads it from the checkpoint at MODEL_PATH)."""
    from transformers import LlamaConfig
    kw = dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008,
              num_hidden_layers=num_layers, num_attention_heads=32, num_key_value_heads=32,
              max_position_embeddings=4096, rms_norm_eps=1e-5, hidden_act="silu",
              tie_word_embeddings=False, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    kw.update(overrides)
    return LlamaConfig(**kw)
