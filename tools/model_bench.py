"""Model-level harness for BASELINE configs 3 and 5: LLaMA-2-7B with every
linear projection of every decoder layer block-circulant (b = 128), prefill and greedy-decode
throughput against the dense model, teacher/student last-token metrics, and a per-projection
parity check of the HIP engine on the model's own activations.

What the reference does (src/bench_all_in_one.py:270-460): cache the dense teacher's last-token
logits, patch, score the student (MSE / KL / cos / top-1 / top-k overlap), then time prefill over
padded batches and model.generate. Here:
  * the 7B architecture is built locally and random-initialised on the GPU in bf16 (no weights or
    tokenizer exist offline), and prompts are synthetic token ids with seeded lengths: the
    metrics show the harness working, not LLaMA quality;
  * patch_linear_with_block_circulant (q/k/v/o/gate/up/down; --targets mlp for the reference's
    MLP-only patch), then fuse_attention_qkv and fuse_mlp_gate_up (one launch for q/k/v; the
    whole MLP in one launch when all its projections are BC, else one for gate/up + SwiGLU);
  * multi-GPU (config 5): one process per GPU under torch.distributed.run; each rank holds the
    whole model and takes a contiguous slice of the prompts (prompt-level replicas, no collective
    in the forward); at the end ONE all-gather (RCCL) of the last-token logits. Throughput is all
    ranks' real tokens / the slowest rank's time.
  * parity: forward hooks capture each BC projection's input and output in the first patched
    layer during one student forward; the output is compared with a plain torch fp32 FFT
    evaluation of the same block-circulant operator (the checker, not the product). Outputs are
    bf16, so each entry also gives rounding_floor = |bf16(ref) - ref| / |ref|: the error of a
    perfect kernel that rounds once; rel_err close to it means the kernel adds little.

Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "llama-fft_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bc_eval as E  # noqa: E402


def reference_bc_fp32(x: torch.Tensor, c: torch.Tensor, bias) -> torch.Tensor:
    """Checker: y = C x in fp32 with torch.fft (patch_llama_fft.py:241-275's sequence)."""
    n_out, n_in, b = c.shape
    xf = torch.fft.rfft(x.float().reshape(-1, n_in, b), dim=-1)
    cf = torch.fft.rfft(c.float(), dim=-1)
    y = torch.fft.irfft(torch.einsum("nif,oif->nof", xf, cf), n=b, dim=-1).reshape(-1, n_out * b)
    return y if bias is None else y + bias.float()


def build_model(args, dev):
    from transformers import LlamaForCausalLM
    cfg = E.llama2_7b_config(args.layers, **json.loads(args.config_overrides))
    cfg._attn_implementation = "sdpa"
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        torch.manual_seed(args.seed)
        with torch.device(dev):
            model = LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(old)
    return model.eval()


COLL_DEV = "cuda"        # where collective operands live: "cpu" under --backend gloo


def sync_max(t: float) -> float:
    if dist.is_initialized():
        v = torch.tensor([t], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return float(v.item())
    return t


def barrier():
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()


@torch.inference_mode()
def prefill(model, batches, warmup, runs):
    """(last-token logits fp32 (P,V), seconds per run over all batches)."""
    lasts = []
    for ids, mask, last in batches:
        lasts.append(E.gather_last_logits(model(input_ids=ids, attention_mask=mask).logits, last).float())
    for _ in range(warmup):
        for ids, mask, _ in batches:
            model(input_ids=ids, attention_mask=mask)
    barrier()
    t0 = time.perf_counter()
    for _ in range(runs):
        for ids, mask, _ in batches:
            model(input_ids=ids, attention_mask=mask)
    barrier()
    return torch.cat(lasts), sync_max((time.perf_counter() - t0) / runs)


@torch.inference_mode()
def decode(model, batches, new_tokens, pad_id):
    kw = dict(max_new_tokens=new_tokens, min_new_tokens=new_tokens, do_sample=False, use_cache=True,
              pad_token_id=pad_id)
    ids, mask, _ = batches[0]
    model.generate(input_ids=ids[:, :8], attention_mask=mask[:, :8], **dict(kw, max_new_tokens=2,
                                                                          min_new_tokens=2))
    barrier()
    t0 = time.perf_counter()
    for ids, mask, _ in batches:
        model.generate(input_ids=ids, attention_mask=mask, **kw)
    barrier()
    return sync_max(time.perf_counter() - t0)


def gather_prompt_logits(last: torch.Tensor, n_prompts: int, group=None) -> torch.Tensor:
    """Config 5's one collective (bench_all_in_one.py:348-389 scores every prompt's last-token
    logits): this rank's (its prompt slice, V) logits to every rank, reassembled in prompt order.
    The slices are bc_eval.prompt_shard's contiguous shard_bounds, as gather_rows expects; RCCL
    all_gather_into_tensor on GPU ranks, gloo's list all-gather in the CPU test."""
    from bcfft.shard import gather_rows
    rows = gather_rows(last.contiguous(), n_prompts, group)
    assert rows.shape[0] == n_prompts
    return rows


def _keep(store, key, pick):
    """A hook that records pick(...) under key once and returns None (a forward hook's return
    value would replace the module's output)."""
    def hook(*args):
        store.setdefault(key, pick(*args))
    return hook


@torch.inference_mode()
def projection_parity(model, layer_idx, batch):
    """rel. Frobenius error of each BC projection of decoder layer layer_idx vs the fp32 checker,
    on the activations of one real forward."""
    import patch_llama_fft as P
    seen, hooks = {}, []
    layer = model.model.layers[layer_idx]
    for name, mod in layer.named_modules():
        if isinstance(mod, P.BlockCirculantLinear):
            hooks.append(mod.register_forward_hook(_keep(seen, name, lambda m, inp, out: (m, inp[0], out))))
    # the fused gate/up launch bypasses gate_proj/up_proj's __call__: capture the MLP input and
    # down_proj's input (= silu(gate(x)) * up(x)) instead
    # the one-launch MLP (bcfft_forward_mlp) bypasses all three projections: capture the MLP's
    # input and output
    mlp_io = {}
    if hasattr(layer.mlp, "_bc_gate_up"):
        hooks.append(layer.mlp.register_forward_hook(_keep(mlp_io, "x", lambda m, inp, out: inp[0])))
        hooks.append(layer.mlp.register_forward_hook(_keep(mlp_io, "y", lambda m, inp, out: out)))
        hooks.append(layer.mlp.down_proj.register_forward_pre_hook(_keep(mlp_io, "h", lambda m, inp: inp[0])))
    ids, mask, _ = batch
    try:
        model(input_ids=ids, attention_mask=mask)
    finally:
        for h in hooks:
            h.remove()

    def score(out, ref):
        # the kernel output is rounded to x's dtype (bf16): also compare with the rounded checker
        ref_r = ref.to(out.dtype).float()
        return {"rel_err": float((out.float() - ref).norm() / ref.norm()),
                "rounding_floor": float((ref_r - ref).norm() / ref.norm()),
                "rel_err_vs_rounded": float((out.float() - ref_r).norm() / ref_r.norm()),
                "tokens": int(out.shape[0])}

    errs = {}
    if "x" in mlp_io and "h" not in mlp_io:           # the whole MLP ran through bcfft_forward_mlp
        g, u, d = layer.mlp.gate_proj, layer.mlp.up_proj, layer.mlp.down_proj
        x = mlp_io["x"].reshape(-1, g.in_features)
        y = mlp_io["y"].reshape(-1, d.out_features)
        gr, ur = reference_bc_fp32(x, g.c, g.bias), reference_bc_fp32(x, u.c, u.bias)
        ref = reference_bc_fp32(torch.nn.functional.silu(gr) * ur, d.c, d.bias)
        errs["mlp(bcfft_forward_mlp)"] = score(y, ref)
        # "rounded": torch's own bf16 sequence (gate, up, silu, product, down rounded to x dtype)
        h_r = (torch.nn.functional.silu(gr.to(y.dtype)) * ur.to(y.dtype))
        ref_r = reference_bc_fp32(h_r, d.c, d.bias).to(y.dtype).float()
        errs["mlp(bcfft_forward_mlp)"].update(rel_err_vs_rounded=float((y.float() - ref_r).norm() / ref_r.norm()),
                                       rounding_floor=float((ref_r - ref).norm() / ref.norm()))
    for name, (m, x, y) in seen.items():
        if name.endswith(("gate_proj", "up_proj")) and "h" in mlp_io:
            continue
        ref = reference_bc_fp32(x.reshape(-1, m.in_features), m.c, m.bias)
        errs[name] = score(y.reshape(-1, m.out_features), ref)
    if "h" in mlp_io:
        g, u = layer.mlp.gate_proj, layer.mlp.up_proj
        x = mlp_io["x"].reshape(-1, g.in_features)
        h = mlp_io["h"].reshape(-1, g.out_features)
        gr, ur = reference_bc_fp32(x, g.c, g.bias), reference_bc_fp32(x, u.c, u.bias)
        ref = torch.nn.functional.silu(gr) * ur
        errs["mlp.gate_up_swiglu(fused)"] = score(h, ref)
        # "rounded" for the fused epilogue = torch's own sequence on the rounded projections
        # (gate, up -> x dtype; silu, product in x dtype), which the kernel reproduces
        ref_r = (torch.nn.functional.silu(gr.to(h.dtype)) * ur.to(h.dtype)).float()
        errs["mlp.gate_up_swiglu(fused)"].update(
            rel_err_vs_rounded=float((h.float() - ref_r).norm() / ref_r.norm()),
            rounding_floor=float((ref_r - ref).norm() / ref.norm()))
    return errs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32, help="decoder layers of the model")
    ap.add_argument("--block-sizes", default="128", help="comma list, as bench_all_in_one's --block_sizes")
    ap.add_argument("--num-layers", type=int, default=-1, help="layers to patch (-1: all)")
    ap.add_argument("--patch-position", default="first", choices=["first", "last"])
    ap.add_argument("--targets", default="all", choices=["all", "mlp"])
    ap.add_argument("--prompts", type=int, default=100, help="prompts over all ranks (prompts_100.txt: 99)")
    ap.add_argument("--max-len", type=int, default=128)
    ap.add_argument("--batch-size", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--new-tokens", type=int, default=32, help="greedy decode length (0: skip)")
    ap.add_argument("--dense", type=int, default=1, help="also time the dense (teacher) model's decode")
    ap.add_argument("--topk", type=int, default=5)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--config-overrides", default="{}", help="JSON LlamaConfig overrides (tests)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group under a launcher: nccl (RCCL, one GPU per rank; the product path) "
                         "or gloo (tests: several ranks sharing one GPU, which RCCL refuses; the logits "
                         "gather then runs on host copies)")
    ap.add_argument("--dump-logits", default="",
                    help="rank 0 saves the student's last-token logits of ALL prompts (after the all-gather "
                         "when distributed) and the teacher's local ones to this .pt file (tests)")
    args = ap.parse_args(argv)
    block_sizes = [int(b) for b in args.block_sizes.split(",") if b.strip()]

    import patch_llama_fft as P
    # under torch.distributed.run (WORLD_SIZE set, any world size, 1 included) the RCCL group is
    # created with device_id before the GPU is touched, and every collective below keys on
    # dist.is_initialized(): the config-5 path runs whenever a launcher started this process
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("model_bench needs a ROCm GPU (the BC engine has no CPU path)")
    global COLL_DEV
    gloo = args.backend == "gloo"
    # gloo: ranks may share a device (the one-GPU test of the world > 1 path)
    dev_index = local % torch.cuda.device_count() if gloo else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    own_pg = launched and not dist.is_initialized()
    if own_pg:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    COLL_DEV = "cpu" if gloo else "cuda"

    if args.prompts < world:
        raise SystemExit(f"--prompts {args.prompts} < {world} ranks: every rank needs a prompt")
    model = build_model(args, dev)
    cfg = model.config
    prompts = E.synthetic_prompts(args.prompts, args.max_len, cfg.vocab_size, seed=args.seed)
    mine = E.prompt_shard(prompts, world, rank)
    batches = [tuple(t.to(dev) for t in b) for b in E.iter_batches(mine, args.batch_size, cfg.pad_token_id)]
    my_tokens = sum(int(a.sum()) for _, a in mine)
    tok = torch.tensor([my_tokens], device=COLL_DEV)
    if dist.is_initialized():
        dist.all_reduce(tok)
    total_tokens = int(tok.item())
    n_patch = cfg.num_hidden_layers if args.num_layers < 0 else args.num_layers
    patched = P._layer_indices(cfg.num_hidden_layers, n_patch, args.patch_position)

    teacher_last, t_dense = prefill(model, batches, args.warmup, args.runs)
    dense_decode_s = decode(model, batches, args.new_tokens, cfg.pad_token_id) if args.dense and args.new_tokens else None

    line = None
    for bi, b in enumerate(block_sizes):
        if bi > 0:                      # patching is in place: rebuild the same seeded dense model
            del model
            torch.cuda.empty_cache()
            model = build_model(args, dev)
        res = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        patch = P.patch_linear_with_block_circulant if args.targets == "all" else P.patch_mlp_with_block_circulant
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):         # the patcher logs every projection
            patch(model, num_layers_to_patch=n_patch, block_size=b, patch_position=args.patch_position)
        n_qkv = P.fuse_attention_qkv(model)
        n_glu = P.fuse_mlp_gate_up(model)
        torch.cuda.synchronize()
        res["patch_s"] = time.perf_counter() - t0
        torch.cuda.empty_cache()

        student_last, t_bc = prefill(model, batches, args.warmup, args.runs)
        metrics = E.last_token_metrics(student_last, teacher_last, args.temperature, args.topk)
        parity = projection_parity(model, patched[0], batches[0]) if patched else {}
        if args.new_tokens:
            res["bc_decode_s"] = decode(model, batches, args.new_tokens, cfg.pad_token_id)

        # config 5's single collective: every rank's last-token logits to every rank (RCCL). The
        # prompt shards are shard_bounds' contiguous slices, so gather_rows reassembles them in order.
        all_last = student_last
        if dist.is_initialized():
            barrier()
            tg = time.perf_counter()
            all_last = gather_prompt_logits(student_last.to(COLL_DEV), args.prompts).to(dev)
            barrier()
            res["allgather_logits_s"] = sync_max(time.perf_counter() - tg)
        if args.dump_logits and rank == 0 and bi == 0:
            torch.save({"student_last": all_last.cpu(), "teacher_last_local": teacher_last.cpu(),
                        "world": world}, args.dump_logits)

        if rank == 0:
            n_prompts_new = args.prompts * args.new_tokens
            line = {
                "metric": "BC-patched LLaMA-2-7B prefill tokens/s",
                "value": round(total_tokens / t_bc, 1), "unit": "tokens/s", "n_gpus": world,
                "higher_is_better": True, "scaling": "weak" if world == 1 else "strong",
                "data": "synthetic prompts (seeded ids, lengths U[max_len/4, max_len]); random-init "
                        "LLaMA-2-7B architecture, bf16 (no weights/tokenizer offline)",
                "config": {"layers": cfg.num_hidden_layers, "hidden": cfg.hidden_size,
                           "intermediate": cfg.intermediate_size, "vocab": cfg.vocab_size,
                           "block_size": b, "targets": args.targets, "patched_layers": len(patched),
                           "patch_position": args.patch_position,
                           "prompts": args.prompts, "max_len": args.max_len,
                           "batch_size": args.batch_size, "tokens": total_tokens,
                           "fused_qkv_layers": n_qkv, "fused_gate_up_layers": n_glu,
                           "parallelism": f"prompt-replicas x{world}"},
                "prefill_ms": round(t_bc * 1e3, 3),
                "dense_prefill_ms": round(t_dense * 1e3, 3),
                "dense_prefill_tokens_per_s": round(total_tokens / t_dense, 1),
                "bc_vs_dense_prefill": round(t_dense / t_bc, 3),
                "patch_s": round(res["patch_s"], 3),
                "teacher_student": metrics,
                "projection_parity_first_patched_layer": parity,
            }
            if "bc_decode_s" in res:
                line["decode_new_tokens_per_s"] = round(n_prompts_new / res["bc_decode_s"], 1)
            if dense_decode_s:
                line["dense_decode_new_tokens_per_s"] = round(n_prompts_new / dense_decode_s, 1)
            if "allgather_logits_s" in res:
                line["allgather_logits_ms"] = round(res["allgather_logits_s"] * 1e3, 3)
                line["value_with_allgather"] = round(total_tokens / (t_bc + res["allgather_logits_s"]), 1)
            print(json.dumps(line), flush=True)
    if own_pg:
        dist.destroy_process_group()
    return line if rank == 0 else None


if __name__ == "__main__":
    main()
