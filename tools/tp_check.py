#!/usr/bin/env python3
"""TP correctness + latency check, one process per rank (torchrun; ranks may share one GPU).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/tp_check.py \
      --out gpurun_out/tp.json [--model test-mistral-shape] [--gguf path]

1. all-reduce numerics: random fp32 vectors of several sizes (decode 1x d ... prefill chunks of
   600 x d, which take the two-shot reduce-scatter + all-gather path and are split into several
   calls), with and without the fused residual, fp32 and bf16 two-shot staging, against torch's
   sum of every rank's input (gathered via gloo); the column all-gather of the vocab-parallel
   lm_head on a rows x (world * slice) matrix;
2. model: a synthetic GGUF (written by rank 0) is loaded sharded on every rank (vocab-parallel
   lm_head) and greedily decoded through prefill (--prompt-len tokens) + per-step decode + graph
   decode loop; rank 0 also loads it unsharded (TP=1) and compares the token streams and logits;
3. timing of the one-shot all-reduce at decode size and of the two-shot at prefill size.
Writes one JSON summary (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/tp.json")
    ap.add_argument("--model", default="test-mistral-shape")
    ap.add_argument("--recipe", default="Q4_K_M")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--prompt-len", type=int, default=21)
    ap.add_argument("--batch", type=int, default=0,
                    help="also decode B >= 5 rows (the skinny-GEMM path, C1 / C2 fused with the next RMSNorm) "
                         "and compare every row's logits against the unsharded engine at the same batch")
    ap.add_argument("--act-q8", action="store_true",
                    help="int8 GEMV activations on both sides (the production decode path: with TP the batch-1 O / "
                         "down all-reduces then run in the GEMV epilogue, EPI_TP_RESID, unless AIOS_TP_FUSE=0)")
    ap.add_argument("--dump-logits", action="store_true", help="store every decode step's logits in the JSON")
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    from aios_amd.parallel.tp import build_tp_engine, create_comm, local_device, worker_loop, TPEngine
    from aios_amd.models.config import get_preset

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = local_device(int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    res = {"world": world, "device_count": torch.cuda.device_count()}
    t_start = time.time()

    def log(msg):  # progress on stderr (rank 0): a silent multi-minute run reads as a hang
        if rank == 0:
            print(f"[tp_check {time.time() - t_start:6.1f}s] {msg}", file=sys.stderr, flush=True)

    log(f"world {world}, {torch.cuda.device_count()} device(s)")

    # ---- 1. collective numerics
    comm = create_comm(rank, world, dev, 64 * 8192)
    g = torch.Generator().manual_seed(1234 + rank)
    errs = []
    st = torch.cuda.current_stream().cuda_stream
    for bf16 in (False, True):
        comm.bf16_payload = bf16
        for n in (4096, 8192, 8 * 8192, 64 * 8192, 600 * 2048, 1000, 3):
            x = torch.randn(n, generator=g)
            resid = torch.randn(n, generator=g)
            allx = [torch.zeros(n) for _ in range(world)]
            dist.all_gather(allx, x)
            want = torch.stack(allx).sum(0)
            xd = x.cuda()
            comm.allreduce(xd.data_ptr(), n, 0, st)
            torch.cuda.synchronize()
            e1 = float((xd.cpu() - want).abs().max())
            xd = x.cuda()
            rd = resid.cuda()
            comm.allreduce(xd.data_ptr(), n, rd.data_ptr(), st)
            torch.cuda.synchronize()
            e2 = float((rd.cpu() - (resid + want)).abs().max())
            two_shot = world > 1 and n >= comm.two_shot_min and n % 4 == 0
            errs.append({"n": n, "bf16": bf16, "two_shot": two_shot, "inplace_err": e1, "fused_resid_err": e2,
                         "scale": float(torch.stack(allx).abs().max())})
    comm.bf16_payload = True
    res["allreduce"] = errs
    log("all-reduce numerics done")
    # column all-gather (vocab-parallel logits): rank r fills its slice, every rank gets all
    gerr = []
    for rows, slice_ in ((1, 512), (3, 4000), (8, 64)):
        ld = slice_ * world
        full = torch.arange(rows * ld, dtype=torch.float32).reshape(rows, ld) * 0.5 - 7
        mine = torch.full((rows, ld), float("nan"))
        mine[:, rank * slice_:(rank + 1) * slice_] = full[:, rank * slice_:(rank + 1) * slice_]
        md = mine.cuda()
        comm.allgather_cols(md.data_ptr(), rows, slice_, ld, st)
        torch.cuda.synchronize()
        gerr.append({"rows": rows, "slice": slice_, "err": float((md.cpu() - full).abs().max())})
    res["allgather"] = gerr
    # fused all-reduce + split-RMSNorm producer (batched TP decode, C1 / C2): residual, bf16(x * g) and
    # per-1024-column sums of squares (tail parts zero); 40 x 2048 exceeds the one-shot size and takes
    # the two-shot all-reduce + add-norm fallback
    from aios_amd.runtime import native

    nerr = []
    for rows, d in ((1, 2048), (6, 4096), (5, 5120), (40, 2048)):
        parts = native.require().resid_norm_parts(d)
        x = torch.randn(rows, d, generator=g)
        resid = torch.randn(rows, d, generator=g)
        gw = torch.rand(d, generator=g) + 0.5
        allx = [torch.zeros(rows, d) for _ in range(world)]
        dist.all_gather(allx, x)
        want = resid + torch.stack(allx).sum(0)
        xd, rd, gd = x.cuda(), resid.cuda(), gw.cuda()
        o16 = torch.zeros(rows, d, dtype=torch.bfloat16, device="cuda")
        pd = torch.full((rows, parts), 7.0, device="cuda")
        comm.allreduce_norm(xd.data_ptr(), rows, d, rd.data_ptr(), gd.data_ptr(), o16.data_ptr(), d, pd.data_ptr(),
                            parts, st)
        torch.cuda.synchronize()
        ncb = d // 1024
        wp = torch.zeros(rows, parts)
        wp[:, :ncb] = (want.reshape(rows, ncb, 1024).double() ** 2).sum(-1).float()
        wx = want * gw
        nerr.append({"rows": rows, "d": d, "parts": parts, "two_shot": world > 1 and rows * d >= comm.two_shot_min,
                     "resid_err": float((rd.cpu() - want).abs().max()),
                     "out16_rel": float((o16.float().cpu() - wx).abs().max() / wx.abs().max()),
                     "part_rel": float((pd.cpu() - wp).abs().max() / wp.abs().max()),
                     "scale": float(torch.stack(allx).abs().max())})
    res["allreduce_norm"] = nerr
    res["comm_error_flag"] = bool(comm.error())
    log("all-gather / all-reduce+norm done")

    # timing at decode size (B=1, d=8192): one-shot; at prefill size (512 x 8192): two-shot
    for n, key, reps in ((8192, "allreduce_us_8192", 500), (512 * 8192, "allreduce_us_512x8192", 20)):
        x = torch.randn(n, device="cuda")
        for _ in range(5):
            comm.allreduce(x.data_ptr(), n, 0, st)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            comm.allreduce(x.data_ptr(), n, 0, st)
        torch.cuda.synchronize()
        res[key] = (time.perf_counter() - t0) / reps * 1e6
    del comm

    # ---- 2. sharded model vs unsharded
    log("loading the sharded model")
    cfg = get_preset(args.model)
    path = os.path.join("/tmp", f"tp_check_{args.model}_{args.recipe}.gguf")
    if rank == 0 and not os.path.exists(path):
        from aios_amd.models.synthetic import write_synthetic_gguf

        write_synthetic_gguf(path, cfg, args.recipe, seed=7)
    dist.barrier()
    # the same activation precision on both sides (fp32 by default; --act-q8: int8 per 32-block,
    # whose blocks a K-sharded GEMV quantises exactly as TP=1 does); greedy stream from TP, then
    # TP=1 teacher-forced on the same tokens, comparing logits at every step
    max_ctx = (args.prompt_len + args.steps + 64 + 127) // 128 * 128
    nb = max(2, args.batch)
    eng, comm = build_tp_engine(cfg, rank, world, dev, path=path, max_ctx=max_ctx, max_slots=nb, max_batch=nb,
                                act_q8=args.act_q8)
    res["vocab_parallel"] = bool(eng.vocab_parallel)
    res["tp_fused"] = bool(getattr(eng, "tp_fused", False))  # C1 / C2 in the GEMV engine's epilogue
    prompt = [cfg.bos_id] + [(11 * i + 5) % (cfg.vocab_size - 3) + 3 for i in range(args.prompt_len - 1)]
    if rank == 0:
        tp = TPEngine(eng, comm)
        logits = np.asarray(tp.prefill(0, prompt, 0, True))
        toks = [int(logits.argmax())]
        step_logits = []
        pos = len(prompt)
        for _ in range(args.steps):
            t = tp.decode([0], [toks[-1]], [pos], [0.0], [0], 0, b"")
            step_logits.append(np.asarray(tp.last_logits(1))[0].copy())
            toks.append(int(t[0]))
            pos += 1
        l2 = np.asarray(tp.prefill(1, prompt, 0, True))
        tp.decode_loop_prepare([1], [int(l2.argmax())], [len(prompt)])
        tp.decode_loop_run(1, args.steps, True)
        tp.synchronize()
        hist = list(tp.decode_loop_history(1, len(prompt) + 1, args.steps))
        B = args.batch
        if B > 1:
            prompts = [[cfg.bos_id] + [(7 * i + 13 * b + 3) % (cfg.vocab_size - 3) + 3 for i in range(args.prompt_len + b)]
                       for b in range(B)]
            btoks = [[int(np.asarray(tp.prefill(b, prompts[b], 0, True)).argmax()) for b in range(B)]]
            blog = []
            bpos = [len(p) for p in prompts]
            for _ in range(args.steps):
                t = tp.decode(list(range(B)), btoks[-1], bpos, [0.0] * B, [0] * B, 0, b"")
                blog.append(np.asarray(tp.last_logits(B)).copy())
                btoks.append([int(v) for v in t])
                bpos = [p + 1 for p in bpos]
        tp.close()
        from aios_amd.runtime.loader import load_engine

        ref, _, _ = load_engine(path, max_ctx=max_ctx, max_slots=nb, max_batch=nb, device=dev, act_q8=args.act_q8)
        rl = np.asarray(ref.prefill(0, prompt, 0, True))
        pos = len(prompt)
        diffs = []
        for i in range(args.steps):
            ref.decode([0], [toks[i]], [pos], [0.0], [0], 0, b"")
            r = np.asarray(ref.last_logits(1))[0]
            diffs.append(float(np.abs(r - step_logits[i]).max()))
            pos += 1
        res["model"] = {
            "tp_tokens": toks, "graph_tokens": [toks[0]] + hist,
            "prefill_logit_max_abs_diff": float(np.abs(logits - rl).max()),
            "decode_logit_max_abs_diff_per_step": diffs, "logit_scale": float(np.abs(rl).max()),
            "graph_tokens_match": [toks[0]] + hist == toks[:len(hist) + 1],
            "act_q8": bool(args.act_q8),
        }
        if args.dump_logits:
            res["model"]["step_logits"] = [[float(v) for v in l] for l in step_logits]
        if B > 1:
            for b in range(B):
                ref.prefill(b, prompts[b], 0, False)
            bpos = [len(p) for p in prompts]
            bd = []
            for i in range(args.steps):
                ref.decode(list(range(B)), btoks[i], bpos, [0.0] * B, [0] * B, 0, b"")
                bd.append(float(np.abs(np.asarray(ref.last_logits(B)) - blog[i]).max()))
                bpos = [p + 1 for p in bpos]
            res["batched"] = {"B": B, "decode_logit_max_abs_diff_per_step": bd,
                              "logit_scale": float(max(np.abs(l).max() for l in blog))}
        res["comm_error_flag_model"] = bool(comm.error())
    else:
        worker_loop(eng, comm)
    dist.barrier()
    if rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
