#!/usr/bin/env python3
"""Strategic-tier benchmark: Llama-3-70B Q4_K_M decode with tensor parallelism (BASELINE config 5).

  python tools/bench_tp.py                                   # TP=1, one GPU
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_tp.py

One process per rank; ranks map to GPUs round-robin (several ranks may share one GPU -- useful
for correctness, meaningless for speed, and flagged as such in the output).  Random-init weights
of the Llama-3-70B architecture in the Q4_K_M per-tensor layout, sharded column/row-parallel;
the decode step (80 layers, 160 fused all-reduce+residual collectives) is captured in a hipGraph
and replayed K times after W warmup steps.  Prints one JSON line (rank 0).
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
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--recipe", default="Q4_K_M")
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--layers", type=int, default=0, help="override layer count (smoke runs only)")
    args = ap.parse_args()
    import torch

    from aios_amd.models.config import get_preset
    from aios_amd.parallel.tp import TPEngine, build_tp_engine, local_device, worker_loop

    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    dev = local_device(int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    cfg = get_preset(args.model)
    if args.layers:
        cfg = cfg.scaled(n_layers=args.layers)
    max_ctx = ((args.prompt + args.warmup + args.steps + 2 + 63) // 64) * 64
    t0 = time.time()
    eng, comm = build_tp_engine(cfg, rank, world, dev, recipe=args.recipe, seed=1234, max_ctx=max_ctx,
                                max_slots=args.batch, max_batch=args.batch)
    load_s = time.time() - t0
    if rank != 0:
        worker_loop(eng, comm)
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
        return
    tp = TPEngine(eng, comm) if world > 1 else eng
    slots = list(range(args.batch))
    toks = []
    for s in slots:
        p = [cfg.bos_id] + [(7 * i + 13 * s) % (cfg.vocab_size - 3) + 3 for i in range(args.prompt - 1)]
        toks.append(int(tp.prefill(s, p, 0, True).argmax()))
    tp.decode_loop_prepare(slots, toks, [args.prompt] * args.batch)
    tp.decode_loop_run(args.batch, args.warmup, True)
    tp.synchronize()
    t0 = time.perf_counter()
    tp.decode_loop_run(args.batch, args.steps, True)
    tp.synchronize()
    dt = time.perf_counter() - t0
    hist = tp.decode_loop_history(args.batch, args.prompt + args.warmup + 1, args.steps)
    assert all(0 <= t < cfg.vocab_size for t in hist)
    if comm.error():
        raise RuntimeError("all-reduce timed out")
    n_dev = torch.cuda.device_count()
    out = {"metric": f"decode tokens/sec {args.model} {args.recipe} TP={world}", "value": round(args.batch * args.steps / dt, 2),
           "unit": "tokens/s", "tp": world, "ms_per_step": round(dt / args.steps * 1e3, 4), "batch": args.batch,
           "steps": args.steps, "warmup": args.warmup, "layers": cfg.n_layers,
           "weight_gb_per_rank": round(eng.weight_bytes / 1e9, 3), "load_s": round(load_s, 1),
           "gpus_visible": n_dev, "ranks_share_gpu": world > n_dev,
           "note": ("ranks share one GPU: correctness/overhead run, not a scaling number" if world > n_dev else
                    "one rank per GPU")}
    if world > 1:
        tp.close()
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
