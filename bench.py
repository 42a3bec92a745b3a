#!/usr/bin/env python3
"""Headline benchmark: decode tokens/sec of Mistral-7B Q4_K_M on MI355X (BASELINE.json metric #1).

One process per GPU (torchrun / torch.distributed, RCCL backend on ROCm).  Each rank serves its
own co-resident replica -- the agent router's request-level data parallelism (SURVEY.md §2.9 DP
row) -- so per-GPU work is fixed as N grows ("weak" scaling) and `value` is the whole-job
aggregate: total decoded tokens / max-over-ranks wall time.  `python bench.py --gpus N` without
torchrun spawns the N ranks itself (a child `torch.distributed.run`, started before this process
touches a GPU); under torchrun `--gpus` must equal WORLD_SIZE.

Secondary `tp_strategic`: the strategic tier -- Llama-3-70B Q4_K_M, batch 1, 128-token prompt --
tensor-parallel over the same N ranks (xGMI collectives inside the captured decode step,
aios_amd/parallel/tp.py), so the 1 -> 8 curve also measures the TP data plane, not only
independent replicas.  When ranks outnumber the visible GPUs they share one (correctness /
overhead run, flagged `ranks_share_gpu`; the persistent decode kernel is then off, since two
grid-resident kernels cannot share the CUs).

Per rank: random-init Mistral-7B weights in the exact Q4_K_M per-tensor layout (Q6_K lm_head and
"more bits" attn_v/ffn_down, Q4_K elsewhere; ~4.1 GB) generated directly in HBM (no network ->
no real checkpoint), a synthetic prompt prefilled into the KV cache, W untimed warmup decode
steps, then exactly K timed decode steps, each the full forward (embed, 32 blocks, lm_head,
on-device greedy sampling) replayed from a captured hipGraph with the sampled token fed back on
device.  Baseline: the reference's GPU target "<100 ms for a 50-token Mistral-7B response"
(docs/phases/04-AI-RUNTIME.md:334) => 500 tok/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_MISTRAL_TOKS = 500.0   # Mistral-7B GPU target => >= 500 tok/s
BASELINE_TINYLLAMA_TOKS = 250.0  # TinyLlama target  => >= 250 tok/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--batch", type=int, default=1, help="concurrent sequences per GPU (decode batch)")
    ap.add_argument("--prompt", type=int, default=128, help="prompt tokens prefilled before decoding")
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--recipe", default="Q4_K_M")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--kv-dtype", default="bf16", help="KV cache dtype: bf16 (default) or fp8_e4m3")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary measurements (TinyLlama, fp32-activation Mistral)")
    ap.add_argument("--fp32-act", action="store_true",
                    help="headline with fp32 activations in the GEMVs instead of int8 (q8_1-style) ones")
    ap.add_argument("--no-tp", action="store_true", help="skip the strategic-tier TP secondary")
    ap.add_argument("--no-serving", action="store_true",
                    help="skip the gRPC operational-tier (config 2) and co-resident tiers (config 4) secondaries")
    ap.add_argument("--no-goal-plan", action="store_true",
                    help="skip the goal->plan latency secondary (BASELINE.json's agent metric)")
    ap.add_argument("--tp-model", default="llama3-70b")
    ap.add_argument("--tp-steps", type=int, default=64)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: set up the ranks and their process group, print one line per rank, "
                         "touch no GPU")
    return ap.parse_args()


def spawn(args) -> int:
    """--gpus N without torchrun: run N ranks under a child torch.distributed.run (nothing in this
    process has touched a GPU; the child's exit code is ours)."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def measure(preset: str, recipe: str, batch: int, prompt: int, steps: int, warmup: int, use_graph: bool, dist,
            device: int, act_q8: bool = True, kv_dtype: str = "bf16"):
    import torch

    from aios_amd.models.config import get_preset
    from aios_amd.runtime.loader import random_engine

    cfg = get_preset(preset)
    max_ctx = ((prompt + warmup + steps + 2 + 63) // 64) * 64
    eng = random_engine(cfg, recipe, seed=1234, max_ctx=max_ctx, max_slots=max(batch, 1), max_batch=batch,
                        device=device, act_q8=act_q8, kv_dtype=kv_dtype)
    slots = list(range(batch))
    toks = []
    for s in slots:
        p = [cfg.bos_id] + [(7 * i + 13 * s) % (cfg.vocab_size - 3) + 3 for i in range(prompt - 1)]
        toks.append(int(eng.prefill(s, p, 0, True).argmax()))
    eng.decode_loop_prepare(slots, toks, [prompt] * batch)
    eng.decode_loop_run(batch, warmup, use_graph)
    eng.synchronize()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    eng.decode_loop_run(batch, steps, use_graph)
    eng.synchronize()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    hist = eng.decode_loop_history(batch, prompt + warmup + 1, steps)
    assert all(0 <= t < cfg.vocab_size for t in hist), "invalid token ids from decode loop"
    info = dict(weight_gb=round(eng.weight_bytes / 1e9, 3), kv_gb=round(eng.kv_bytes / 1e9, 3),
                workspace_gb=round(eng.workspace_bytes / 1e9, 3))
    del eng
    return dt, info


def measure_goal_plan(goals: int = 16, timeout_s: float = 90.0):
    """BASELINE.json's agent metric: p50 goal -> plan latency of tactical goals through the real
    planner (classification, LLM decomposition over gRPC, task persistence) on an in-process runtime
    serving the synthetic Mistral-7B tier (tools/bench_goal_plan.py; reference path
    agent-core/src/task_planner.rs:163-218).  Bounded: a run past timeout_s reports an error."""
    import argparse as _ap
    import asyncio

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    from bench_goal_plan import main_async

    # every plan is exactly 300 tokens (the top of the reference's typical plan, task_planner.rs:168);
    # + goal_plan_burst: 3 tactical goals submitted at once, 300 tokens each
    ns = _ap.Namespace(model="mistral-7b", goals=goals, warmup=2, burst=3, plan_tokens=300, burst_plan_tokens=300,
                       fixed_length=True)
    return asyncio.run(asyncio.wait_for(main_async(ns), timeout_s))


def measure_grpc(timeout_s: float = 120.0):
    """BASELINE.json config 2: TinyLlama-1.1B BF16, the operational tier, tokens/s through
    AIRuntime.StreamInfer / Infer on loopback gRPC (tools/bench_grpc.py; reference path
    runtime/src/grpc_service.rs:33-177).  Bounded: a run past timeout_s reports an error."""
    import argparse as _ap
    import asyncio

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    from bench_grpc import main_async

    ns = _ap.Namespace(tokens=256, reps=3, recipe="BF16")
    return asyncio.run(asyncio.wait_for(main_async(ns), timeout_s))


def measure_coresident(steps: int = 256, prompt: int = 128, cu_split: int = 0):
    """BASELINE.json config 4: TinyLlama-1.1B and Mistral-7B resident together on one GPU, each
    replaying its decode graph on its own stream, dispatched concurrently from two host threads
    (tools/bench_coresident.py): per-tier tok/s alone and concurrent, the aggregate, HBM per tier.
    cu_split > 0: each tier on its own CUs (CU-masked streams, grids sized to them)."""
    import argparse as _ap

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    from bench_coresident import run

    return run(_ap.Namespace(steps=steps, prompt=prompt, cu_split=cu_split, priority=""))


def measure_tp(args, rank: int, world: int, device: int, gloo):
    """Strategic tier: Llama-3-70B TP=world, batch 1 (tools/bench_tp.py logic); seconds of the
    timed steps on the leader (None on workers)."""
    from aios_amd.models.config import get_preset
    from aios_amd.parallel.tp import TPEngine, build_tp_engine, worker_loop

    cfg = get_preset(args.tp_model)
    steps, warmup = args.tp_steps, 8
    max_ctx = ((args.prompt + warmup + steps + 2 + 63) // 64) * 64
    eng, comm = build_tp_engine(cfg, rank, world, device, recipe=args.recipe, seed=1234, max_ctx=max_ctx,
                                max_slots=1, max_batch=1, group=gloo)
    if rank != 0:
        worker_loop(eng, comm, group=gloo)
        del eng
        return None, None
    tp = TPEngine(eng, comm, group=gloo) if world > 1 else eng
    try:
        p = [cfg.bos_id] + [(7 * i) % (cfg.vocab_size - 3) + 3 for i in range(args.prompt - 1)]
        tok = int(tp.prefill(0, p, 0, True).argmax())
        tp.decode_loop_prepare([0], [tok], [args.prompt])
        tp.decode_loop_run(1, warmup, True)
        tp.synchronize()
        t0 = time.perf_counter()
        tp.decode_loop_run(1, steps, True)
        tp.synchronize()
        dt = time.perf_counter() - t0
        if comm.error():
            raise RuntimeError("TP all-reduce timed out")
        info = {"weight_gb_per_rank": round(eng.weight_bytes / 1e9, 3)}
    finally:
        if world > 1:
            tp.close()  # releases the workers' command loop whatever happened on the leader
    del eng
    return dt, info


def measure_collectives(rank: int, world: int, device: int, gloo):
    """All-reduce latency of the two TP data planes at the decode / prefill message sizes the
    engine issues: 16 KB (B=1 d=4096), 64 KB (B=4 or d=16384) and 32 MB (a 2k-token prefill chunk's
    partial), xGMI one-shot / two-shot kernels (XgmiComm) vs librccl (RcclComm); max over ranks."""
    import torch
    import torch.distributed as td

    from aios_amd.parallel.tp import create_comm

    res = {}
    dev = torch.device("cuda", device)
    for kind in ("xgmi", "rccl"):
        try:
            comm = create_comm(rank, world, device, 8 << 20, gloo, kind=kind)
        except Exception as e:  # noqa: BLE001
            res[f"{kind}_error"] = f"{type(e).__name__}: {e}"[:200]
            continue
        st = torch.cuda.current_stream(dev).cuda_stream
        for n, key in ((4096, "16KB"), (16384, "64KB"), (8 << 20, "32MB")):
            x = torch.randn(n, device=dev)
            for _ in range(5):
                comm.allreduce(x.data_ptr(), n, 0, st)
            torch.cuda.synchronize(dev)
            td.barrier(group=gloo)
            reps = 200 if n < (1 << 20) else 20
            t0 = time.perf_counter()
            for _ in range(reps):
                comm.allreduce(x.data_ptr(), n, 0, st)
            torch.cuda.synchronize(dev)
            t = torch.tensor([(time.perf_counter() - t0) / reps * 1e6])
            td.all_reduce(t, op=td.ReduceOp.MAX, group=gloo)
            res[f"{kind}_allreduce_us_{key}"] = round(float(t[0]), 2)
        del comm
    return res


def main():
    args = parse()
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        sys.exit(spawn(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch N ranks for --gpus N)")
    import torch

    n_dev = max(1, torch.cuda.device_count())  # counting devices does not initialise the GPU
    if args.dry_run and os.environ.get("AIOS_BENCH_DEVICES"):  # (launcher tests: a node's device count)
        n_dev = int(os.environ["AIOS_BENCH_DEVICES"])
    share = world > n_dev                      # more ranks than GPUs: ranks share (not a scaling run)
    device = local % n_dev
    dist = gloo = None
    if args.dry_run:
        if world > 1:
            import torch.distributed as td

            td.init_process_group("gloo")
            td.barrier()
        print(json.dumps({"rank": rank, "world": world, "device": device, "ranks_share_gpu": share}), flush=True)
        return
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as td

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if share:  # RCCL refuses two ranks on one GPU
            td.init_process_group("gloo")
        else:
            td.init_process_group("nccl", device_id=torch.device("cuda", device))
        import datetime

        # the TP leader's command channel; bounded, so a rank lost in the secondary cannot hold the run
        gloo = td.new_group(backend="gloo", timeout=datetime.timedelta(seconds=600))
        dist = td

    act_q8 = not args.fp32_act
    dt, info = measure(args.model, args.recipe, args.batch, args.prompt, args.steps, args.warmup,
                       not args.no_graph, dist, device, act_q8, args.kv_dtype)
    secondary = other_act = tp_dt = tp_info = None
    if not args.no_secondary:
        secondary, _ = measure("tinyllama-1.1b", "Q4_K_M", 1, args.prompt, args.steps, args.warmup,
                               not args.no_graph, dist, device)
        # the same Mistral decode with the other GEMV activation precision
        other_act, _ = measure(args.model, args.recipe, args.batch, args.prompt, args.steps, args.warmup,
                               not args.no_graph, dist, device, not act_q8)
        if not args.no_tp:
            if dist is not None:
                dist.barrier()
            # a failure of the secondary (e.g. a peer mapping the node refuses) is reported in the JSON,
            # it never costs the headline measurement above
            try:
                tp_dt, tp_info = measure_tp(args, rank, world, device, gloo)
            except Exception as e:  # noqa: BLE001
                tp_dt, tp_info = None, {"error": f"{type(e).__name__}: {e}"[:300]}
                print(f"[rank {rank}] tp_strategic failed: {tp_info['error']}", file=sys.stderr, flush=True)

    collectives = None
    if world > 1 and not share and not args.no_secondary and not args.no_tp:
        try:
            collectives = measure_collectives(rank, world, device, gloo)
        except Exception as e:  # noqa: BLE001
            collectives = {"error": f"{type(e).__name__}: {e}"[:300]}
            print(f"[rank {rank}] collectives failed: {collectives['error']}", file=sys.stderr, flush=True)

    goal_plan = None
    if not args.no_secondary and not args.no_goal_plan and rank == 0:
        try:
            goal_plan = measure_goal_plan()
        except Exception as e:  # noqa: BLE001  (reported, never costs the headline)
            goal_plan = {"error": f"{type(e).__name__}: {e}"[:300]}
            print(f"goal_plan failed: {goal_plan['error']}", file=sys.stderr, flush=True)

    # BASELINE configs 2 and 4 (rank 0; each bounded, a failure is reported, never costs the headline)
    grpc_res = coresident = None
    if not args.no_secondary and not args.no_serving and rank == 0:
        try:
            edt, _ = measure("tinyllama-1.1b", "BF16", 1, args.prompt, 256, 16, not args.no_graph, None, device)
            grpc_res = measure_grpc()
            grpc_res["engine_tok_s"] = round(256 / edt, 1)
        except Exception as e:  # noqa: BLE001
            grpc_res = {"error": f"{type(e).__name__}: {e}"[:300]}
            print(f"tinyllama_bf16_grpc failed: {grpc_res['error']}", file=sys.stderr, flush=True)
        try:
            coresident = measure_coresident()
            # the same with each tier on its own CUs (TinyLlama 128 / Mistral 128: the split with the
            # highest aggregate of 64 / 96 / 128 measured, profiles/coresident_r6.txt)
            try:
                part = measure_coresident(cu_split=128)
                coresident["cu_partitioned"] = {k: part[k] for k in part if k.endswith("_tok_s") or k == "cu_split"}
            except Exception as e:  # noqa: BLE001
                coresident["cu_partitioned"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        except Exception as e:  # noqa: BLE001
            coresident = {"error": f"{type(e).__name__}: {e}"[:300]}
            print(f"coresident failed: {coresident['error']}", file=sys.stderr, flush=True)

    # max over ranks
    if dist is not None:
        t = torch.tensor([dt, secondary or 0.0, other_act or 0.0], dtype=torch.float64)
        if not share:
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
        secondary = float(t[1]) if secondary is not None else None
        other_act = float(t[2]) if other_act is not None else None
    n = world
    total_tokens = n * args.batch * args.steps
    value = total_tokens / dt
    if rank == 0:
        headline = args.model == "mistral-7b" and args.recipe == "Q4_K_M"
        out = {
            # (another --model / --recipe is a side measurement: labelled as such, no baseline ratio)
            "metric": "decode tokens/sec Mistral-7B Q4_K (aggregate over GPUs)" if headline else
                      f"decode tokens/sec {args.model} {args.recipe} (aggregate over GPUs)",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (BASELINE_MISTRAL_TOKS * 1.0), 3) if headline else None,
            # weights Q4_K_M; GEMV activations int8 per 32-block with fp32 scales (llama.cpp's q8_1
            # mul_mat_vec_q precision, the reference's) or fp32 with --fp32-act; fp32 accumulate
            "dtype": "q8_1-act/Q4_K_M" if act_q8 else "fp32-act/Q4_K_M",
            "data": "synthetic (random-init Q4_K_M weights of the Mistral-7B architecture, synthetic prompt)" if headline
                    else f"synthetic (random-init {args.recipe} weights of the {args.model} architecture, synthetic prompt)",
            "config": {
                "model": "Mistral-7B-Instruct-v0.2 Q4_K_M (architecture: d4096 L32 H32/8 ff14336 V32000)" if headline
                         else f"{args.model} {args.recipe}",
                "global_batch": n * args.batch,
                "seq_len": args.prompt + args.warmup + args.steps,
                "parallelism": f"dp{n}",
                "weights": args.recipe,
                "activations": ("int8 per-32-block activations with fp32 scales in the quantised GEMVs "
                                "(q8_1 as llama.cpp), fp32 residual stream, fp32 accumulate" if act_q8 else
                                "fp32 activations in the GEMVs, fp32 accumulate") +
                               "; int8 GEMV engine up to B = 4, bf16 MFMA operands for B >= 5; attention: " +
                               ("fp8 e4m3 KV cache (per-layer scales)" if args.kv_dtype != "bf16" else "bf16 KV cache") +
                               ", bf16-rounded q, fp32 softmax",
                "per_gpu_batch": args.batch,
                "prompt_tokens": args.prompt,
                "hipgraph": not args.no_graph,
                "ranks_share_gpu": share,
                **info,
            },
        }
        if secondary is not None:
            tl = n * args.steps / secondary
            out["secondary"] = {
                "metric": "decode tokens/sec TinyLlama-1.1B Q4_K_M (aggregate)",
                "value": round(tl, 2),
                "ms_per_step": round(secondary / args.steps * 1e3, 4),
                "vs_baseline": round(tl / BASELINE_TINYLLAMA_TOKS, 3),
            }
        if other_act is not None:
            v2 = n * args.batch * args.steps / other_act
            out["secondary_other_activations"] = {
                "metric": "decode tokens/sec Mistral-7B Q4_K with " + ("fp32" if act_q8 else "int8 (q8_1)") +
                          " GEMV activations (aggregate)",
                "value": round(v2, 2),
                "ms_per_step": round(other_act / args.steps * 1e3, 4),
                "vs_baseline": round(v2 / BASELINE_MISTRAL_TOKS, 3),
            }
        if tp_dt is not None:
            out["tp_strategic"] = {
                "metric": f"decode tokens/sec {args.tp_model} {args.recipe} TP={world} (batch 1)",
                "value": round(args.tp_steps / tp_dt, 2),
                "ms_per_step": round(tp_dt / args.tp_steps * 1e3, 4),
                "tp": world, "ranks_share_gpu": share, **(tp_info or {}),
            }
        elif tp_info and "error" in tp_info:
            out["tp_strategic"] = {"metric": f"decode tokens/sec {args.tp_model} {args.recipe} TP={world} (batch 1)",
                                   "value": None, "tp": world, "error": tp_info["error"]}
        if goal_plan is not None:
            if "error" in goal_plan:
                out["goal_plan_p50_ms"] = None
                out["goal_plan"] = goal_plan
            else:
                out["goal_plan_p50_ms"] = goal_plan["value"]
                out["goal_plan"] = {k: goal_plan[k] for k in ("metric", "p90_ms", "goals", "tasks_per_goal",
                                                              "reactive_p50_ms", "plan_tokens_cap", "plan_tokens_p50",
                                                              "plan_tokens_min_max", "ms_per_token", "model",
                                                              "baseline_ms")}
                b = goal_plan.get("burst", {})
                out["goal_plan_burst"] = {"metric": "goal->plan latency, 3 tactical goals submitted at once",
                                          "p50_ms": b.get("p50_ms"), "p90_ms": b.get("p90_ms"),
                                          "goals": b.get("concurrent_goals"), "plan_tokens_cap": b.get("plan_tokens_cap"),
                                          "plan_tokens_total": b.get("plan_tokens_total"), "wall_s": b.get("wall_s")}
        if collectives is not None:
            out["collectives"] = collectives
        if grpc_res is not None:
            out["tinyllama_bf16_grpc"] = grpc_res
        if coresident is not None:
            out["coresident"] = coresident
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
