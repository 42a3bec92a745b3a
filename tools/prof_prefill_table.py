#!/usr/bin/env python3
"""Per-projection table of ONE prefill chunk from a rocprofv3 kernel trace (the last run in the
trace): median kernel time per role over the layers and the achieved TFLOP/s of each GEMM.

  python tools/prof_prefill_table.py gpurun_out/pfa/run_kernel_trace.csv --tokens 2048 \
      [--model mistral-7b]

Roles per layer (engine.hip prefill_layer order): rmsnorm, QKV GEMM, qkv_post (RoPE + KV write),
attention, O GEMM (+ residual), rmsnorm, gate/up GEMM (+ SwiGLU), down GEMM (+ residual)."""
import argparse
import csv
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tokens", type=int, default=2048)
    ap.add_argument("--model", default="mistral-7b")
    args = ap.parse_args()
    from aios_amd.models.config import get_preset

    cfg = get_preset(args.model)
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0]
    attn = [i for i, r in enumerate(rows) if "attn_prefill_kernel" in name(r)]
    L = cfg.n_layers
    if len(attn) < L:
        raise SystemExit(f"{len(attn)} prefill attention launches in the trace, need {L}")
    last = attn[-L:]
    # window: from the layer-0 norm before the first attention of the last run to the last down GEMM
    lo = last[0]
    while lo > 0 and "rmsnorm" not in name(rows[lo]):
        lo -= 1
    hi = last[-1]
    n_after = 0
    while hi + 1 < len(rows) and n_after < 4:
        hi += 1
        if "gemm" in name(rows[hi]) or "rmsnorm" in name(rows[hi]):
            n_after += 1 if "gemm" in name(rows[hi]) else 0
    win = rows[lo:hi + 1]
    d, hd = cfg.d_model, cfg.head_dim
    qd, kvd = cfg.n_heads * hd, cfg.n_kv_heads * hd
    flops = {"qkv": 2 * args.tokens * d * (qd + 2 * kvd), "o": 2 * args.tokens * qd * d,
             "gate_up": 2 * args.tokens * d * 2 * cfg.d_ff, "down": 2 * args.tokens * cfg.d_ff * d,
             "attention": 4 * cfg.n_heads * hd * args.tokens * args.tokens / 2}
    roles = {}
    for li, a in enumerate(last):
        ai = a - lo
        seq = win[:ai][::-1]  # kernels before this attention (nearest first)
        before = [r for r in seq][:3]
        after = win[ai + 1:ai + 8]
        pick = {}
        for r in before:
            n = name(r)
            if "qkv_post" in n:
                pick.setdefault("qkv_post", r)
            elif "gemm" in n:
                pick.setdefault("qkv", r)
            elif "rmsnorm" in n:
                pick.setdefault("attn_norm", r)
        pick["attention"] = win[ai]
        g = [r for r in after if "gemm" in name(r)]
        for role, r in zip(("o", "gate_up", "down"), g):
            pick[role] = r
        nrm = [r for r in after if "rmsnorm" in name(r)]
        if nrm:
            pick["ffn_norm"] = nrm[0]
        for role, r in pick.items():
            roles.setdefault(role, []).append((r, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    wall = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
    ksum = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in win)
    print(f"# {args.model}, one {args.tokens}-token prefill chunk (last run in {os.path.basename(args.trace)}): "
          f"{len(win)} kernels, wall {wall / 1e3:.2f} ms, sum of kernel times {ksum / 1e3:.2f} ms")
    print(f"{'role':10s} {'median us':>10s} {'x layers':>9s} {'share':>6s} {'TFLOP/s':>8s}  kernel")
    order = ["attn_norm", "qkv", "qkv_post", "attention", "o", "ffn_norm", "gate_up", "down"]
    for role in order:
        if role not in roles:
            continue
        ts = [t for _, t in roles[role]]
        med = statistics.median(ts)
        tf = f"{flops[role] / (med * 1e-6) / 1e12:8.0f}" if role in flops else " " * 8
        kn = name(roles[role][0][0])[:58]
        print(f"{role:10s} {med:10.1f} {len(ts):9d} {100 * sum(ts) / ksum:5.1f}% {tf}  {kn}")
    others = set(name(r) for r in win) - {name(r) for v in roles.values() for r, _ in v}
    if others:
        print("# other kernels in the window:", ", ".join(sorted(o[:50] for o in others)))
    print("# every kernel above is an aios:: HIP kernel (no vendor GEMM library in the prefill path)")


if __name__ == "__main__":
    main()
