"""Decode-GEMV phase anatomy on MI355X: per Mistral-7B projection, the row-pair int8 GEMV vs the
CU-balanced register-streaming one (kernels/gemv_cu.h) vs the LDS-DMA loader/consumer engine
(kernels/gemv_lds.h, the default), all graph-replayed over rotating weight copies (> the 256 MB
Infinity Cache, so the bytes come from HBM as in the decode step), plus the default kernel's
in-kernel phase timestamps (s_memrealtime, 10 ns ticks) across its workgroups: start skew, first loads
issued, x staged, barrier, compute done, epilogue done.

python tools/gemv_cu_probe.py [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from aios_amd.gguf.quants import BLOCK_INFO, GGMLType
from aios_amd.runtime import native

Q4, Q6 = GGMLType.Q4_K, GGMLType.Q6_K
SHAPES = [  # name, [(fmt, rows)], K, norm, epi
    ("qkv", [(Q4, 5120), (Q6, 1024)], 4096, True, "STORE"),
    ("o", [(Q4, 4096)], 4096, False, "RESID"),
    ("gate_up", [(Q4, 28672)], 4096, True, "SWIGLU"),
    ("down_q6k", [(Q6, 4096)], 14336, False, "RESID"),
    ("down_q4k", [(Q4, 4096)], 14336, False, "RESID"),
    ("lm_head", [(Q6, 32000)], 4096, True, "STORE"),
    # diagnostics (--only): QKV with V in Q4_K too (no mixed format), QKV without the RMSNorm,
    # O with one
    ("qkv_q4", [(Q4, 6144)], 4096, True, "STORE"),
    ("qkv_nonorm", [(Q4, 5120), (Q6, 1024)], 4096, False, "STORE"),
    ("o_norm", [(Q4, 4096)], 4096, True, "RESID"),
    ("v_q6", [(Q6, 1024)], 4096, True, "STORE"),
    ("qk_q4", [(Q4, 5120)], 4096, True, "STORE"),
    # TinyLlama-1.1B (--only tl_...): QKV mixed / all-Q4_K / without the norm, O, gate/up, down
    ("tl_qkv", [(Q4, 2304), (Q6, 256)], 2048, True, "STORE"),
    ("tl_qkv_q4", [(Q4, 2560)], 2048, True, "STORE"),
    ("tl_qkv_nonorm", [(Q4, 2304), (Q6, 256)], 2048, False, "STORE"),
    ("tl_o", [(Q4, 2048)], 2048, False, "RESID"),
    ("tl_gu", [(Q4, 11264)], 2048, True, "SWIGLU"),
    ("tl_down", [(Q4, 2048)], 5632, False, "RESID"),
]


def pct(v, q):
    return float(np.percentile(v, q))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    E = native.require()
    res = []
    for name, segs, K, norm, epi in SHAPES:
        if (args.only and name not in args.only.split(",")) or (not args.only and (name.startswith("tl_") or name in (
                "qkv_q4", "qkv_nonorm", "o_norm", "v_q6", "qk_q4"))):
            continue
        nbytes = sum(BLOCK_INFO[t][1] * r * K // 256 for t, r in segs)
        nrot = int(os.environ.get("NROT", 0)) or max(2, (640 << 20) // nbytes + 1)  # NROT=1: MALL-resident weights
        mats = []
        for i in range(nrot):
            ms = []
            for j, (t, r) in enumerate(segs):
                m = E.QMatrix(int(t), r, K, np.zeros(BLOCK_INFO[t][1] * r * K // 256, dtype=np.uint8))
                m.fill_random(7 + 3 * i + j, 0.02)
                ms.append(m)
            mats.append(ms)
        N = sum(r for _, r in segs)
        B = int(os.environ.get("PROBE_B", 1))  # batch rows (B = 2..4: the engine's batched consumers)
        x = torch.randn(B, K, device="cuda")
        nw = torch.rand(K, device="cuda") + 0.5
        y = torch.zeros(B, N, device="cuda")
        epic = getattr(E, "EPI_" + epi)
        ldy = N // 2 if epi == "SWIGLU" else N

        # PROBE_XDIRTY: x rewritten before every launch, as the decode step's residual producers do --
        # "store" (plain stores, torch mul_) or "atomic" (memory-side float atomics, torch index_add_);
        # the writer's own time (a graph of writers alone) is subtracted
        xdirty = os.environ.get("PROBE_XDIRTY", "")
        xidx = torch.arange(K, device="cuda")
        xzero = torch.zeros(B, K, device="cuda")

        def writer():
            if xdirty == "store":
                x.mul_(1.0)
            elif xdirty == "atomic":
                x.index_add_(1, xidx, xzero)

        def launch(ms, sel, ts=0):
            writer()
            st = torch.cuda.current_stream().cuda_stream
            # sel 4: the LDS engine with its consumers skipping the dot work (bare ring cadence)
            E.gemv(ms, B, x.data_ptr(), K, nw.data_ptr() if norm else 0, 1e-5, y.data_ptr(), ldy, epic, st, 0, 1,
                   kernel_sel=3 if sel == 4 else sel, tune_dbg=0x10000 if sel == 4 else 0, dbg_ts=ts,
                   tune_u=int(os.environ.get("PROBE_U", 0)))  # PROBE_U: the row kernel's U (12: U 2 unbuffered)

        row = dict(shape=name, B=B, mb=round(nbytes / 1e6, 1))
        sels = ((1, "rows"), (2, "cu"), (3, "lds"), (4, "ring"), (0, "auto")) if B == 1 else ((3, "lds"), (1, "rows"))
        for sel, tag in sels:
            for ms in mats:
                launch(ms, sel)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            nrep = int(os.environ.get("NREP", 1))  # > 1 with a small NROT: Infinity-Cache-resident weights
            with torch.cuda.graph(g):
                for _ in range(nrep):
                    for ms in mats:
                        launch(ms, sel)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (reps * nrot * nrep)
            if xdirty and "writer_us" not in row:
                gw = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gw):
                    for _ in range(nrep * nrot):
                        writer()
                gw.replay()
                torch.cuda.synchronize()
                e0.record()
                for _ in range(reps):
                    gw.replay()
                e1.record()
                torch.cuda.synchronize()
                row["writer_us"] = round(e0.elapsed_time(e1) * 1e3 / (reps * nrot * nrep), 2)
            if xdirty:
                us -= row["writer_us"]
            row[tag + "_us"] = round(us, 2)
            row[tag + "_tbs"] = round(nbytes / us / 1e6, 2)
        row["floor_us"] = round(E.bench_stream_read(nbytes // 4096 * 4096, nrot, 1, 4, 512, 20), 2)
        # phase stamps of one cold launch (the copy least recently touched); STAMP_SEL=1: the row
        # kernel's stamps (start, loads issued, x staged, barrier, first pair computed, done)
        G = 256
        ssel = int(os.environ.get("STAMP_SEL", 3))
        ts = torch.zeros(G * 2 * 8, dtype=torch.int64, device="cuda")
        launch(mats[0], ssel)  # warm the code path
        for ms in mats[1:]:
            launch(ms, ssel)
        torch.cuda.synchronize()
        launch(mats[0], ssel, ts.data_ptr())
        torch.cuda.synchronize()
        t = ts.view(G, 2, 8).cpu().numpy().astype(np.float64)
        live = t[:, 0, 0] > 0
        t = t[live]
        if not live.any():  # production build: the stamps are compiled out (AIOS_BUILD_PROBES=1 for them)
            res.append(row)
            print(json.dumps(row), flush=True)
            del mats
            torch.cuda.empty_cache()
            continue
        t0 = t[:, :, 0][t[:, :, 0] > 0].min()
        rel = (t - t0) / 100.0  # 100 MHz -> us
        if ssel == 1:
            phases = {"start": rel[:, 0, 0], "loads_issued": rel[:, 0, 1], "x_staged": rel[:, 0, 2],
                      "barrier": rel[:, 0, 3], "pair_w0": rel[:, 0, 4], "pair_wlast": rel[:, 1, 4],
                      "done_w0": rel[:, 0, 5], "done_wlast": rel[:, 1, 5]}
        else:
            phases = {"start": rel[:, 0, 0], "loads_issued": rel[:, 0, 1], "x_staged": rel[:, 0, 2],
                      "barrier": rel[:, 0, 3], "compute_w0": rel[:, 0, 4], "compute_w15": rel[:, 1, 4],
                      "final_barrier": rel[:, 0, 5], "epilogue": rel[:, 0, 6]}
        row["stamps_us"] = {k: [round(pct(v, q), 2) for q in (0, 50, 100)] for k, v in phases.items()}
        res.append(row)
        print(json.dumps(row), flush=True)
        del mats
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
