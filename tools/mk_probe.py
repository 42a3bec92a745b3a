#!/usr/bin/env python3
"""Phase breakdown of the persistent decode step (kernels/decode_mk.hip) from in-kernel stamps.

Per stage kind (QKV / ATT / O / GU / DOWN / LM), medians over layers of the per-CU phase spans:
  wait   stage start -> the previous stage's counter matched (wave 0 poll)
  stage  counter matched -> input staged (B_in)
  slots  B_in -> last slot step (the weight stream of the stage)
  epi    epilogue + arrival
and the spread of stage completion over CUs.  One JSON line per kind + a total.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KINDS = ["QKV", "ATT", "O", "GU", "DOWN"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dbg", type=int, nargs="*", default=[0],
                    help="probe modes: 0 real, 1 consumers skip the dot products, 2 loaders issue no DMA")
    args = ap.parse_args()
    from aios_amd.models.config import get_preset
    from aios_amd.runtime.loader import random_engine

    cfg = get_preset(args.model)
    eng = random_engine(cfg, "Q4_K_M", seed=1234, max_ctx=args.prompt + 64, max_slots=1, max_batch=1)
    p = [cfg.bos_id] + [(7 * i) % (cfg.vocab_size - 3) + 3 for i in range(args.prompt - 1)]
    tok = int(eng.prefill(0, p, 0, True).argmax())
    eng.decode_loop_prepare([0], [tok], [args.prompt])
    eng.decode_loop_run(1, 8, True)
    eng.synchronize()
    L = cfg.n_layers
    for rep, dbg in [(r, d) for d in args.dbg for r in range(args.reps)]:
        ts = eng.mk_probe(dbg).astype(np.int64)  # [G][S][8] ticks of 10 ns
        t0 = ts[:, 0, 0].min()
        us = (ts - t0) / 100.0
        G, S, _ = ts.shape
        kind = [KINDS[s % 5] if s < 5 * L else "LM" for s in range(S)]
        rows = {}
        for k in KINDS + ["LM"]:
            ss = [s for s in range(S) if kind[s] == k]
            if not ss:
                continue
            a = us[:, ss, :]
            if k == "ATT":
                ph = {"wait": a[:, :, 1] - a[:, :, 0], "rest": a[:, :, 5] - a[:, :, 2]}
            else:
                ph = {"wait": a[:, :, 1] - a[:, :, 0], "stage": a[:, :, 3] - a[:, :, 2],
                      "slots": a[:, :, 4] - a[:, :, 3], "epi": a[:, :, 5] - a[:, :, 4],
                      "loader_stage": a[:, :, 7] - a[:, :, 6]}
            span = a[:, :, 5].max(axis=0) - a[:, :, 0].min(axis=0)  # stage start (first CU) -> end (last CU)
            rows[k] = {n: round(float(np.median(v)), 2) for n, v in ph.items()}
            rows[k]["p90_wait"] = round(float(np.percentile(ph["wait"], 90)), 2)
            rows[k]["stage_span_med"] = round(float(np.median(span)), 2)
            rows[k]["end_skew"] = round(float(np.median(a[:, :, 5].max(axis=0) - a[:, :, 5].min(axis=0))), 2)
        total = float(us[:, -1, 5].max())
        print(json.dumps({"rep": rep, "dbg": dbg, "total_us": round(total, 1), "per_layer_us": round(total / L, 2), **rows}),
              flush=True)


if __name__ == "__main__":
    main()
