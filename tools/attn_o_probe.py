"""Fused attention -> O launch (kernels/attn_o.hip) probe: a 2-layer random Mistral-7B engine,
batch-1 decode steps timed eagerly and through the graph loop, then layer 0's counter block (the
per-XCD counts, the XCD-dealing error flag and -- AIOS_ATTN_XCD=3 -- every workgroup's physical
XCD)."""
import dataclasses
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("AIOS_GEMM_PF_TUNE", "0")
from aios_amd.models.config import get_preset  # noqa: E402
from aios_amd.runtime.loader import random_engine  # noqa: E402

ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 140
cfg = dataclasses.replace(get_preset("mistral-7b"), n_layers=2)
eng = random_engine(cfg, "Q4_K_M", seed=3, max_ctx=1024, max_slots=1, max_batch=1)
prompt = [1] + [(7 * i) % (cfg.vocab_size - 3) + 3 for i in range(ctx - 1)]
tok = int(np.argmax(eng.prefill(0, prompt, 0, True)))
for i in range(3):
    t0 = time.perf_counter()
    tok = eng.decode([0], [tok], [ctx + i])[0]
    eng.synchronize()
    print(f"decode step {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
for l in range(2):
    c = np.asarray(eng.attn_o_counters(l))
    print(f"layer {l}: short counts {c[0:256:32].tolist()} long {c[256:512:32].tolist()}")
    if c[768] != 0:
        x = c[768:1024] - 100
        r = (x[0] - 0) % 8
        print(f"  xcc of wg b == (b + {r}) % 8 for all b:", bool(np.all(x == (np.arange(256) + r) % 8)), x[:12].tolist())
