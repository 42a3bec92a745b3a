"""Device sampler timing (aios::sample_kernel) per configuration: B = 1 row of a 32000-logit vocabulary,
greedy / temperature / top-k / top-p, with and without a grammar mask (allowed-token bitmap).

  python tools/sample_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from aios_amd.runtime import native


def main():
    only = os.environ.get("SAMPLE_ONLY", "")
    E = native.require()
    V, B = 32000, 1
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(0)
    logits = (torch.randn(B, V, generator=g) * 3).cuda()
    allowed = torch.zeros(V, dtype=torch.bool)
    allowed[torch.randperm(V, generator=g)[:300]] = True  # a JSON-grammar-like mask: a few hundred tokens open
    bits = torch.zeros((V + 7) // 8, dtype=torch.uint8)
    for i in allowed.nonzero().flatten().tolist():
        bits[i >> 3] |= 1 << (i & 7)
    maskd = bits.repeat(B, 1).cuda()
    pos = torch.zeros(B, dtype=torch.int32, device="cuda")
    tok = torch.zeros(B, dtype=torch.int32, device="cuda")
    out = []
    for name, temp, tk, tp, mask in [("greedy", 0.0, 0, 1.0, False), ("greedy+mask", 0.0, 0, 1.0, True),
                                     ("temp0.7", 0.7, 0, 1.0, False), ("temp0.7 k40 p0.95", 0.7, 40, 0.95, False),
                                     ("temp0.7 k40 p0.95 +mask", 0.7, 40, 0.95, True),
                                     ("temp0.7 p0.95", 0.7, 0, 0.95, False)]:
        if only and name != only:
            continue
        t = torch.full((B,), temp, device="cuda")
        k = torch.full((B,), tk, dtype=torch.int32, device="cuda")
        p = torch.full((B,), tp, device="cuda")

        def run():
            E.sample(logits.data_ptr(), V, B, V, t.data_ptr(), k.data_ptr(), 5, tok.data_ptr(), pos.data_ptr(),
                     maskd.data_ptr() if mask else 0, st, p.data_ptr())

        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            run()
        e1.record()
        torch.cuda.synchronize()
        row = {"config": name, "us": round(e0.elapsed_time(e1) * 1e3 / 200, 2), "token": int(tok[0])}
        # phase stamps (s_memrealtime, 100 MHz) of one launch: per slice workgroup, us from the first entry
        ns = (V + 4095) // 4096
        ts = torch.zeros(B * ns * 16, dtype=torch.int64, device="cuda")
        E.sample(logits.data_ptr(), V, B, V, t.data_ptr(), k.data_ptr(), 5, tok.data_ptr(), pos.data_ptr(),
                 maskd.data_ptr() if mask else 0, st, p.data_ptr(), ts.data_ptr())
        torch.cuda.synchronize()
        tv = ts.view(ns, 16).cpu()
        if int(tv[:, 0].max()) == 0:  # production build: the stamps are compiled out (AIOS_BUILD_PROBES=1)
            out.append(row)
            print(json.dumps(row), flush=True)
            continue
        t0 = int(tv[:, 0][tv[:, 0] > 0].min())
        row["stamps_us"] = {str(kk): [round((int(x) - t0) / 100, 2) for x in tv[:, kk].tolist() if int(x) > 0]
                            for kk in range(11) if int(tv[:, kk].max()) > 0}
        row["candidates"], row["survivors"] = int(tv[:, 12].max()), int(tv[:, 13].max())
        out.append(row)
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
