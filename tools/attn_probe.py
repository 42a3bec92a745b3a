"""Decode-attention microbenchmark on the GPU: per-launch time (hipGraph of back-to-back launches)
of attn_decode over context lengths x split sizes.  python tools/attn_probe.py
--stamps (needs a probe build: AIOS_BUILD_PROBES=1 with the build dir removed -- production builds
compile the stamps out): per-phase in-kernel timestamps (s_memrealtime, AttnDecodeArgs.ts) of one launch with the
K/V cache evicted from the Infinity Cache first (a 512 MB write in between), median / max over the
workgroups: entry -> seq_len known -> first pass computed -> waves merged -> partial published ->
combine weights ready -> done."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from aios_amd.runtime import native


def graph_time(fn, n=64, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * n)


def stamps(E):
    H, Hkv, hd, max_ctx = 32, 8, 128, 4096
    kc = (torch.randn(1, Hkv, max_ctx, hd) * 0.5).to(torch.bfloat16).cuda()
    vc = torch.randn(1, Hkv, max_ctx, hd).to(torch.bfloat16).cuda()
    q = torch.randn(1, H, hd, device="cuda")
    slot = torch.zeros(1, dtype=torch.int32, device="cuda")
    nch = max_ctx // E.ATTN_CHUNK
    opart = torch.empty(1, H, nch, hd, device="cuda")
    ml = torch.empty(1, H, nch, 2, device="cuda")
    out = torch.empty(1, H * hd, device="cuda")
    cnt = torch.zeros(1, H, dtype=torch.int32, device="cuda")
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    ts = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    names = ["entry", "seq_len", "pass1", "merged", "published", "weights", "done"]
    for L, comb in ((153, 1), (1000, 2), (1000, 1), (4000, 2), (4000, 1)):
        # AIOS_ATTN_COMBINE: 2 = two-round-trip split-K combine, 1 = one round trip (round 4)
        os.environ["AIOS_ATTN_COMBINE"] = str(comb)
        seq = torch.tensor([L], dtype=torch.int32, device="cuda")
        run = lambda t=0: E.attn_decode(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), seq.data_ptr(), slot.data_ptr(),
                                        1, H, Hkv, hd, max_ctx, nch, 1 / math.sqrt(hd), opart.data_ptr(), ml.data_ptr(),
                                        out.data_ptr(), cnt.data_ptr(), torch.cuda.current_stream().cuda_stream, 0,
                                        ts=t)
        run()
        rows = []
        for rep in range(5):
            flush.fill_(rep)
            ts.zero_()
            torch.cuda.synchronize()
            run(ts.data_ptr())
            torch.cuda.synchronize()
            t = ts.view(-1, 8).cpu().numpy().astype("float64")
            t = t[t[:, 0] > 0]
            rows.append((t - t[:, 0].min()) / 100.0)  # 100 MHz ticks -> us from the first entry
        import numpy as np
        t = np.concatenate(rows[1:])
        res = {}
        for k, n in enumerate(names):
            v = t[:, k][t[:, k] > 0] if k else t[:, 0]
            if len(v):
                res[n] = [round(float(np.median(v)), 2), round(float(v.max()), 2)]
        us = graph_time(lambda: run())
        print(json.dumps({"len": L, "combine_trips": comb, "graph_us": round(us, 2), "workgroups": int(len(t) / 4),
                          "phase_us_median_max": res}), flush=True)
    os.environ.pop("AIOS_ATTN_COMBINE")


def main():
    E = native.require()
    if "--stamps" in sys.argv:
        stamps(E)
        return
    H, Hkv, hd = 32, 8, 128
    for max_ctx in (512, 4096):
        kc = (torch.randn(1, Hkv, max_ctx, hd) * 0.5).to(torch.bfloat16).cuda()
        vc = torch.randn(1, Hkv, max_ctx, hd).to(torch.bfloat16).cuda()
        q = torch.randn(1, H, hd, device="cuda")
        slot = torch.zeros(1, dtype=torch.int32, device="cuda")
        nch = max_ctx // E.ATTN_CHUNK
        opart = torch.empty(1, H, nch, hd, device="cuda")
        ml = torch.empty(1, H, nch, 2, device="cuda")
        out = torch.empty(1, H * hd, device="cuda")
        cnt = torch.zeros(1, H, dtype=torch.int32, device="cuda")
        for L in (64, 130, 153, 256, 400, 1000, 2000, 4000):
            if L > max_ctx:
                continue
            seq = torch.tensor([L], dtype=torch.int32, device="cuda")
            row = []
            for P in (0, 8, 16, 32, 64):
                if P > nch:
                    continue
                split = P * E.ATTN_CHUNK
                fn = lambda: E.attn_decode(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), seq.data_ptr(), slot.data_ptr(),
                                           1, H, Hkv, hd, max_ctx, nch, 1 / math.sqrt(hd), opart.data_ptr(),
                                           ml.data_ptr(), out.data_ptr(), cnt.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream, split)
                row.append(f"P{P}={graph_time(fn):6.2f}")
            # split-shape knobs at the launcher's P: passes per workgroup x short-mode splits
            for ppw in (1, 2):
                for sp in (1, 2, 4):
                    os.environ["AIOS_ATTN_PPW"], os.environ["AIOS_ATTN_SHORT_P"] = str(ppw), str(sp)
                    fn = lambda: E.attn_decode(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), seq.data_ptr(),
                                               slot.data_ptr(), 1, H, Hkv, hd, max_ctx, nch, 1 / math.sqrt(hd),
                                               opart.data_ptr(), ml.data_ptr(), out.data_ptr(), cnt.data_ptr(),
                                               torch.cuda.current_stream().cuda_stream, 0)
                    row.append(f"w{ppw}s{sp}={graph_time(fn):6.2f}")
            os.environ.pop("AIOS_ATTN_PPW")
            os.environ.pop("AIOS_ATTN_SHORT_P")
            kv_mb = 2 * Hkv * L * hd * 2 / 1e6
            row.append(f"KV={kv_mb:.2f}MB")
            print(f"max_ctx={max_ctx:5d} len={L:5d}  " + "  ".join(row), flush=True)
    print("launch chain graph (256 blocks): %.2f us/kernel" % E.bench_launch_chain(200, 256, 1, 20))


if __name__ == "__main__":
    main()
