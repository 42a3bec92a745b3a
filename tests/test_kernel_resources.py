"""Static check of the built engine (no GPU): no decode-path kernel may use scratch memory.

Round 4 found two such regressions only through same-box benchmarks (a register left unwritten on
one side of a branch sent the batch-1 engine's x prefetch to 80 B/lane of scratch: -15 % decode;
a per-lane K/V cache pointer select put 24 B in every batched GEMV).  tools/kernel_resources.py
reads the AMDGPU metadata of every kernel in the .so's offload bundles."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools import kernel_resources as kr  # noqa: E402


def _so():
    try:
        return kr._engine_so()
    except FileNotFoundError:
        return None


@pytest.mark.skipif(_so() is None, reason="engine not built")
def test_hot_kernels_use_no_scratch():
    pytest.importorskip("msgpack")
    rows = kr.kernels(_so())
    assert len(rows) > 100  # the whole kernel set was read
    names = {r["name"] for r in rows}
    # the decode path's kernels are all present ...
    for must in ("gemv_lds_b1<12, 12, 1, 1>", "gemv_q8_rows<12, 14, 1, 2, 1>", "attn_decode_kernel<128, 4, false>",
                 "attn_decode_kernel<128, 4, true>", "gemv_lds16<1, 3, 2>", "gemm_ring_kernel<12, 12, 1, 2, true>"):
        assert any(must in n for n in names), must
    # ... and none of them spills to scratch
    bad = kr.hot_with_scratch(rows)
    assert not bad, [(r["name"], r["scratch"]) for r in bad]
