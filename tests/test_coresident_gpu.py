"""GPU: co-resident model tiers (BASELINE.json config 4: TinyLlama + Mistral co-resident in HBM,
concurrent agent-router dispatch, hipGraph decode).  Two engines on one GPU, each with its own
non-blocking HIP stream and captured decode graph, decoding at the same time from two host
threads, must produce exactly the tokens each produces alone (stream isolation: no shared
scratch, counters or graph state between engines)."""
import threading

import numpy as np
import pytest

from aios_amd.models.config import get_preset

pytestmark = pytest.mark.gpu


def _engine(preset, seed):
    from aios_amd.runtime.loader import random_engine

    cfg = get_preset(preset)
    return cfg, random_engine(cfg, "Q4_K_M", seed=seed, max_ctx=256, max_slots=1, max_batch=1)


def _decode(eng, cfg, steps, prompt_len=20):
    prompt = [cfg.bos_id] + [(5 * i + 3) % (cfg.vocab_size - 3) + 3 for i in range(prompt_len - 1)]
    first = int(np.argmax(eng.prefill(0, prompt, 0, True)))
    eng.decode_loop_prepare([0], [first], [prompt_len])
    eng.decode_loop_run(1, steps, True)
    eng.synchronize()
    return list(eng.decode_loop_history(1, prompt_len + 1, steps))


def test_coresident_engines_decode_concurrently_and_match_alone():
    small_cfg, small = _engine("test-small", 5)
    big_cfg, big = _engine("test-mistral-shape", 6)
    alone = (_decode(small, small_cfg, 48), _decode(big, big_cfg, 48))
    out = [None, None]

    def run(i, eng, cfg):
        for _ in range(3):  # several overlapping rounds
            out[i] = _decode(eng, cfg, 48)

    ts = [threading.Thread(target=run, args=(0, small, small_cfg)), threading.Thread(target=run, args=(1, big, big_cfg))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert out[0] == alone[0] and out[1] == alone[1]


@pytest.mark.parametrize("split", [64, 128])
def test_cu_masked_tiers_match_unmasked(split):
    """each tier on its own CUs (CU-masked stream, grids sized to the mask) decodes
    exactly the tokens of the unmasked engine, alone and concurrently with the other tier."""
    from aios_amd.runtime.loader import random_engine
    from aios_amd.runtime.native import cu_mask_words, require

    total = require().device_cu_count()
    small_cfg, big_cfg = get_preset("test-small"), get_preset("test-mistral-shape")
    ref_small, ref_big = _engine("test-small", 5)[1], _engine("test-mistral-shape", 6)[1]
    want = (_decode(ref_small, small_cfg, 48), _decode(ref_big, big_cfg, 48))
    del ref_small, ref_big
    small = random_engine(small_cfg, "Q4_K_M", seed=5, max_ctx=256, max_slots=1, max_batch=1,
                          cu_mask=cu_mask_words(split, 0, total))
    big = random_engine(big_cfg, "Q4_K_M", seed=6, max_ctx=256, max_slots=1, max_batch=1,
                        cu_mask=cu_mask_words(total - split, split // 8, total))
    assert (_decode(small, small_cfg, 48), _decode(big, big_cfg, 48)) == want
    out = [None, None]

    def run(i, eng, cfg):
        for _ in range(3):
            out[i] = _decode(eng, cfg, 48)

    ts = [threading.Thread(target=run, args=(0, small, small_cfg)), threading.Thread(target=run, args=(1, big, big_cfg))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert tuple(out) == want
