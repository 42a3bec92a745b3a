"""CPU tests: fp32 reference forward (the numerics oracle) is self-consistent."""
import torch

from aios_amd.models.config import get_preset
from aios_amd.models.reference import ReferenceModel
from aios_amd.models.synthetic import write_synthetic_gguf


def test_incremental_equals_full(tmp_path):
    cfg = get_preset("test-tiny")
    p = write_synthetic_gguf(str(tmp_path / "m.gguf"), cfg, "Q8_0", seed=3)
    ref = ReferenceModel.from_gguf(p)
    toks = [1, 50, 60, 70, 80, 90, 100]
    full = ref.forward(toks)
    cache = ref.new_cache()
    a = ref.forward(toks[:4], cache)
    b = ref.forward(toks[4:], cache)
    inc = torch.cat([a, b], 0)
    assert torch.allclose(full, inc, atol=1e-4, rtol=1e-4)


def test_greedy_runs(tmp_path):
    cfg = get_preset("test-tiny")
    p = write_synthetic_gguf(str(tmp_path / "m.gguf"), cfg, "Q4_0", seed=1)
    ref = ReferenceModel.from_gguf(p)
    out = ref.greedy([1, 10, 20], 5)
    assert len(out) == 5 and all(0 <= t < cfg.vocab_size for t in out)
