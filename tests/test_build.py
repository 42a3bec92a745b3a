"""A clean build (no cached objects) of the gfx950 engine compiles and links -- the driver's build()
reuses in-tree objects by mtime, so this is the check that the sources alone still build
(VERDICT r4).  CPU only: hipcc cross-compiles for gfx950 without a GPU.  Several minutes (the
GEMV translation units dominate); AIOS_SKIP_CLEAN_BUILD=1 skips it."""
import os
import shutil

import pytest


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
@pytest.mark.skipif(os.environ.get("AIOS_SKIP_CLEAN_BUILD") == "1", reason="AIOS_SKIP_CLEAN_BUILD=1")
def test_clean_build_compiles_and_links(tmp_path):
    from aios_amd import _build

    out = tmp_path / ("_engine" + _build.ext_suffix())
    so = _build.build(verbose=False, build_dir=tmp_path / "obj", out=out)
    assert so == out and out.stat().st_size > 1_000_000
    objs = sorted(p.name for p in (tmp_path / "obj").iterdir())
    assert len(objs) == len(_build._sources())
    # the extension exports the pybind11 module init and carries gfx950 code objects
    data = out.read_bytes()
    assert b"PyInit__engine" in data and b"gfx950" in data
