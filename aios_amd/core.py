"""Loader for the native control-plane core (`aios_amd/_core*.so`, sources in aios_amd/native).

The core is host-only C++ (no HIP), so it builds and runs on CPU-only hosts as well; the first
import on a fresh checkout compiles it in-tree (≈20 s) unless AIOS_NO_AUTOBUILD=1.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

_mod = None


def load(build_if_missing: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    so = os.environ.get("AIOS_CORE_SO")  # e.g. the sanitizer build (scripts/sanitize.sh)
    if so:
        spec = importlib.util.spec_from_file_location("aios_amd._core", so)
        _mod = importlib.util.module_from_spec(spec)
        sys.modules["aios_amd._core"] = _mod
        spec.loader.exec_module(_mod)
        return _mod
    try:
        _mod = importlib.import_module("aios_amd._core")
        return _mod
    except ImportError as e:
        err = e
    if build_if_missing and os.environ.get("AIOS_NO_AUTOBUILD") != "1":
        from . import _build

        _build.build_core(verbose=False)
        importlib.invalidate_caches()
        _mod = importlib.import_module("aios_amd._core")
        return _mod
    raise ImportError(f"aios_amd control-plane core not built: {err}")
