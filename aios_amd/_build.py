"""Native build: compile the gfx950 HIP kernels + C++ engine + pybind11 bindings in-tree.

`python -m aios_amd._build` (or `__graft_entry__.build()`) drives hipcc directly -- no hipify,
no torch.utils.cpp_extension -- producing `aios_amd/_engine*.so` next to the package so the
snapshot that travels to the GPU box carries it.  Objects are cached under `build/` and
rebuilt when a source or any header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("AIOS_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required)")


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def target_path() -> Path:
    return PKG / ("_engine" + ext_suffix())


def _sources():
    srcs = sorted((CSRC / "kernels").glob("*.hip")) + [CSRC / "engine.hip", CSRC / "grammar.cpp", CSRC / "rccl_comm.cpp",
                                                      CSRC / "bindings.cpp"]
    return srcs


def _headers():
    return list(CSRC.rglob("*.h"))


def _flags():
    import pybind11

    return [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "-Wno-unused-result",
        "-Wno-pass-failed",
        f"-I{CSRC}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
    ] + (["-DAIOS_GEMV_PROBES=1", "-DAIOS_ATTN_PROBES=1", "-DAIOS_SAMPLE_PROBES=1"] if os.environ.get("AIOS_BUILD_PROBES") == "1" else [])
    # (AIOS_BUILD_PROBES=1: the microbenchmark / phase-stamp hooks the probe tools use -- tools/attn_probe.py
    # --stamps, tools/gemv_cu_probe.py ring mode; compiled out of production builds)


# The GEMV ring consumers add one lane's row sum to an LDS accumulator per step; LLVM's atomic
# optimizer wraps every such uniform-address atomic in a readlane waterfall loop (~15 instructions
# per group in a VALU-issue-bound loop) although only one lane is active.  Off for the GEMV objects
# (elementwise.hip's many-lane candidate counters keep it).
_NO_ATOMIC_OPT = ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]
_FILE_FLAGS = {n: _NO_ATOMIC_OPT for n in ("gemv_kquant.hip", "gemv_kquant2.hip", "gemv_legacy.hip")}
# The prefill GEMM's weight decode beside MFMAs: LLVM's SLP vectoriser packs the fmaf pairs into
# v_pk_fma_f32, which costs ~+22 cycles per instruction when issued between MFMAs (MI355X guide,
# price list 'packed f32 VALU ... an anti-lever beside MFMAs'); plain v_fma_f32 instead.
for _n in ("gemm_pf.hip", "gemm_pf_q4k.hip", "gemm_pf_q6k.hip", "gemm_pf_mix.hip", "gemm_pf_bf16.hip", "gemm_pf_q5k.hip",
           "gemm_pf_q8q4.hip"):
    _FILE_FLAGS[_n] = ["-fno-slp-vectorize"]


def _deps(src: Path, seen=None) -> set:
    """src plus every quoted #include it reaches (resolved next to the includer or under csrc/)."""
    import re

    seen = set() if seen is None else seen
    if src in seen or not src.exists():
        return seen
    seen.add(src)
    for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', src.read_text(errors="ignore"), re.M):
        for base in (src.parent, CSRC):
            cand = (base / inc).resolve()
            if cand.exists():
                _deps(cand, seen)
                break
    return seen


def _compile(src: Path, flags, hipcc, build_dir: Path = None) -> Path:
    obj = (build_dir or BUILD) / (src.stem + ".o")
    newest_dep = max(d.stat().st_mtime for d in _deps(src))
    if obj.exists() and obj.stat().st_mtime >= newest_dep:
        return obj
    cmd = [hipcc, *flags, *_FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
    if src.suffix == ".cpp":
        cmd = [hipcc, *flags, "-x", "hip", "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    return obj


def build(verbose: bool = True, jobs: int | None = None, build_dir: Path | None = None, out: Path | None = None) -> Path:
    """Compile every HIP / C++ source of the engine for gfx950 (incrementally: an object is rebuilt when
    its source or a header it includes is newer) and link the extension.  build_dir / out: a clean
    build elsewhere (tests/test_build.py), leaving the in-tree objects and .so alone."""
    build_dir = Path(build_dir) if build_dir else BUILD
    build_dir.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    flags = _flags()
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, hipcc, build_dir), srcs))
    out = Path(out) if out else target_path()
    newest = max(o.stat().st_mtime for o in objs)
    if not out.exists() or out.stat().st_mtime < newest:
        tmp = out.with_suffix(".tmp.so")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
               "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, out)
    if verbose:
        print(f"[aios_amd] native engine: {out} ({out.stat().st_size / 1e6:.1f} MB, {ARCH})")
    return out


# ------------------------------------------------------------------------------ control-plane core
NATIVE = PKG / "native"


def core_target_path() -> Path:
    return PKG / ("_core" + ext_suffix())


def _sqlite_lib() -> str:
    for c in ("/lib/x86_64-linux-gnu/libsqlite3.so.0", "/usr/lib/x86_64-linux-gnu/libsqlite3.so.0",
              "/usr/lib64/libsqlite3.so.0"):
        if os.path.exists(c):
            return c
    raise RuntimeError("libsqlite3.so.0 not found")


def core_sanitized_path(sanitize: str) -> Path:
    return ROOT / "build" / ("core-" + sanitize.replace(",", "-")) / ("_core" + ext_suffix())


def build_core(verbose: bool = True, jobs: int | None = None, sanitize: str = "") -> Path:
    """Host-only C++17 build of aios_amd/native (tools / memory / orchestrator cores + bindings)
    into `aios_amd/_core*.so`, linked against the system libsqlite3 and OpenSSL libcrypto.

    sanitize="address,undefined" builds an instrumented copy under build/core-address-undefined/
    instead (loaded by aios_amd.core when AIOS_CORE_SO points at it; scripts/sanitize.sh)."""
    import pybind11

    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    out_dir = ROOT / "build" / ("core" + ("-san-" + sanitize.replace(",", "-") if sanitize else ""))
    out_dir.mkdir(parents=True, exist_ok=True)
    flags = ["-std=c++17", "-O2", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
             f"-I{NATIVE}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    san = [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-g"] if sanitize else []
    flags += san
    srcs = sorted(NATIVE.glob("*.cpp"))
    hdrs = list(NATIVE.glob("*.h"))

    def comp(src: Path) -> Path:
        obj = out_dir / (src.stem + ".o")
        newest = max([src.stat().st_mtime] + [h.stat().st_mtime for h in hdrs])
        if obj.exists() and obj.stat().st_mtime >= newest:
            return obj
        r = subprocess.run([cxx, *flags, "-c", str(src), "-o", str(obj)], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"c++ failed for {src.name}:\n{r.stderr[-6000:]}")
        return obj

    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(comp, srcs))
    out = core_sanitized_path(sanitize) if sanitize else core_target_path()
    out.parent.mkdir(parents=True, exist_ok=True)
    newest = max(o.stat().st_mtime for o in objs)
    if not out.exists() or out.stat().st_mtime < newest:
        tmp = out.with_suffix(".tmp.so")
        cmd = [cxx, "-shared", "-fPIC", *san, "-o", str(tmp), *map(str, objs), _sqlite_lib(), "-lcrypto", "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"core link failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, out)
    if verbose:
        print(f"[aios_amd] control-plane core: {out} ({out.stat().st_size / 1e6:.1f} MB)")
    return out


def initd_target_path() -> Path:
    return PKG / "bin" / "aios-init"


def build_initd(verbose: bool = True) -> Path:
    """Static-ish C++17 build of the init / supervisor daemon (aios_amd/native/initd)."""
    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    out = initd_target_path()
    out.parent.mkdir(parents=True, exist_ok=True)
    srcs = [NATIVE / "initd" / "initd.cpp", NATIVE / "json.cpp"]
    deps = srcs + [NATIVE / "json.h"]
    if not out.exists() or out.stat().st_mtime < max(d.stat().st_mtime for d in deps):
        tmp = out.with_suffix(".tmp")
        r = subprocess.run([cxx, "-std=c++17", "-O2", "-Wall", f"-I{NATIVE}", "-o", str(tmp), *map(str, srcs),
                            "-lpthread"], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"aios-init build failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, out)
    if verbose:
        print(f"[aios_amd] init daemon: {out}")
    return out


if __name__ == "__main__":
    build()
    build_core()
    build_initd()
    sys.exit(0)
