#!/usr/bin/env python3
"""Per-kernel resource table of the built engine (.so): VGPRs/AGPRs, SGPRs, LDS, scratch, spills.

Reads the gfx950 code objects out of the .so's `.hip_fatbin` section (clang offload bundles) and the
AMDGPU metadata note (msgpack) of each -- no GPU, no ROCm tool needed.  The check that matters:
a decode-path kernel with a non-zero private segment (scratch) runs ~15 % slower per token (round 4:
one float4 left unwritten on one side of a branch sent the B = 1 engine's x prefetch to scratch).

  python tools/kernel_resources.py                     # table of every kernel with scratch
  python tools/kernel_resources.py --all --grep gemv_lds
  python tools/kernel_resources.py --check             # exit 1 if a HOT kernel uses scratch
"""
import argparse
import fnmatch
import os
import re
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "aios_amd")

# decode-path kernel templates that must never touch scratch (mangled-name globs over the
# demangled text); the batch>1 row-pair GEMV variants are fallbacks and are reported, not enforced
HOT = [
    "aios::gemv_lds_b1<*, *, 1, *>*",
    "aios::gemv_lds16<*",
    "aios::gemv_q8_rows<*, *, 1, 2, 1>*",
    "aios::gemv_q8_rows<*, *, 1, 1, *>*",
    "aios::gemv_q8_rows<*, *, 1, 2, 2>*",
    "aios::attn_decode_kernel<*",
    "aios::gemm_skinny_kernel<*",
    "aios::gemm_ring_kernel<*",
    "aios::sample_kernel*",
    "aios::get_rows_step_kernel*",
]


def _engine_so():
    for f in sorted(os.listdir(SO)):
        if f.startswith("_engine") and f.endswith(".so"):
            return os.path.join(SO, f)
    raise FileNotFoundError("no built engine under aios_amd/ (run __graft_entry__.build())")


def _section(elf: bytes, want: str) -> bytes:
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    strtab = hdrs[shstrndx]
    for h in hdrs:
        name_off = strtab[4] + h[0]
        name = elf[name_off:elf.index(b"\0", name_off)].decode()
        if name == want:
            return elf[h[4]:h[4] + h[5]]
    return b""


def _code_objects(fat: bytes):
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = fat.find(magic)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        off = pos + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", fat, off)
            triple = fat[off + 24:off + 24 + tl].decode()
            off += 24 + tl
            if "gfx950" in triple and es:
                yield fat[pos + eo:pos + eo + es]
        pos = fat.find(magic, pos + 24)


def _notes(elf: bytes):
    import msgpack

    note = _section(elf, ".note")
    i = 0
    while i + 12 <= len(note):
        nsz, dsz, typ = struct.unpack_from("<III", note, i)
        name = note[i + 12:i + 12 + nsz]
        d0 = i + 12 + ((nsz + 3) & ~3)
        if name.startswith(b"AMDGPU") and typ == 32:
            return msgpack.unpackb(note[d0:d0 + dsz], raw=False)
        i = d0 + ((dsz + 3) & ~3)
    return {}


def _demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, timeout=30).stdout
        return out.splitlines()
    except (OSError, subprocess.SubprocessError):
        return list(names)


def kernels(so_path=None):
    so = open(so_path or _engine_so(), "rb").read()
    fat = _section(so, ".hip_fatbin")
    rows = {}
    for co in _code_objects(fat):
        for k in _notes(co).get("amdhsa.kernels", []):
            rows[k[".name"]] = k
    names = sorted(rows)
    out = []
    for mangled, dem in zip(names, _demangle(names)):
        k = rows[mangled]
        out.append(dict(name=re.sub(r"\(.*", "", dem), mangled=mangled, vgpr=k.get(".vgpr_count", 0),
                        agpr=k.get(".agpr_count", 0), sgpr=k.get(".sgpr_count", 0),
                        lds=k.get(".group_segment_fixed_size", 0), scratch=k.get(".private_segment_fixed_size", 0),
                        vspill=k.get(".vgpr_spill_count", 0), sspill=k.get(".sgpr_spill_count", 0),
                        wg=k.get(".max_flat_workgroup_size", 0)))
    return out


def hot_with_scratch(rows):
    return [r for r in rows if r["scratch"] and any(fnmatch.fnmatchcase(r["name"], "void " + p) or
                                                     fnmatch.fnmatchcase(r["name"], p) for p in HOT)]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--so", default=None)
    ap.add_argument("--all", action="store_true", help="every kernel, not only those with scratch")
    ap.add_argument("--grep", default=None)
    ap.add_argument("--check", action="store_true", help="exit 1 when a hot decode kernel uses scratch")
    a = ap.parse_args(argv)
    rows = kernels(a.so)
    show = [r for r in rows if (a.all or r["scratch"]) and (not a.grep or a.grep in r["name"])]
    print(f"{'scratch':>7} {'vgpr':>4} {'agpr':>4} {'sgpr':>4} {'lds':>6} {'spill':>5}  kernel")
    for r in show:
        print(f"{r['scratch']:>7} {r['vgpr']:>4} {r['agpr']:>4} {r['sgpr']:>4} {r['lds']:>6} "
              f"{r['vspill'] + r['sspill']:>5}  {r['name']}")
    print(f"# {len(rows)} kernels, {sum(1 for r in rows if r['scratch'])} with scratch")
    if a.check:
        bad = hot_with_scratch(rows)
        for r in bad:
            print(f"HOT KERNEL USES SCRATCH: {r['scratch']} B  {r['name']}", file=sys.stderr)
        return 1 if bad else 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
