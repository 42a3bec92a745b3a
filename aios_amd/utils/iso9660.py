"""ISO 9660 images without root or mkisofs: the aiOS boot medium as a data disc (scripts/build-iso.sh --data).

The early init finds its medium by the ISO 9660 volume id "AIOS" (distro/initramfs/init.c `label_is`,
sector 16, offset 40) and mounts it read-only; this writer produces that medium from a staging tree when
no grub-mkrescue / xorriso is available (the image then carries no boot catalog: the kernel and initramfs
on it are started by an external loader -- qemu -kernel / -initrd, PXE, kexec).  Interchange level 2:
upper-case d-character names of up to 30 characters with ";1" (Linux shows them lower-case), one extent
per file, both path tables, fixed timestamps, sorted entries -- the same tree always gives the same image.

  python -m aios_amd.utils.iso9660 --root build/distro/iso --out build/aios-mi355x.iso [--volid AIOS]
  python -m aios_amd.utils.iso9660 --list build/aios-mi355x.iso
"""
import argparse
import os
import re
import struct
import sys

SECTOR = 2048
_DATE7 = bytes([126, 1, 1, 0, 0, 0, 0])  # 2026-01-01 00:00:00 UTC
_DATE17 = b"2026010100000000\x00"
_NODATE17 = b"0" * 16 + b"\x00"


def _both16(v: int) -> bytes:
    return struct.pack("<H", v) + struct.pack(">H", v)


def _both32(v: int) -> bytes:
    return struct.pack("<I", v) + struct.pack(">I", v)


def iso_name(name: str, is_dir: bool) -> str:
    """A host name as an interchange-level-2 identifier: upper case, [A-Z0-9_] plus one '.', <= 30 chars."""
    base, _, ext = name.upper().rpartition(".") if ("." in name and not is_dir) else (name.upper(), "", "")
    clean = lambda s: re.sub(r"[^A-Z0-9_]", "_", s)  # noqa: E731
    base, ext = clean(base), clean(ext)
    if is_dir:
        return base[:30]
    ext = ext[:8]
    base = base[:max(1, 30 - len(ext) - 1)]
    return f"{base}.{ext};1"


def _record(ident: bytes, lba: int, size: int, is_dir: bool) -> bytes:
    n = 33 + len(ident)
    pad = b"\x00" if n % 2 else b""
    return (bytes([n + len(pad), 0]) + _both32(lba) + _both32(size) + _DATE7 + bytes([2 if is_dir else 0, 0, 0])
            + _both16(1) + bytes([len(ident)]) + ident + pad)


class _Dir:
    def __init__(self, path, name, parent):
        self.path, self.name, self.parent = path, name, parent
        self.dirs, self.files = [], []  # (_Dir) / (iso name, host path, size)
        self.lba = self.size = self.number = 0

    def entries(self):
        out = [(d.name, d) for d in self.dirs] + [(f[0], f) for f in self.files]
        return sorted(out, key=lambda e: e[0])

    def extent_size(self) -> int:
        """Bytes of this directory's records: none straddles a sector boundary."""
        used = 34 + 34  # "." and ".."
        for name, _ in self.entries():
            n = 33 + len(name) + (0 if len(name) % 2 else 1)
            if used % SECTOR + n > SECTOR:
                used += SECTOR - used % SECTOR
            used += n
        return (used + SECTOR - 1) // SECTOR * SECTOR


def _scan(root: str):
    top = _Dir(root, "\x00", None)
    todo = [top]
    order = []
    while todo:  # breadth first: the path tables' order
        d = todo.pop(0)
        order.append(d)
        seen = set()
        for e in sorted(os.scandir(d.path), key=lambda e: e.name):
            if e.is_symlink():
                continue
            name = iso_name(e.name, e.is_dir())
            if name in seen:
                raise ValueError(f"{e.path}: ISO name {name} collides with a sibling")
            seen.add(name)
            if e.is_dir():
                sub = _Dir(e.path, name, d)
                d.dirs.append(sub)
            elif e.is_file():
                size = e.stat().st_size
                if size >= 1 << 32:  # one extent per file (no level-3 multi-extent files)
                    raise ValueError(f"{e.path}: {size} bytes does not fit one ISO 9660 extent (< 4 GiB)")
                d.files.append((name, e.path, size))
        d.dirs.sort(key=lambda x: x.name)
        todo.extend(d.dirs)
    for i, d in enumerate(order):
        d.number = i + 1
    return order


def _path_table(order, big_endian: bool) -> bytes:
    out = bytearray()
    for d in order:
        ident = b"\x00" if d.parent is None else d.name.encode()
        parent = 1 if d.parent is None else d.parent.number
        lba = struct.pack(">I" if big_endian else "<I", d.lba)
        out += bytes([len(ident), 0]) + lba + struct.pack(">H" if big_endian else "<H", parent) + ident
        if len(ident) % 2:
            out += b"\x00"
    return bytes(out)


def write_iso(root: str, out_path: str, volid: str = "AIOS") -> int:
    """Write the tree under `root` as an ISO 9660 image; returns its size in bytes."""
    order = _scan(root)
    pt_size = len(_path_table(order, False))
    pt_sectors = (pt_size + SECTOR - 1) // SECTOR
    lba = 18  # 16 system-area sectors, the primary descriptor, the terminator
    l_pt, m_pt = lba, lba + pt_sectors
    lba += 2 * pt_sectors
    for d in order:
        d.size = d.extent_size()
        d.lba = lba
        lba += d.size // SECTOR
    files = []
    for d in order:
        for name, path, size in sorted(d.files):
            files.append((d, name, path, size, lba))
            lba += (size + SECTOR - 1) // SECTOR
    file_lba = {(id(d), name): (flba, size) for d, name, _, size, flba in files}
    total = lba

    with open(out_path, "wb") as f:
        f.write(b"\x00" * 16 * SECTOR)
        root_rec = _record(b"\x00", order[0].lba, order[0].size, True)
        pvd = (b"\x01CD001\x01\x00" + b"AIOS".ljust(32) + volid.upper().encode()[:32].ljust(32) + b"\x00" * 8
               + _both32(total) + b"\x00" * 32 + _both16(1) + _both16(1) + _both16(SECTOR) + _both32(pt_size)
               + struct.pack("<I", l_pt) + b"\x00" * 4 + struct.pack(">I", m_pt) + b"\x00" * 4 + root_rec
               + b" " * 128 + b"AIOS-MI355X".ljust(128) + b" " * 128 + b"AIOS_AMD.UTILS.ISO9660".ljust(128)
               + b" " * 37 * 3 + _DATE17 + _DATE17 + _NODATE17 + _DATE17 + b"\x01\x00")
        f.write(pvd.ljust(SECTOR, b"\x00"))
        f.write(b"\xffCD001\x01".ljust(SECTOR, b"\x00"))
        f.write(_path_table(order, False).ljust(pt_sectors * SECTOR, b"\x00"))
        f.write(_path_table(order, True).ljust(pt_sectors * SECTOR, b"\x00"))
        for d in order:
            buf = bytearray()
            parent = d.parent or d
            for rec in (_record(b"\x00", d.lba, d.size, True), _record(b"\x01", parent.lba, parent.size, True)):
                buf += rec
            for name, ent in d.entries():
                if isinstance(ent, _Dir):
                    rec = _record(name.encode(), ent.lba, ent.size, True)
                else:
                    flba, size = file_lba[(id(d), name)]
                    rec = _record(name.encode(), flba if size else 0, size, False)
                if len(buf) % SECTOR + len(rec) > SECTOR:
                    buf += b"\x00" * (SECTOR - len(buf) % SECTOR)
                buf += rec
            f.write(bytes(buf).ljust(d.size, b"\x00"))
        for d, name, path, size, flba in files:
            assert f.tell() == flba * SECTOR or size == 0
            if not size:
                continue
            with open(path, "rb") as src:
                while True:
                    chunk = src.read(1 << 20)
                    if not chunk:
                        break
                    f.write(chunk)
            f.write(b"\x00" * ((SECTOR - size % SECTOR) % SECTOR))
        assert f.tell() == total * SECTOR
    return total * SECTOR


def read_iso(path: str):
    """(volume id, {path: bytes}) of an image written by write_iso (or any plain level-1/2 image),
    parsed from the primary descriptor and the directory records -- not from the path tables."""
    with open(path, "rb") as f:
        data = f.read()
    pvd = data[16 * SECTOR: 17 * SECTOR]
    if pvd[1:6] != b"CD001" or pvd[0] != 1:
        raise ValueError("no primary volume descriptor")
    volid = pvd[40:72].decode().rstrip()
    out = {}

    def walk(lba, size, prefix):
        pos, end = lba * SECTOR, lba * SECTOR + size
        while pos < end:
            n = data[pos]
            if n == 0:  # the rest of this sector is padding
                pos = (pos // SECTOR + 1) * SECTOR
                continue
            elba, esize = struct.unpack("<I", data[pos + 2:pos + 6])[0], struct.unpack("<I", data[pos + 10:pos + 14])[0]
            flags, nlen = data[pos + 25], data[pos + 32]
            ident = data[pos + 33:pos + 33 + nlen]
            if ident not in (b"\x00", b"\x01"):
                name = ident.decode().split(";")[0].lower()
                if not flags & 2 and name.endswith("."):
                    name = name[:-1]  # "VMLINUZ.;1" -> vmlinuz, as Linux's isofs shows it
                if flags & 2:
                    walk(elba, esize, prefix + name + "/")
                else:
                    out[prefix + name] = data[elba * SECTOR: elba * SECTOR + esize]
            pos += n

    r = pvd[156:190]
    walk(struct.unpack("<I", r[2:6])[0], struct.unpack("<I", r[10:14])[0], "")
    return volid, out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--root")
    ap.add_argument("--out")
    ap.add_argument("--volid", default="AIOS")
    ap.add_argument("--list")
    a = ap.parse_args(argv)
    if a.list:
        volid, files = read_iso(a.list)
        print(f"volume {volid}")
        for name, body in sorted(files.items()):
            print(f"{len(body):12d} {name}")
        return 0
    if not a.root or not a.out:
        ap.error("--root and --out (or --list)")
    n = write_iso(a.root, a.out, a.volid)
    print(f"{a.out}: {n} bytes, volume {a.volid}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
