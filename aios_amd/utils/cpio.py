"""newc ("070701") cpio archives, the format the Linux kernel unpacks an initramfs from.

Written without root and without the cpio tool: every entry is recorded as owned by root (uid / gid 0)
with the source tree's modes, in a sorted, deterministic order (mtime 0), so the same tree always gives
the same image (scripts/build-initramfs.sh).  `read_newc` parses an archive back (tests, `--list`).

  python -m aios_amd.utils.cpio --root build/distro/initramfs --out build/distro/initramfs.img [--gzip]
  python -m aios_amd.utils.cpio --list build/distro/initramfs.img
"""
import argparse
import gzip
import io
import os
import stat
import sys

MAGIC = b"070701"
TRAILER = "TRAILER!!!"


def _pad4(n: int) -> int:
    return (4 - n % 4) % 4


def _header(name: bytes, ino: int, mode: int, nlink: int, size: int, rdev: int = 0) -> bytes:
    fields = [ino, mode, 0, 0, nlink, 0, size, 0, 0, (rdev >> 8) & 0xfff, rdev & 0xff, len(name) + 1, 0]
    return MAGIC + b"".join(b"%08X" % f for f in fields)


def _entry(out, name: str, ino: int, mode: int, data: bytes = b"", nlink: int = 1, rdev: int = 0):
    nb = name.encode()
    hdr = _header(nb, ino, mode, nlink, len(data), rdev) + nb + b"\0"
    out.write(hdr + b"\0" * _pad4(len(hdr)))
    out.write(data + b"\0" * _pad4(len(data)))


def write_newc(root: str, extra_nodes=(("dev/console", 0o600, 5, 1),)) -> bytes:
    """The tree under `root` as a newc archive.  `extra_nodes`: (path, perm, major, minor) character
    devices created in the archive (the kernel needs /dev/console before devtmpfs is mounted)."""
    out = io.BytesIO()
    ino = 1
    paths = []
    for dirpath, dirnames, filenames in os.walk(root):
        dirnames.sort()
        rel = os.path.relpath(dirpath, root)
        if rel != ".":
            paths.append(rel)
        for f in sorted(filenames):
            paths.append(os.path.normpath(os.path.join(rel, f)))
    for rel in sorted(paths):
        full = os.path.join(root, rel)
        st = os.lstat(full)
        if stat.S_ISDIR(st.st_mode):
            _entry(out, rel, ino, stat.S_IFDIR | (st.st_mode & 0o7777), nlink=2)
        elif stat.S_ISLNK(st.st_mode):
            _entry(out, rel, ino, stat.S_IFLNK | 0o777, os.readlink(full).encode())
        elif stat.S_ISREG(st.st_mode):
            with open(full, "rb") as f:
                _entry(out, rel, ino, stat.S_IFREG | (st.st_mode & 0o7777), f.read())
        else:
            continue  # device nodes of the staging tree: declared through extra_nodes instead
        ino += 1
    for path, perm, major, minor in extra_nodes:
        if path not in paths:
            _entry(out, path, ino, stat.S_IFCHR | perm, rdev=(major << 8) | minor)
            ino += 1
    _entry(out, TRAILER, 0, 0, nlink=1)
    data = out.getvalue()
    return data + b"\0" * _pad4(len(data))


def read_newc(data: bytes):
    """[(name, mode, size, bytes)] of an (optionally gzip-compressed) newc archive."""
    if data[:2] == b"\x1f\x8b":
        data = gzip.decompress(data)
    out, pos = [], 0
    while True:
        if data[pos:pos + 6] != MAGIC:
            raise ValueError(f"bad cpio magic at {pos}")
        f = [int(data[pos + 6 + 8 * i: pos + 14 + 8 * i], 16) for i in range(13)]
        mode, size, namesize = f[1], f[6], f[11]
        npos = pos + 110
        name = data[npos:npos + namesize - 1].decode()
        dpos = npos + namesize
        dpos += _pad4(dpos)
        if name == TRAILER:
            return out
        out.append((name, mode, size, data[dpos:dpos + size]))
        pos = dpos + size
        pos += _pad4(pos)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--root")
    ap.add_argument("--out")
    ap.add_argument("--gzip", action="store_true")
    ap.add_argument("--list")
    a = ap.parse_args(argv)
    if a.list:
        with open(a.list, "rb") as f:
            for name, mode, size, _ in read_newc(f.read()):
                print(f"{mode:07o} {size:10d} {name}")
        return 0
    if not a.root or not a.out:
        ap.error("--root and --out (or --list)")
    data = write_newc(a.root)
    if a.gzip:
        data = gzip.compress(data, compresslevel=9, mtime=0)
    with open(a.out, "wb") as f:
        f.write(data)
    print(f"{a.out}: {len(data)} bytes")
    return 0


if __name__ == "__main__":
    sys.exit(main())
