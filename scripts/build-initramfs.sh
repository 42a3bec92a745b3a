#!/usr/bin/env bash
# Minimal initramfs: a static early init (distro/initramfs/init.c -- no busybox needed) + the modules needed to
# reach the root image (NVMe / virtio / iso9660 / squashfs / overlay / loop; amdgpu is loaded later by
# aios-init's hardware phase).  /init mounts the squashfs root read-only under a tmpfs overlay and
# switch_roots into /usr/sbin/aios-init.  The newc archive is written by aios_amd.utils.cpio: no root, no
# cpio tool, deterministic (every entry root-owned, mtime 0).  With --busybox and a static busybox on PATH,
# /init is the busybox script of the same plan instead and /bin/sh is the rescue shell.
#   scripts/build-initramfs.sh [--out build/distro] [--modules build/distro/modules] [--busybox] [--dry-run]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/distro"; MODS=""; DRY=0; BB=0
while [ $# -gt 0 ]; do
  case "$1" in
    --out) OUT="$2"; shift ;; --modules) MODS="$2"; shift ;; --dry-run) DRY=1 ;; --busybox) BB=1 ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
MODS="${MODS:-$OUT/modules}"
W="$OUT/initramfs"
CC="${CC:-gcc}"
PY="${PYTHON:-python3}"
run() { echo "+ $*"; [ "$DRY" = 1 ] || "$@"; }
run rm -rf "$W"
run mkdir -p "$W"/{bin,sbin,proc,sys,dev,run,mnt/medium,mnt/ro,mnt/rw,newroot,lib/modules}
for m in nvme nvme-core virtio_blk virtio_pci isofs squashfs overlay loop; do
  f="$(find "$MODS" -name "$m.ko*" 2>/dev/null | head -n 1 || true)"
  [ -n "$f" ] && run cp "$f" "$W/lib/modules/"
done
if [ "$BB" = 1 ]; then
  BUSYBOX="$(command -v busybox || true)"
  [ "$DRY" = 1 ] || [ -n "$BUSYBOX" ] || { echo "--busybox: a static busybox is required" >&2; exit 1; }
  run cp "${BUSYBOX:-/bin/busybox}" "$W/bin/busybox"
  init_script() {
    cat <<'INIT'
#!/bin/busybox sh
/bin/busybox --install -s /bin
mount -t proc proc /proc; mount -t sysfs sysfs /sys; mount -t devtmpfs dev /dev
for m in /lib/modules/*.ko*; do insmod "$m" 2>/dev/null; done
for i in $(seq 1 30); do
  dev=$(findfs LABEL=AIOS 2>/dev/null) && break
  sleep 0.5
done
[ -n "$dev" ] || dev=/dev/nvme0n1p1
mount -o ro "$dev" /mnt/medium || exec sh
if [ -f /mnt/medium/rootfs.squashfs ]; then
  mount -t squashfs -o loop,ro /mnt/medium/rootfs.squashfs /mnt/ro || exec sh
else
  mount -t ext4 -o loop,ro /mnt/medium/rootfs.ext4 /mnt/ro || exec sh
fi
mount -t tmpfs tmpfs /mnt/rw; mkdir -p /mnt/rw/upper /mnt/rw/work
mount -t overlay overlay -o lowerdir=/mnt/ro,upperdir=/mnt/rw/upper,workdir=/mnt/rw/work /newroot || exec sh
grep -q aios.debug_shell=1 /proc/cmdline && exec sh
for kv in $(cat /proc/cmdline); do
  case "$kv" in aios.*=*)
    k=$(echo "${kv%%=*}" | sed 's/^aios\.//' | tr 'a-z.' 'A-Z_'); export "AIOS_$k=${kv#*=}" ;;
  esac
done
exec switch_root /newroot /usr/sbin/aios-init
INIT
  }
  if [ "$DRY" = 1 ]; then echo "+ write $W/init"; else init_script > "$W/init"; chmod 755 "$W/init"; fi
else
  # the static early init: one binary, no libc or shell in the image
  run "$CC" -static -O2 -Wall -o "$W/init" "$ROOT/distro/initramfs/init.c"
  run strip "$W/init"
fi
run env PYTHONPATH="$ROOT" "$PY" -m aios_amd.utils.cpio --root "$W" --out "$OUT/initramfs.img" --gzip
echo "initramfs -> $OUT/initramfs.img"
