#!/usr/bin/env bash
# Minimal initramfs: busybox + the modules needed to reach the root image (NVMe / virtio / iso9660 /
# squashfs / overlay; amdgpu is loaded later by aios-init's hardware phase).  /init mounts the
# squashfs root read-only under a tmpfs overlay and switch_roots into /usr/sbin/aios-init.
#   scripts/build-initramfs.sh [--out build/distro] [--modules build/distro/modules] [--dry-run]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/distro"; MODS=""; DRY=0
while [ $# -gt 0 ]; do
  case "$1" in
    --out) OUT="$2"; shift ;; --modules) MODS="$2"; shift ;; --dry-run) DRY=1 ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
MODS="${MODS:-$OUT/modules}"
W="$OUT/initramfs"
run() { echo "+ $*"; [ "$DRY" = 1 ] || "$@"; }
BUSYBOX="$(command -v busybox || true)"
[ "$DRY" = 1 ] || [ -n "$BUSYBOX" ] || { echo "busybox (static) required" >&2; exit 1; }
run rm -rf "$W"
run mkdir -p "$W"/{bin,sbin,proc,sys,dev,run,mnt/ro,mnt/rw,newroot,lib/modules}
run cp "${BUSYBOX:-/bin/busybox}" "$W/bin/busybox"
for m in nvme nvme-core virtio_blk virtio_pci isofs squashfs overlay loop; do
  f="$(find "$MODS" -name "$m.ko*" 2>/dev/null | head -n 1 || true)"
  [ -n "$f" ] && run cp "$f" "$W/lib/modules/"
done
init_script() {
  cat <<'INIT'
#!/bin/busybox sh
/bin/busybox --install -s /bin
mount -t proc proc /proc; mount -t sysfs sysfs /sys; mount -t devtmpfs dev /dev
for m in /lib/modules/*.ko*; do insmod "$m" 2>/dev/null; done
# the boot medium carrying rootfs.squashfs (ISO label AIOS, or the first NVMe partition)
for i in $(seq 1 30); do
  dev=$(findfs LABEL=AIOS 2>/dev/null) && break
  sleep 0.5
done
[ -n "$dev" ] || dev=/dev/nvme0n1p1
mkdir -p /mnt/medium; mount -o ro "$dev" /mnt/medium || exec sh
mount -t squashfs -o loop,ro /mnt/medium/rootfs.squashfs /mnt/ro || exec sh
mount -t tmpfs tmpfs /mnt/rw; mkdir -p /mnt/rw/upper /mnt/rw/work
mount -t overlay overlay -o lowerdir=/mnt/ro,upperdir=/mnt/rw/upper,workdir=/mnt/rw/work /newroot || exec sh
grep -q aios.debug_shell=1 /proc/cmdline && exec sh
# aios.<key>=<value> kernel parameters -> AIOS_<KEY>=<value> for aios-init and its daemons
for kv in $(cat /proc/cmdline); do
  case "$kv" in aios.*=*)
    k=$(echo "${kv%%=*}" | sed 's/^aios\.//' | tr 'a-z.' 'A-Z_'); export "AIOS_$k=${kv#*=}" ;;
  esac
done
[ -f /newroot/etc/aios/environment ] && . /newroot/etc/aios/environment && export $(cut -d= -f1 /newroot/etc/aios/environment)
exec switch_root /newroot /usr/sbin/aios-init
INIT
}
if [ "$DRY" = 1 ]; then echo "+ write $W/init"; else init_script > "$W/init"; chmod 755 "$W/init"; fi
if [ "$DRY" = 1 ]; then
  echo "+ (cd $W && find . | cpio -o -H newc | zstd -19) > $OUT/initramfs.img"
else
  (cd "$W" && find . | cpio -o -H newc 2>/dev/null | zstd -19 -q) > "$OUT/initramfs.img"
fi
echo "initramfs -> $OUT/initramfs.img"
