#!/usr/bin/env bash
# Bootable hybrid ISO (BIOS + UEFI, GRUB): kernel + initramfs + rootfs.squashfs, label AIOS.
#   scripts/build-iso.sh [--out build/distro] [--iso build/aios-mi355x.iso] [--data] [--dry-run]
# Runs the kernel / rootfs / initramfs builds first when their outputs are missing.
# --data (or no grub-mkrescue on PATH): a non-bootable data medium written by aios_amd.utils.iso9660 --
# no root, no ISO tools -- holding whatever of vmlinuz / initramfs.img / rootfs.squashfs / rootfs.ext4 /
# aios-overlay.ext4 exists (the initramfs is built offline when missing); volume id AIOS, so the early
# init finds it; the kernel and initramfs are then started by an external loader (qemu -kernel/-initrd).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/distro"; ISO="$ROOT/build/aios-mi355x.iso"; DRY=0; PASS=(); DATA=0
while [ $# -gt 0 ]; do
  case "$1" in
    --out) OUT="$2"; shift ;; --iso) ISO="$2"; shift ;; --dry-run) DRY=1; PASS+=(--dry-run) ;; --data) DATA=1 ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
run() { echo "+ $*"; [ "$DRY" = 1 ] || "$@"; }
command -v grub-mkrescue >/dev/null 2>&1 || [ "$DRY" = 1 ] || DATA=1
if [ "$DATA" = 1 ]; then
  [ -f "$OUT/initramfs.img" ] || "$ROOT/scripts/build-initramfs.sh" --out "$OUT" "${PASS[@]}"
  S="$OUT/iso-data"
  run rm -rf "$S"
  run mkdir -p "$S/boot"
  for f in vmlinuz initramfs.img; do if [ -f "$OUT/$f" ]; then run cp "$OUT/$f" "$S/boot/$f"; fi; done
  for f in rootfs.squashfs rootfs.ext4 aios-overlay.ext4; do if [ -f "$OUT/$f" ]; then run cp "$OUT/$f" "$S/$f"; fi; done
  run env PYTHONPATH="$ROOT" "${PYTHON:-python3}" -m aios_amd.utils.iso9660 --root "$S" --out "$ISO" --volid AIOS
  echo "data iso -> $ISO"
  exit 0
fi
[ -f "$OUT/vmlinuz" ] || "$ROOT/scripts/build-kernel.sh" --out "$OUT" "${PASS[@]}"
[ -f "$OUT/rootfs.squashfs" ] || "$ROOT/scripts/build-rootfs.sh" --out "$OUT" "${PASS[@]}"
[ -f "$OUT/initramfs.img" ] || "$ROOT/scripts/build-initramfs.sh" --out "$OUT" "${PASS[@]}"
S="$OUT/iso"
run rm -rf "$S"
run mkdir -p "$S/boot/grub"
run cp "$OUT/vmlinuz" "$S/boot/vmlinuz"
run cp "$OUT/initramfs.img" "$S/boot/initramfs.img"
run cp "$OUT/rootfs.squashfs" "$S/rootfs.squashfs"
run cp "$ROOT/deploy/boot/grub/grub.cfg" "$S/boot/grub/grub.cfg"
run grub-mkrescue -o "$ISO" "$S" -- -volid AIOS
echo "iso -> $ISO"
