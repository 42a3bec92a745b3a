#!/usr/bin/env bash
# Bootable hybrid ISO (BIOS + UEFI, GRUB): kernel + initramfs + rootfs.squashfs, label AIOS.
#   scripts/build-iso.sh [--out build/distro] [--iso build/aios-mi355x.iso] [--dry-run]
# Runs the kernel / rootfs / initramfs builds first when their outputs are missing.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/distro"; ISO="$ROOT/build/aios-mi355x.iso"; DRY=0; PASS=()
while [ $# -gt 0 ]; do
  case "$1" in
    --out) OUT="$2"; shift ;; --iso) ISO="$2"; shift ;; --dry-run) DRY=1; PASS+=(--dry-run) ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
run() { echo "+ $*"; [ "$DRY" = 1 ] || "$@"; }
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
