#!/usr/bin/env bash
# Build the aiOS MI355X kernel: a stock Linux tree + distro/kernel/aios-mi355x.config merged on the
# x86_64 defconfig (amdgpu/KFD/HMM/P2P/IOMMU-pt, AppArmor, squashfs+overlay root).
#   scripts/build-kernel.sh [--src DIR | --version 6.12.9] [--out build/distro] [--jobs N] [--dry-run]
# Without --src the release tarball is fetched from kernel.org (needs network).  Outputs
# <out>/vmlinuz, <out>/modules/ (modules_install), <out>/kernel.config.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
VERSION="6.12.9"; SRC=""; OUT="$ROOT/build/distro"; JOBS="$(nproc)"; DRY=0
while [ $# -gt 0 ]; do
  case "$1" in
    --src) SRC="$2"; shift ;; --version) VERSION="$2"; shift ;; --out) OUT="$2"; shift ;;
    --jobs) JOBS="$2"; shift ;; --dry-run) DRY=1 ;; *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
FRAG="$ROOT/distro/kernel/aios-mi355x.config"
run() { echo "+ $*"; [ "$DRY" = 1 ] || "$@"; }
[ -f "$FRAG" ] || { echo "missing $FRAG" >&2; exit 1; }
if [ -z "$SRC" ]; then
  SRC="$ROOT/build/kernel/linux-$VERSION"
  if [ ! -d "$SRC" ]; then
    run mkdir -p "$ROOT/build/kernel"
    run curl -fL -o "$ROOT/build/kernel/linux-$VERSION.tar.xz" \
      "https://cdn.kernel.org/pub/linux/kernel/v${VERSION%%.*}.x/linux-$VERSION.tar.xz"
    run tar -C "$ROOT/build/kernel" -xf "$ROOT/build/kernel/linux-$VERSION.tar.xz"
  fi
fi
run mkdir -p "$OUT/modules"
run make -C "$SRC" ARCH=x86_64 defconfig
run "$SRC/scripts/kconfig/merge_config.sh" -m -O "$SRC" "$SRC/.config" "$FRAG"
run make -C "$SRC" ARCH=x86_64 olddefconfig
# every fragment option must have survived the merge (a missing dependency silently drops one)
if [ "$DRY" = 0 ]; then
  miss=0
  while IFS= read -r line; do
    case "$line" in CONFIG_*=y|CONFIG_*=m)
      grep -qx "$line" "$SRC/.config" || { echo "kernel option not applied: $line" >&2; miss=1; } ;;
    esac
  done < "$FRAG"
  [ "$miss" = 0 ] || exit 1
fi
run make -C "$SRC" ARCH=x86_64 -j"$JOBS" bzImage modules
run make -C "$SRC" ARCH=x86_64 INSTALL_MOD_PATH="$OUT/modules" modules_install
run cp "$SRC/arch/x86/boot/bzImage" "$OUT/vmlinuz"
run cp "$SRC/.config" "$OUT/kernel.config"
echo "kernel -> $OUT/vmlinuz"
