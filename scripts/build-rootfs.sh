#!/usr/bin/env bash
# Assemble the aiOS root filesystem (squashfs): a minimal Ubuntu 22.04 userland (debootstrap),
# the ROCm *runtime* (HIP runtime, HSA, rocm-smi, RCCL -- no compilers), Python with the
# aios_amd package and its prebuilt gfx950 extensions, aios-init as /usr/sbin/aios-init, the
# node config, agent TOMLs, security policy, AppArmor profile and systemd-free boot.
#   scripts/build-rootfs.sh [--out build/distro] [--rocm /opt/rocm] [--suite jammy] [--dry-run] [--overlay-only]
#                           [--base DIR]
# --overlay-only: only the aiOS layer (framework + built extensions, aios-init, configs, environment), no
# debootstrap / chroot / root needed: staged under OUT/overlay and packed as an ext4 image (mkfs.ext4 -d,
# label AIOS-OVL) to lay over any Ubuntu 22.04 + ROCm userland.
# --base DIR: an existing userland tree (e.g. an exported Ubuntu 22.04 + ROCm-runtime container rootfs)
# with the aiOS layer laid over it, packed as OUT/rootfs.ext4 (label AIOS-ROOT) -- the root image the
# early init mounts when the medium has no squashfs; no debootstrap, chroot or root (files keep the
# owners they have in DIR).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/distro"; ROCM="${ROCM_PATH:-/opt/rocm}"; SUITE="jammy"; DRY=0; OVL=0; BASE=""
MIRROR="${AIOS_APT_MIRROR:-http://archive.ubuntu.com/ubuntu}"
while [ $# -gt 0 ]; do
  case "$1" in
    --out) OUT="$2"; shift ;; --rocm) ROCM="$2"; shift ;; --suite) SUITE="$2"; shift ;;
    --dry-run) DRY=1 ;; --overlay-only) OVL=1 ;; --base) BASE="$2"; OVL=1; shift ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
RFS="$OUT/rootfs"
run() { echo "+ $*"; [ "$DRY" = 1 ] || "$@"; }
cat_env() {
  cat <<ENV
PYTHONPATH=/usr/lib/aios
AIOS_PYTHON=/usr/lib/aios/venv/bin/python3
AIOS_CONFIG=/etc/aios/config.toml
LD_LIBRARY_PATH=/opt/rocm/lib
HSA_ENABLE_IPC_MODE_LEGACY=0
ENV
}
if [ "$OVL" = 1 ]; then
  O="$OUT/overlay"
  run rm -rf "$O"
  run mkdir -p "$O/usr/lib/aios" "$O/usr/sbin" "$O/etc/aios" "$O/etc/apparmor.d" "$O/var/lib/aios/models" "$O/var/log/aios"
  # the package without build caches (bytecode, object files)
  run tar -C "$ROOT" --exclude='__pycache__' --exclude='*.pyc' --exclude='build' -cf "$OUT/aios_amd.tar" aios_amd
  run tar -C "$O/usr/lib/aios" -xf "$OUT/aios_amd.tar"
  run rm -f "$OUT/aios_amd.tar"
  [ -e "$ROOT/aios_amd/bin/aios-init" ] && run cp "$ROOT/aios_amd/bin/aios-init" "$O/usr/sbin/aios-init"
  run cp "$ROOT/config/default-config.toml" "$O/etc/aios/config.toml"
  run cp -a "$ROOT/deploy/etc/aios/." "$O/etc/aios/"
  run cp -a "$ROOT/deploy/etc/apparmor.d/." "$O/etc/apparmor.d/"
  if [ "$DRY" = 1 ]; then echo "+ write $O/etc/aios/environment"; else cat_env > "$O/etc/aios/environment"; fi
  if [ -n "$BASE" ]; then
    [ "$DRY" = 1 ] || [ -d "$BASE" ] || { echo "--base: $BASE is not a directory" >&2; exit 1; }
    S="$OUT/rootfs-stage"
    run rm -rf "$S"
    run mkdir -p "$S"
    run cp -a "$BASE/." "$S/"
    run cp -a "$O/." "$S/"
    SZ=$(( $(du -sm "$S" 2>/dev/null | cut -f1 || echo 64) * 5 / 4 + 64 ))
    run rm -f "$OUT/rootfs.ext4"
    run mkfs.ext4 -q -F -L AIOS-ROOT -d "$S" "$OUT/rootfs.ext4" "${SZ}M"
    run rm -rf "$S"
    echo "rootfs -> $OUT/rootfs.ext4"
    exit 0
  fi
  SZ=$(( $(du -sm "$O" 2>/dev/null | cut -f1 || echo 64) * 5 / 4 + 32 ))
  run rm -f "$OUT/aios-overlay.ext4"
  run mkfs.ext4 -q -F -L AIOS-OVL -d "$O" "$OUT/aios-overlay.ext4" "${SZ}M"
  echo "overlay -> $OUT/aios-overlay.ext4"
  exit 0
fi
[ "$DRY" = 1 ] || [ "$(id -u)" = 0 ] || { echo "build-rootfs needs root (debootstrap, chroot)" >&2; exit 1; }

run mkdir -p "$RFS"
run debootstrap --variant=minbase --include=python3,python3-venv,ca-certificates,iproute2,nftables,apparmor,kmod,udev,util-linux,procps,openssl,sqlite3 "$SUITE" "$RFS" "$MIRROR"

# ROCm runtime: only the shared libraries the engine, torch and RCCL load, plus rocm-smi
for d in lib lib64 share/amd_smi bin/rocm-smi bin/amd-smi; do
  [ -e "$ROCM/$d" ] && run mkdir -p "$RFS/opt/rocm/$(dirname "$d")" && run cp -a "$ROCM/$d" "$RFS/opt/rocm/$d"
done
run rm -rf "$RFS/opt/rocm/lib/llvm" "$RFS/opt/rocm/lib/cmake"  # compilers / cmake files stay on the build host

# the framework: package, built extensions (.so), aios-init, configs
run mkdir -p "$RFS/usr/lib/aios" "$RFS/usr/sbin" "$RFS/etc/aios" "$RFS/var/lib/aios/models" "$RFS/var/log/aios"
run cp -a "$ROOT/aios_amd" "$RFS/usr/lib/aios/"
run cp "$ROOT/aios_amd/bin/aios-init" "$RFS/usr/sbin/aios-init"
run cp "$ROOT/config/default-config.toml" "$RFS/etc/aios/config.toml"
run cp -a "$ROOT/deploy/etc/aios/." "$RFS/etc/aios/"
run cp -a "$ROOT/deploy/etc/apparmor.d/." "$RFS/etc/apparmor.d/"
run chroot "$RFS" python3 -m venv /usr/lib/aios/venv
run chroot "$RFS" /usr/lib/aios/venv/bin/pip install --no-index --find-links /usr/lib/aios/wheels \
    grpcio protobuf aiohttp numpy torch
if [ "$DRY" = 1 ]; then echo "+ write $RFS/etc/aios/environment"; cat_env; else cat_env > "$RFS/etc/aios/environment"; fi
run mksquashfs "$RFS" "$OUT/rootfs.squashfs" -comp zstd -Xcompression-level 15 -noappend
echo "rootfs -> $OUT/rootfs.squashfs"
