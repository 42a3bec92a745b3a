#!/usr/bin/env bash
# Assemble the aiOS root filesystem (squashfs): a minimal Ubuntu 22.04 userland (debootstrap),
# the ROCm *runtime* (HIP runtime, HSA, rocm-smi, RCCL -- no compilers), Python with the
# aios_amd package and its prebuilt gfx950 extensions, aios-init as /usr/sbin/aios-init, the
# node config, agent TOMLs, security policy, AppArmor profile and systemd-free boot.
#   scripts/build-rootfs.sh [--out build/distro] [--rocm /opt/rocm] [--suite jammy] [--dry-run]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/distro"; ROCM="${ROCM_PATH:-/opt/rocm}"; SUITE="jammy"; DRY=0
MIRROR="${AIOS_APT_MIRROR:-http://archive.ubuntu.com/ubuntu}"
while [ $# -gt 0 ]; do
  case "$1" in
    --out) OUT="$2"; shift ;; --rocm) ROCM="$2"; shift ;; --suite) SUITE="$2"; shift ;;
    --dry-run) DRY=1 ;; *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
RFS="$OUT/rootfs"
run() { echo "+ $*"; [ "$DRY" = 1 ] || "$@"; }
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
cat_env() {
  cat <<ENV
PYTHONPATH=/usr/lib/aios
AIOS_PYTHON=/usr/lib/aios/venv/bin/python3
AIOS_CONFIG=/etc/aios/config.toml
LD_LIBRARY_PATH=/opt/rocm/lib
HSA_ENABLE_IPC_MODE_LEGACY=0
ENV
}
if [ "$DRY" = 1 ]; then echo "+ write $RFS/etc/aios/environment"; cat_env; else cat_env > "$RFS/etc/aios/environment"; fi
run mksquashfs "$RFS" "$OUT/rootfs.squashfs" -comp zstd -Xcompression-level 15 -noappend
echo "rootfs -> $OUT/rootfs.squashfs"
