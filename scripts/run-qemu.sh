#!/usr/bin/env bash
# Boot the aiOS ISO in QEMU/KVM for a smoke test of the boot path (no GPU in the VM: the boot
# entry selects the CPU runtime backend).  With --check the VM is stopped once aios-init logs
# "boot complete" on the serial console, and the exit code says whether it got there.
#   scripts/run-qemu.sh [--iso build/aios-mi355x.iso] [--mem 16G] [--cpus 8] [--check] [--timeout 300]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
ISO="$ROOT/build/aios-mi355x.iso"; MEM=16G; CPUS=8; CHECK=0; TIMEOUT=300
while [ $# -gt 0 ]; do
  case "$1" in
    --iso) ISO="$2"; shift ;; --mem) MEM="$2"; shift ;; --cpus) CPUS="$2"; shift ;;
    --check) CHECK=1 ;; --timeout) TIMEOUT="$2"; shift ;; *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
[ -f "$ISO" ] || { echo "no ISO at $ISO (scripts/build-iso.sh)" >&2; exit 1; }
ACCEL=(-accel tcg); [ -w /dev/kvm ] && ACCEL=(-accel kvm -cpu host)
ARGS=("${ACCEL[@]}" -m "$MEM" -smp "$CPUS" -cdrom "$ISO" -boot d -nographic -serial mon:stdio
      -nic user,model=virtio-net-pci,hostfwd=tcp::19090-:9090,hostfwd=tcp::50051-:50051)
if [ "$CHECK" = 0 ]; then exec qemu-system-x86_64 "${ARGS[@]}"; fi
LOG="$(mktemp)"
qemu-system-x86_64 "${ARGS[@]}" > "$LOG" 2>&1 &
QPID=$!
for _ in $(seq 1 "$TIMEOUT"); do
  if grep -q "boot complete" "$LOG"; then kill "$QPID"; echo "boot OK"; exit 0; fi
  kill -0 "$QPID" 2>/dev/null || break
  sleep 1
done
kill "$QPID" 2>/dev/null || true
tail -n 40 "$LOG"; echo "boot did not complete" >&2; exit 1
