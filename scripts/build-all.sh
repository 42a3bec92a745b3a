#!/usr/bin/env bash
# Build everything for an MI355X node: gfx950 HIP engine, C++ control-plane core, aios-init;
# run the CPU test suite; optionally package a release tarball.
#   scripts/build-all.sh [--skip-tests] [--package] [--arch gfx950]
set -euo pipefail
cd "$(dirname "$0")/.."
SKIP_TESTS=0; PACKAGE=0
while [ $# -gt 0 ]; do
  case "$1" in
    --skip-tests) SKIP_TESTS=1 ;;
    --package) PACKAGE=1 ;;
    --arch) export AIOS_OFFLOAD_ARCH="$2"; shift ;;
    *) echo "unknown flag $1"; exit 2 ;;
  esac
  shift
done
echo "[1/4] native engine (HIP, ${AIOS_OFFLOAD_ARCH:-gfx950})"
python3 -c "from aios_amd import _build; _build.build()"
echo "[2/4] control-plane core + aios-init (C++17)"
python3 -c "from aios_amd import _build; _build.build_core(); _build.build_initd()"
echo "[3/4] proto files for external tooling"
scripts/gen-proto.sh build/proto >/dev/null
if [ "$SKIP_TESTS" = 0 ]; then
  echo "[4/4] CPU tests"
  python3 -m pytest tests -q -m "not gpu"
fi
if [ "$PACKAGE" = 1 ]; then
  scripts/create-release.sh
fi
