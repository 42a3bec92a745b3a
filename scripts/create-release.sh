#!/usr/bin/env bash
# Package a release: built package (gfx950 engine, core, aios-init), config, deploy assets,
# scripts, checksums and notes -> dist/aios-mi355x-<version>.tar.gz
set -euo pipefail
cd "$(dirname "$0")/.."
VER=${1:-$(git describe --tags --always 2>/dev/null || echo dev)}
OUT=dist/aios-mi355x-$VER; rm -rf "$OUT"; mkdir -p "$OUT"
cp -a aios_amd config deploy scripts tools README.md "$OUT/"
find "$OUT" -name __pycache__ -prune -exec rm -rf {} +
( cd dist && tar czf "aios-mi355x-$VER.tar.gz" "aios-mi355x-$VER" && sha256sum "aios-mi355x-$VER.tar.gz" > SHA256SUMS )
git log --oneline -20 > "dist/RELEASE_NOTES-$VER.txt" 2>/dev/null || true
echo "dist/aios-mi355x-$VER.tar.gz"
