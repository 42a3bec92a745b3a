#!/usr/bin/env bash
# Render the gRPC contract (aios_amd/rpc/schema.py) as standard .proto files (grpcurl, other
# languages).  The runtime builds its descriptors from the same spec, so nothing is generated
# into the package (replaces the reference's grpc_tools.protoc step).
set -euo pipefail
cd "$(dirname "$0")/.."
python3 -m aios_amd.rpc.schema "${1:-build/proto}"
