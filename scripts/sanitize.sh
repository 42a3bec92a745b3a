#!/usr/bin/env bash
# Host-code sanitizers (SURVEY.md §5 "race detection / sanitizers"): build the control-plane core
# and aios-init with ASan + UBSan and run the native-core, security and control-plane test suites
# against the instrumented build.  GPU code is not instrumented (GPU ASan is not available here).
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "from aios_amd import _build; _build.build_core(verbose=True, sanitize='address,undefined')"
SO=$(python -c "from aios_amd import _build; print(_build.core_sanitized_path('address,undefined'))")
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -Iaios_amd/native \
    -o build/aios-init-asan aios_amd/native/initd/initd.cpp aios_amd/native/json.cpp -lpthread
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:strict_string_checks=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export AIOS_CORE_SO="$SO" AIOS_INIT_BIN="$PWD/build/aios-init-asan"
python -m pytest -q -p no:cacheprovider tests/test_native_core.py tests/test_security.py tests/test_initd.py \
    tests/test_control_plane.py tests/test_agents.py tests/test_runtime.py "$@"
echo "sanitizers: clean"
