#!/usr/bin/env bash
# Host-code sanitizers (SURVEY.md §5 "race detection / sanitizers").  GPU code is not instrumented
# (GPU ASan / XNACK runs are not available on this pool).
#   scripts/sanitize.sh            ASan + UBSan build of the control-plane core and aios-init; the
#                                  native-core, security, control-plane, agent and runtime suites
#   scripts/sanitize.sh --thread   ThreadSanitizer build of the core; the concurrency suite (8
#                                  threads hammering shared stores with the GIL released) and the
#                                  in-process native-core tests
set -euo pipefail
cd "$(dirname "$0")/.."
if [ "${1:-}" = "--thread" ]; then
  shift
  python -c "from aios_amd import _build; _build.build_core(verbose=True, sanitize='thread')"
  SO=$(python -c "from aios_amd import _build; print(_build.core_sanitized_path('thread'))")
  export LD_PRELOAD="$(gcc -print-file-name=libtsan.so)"
  # python itself is not instrumented: only races inside the core's own accesses are reported
  export TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0:second_deadlock_stack=1"
  export AIOS_CORE_SO="$SO"
  # (the tests that spawn child processes are left out: a child inheriting the TSan preload after a
  # multi-threaded fork can deadlock inside the runtime, which is a harness artefact, not a race)
  python -m pytest -q -p no:cacheprovider tests/test_native_concurrency.py tests/test_native_core.py \
      -k "not plugin and not sandbox and not run_cmd and not monitor" "$@"
  echo "thread sanitizer: clean"
  exit 0
fi
python -c "from aios_amd import _build; _build.build_core(verbose=True, sanitize='address,undefined')"
SO=$(python -c "from aios_amd import _build; print(_build.core_sanitized_path('address,undefined'))")
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -Iaios_amd/native \
    -o build/aios-init-asan aios_amd/native/initd/initd.cpp aios_amd/native/json.cpp -lpthread
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:strict_string_checks=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export AIOS_CORE_SO="$SO" AIOS_INIT_BIN="$PWD/build/aios-init-asan"
python -m pytest -q -p no:cacheprovider tests/test_native_core.py tests/test_security.py tests/test_initd.py \
    tests/test_control_plane.py tests/test_agents.py tests/test_runtime.py tests/test_native_concurrency.py "$@"
echo "sanitizers: clean"
