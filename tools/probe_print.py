"""Pretty-print tools/gemv_cu_probe.py JSON lines (stdin): per-kernel times and stamp percentiles."""
import json
import sys

for line in sys.stdin:
    try:
        d = json.loads(line)
    except Exception:
        print(line.rstrip())
        continue
    print(d.get("shape"), {k: v for k, v in d.items() if k.endswith("_us") and k != "stamps_us"})
    for k, v in d.get("stamps_us", {}).items():
        print("   ", k, v)
