"""Print the *_us columns of tools/gemv_cu_probe.py JSON lines: python tools/probe_summary.py FILE"""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("{"):
        r = json.loads(line)
        print(r["shape"], {k: v for k, v in r.items() if k.endswith("_us")})
