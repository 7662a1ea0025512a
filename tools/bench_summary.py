#!/usr/bin/env python3
"""One line per bench.py JSON log: headline and sub-record images/s (A/B scripts)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        line = [ln for ln in open(path) if ln.startswith("{")][-1]
        d = json.loads(line)
    except (OSError, IndexError, ValueError) as e:
        print(f"{path}: no record ({e})")
        continue
    parts = [f"{d['config']['model']} {d['value']:.0f}"]
    for m, r in (d.get("models") or {}).items():
        parts.append(f"{m} {r['value']:.0f}")
    if d.get("service"):
        parts.append(f"service {d['service'].get('value', 0):.0f}")
    print(f"{path}: " + "  ".join(parts))
