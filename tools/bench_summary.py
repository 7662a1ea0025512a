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
        sp = d["service"].get("store_images_pass")
        if sp:
            parts.append(f"store-images {sp.get('value', 0):.0f} (x{sp.get('vs_synthetic_service')}, "
                         f"decode {sp.get('store_path', {}).get('decode_rate_img_s')}/s)" if "value" in sp
                         else f"store-images error {sp.get('error', '')[:120]}")
    print(f"{path}: " + "  ".join(parts))
