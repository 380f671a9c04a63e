#!/usr/bin/env python3
"""One-line summary of a tools/tune.py log: variant -> median us (compact)."""
import json
import sys

out = []
for line in open(sys.argv[1]):
    try:
        r = json.loads(line)
    except ValueError:
        continue
    if "us_median" not in r or r["variant"].startswith("torch"):
        continue
    kind, opts = json.loads(r["variant"])
    tag = kind[0] + "".join(f"{k[0]}{v}" for k, v in opts.items()) if opts else kind + "-default"
    out.append(f"{tag}={r['us_median']}")
print(" ".join(out))
