#!/usr/bin/env python3
"""One line per bench.py JSON: value, ms/iter and the x-tile / column-pass classes.
usage: python tools/ab_summary.py FILE.json ..."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    k = d.get("kernel_ms") or {}
    g = lambda c: k.get(c, {}).get("avg_ms", float("nan"))
    pw = (d.get("pointwise") or {}).get("frac", float("nan"))
    print(f"{f}: {d['value']:.1f} Mvox/s  {d['ms_per_step']:.3f} ms/iter  quotient {g('x_quotient'):.4f}  "
          f"update {g('x_update'):.4f}  y {g('y_pass'):.4f}  z {g('z_convolve'):.4f}  pointwise {pw:.3f}")
