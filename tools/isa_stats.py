#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing: python tools/isa_stats.py FILE.s NAME_SUBSTRING"""
import sys
from collections import Counter

src, want = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and ":" in l and want in l.split(":")[0])
body = []
for l in lines[start + 1:]:
    if l.startswith(".Lfunc_end"):
        break
    t = l.strip()
    if t and not t.startswith((".", ";", "//")) and not t.endswith(":"):
        body.append(t.split()[0])
c = Counter(body)
print(want, "instructions:", len(body))
print("VALU", sum(v for k, v in c.items() if k.startswith("v_")), "SALU", sum(v for k, v in c.items() if k.startswith("s_")),
      "DS", sum(v for k, v in c.items() if k.startswith("ds_")), "VMEM", sum(v for k, v in c.items() if k.startswith(("global_", "buffer_"))))
print(sorted(c.items(), key=lambda x: -x[1])[:45])
