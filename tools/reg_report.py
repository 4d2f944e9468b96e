#!/usr/bin/env python3
"""Register / spill / occupancy per kernel from a hipcc -Rpass-analysis=kernel-resource-usage log.
usage: python tools/reg_report.py BUILD.log [NAME_SUBSTRING]"""
import re
import sys

want = sys.argv[2] if len(sys.argv) > 2 else ""
cur, out = None, {}
for l in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        out[cur] = {}
        continue
    for key, pat in (("vgpr", r"remark:\s+VGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, l)
        if m and cur:
            out[cur][key] = int(m.group(1))
for f, d in out.items():
    if want in f:
        print(f[:110], d)
