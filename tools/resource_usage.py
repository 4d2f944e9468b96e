#!/usr/bin/env python3
"""Per-kernel register / spill summary of a hipcc -Rpass-analysis=kernel-resource-usage log.

usage: python tools/resource_usage.py LOG [name-substring ...]
"""
import re
import sys


def parse(path):
    info, cur = {}, None
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            info[cur] = {}
            continue
        m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            info[cur][m.group(1).split(" [")[0].replace(" ", "_")] = int(m.group(2))
    return info


if __name__ == "__main__":
    info = parse(sys.argv[1])
    pats = sys.argv[2:]
    for f, d in info.items():
        if all(p in f for p in pats):
            print(f"{f[:90]:90s} " + " ".join(f"{k}={v}" for k, v in d.items()))
