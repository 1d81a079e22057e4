#!/usr/bin/env python3
"""Table of the kernel-resource-usage remarks hipcc prints (-Rpass-analysis=kernel-resource-usage) on stderr:
   tools/ru_table.py <remarks.txt> [name-substring]   ->  kernel  VGPRs  spills  scratch  waves/SIMD"""
import re
import subprocess
import sys


def parse(path):
    d, cur = {}, None
    for ln in open(path, errors="replace"):
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = m.group(1)
            d[cur] = {}
            continue
        m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|"
                      r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", ln)
        if m and cur:
            d[cur][m.group(1)] = int(m.group(2))
    return d


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
        return dict(zip(names, out))
    except OSError:
        return {n: n for n in names}


if __name__ == "__main__":
    d = parse(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    names = [k for k in d if sub in k]
    dm = demangle(names)
    for k in names:
        e = d[k]
        m = re.search(r"(k_\w+)<([^>]*)>", dm[k])
        nm = "%s<%s>" % (m.group(1), m.group(2).replace(" ", "")) if m else dm[k]
        print("%-48s VGPR %3d  spillV %3d  spillS %3d  scratch %4d  waves %d" % (
            nm[:48], e.get("VGPRs", -1), e.get("VGPRs Spill", -1), e.get("SGPRs Spill", -1),
            e.get("ScratchSize [bytes/lane]", -1), e.get("Occupancy [waves/SIMD]", -1)))
