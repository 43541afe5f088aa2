#!/usr/bin/env python
"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` remarks (stderr of a --cuda-device-only
compile) per kernel: VGPRs, SGPRs, scratch bytes per lane, occupancy, spills, LDS.
usage: scripts/kres_usage.py <remarks.txt> [substring ...]"""
import re
import subprocess
import sys


def main():
    txt = open(sys.argv[1]).read()
    keys = sys.argv[2:]
    fields = {"v": "VGPRs", "s": "SGPRs", "scratch": r"ScratchSize \[bytes/lane\]", "occ": r"Occupancy \[waves/SIMD\]",
              "sspill": "SGPRs Spill", "vspill": "VGPRs Spill", "lds": r"LDS Size \[bytes/block\]"}
    for b in re.split(r"remark: .*?Function Name: ", txt)[1:]:
        name = b.split("\n")[0].strip()
        if keys and not any(k in name for k in keys):
            continue
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        vals = []
        for k, pat in fields.items():
            m = re.search(pat + r": (\d+)", b)
            vals.append(f"{k}{m.group(1) if m else '?'}")
        print(f"{dn.split('(')[0][:60]:60s} " + " ".join(vals))


if __name__ == "__main__":
    main()
