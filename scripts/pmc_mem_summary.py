#!/usr/bin/env python3
"""Per-kernel averages of the counters collected by scripts/pmc_mem.sh.
usage: scripts/pmc_mem_summary.py gpurun_out/pmc_mem [out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"dxrpt::(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else None


def main(d, out=None):
    acc = defaultdict(lambda: defaultdict(list))
    for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        with open(p) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                if k:
                    acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    for k, cs in sorted(res.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:40s} {v:16.1f}")
        if cs.get("SQ_INSTS_VMEM_RD"):
            print(f"   {'avg VMEM latency (quad-cycles)':40s} {cs.get('SQ_INST_LEVEL_VMEM', 0) / cs['SQ_INSTS_VMEM_RD']:16.1f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=2)


if __name__ == "__main__":
    main(*sys.argv[1:])
