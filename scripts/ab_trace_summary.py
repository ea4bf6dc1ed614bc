#!/usr/bin/env python3
"""Per-depth median dispatch durations from scripts/ab_trace.sh output.

Frames launch raygen, then per depth d = 1..L-1: trace, shade, shadow, resolve, then accumulate;
the d-th traversal dispatch of each kind inside a frame is depth d.
    python scripts/ab_trace_summary.py gpurun_out/abtrace
"""
import csv
import glob
import os
import re
import statistics
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abtrace"
for d in sorted(glob.glob(os.path.join(root, "*"))):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        continue
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    per = defaultdict(list)
    depth = defaultdict(int)
    for s, e, n in rows:
        m = re.search(r"dxrpt::(k_\w+)", n)
        if not m:
            continue
        k = m.group(1)
        if k == "k_raygen":
            depth.clear()
            continue
        if k in ("k_accumulate",):
            continue
        kind = {"k_traverse8p": None}.get(k, k)
        if k == "k_traverse8p":
            kind = "k_shadow" if "true>" in n.split(",")[-1] or re.search(r"k_traverse8p<\w+, true>", n) else "k_trace"
        depth[kind] += 1
        per[(kind, depth[kind])].append((e - s) / 1e6)
    print(os.path.basename(d))
    for (kind, dep), v in sorted(per.items()):
        print(f"  {kind:10s} d{dep}: median {statistics.median(v):.3f} ms  (n={len(v)})")
