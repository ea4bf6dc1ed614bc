#!/usr/bin/env python3
"""Per-kernel average of each counter in a rocprofv3 --pmc output directory (scripts/pmc_ab.sh)."""
import csv
import glob
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from scripts.pmc_summary import short  # noqa: E402

acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k and k.startswith("k_path"):
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    print(sys.argv[2], k, " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(d.items())))
