#!/bin/bash
# rocprofv3 kernel trace of the split schedule on a few configs: per-kernel (head / tail per depth) durations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/kt_split
mkdir -p $OUT
for c in ${CONFIGS:-metric c3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$c -o run -- python3 scripts/time_frames.py --config $c \
      --rounds 1 --frames 8 --opt MEGAKERNEL_SPLIT=${MSPLIT:-1} --opt FRAME_OVERLAP=${OVERLAP:-0} > $OUT/$c.txt 2>&1 || exit $?
  python3 - "$OUT/$c" "$c" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "k_path" not in n:
        continue
    key = n.split("(")[0][:60]
    # the tail's depth is an argument: distinguish launches by order within a frame instead
    by[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for k, v in by.items():
    d = [(e - s) / 1e6 for s, e in v]
    print(f"{sys.argv[2]:7s} {k:60s} n={len(d):4d} mean {sum(d)/len(d):.4f} ms")
# per-launch sequence of the last frame
allk = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows if "k_path" in r["Kernel_Name"])
heads = [i for i, x in enumerate(allk) if "head" in x[2]]
if heads:
    last = allk[heads[-2]:heads[-1]]
    t0 = last[0][0]
    for s, e, n in last:
        print(f"   {n[:40]:40s} start {(s - t0) / 1e6:.4f} dur {(e - s) / 1e6:.4f} ms")
PY
done
