#!/usr/bin/env python3
"""Summarise the rocprofv3 outputs of scripts/profile.sh (kernel trace + stats of bench.py, then one
rocprofv3 --pmc pass per counter group over the same command) into profiles/<round>_*.

bench.py runs, in one process: a census frame (the counting instantiations of the timed schedule --
k_path_head<5, true> + k_path_tail<7, true>, or k_path<occ, true> -- on the caller's stream), a
frame-at-a-time pass (DXRPT_OPT_FRAME_OVERLAP 0: every kernel on the caller's stream, one launch at a
time -- the per-launch durations of the bench line's roofline), then the timed overlapped frames (the
kernels on two internal slot streams).  Per kernel kind (k_path_head / k_path_tail / k_path) this writes:
  - avg_ms: the kernel trace's average duration of the launches on the caller's stream (the queue of
    the census kernel), i.e. the frame-at-a-time launches, which bench.py's roofline times with HIP events;
    avg_ms_all: over every launch (overlapped launches share the GPU with the neighbour frame);
  - per-launch counters of those launches;
  - profiles/<round>_kernel_stats[_<config>].csv: rocprofv3's statistics columns over those caller-stream
    launches only (the non-overlapped per-launch durations), <round>_kernel_stats_all[_<config>].csv:
    rocprofv3's own statistics over every launch, <round>_kernel_trace[_<config>].csv: the raw trace.  l2_fabric_bytes_per_launch = FETCH_SIZE + WRITE_SIZE (KiB x 1024,
    RAW: no x2 read correction -- MI355X_MICROARCH.md calibrates that on 16-B/lane streaming reads only, and
    these are scattered gathers): L2 -> fabric traffic, Infinity-Cache hits included, so not HBM bytes.
usage: PMC_CONFIG_TAG=<config> PMC_CONFIG="<scene>-proxy WxH L=n" scripts/pmc_summary.py gpurun_out/prof_<config> <round>
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

CONFIG = os.environ.get("PMC_CONFIG", "sponza-proxy 1920x1080 L=3")
TAG = os.environ.get("PMC_CONFIG_TAG", "metric")


def short(name):
    """'void dxrpt::k_path_tail<7>(dxrpt::KArgs, int)' -> 'k_path_tail<7>'"""
    m = re.search(r"dxrpt::(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else None


PATH_KINDS = ("k_path", "k_path_head", "k_path_tail")


def is_census(k):
    """The counting instantiations k_path<occ, true, ...>, k_path_head<occ, true>, k_path_tail<occ, true>."""
    if k is None or "<" not in k or k.split("<")[0] not in PATH_KINDS:
        return False
    return k[k.index("<") + 1:-1].split(", ")[1:2] == ["true"]


def kind(k):
    """Kernel kind of a short name; None for a census instantiation."""
    if k is None or is_census(k):
        return None
    return k.split("<")[0]


def census_queue(rows, qcol):
    """The caller's stream: the queue the (non-overlapped) census frame ran on."""
    for r in rows:
        if is_census(short(r["Kernel_Name"])):
            return r[qcol]
    return None


def write_stats(rows, q0, path):
    """rocprofv3's kernel-stats columns over the launches on queue q0 (the caller's stream)."""
    import statistics
    per = defaultdict(list)
    for r in rows:
        if r["Queue_Id"] == q0:
            per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in per.values()) or 1
    with open(path, "w") as g:
        g.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev","Launches"\n')
        for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            sd = statistics.pstdev(v) if len(v) > 1 else 0.0
            g.write(f'"{name}",{len(v)},{sum(v)},{sum(v) / len(v):.6f},{100.0 * sum(v) / total:.4g},{min(v)},{max(v)},{sd:.6f},'
                    f'"caller stream"\n')


def main(prof, rnd):
    os.makedirs("profiles", exist_ok=True)
    sfx = "" if TAG == "metric" else "_" + TAG
    # kernel trace: per-kind durations, caller-stream launches vs all
    rows = list(csv.DictReader(open(os.path.join(prof, "kt", "run_kernel_trace.csv"))))
    q0 = census_queue(rows, "Queue_Id")
    dur = defaultdict(lambda: {"caller": [], "all": [], "names": set(), "vgpr": None, "scratch": None})
    for r in rows:
        k = short(r["Kernel_Name"])
        kd = kind(k)
        if kd not in ("k_path", "k_path_head", "k_path_tail"):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        e = dur[kd]
        e["all"].append(d)
        e["names"].add(k)
        e["vgpr"], e["scratch"] = int(r["VGPR_Count"]), int(r["Scratch_Size"])
        if r["Queue_Id"] == q0:
            e["caller"].append(d)
    # PMC passes: per-launch averages of the caller-queue launches of each kind
    pmc = defaultdict(lambda: defaultdict(list))
    pmc_all = defaultdict(lambda: defaultdict(list))
    for dname in sorted(os.listdir(prof)):
        p = os.path.join(prof, dname, "run_counter_collection.csv")
        if not (dname.startswith("pmc_") and os.path.exists(p)):
            continue
        prow = list(csv.DictReader(open(p)))
        pq = census_queue(prow, "Queue_Id")
        for r in prow:
            kd = kind(short(r["Kernel_Name"]))
            if kd not in ("k_path", "k_path_head", "k_path_tail"):
                continue
            v = float(r["Counter_Value"])
            pmc_all[kd][r["Counter_Name"]].append(v)
            if r["Queue_Id"] == pq:
                pmc[kd][r["Counter_Name"]].append(v)
    by_kind = {}
    for kd, e in dur.items():
        c = {n: sum(v) / len(v) for n, v in pmc[kd].items() if v}
        s = {"kernels": sorted(e["names"]), "calls": len(e["caller"]), "calls_all": len(e["all"]),
             "avg_ms": sum(e["caller"]) / len(e["caller"]) if e["caller"] else None,
             "avg_ms_all": sum(e["all"]) / len(e["all"]), "vgpr": e["vgpr"], "scratch_bytes_per_lane": e["scratch"],
             "counters_per_launch": c}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            s["l2_fabric_bytes_per_launch"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        if "WRITE_SIZE" in c:
            s["write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in c:
            s["fetch_bytes_per_launch_raw"] = c["FETCH_SIZE"] * 1024
        if c.get("SQ_WAVE_CYCLES"):
            s["wait_any_per_wave_cycle"] = c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
            s["active_inst_any_per_wave_cycle"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_ACTIVE_INST_VALU"):
            s["valu_lane_utilisation"] = c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (c["SQ_ACTIVE_INST_VALU"] * 64.0)
        if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
            s["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        by_kind[kd] = s
    out = {"config": CONFIG, "source": f"rocprofv3 --kernel-trace --stats and --pmc passes of bench.py ({prof})",
           "queue": "caller-stream launches (the bench's frame-at-a-time pass; the census kernel's queue)",
           "traffic": "l2_fabric_bytes = FETCH_SIZE + WRITE_SIZE raw (L2 -> fabric requests; Infinity-Cache hits "
                      "included; no x2 read correction)",
           "kernels_by_kind": by_kind}
    with open(f"profiles/{rnd}_launch_{TAG}.json", "w") as f:
        json.dump(out, f, indent=2)
    # kernel statistics of the frame-at-a-time (caller-stream) launches only -- the per-launch durations
    # the roofline uses; rocprofv3's own statistics over every launch (overlapped ones included) beside
    # them, and the raw trace for recomputation
    write_stats(rows, q0, f"profiles/{rnd}_kernel_stats{sfx}.csv")
    with open(os.path.join(prof, "kt", "run_kernel_stats.csv")) as f, open(f"profiles/{rnd}_kernel_stats_all{sfx}.csv", "w") as g:
        g.write(f.read())
    with open(os.path.join(prof, "kt", "run_kernel_trace.csv")) as f, open(f"profiles/{rnd}_kernel_trace{sfx}.csv", "w") as g:
        g.write(f.read())
    for kd, s in sorted(by_kind.items()):
        print(f"{TAG:7s} {kd:12s} {','.join(s['kernels']):28s} launches {s['calls']:4d} avg {s['avg_ms'] or 0:8.4f} ms "
              f"(all {s['avg_ms_all']:.4f})  fabric {s.get('l2_fabric_bytes_per_launch', 0) / 1e9:6.3f} GB "
              f"writes {s.get('write_bytes_per_launch', 0) / 1e9:6.3f} GB  L2 hit {s.get('l2_hit_rate', 0):.3f} "
              f"wait {s.get('wait_any_per_wave_cycle', 0):.3f} lanes {s.get('valu_lane_utilisation', 0):.3f} "
              f"vgpr {s['vgpr']} scratch {s['scratch_bytes_per_lane']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
