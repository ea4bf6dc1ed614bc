#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of scripts/profile.sh into profiles/<round>_*.

Per kernel: launches, average duration (kernel trace), and per-launch PMC averages.  HBM traffic per
launch follows MI355X_MICROARCH.md section HBM: FETCH_SIZE and WRITE_SIZE come from separate passes,
are in KiB, and on gfx950 FETCH_SIZE reports half the bytes of 16-B/lane reads, so the read side is
doubled (our traversal loads are 16-B/lane dwordx4; the guide marks other shapes uncalibrated, so the
raw value is kept next to the corrected one).
usage: scripts/pmc_summary.py gpurun_out/prof r01
"""
import csv
import json
import os
import sys
from collections import defaultdict

CONFIG = os.environ.get("PMC_CONFIG", "sponza-proxy 1920x1080 L=3")


def short(name):
    """'void dxrpt::k_trace<false, 8, 8>(dxrpt::KArgs, int)' -> 'k_trace<false, 8, 8>'"""
    import re
    m = re.search(r"dxrpt::(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else None


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k:
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def main(prof, rnd):
    stats = {}
    with open(os.path.join(prof, "kt", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            if k:
                stats[k] = {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) / 1e6,
                            "total_ms": float(row["TotalDurationNs"]) / 1e6, "pct": float(row["Percentage"])}
    pmc = {}
    for d in sorted(os.listdir(prof)):
        p = os.path.join(prof, d, "run_counter_collection.csv")
        if d.startswith("pmc_") and os.path.exists(p):
            for k, cs in counters(p).items():
                pmc.setdefault(k, {}).update(cs)
    out = {"config": CONFIG, "source": f"rocprofv3 via scripts/profile.sh ({prof})", "kernels": {}}
    for k in sorted(set(stats) | set(pmc)):
        e = dict(stats.get(k, {}))
        c = pmc.get(k, {})
        e["pmc"] = c
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_read_bytes_raw"] = c["FETCH_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            e["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
        if c.get("SQ_WAVE_CYCLES"):
            e["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
            e["issue_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        out["kernels"][k] = e
    os.makedirs("profiles", exist_ok=True)
    sfx = "" if os.environ.get("PMC_CONFIG_TAG", "metric") == "metric" else "_" + os.environ["PMC_CONFIG_TAG"]
    with open(f"profiles/{rnd}_kernels{sfx}.json", "w") as f:
        json.dump(out, f, indent=2)
    # the timed kinds (DXRPT_K_TRACE / DXRPT_K_SHADOW): the uninstrumented instantiations of the frame
    # (packet and per-lane variants), launch-weighted
    for kind, prefixes in (("k_trace", ("k_trace<false", "k_trace_packet")),
                           ("k_shadow", ("k_shadow<false", "k_shadow_packet")), ("k_path", ("k_path<",))):
        # k_path<occ, persistent, lds, group, kCount = true, order> is the bench's one instrumented census
        # frame, not a timed launch
        cands = [k for k in out["kernels"] if k.startswith(prefixes)
                 and not (kind == "k_path" and k[k.index("<") + 1:-1].split(", ")[4:5] == ["true"])]
        if not cands:
            continue
        calls = sum(out["kernels"][k].get("calls", 0) for k in cands)

        def wavg(key):
            vals = [(out["kernels"][k].get("calls", 0), out["kernels"][k].get(key)) for k in cands]
            if not calls or any(v is None for _, v in vals):
                return None
            return sum(c * v for c, v in vals) / calls

        def wavg_pmc(counter):
            vals = [(out["kernels"][k].get("calls", 0), out["kernels"][k]["pmc"].get(counter)) for k in cands]
            if not calls or any(v is None for _, v in vals):
                return None
            return sum(c * v for c, v in vals) / calls
        with open(f"profiles/{rnd}_pmc_{kind}{sfx}.json", "w") as f:
            json.dump({"config": CONFIG, "kernel": " + ".join(sorted(cands)), "calls": calls,
                       "avg_ms": (sum(out["kernels"][k].get("total_ms", 0.0) for k in cands) / calls) if calls else None,
                       "per_kernel_avg_ms": {k: out["kernels"][k].get("avg_ms") for k in cands},
                       "hbm_bytes_per_launch": wavg("hbm_bytes_per_launch"),
                       "hbm_read_bytes_raw": wavg("hbm_read_bytes_raw"), "l2_hit_rate": wavg("l2_hit_rate"),
                       "hbm_write_bytes_per_launch": wavg("hbm_write_bytes"),
                       "wait_any_per_wave_cycle": wavg("wait_any_frac"),
                       "active_inst_any_per_wave_cycle": wavg("issue_frac"),
                       "counters_per_launch": ({c: wavg_pmc(c) for c in sorted(out["kernels"][cands[0]]["pmc"])}
                                               if cands else {}),
                       "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 16-B/lane read correction) + WRITE_SIZE KiB x1024"},
                      f, indent=2)
    # per FRAME of the megakernel schedule (k_path, or the split schedule's k_path_head + k_path_tail per
    # depth): counters summed over every megakernel launch (the census frame's counting k_path excluded)
    # and divided by the frames (launches of the frame's first kernel)
    fam = [k for k in out["kernels"] if k.startswith(("k_path<", "k_path_head<", "k_path_tail<"))
           and not (k.startswith("k_path<") and k[k.index("<") + 1:-1].split(", ")[4:5] == ["true"])]
    firsts = [k for k in fam if k.startswith(("k_path<", "k_path_head<"))]
    frames = sum(out["kernels"][k].get("calls", 0) for k in firsts)
    if fam and frames:
        tot = defaultdict(float)
        ms = 0.0
        for k in fam:
            e = out["kernels"][k]
            n = e.get("calls", 0)
            ms += e.get("total_ms", 0.0)
            for c, v in e["pmc"].items():
                tot[c] += v * n
        pf = {c: v / frames for c, v in tot.items()}
        fr = {"config": CONFIG, "kernels": sorted(fam), "frames": frames, "ms_per_frame": ms / frames,
              "per_kernel": {k: {"calls": out["kernels"][k].get("calls"), "avg_ms": out["kernels"][k].get("avg_ms")}
                             for k in fam},
              "counters_per_frame": pf,
              "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 16-B/lane read correction) + WRITE_SIZE KiB x1024"}
        if "FETCH_SIZE" in pf and "WRITE_SIZE" in pf:
            fr["hbm_read_bytes_raw"] = pf["FETCH_SIZE"] * 1024
            fr["hbm_write_bytes"] = pf["WRITE_SIZE"] * 1024
            fr["hbm_bytes_per_frame"] = pf["FETCH_SIZE"] * 1024 * 2 + pf["WRITE_SIZE"] * 1024
        if pf.get("SQ_WAVE_CYCLES"):
            fr["wait_any_per_wave_cycle"] = pf.get("SQ_WAIT_ANY", 0.0) / pf["SQ_WAVE_CYCLES"]
            fr["active_inst_any_per_wave_cycle"] = pf.get("SQ_ACTIVE_INST_ANY", 0.0) / pf["SQ_WAVE_CYCLES"]
        if pf.get("SQ_ACTIVE_INST_VALU"):
            fr["valu_lane_utilisation"] = pf.get("SQ_THREAD_CYCLES_VALU", 0.0) / (pf["SQ_ACTIVE_INST_VALU"] * 64.0)
        if pf.get("TCC_HIT_sum", 0) + pf.get("TCC_MISS_sum", 0) > 0:
            fr["l2_hit_rate"] = pf["TCC_HIT_sum"] / (pf["TCC_HIT_sum"] + pf["TCC_MISS_sum"])
        tag = os.environ.get("PMC_CONFIG_TAG", "metric")
        with open(f"profiles/{rnd}_pmc_frame_{tag}.json", "w") as f:
            json.dump(fr, f, indent=2)
        print(f"per frame ({tag}): {fr['ms_per_frame']:.4f} ms, HBM {fr.get('hbm_bytes_per_frame', 0) / 1e9:.3f} GB "
              f"(writes {fr.get('hbm_write_bytes', 0) / 1e9:.3f}), L2 hit {fr.get('l2_hit_rate', 0):.3f}, "
              f"wait {fr.get('wait_any_per_wave_cycle', 0):.3f}, lanes {fr.get('valu_lane_utilisation', 0):.3f}")
    for src in ("kt/run_kernel_stats.csv",):
        tag = os.environ.get("PMC_CONFIG_TAG", "metric")
        with open(os.path.join(prof, src)) as f, open(f"profiles/{rnd}_kernel_stats{'' if tag == 'metric' else '_' + tag}.csv", "w") as g:
            g.write(f.read())
    for k, e in out["kernels"].items():
        print(f"{k:26s} calls {e.get('calls', 0):4d} avg {e.get('avg_ms', 0):8.4f} ms  "
              f"hbm/launch {e.get('hbm_bytes_per_launch', 0) / 1e6:9.1f} MB  L2 hit {e.get('l2_hit_rate', 0):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
