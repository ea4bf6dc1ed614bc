#!/usr/bin/env python3
"""Writes profiles/AB_INDEX.md: one row per A/B record under profiles/ (r01-r06 *_ab_*.txt) with the
record's own header comment -- what was compared and what shipped.  The one-off r0*_ab_*.sh scripts that
produced r01-r05's records were folded into scripts/ab.sh (BUILDS / CASES / ROUNDS) in r06; the records
keep their original script names in their headers."""
import glob
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header(path, n=4):
    out = []
    for line in open(path, errors="replace"):
        line = line.rstrip("\n")
        if not line.startswith("#"):
            break
        out.append(line.lstrip("# ").strip())
        if len(out) >= n:
            break
    return " ".join(out)


def design_mentions(name, design):
    """The DESIGN.md sentence(s) citing the record (its conclusion as the design text states it)."""
    stem = name[:-4]
    out = []
    for m in re.finditer(re.escape(stem) + r"[\w*,{}]*\.txt|" + re.escape(stem) + r"\b", design):
        a = max(design.rfind(". ", 0, m.start()), design.rfind("\n\n", 0, m.start()), design.rfind("| ", 0, m.start()))
        b = design.find(". ", m.end())
        frag = re.sub(r"\s+", " ", design[a + 2:b + 1 if b > 0 else m.end() + 200]).strip()
        if frag and frag not in out:
            out.append(frag[:400])
        if len(out) >= 2:
            break
    return " / ".join(out)


def main():
    design = open(os.path.join(REPO, "DESIGN.md")).read()
    rows = []
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "r0*_ab_*.txt"))):
        name = os.path.basename(p)
        h = header(p)
        if not h:
            first = next((l.strip() for l in open(p, errors="replace") if l.strip()), "")
            d = design_mentions(name, design)
            h = ("DESIGN.md: " + d) if d else "(raw timings, no header) " + re.sub(r"\s+", " ", first)[:160]
        rows.append(f"| `{name}` | {h.replace('|', '/')} |")
    text = ("# A/B records index\n\n"
            "Every A/B experiment kept under `profiles/` (timings from `scripts/time_frames.py`, counters from\n"
            "`scripts/pmc_ab.sh`), with the record's own header: what was compared, and the outcome where the\n"
            "header states one.  r01-r05's one-off `scripts/r0*_ab_*.sh` drivers were folded into the\n"
            "parametrised `scripts/ab.sh` in r06 (BUILDS = kernel builds from `make variant`, CASES =\n"
            "time_frames.py argument sets, ROUNDS); regenerate this file with `python scripts/ab_index.py`.\n\n"
            f"{len(rows)} records.\n\n| record | what / outcome |\n|---|---|\n" + "\n".join(rows) + "\n")
    open(os.path.join(REPO, "profiles", "AB_INDEX.md"), "w").write(text)
    print(f"{len(rows)} records")


if __name__ == "__main__":
    main()
