#!/usr/bin/env python
"""Per-kernel mean of rocprofv3 PMC counters (any counters) from one or more --pmc output dirs.

    python tools/sq_summary.py OUT.json DIR [DIR ...]

Prints/writes {kernel_short_name: {grid: {counter: mean_per_dispatch, "dispatches": n}}}. SQ_*CYCLES /
SQ_WAIT_* / SQ_ACTIVE_INST_* are quad-cycles summed over waves (MI355X_MICROARCH.md, PMC table)."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"yanerf(?:\d+|::)([a-z_0-9]+?)(?:I|E)", name) or re.search(r"([a-z_]+_kernel)", name)
    base = m.group(1) if m else name[:40]
    if "ItE" in name or "ItLb" in name or "<unsigned short" in name:
        base += "<bf16>"
    elif "IfE" in name or "IfLb" in name or "<float" in name:
        base += "<f32>"
    if "Lb1E" in name or ", true>" in name:
        base += "<train>"
    elif "Lb0E" in name or ", false>" in name:
        base += "<infer>"
    return base


def main():
    out = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    disp = defaultdict(lambda: defaultdict(lambda: defaultdict(set)))
    for d in sys.argv[2:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                g = int(r.get("Grid_Size", 0) or 0)
                did = (d, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                acc[k][g][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k][g][r["Counter_Name"]].add(did)
    res = {}
    for k, gs in acc.items():
        res[k] = {}
        for g, cs in gs.items():
            res[k][str(g)] = {c: v / len(disp[k][g][c]) for c, v in cs.items()}
            res[k][str(g)]["dispatches"] = max(len(x) for x in disp[k][g].values())
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
