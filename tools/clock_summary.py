#!/usr/bin/env python
"""Per-kernel effective clock from a rocprofv3 --pmc GRBM_GUI_ACTIVE/GRBM_COUNT run: counter value per dispatch
divided by the dispatch's duration (kernel trace of the same run), so a counter summed over the 8 XCDs shows as
8 x the clock. Prints JSON {kernel@grid: {counter: {"per_dispatch": v, "per_ns": v / ns}, "ms": duration}}."""
import collections
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    dur = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                     r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            did = r.get("Dispatch_Id")
            if did not in dur:
                continue
            ns, name, grid = dur[did]
            if "mlp" not in name:
                continue
            acc[f"{name}@{grid}"][r["Counter_Name"]].append((float(r["Counter_Value"]), ns))
    out = {}
    for k, cs in acc.items():
        o = {}
        for c, v in cs.items():
            tot_v = sum(x for x, _ in v)
            tot_ns = sum(n for _, n in v)
            o[c] = {"per_dispatch": tot_v / len(v), "per_ns": tot_v / tot_ns}
            o["ms"] = tot_ns / len(v) / 1e6
        out[k] = o
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
