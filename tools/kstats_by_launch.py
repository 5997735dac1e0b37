#!/usr/bin/env python
"""Per-launch-shape kernel summary from a rocprofv3 kernel trace: the --stats summary averages every launch of a
kernel (coarse and fine passes, training and inference instantiations together); this splits them by grid size so
the fine-pass MLP launches can be compared with bench.py's HIP-event timing.

    python tools/kstats_by_launch.py <dir with *kernel_trace.csv> [out.json]
"""
import collections
import csv
import glob
import json
import sys


def main():
    files = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)
    d = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            d[(name, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    # launches of one kernel and grid can still be two passes (the fp32 / x3 dW of the coarse and fine pass have the
    # same tiles x point splits): a group whose sorted durations jump by > 1.8x between neighbours is split there
    groups = []
    for (name, grid), v in d.items():
        v = sorted(v)
        # (the largest jump among cuts that leave >= 3 launches on each side: a few stray short launches below the
        # coarse pass must not hide the coarse / fine jump)
        cut = max(range(3, len(v) - 2), key=lambda i: v[i] / max(v[i - 1], 1e-9), default=None)
        if cut is not None and v[cut] / max(v[cut - 1], 1e-9) > 1.8:
            groups += [(name, grid, v[:cut], "lower mode"), (name, grid, v[cut:], "upper mode")]
        else:
            groups.append((name, grid, v, None))
    rows = []
    for name, grid, v, mode in sorted(groups, key=lambda g: -sum(g[2])):
        r = {"kernel": name, "grid_threads": grid, "launches": len(v), "median_us": round(v[len(v) // 2], 1),
             "mean_us": round(sum(v) / len(v), 1), "total_ms": round(sum(v) / 1e3, 2)}
        if mode:
            r["mode"] = mode
        rows.append(r)
    for r in rows[:30]:
        print(f"{r['kernel'][:60]:60s} grid={r['grid_threads']:>9d} n={r['launches']:5d} "
              f"median={r['median_us']:9.1f} us mean={r['mean_us']:9.1f} us")
    if len(sys.argv) > 2:
        json.dump(rows, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
