#!/usr/bin/env python
"""Timeline of one training step from a rocprofv3 kernel trace: every kernel of the step with its start offset,
duration and stream (queue), plus the idle gaps on the GPU (no kernel running). Steps are delimited by the Adam
kernel (the step's last launch). Development tool for finding the critical path of the fused step.

    python tools/step_timeline.py <dir with *kernel_trace.csv> [step_index_from_end=3] [out.json]
"""
import csv
import glob
import json
import sys


def main():
    files = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("yanerf::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?"),
                         int(r["Grid_Size_X"])))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if r[2].startswith(("adam_kernel", "adam_table_kernel",
                                                                "adam_table_step_kernel"))]
    if len(ends) < back + 1:
        print("not enough steps")
        return
    a, b = ends[-back - 1] + 1, ends[-back] + 1
    step = rows[a:b]
    t0 = step[0][0]
    out = []
    busy_until = t0
    idle = 0
    for s, e, n, q, g in step:
        gap = max(0, s - busy_until)
        idle += gap
        busy_until = max(busy_until, e)
        out.append({"kernel": n[:70], "queue": q, "grid": g, "start_us": round((s - t0) / 1e3, 1),
                    "dur_us": round((e - s) / 1e3, 1), "gap_before_us": round(gap / 1e3, 1)})
        print(f"{(s - t0) / 1e3:9.1f} +{(e - s) / 1e3:8.1f} us  q={q:>3s} gap={gap / 1e3:6.1f}  {n[:70]} grid={g}")
    total = (step[-1][1] - t0) / 1e3
    print(f"step span {total:.1f} us, GPU idle {idle / 1e3:.1f} us")
    if len(sys.argv) > 3:
        json.dump({"step_span_us": total, "idle_us": idle / 1e3, "kernels": out}, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
