"""The evidence tools' launch selection (CPU): tools/pmc_summary.py keeps the fine pass when the coarse and fine dW
launches share a grid, tools/kstats_by_launch.py splits such a group into its two duration modes. The bench's
`roofline.traffic` and the per-launch trace summaries under profiles/ come from these."""
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _write(path, header, rows):
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_pmc_summary_keeps_fine_mode(tmp_path):
    hdr = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"]
    # 3 fine (3000 KB) and 3 coarse (1000 KB) dW launches with one grid, plus a smaller-grid launch of another size
    fetch = [[i, "mlp_dw_kernel<float>", 786432, "FETCH_SIZE", 3000.0 if i % 2 else 1000.0] for i in range(6)]
    fetch.append([9, "mlp_dw_kernel<float>", 1024, "FETCH_SIZE", 5.0])
    write = [[i, "mlp_dw_kernel<float>", 786432, "WRITE_SIZE", 100.0] for i in range(6)]
    _write(tmp_path / "f" / "run_counter_collection.csv", hdr, fetch)
    _write(tmp_path / "w" / "run_counter_collection.csv", hdr, write)
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_summary.py"), str(tmp_path / "f"), str(tmp_path / "w"),
                    "mlp_dw_kernel", str(out)], check=True, capture_output=True)
    r = json.loads(out.read_text())
    assert r["launches"] == [3, 6]
    assert r["fetch_size_kb_raw"] == 3000.0 and r["hbm_read_bytes_per_launch"] == 2 * 3000.0 * 1024


def test_kstats_by_launch_splits_modes(tmp_path):
    hdr = ["Kernel_Name", "Grid_Size_X", "Start_Timestamp", "End_Timestamp"]
    rows = [["void k<float>(int)", 100, 0, 8_000_000]] * 4 + [["void k<float>(int)", 100, 0, 2_600_000]] * 4
    rows += [["void j(int)", 50, 0, 1000]] * 3
    _write(tmp_path / "t" / "run_kernel_trace.csv", hdr, rows)
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "kstats_by_launch.py"), str(tmp_path / "t"), str(out)],
                   check=True, capture_output=True)
    r = json.loads(out.read_text())
    k = {(x["kernel"], x.get("mode")): x for x in r}
    assert k[("k<float>", "upper mode")]["median_us"] == 8000.0 and k[("k<float>", "upper mode")]["launches"] == 4
    assert k[("k<float>", "lower mode")]["median_us"] == 2600.0
    assert k[("j", None)]["launches"] == 3


def test_kstats_by_launch_split_ignores_stray_short_launches(tmp_path):
    # two stray short launches of the same grid (a smaller job on the same tiles x splits) below the coarse mode: the
    # coarse / fine jump is still the split
    hdr = ["Kernel_Name", "Grid_Size_X", "Start_Timestamp", "End_Timestamp"]
    rows = [["void k<float>(int)", 100, 0, 7_400_000]] * 5 + [["void k<float>(int)", 100, 0, 2_450_000]] * 5
    rows += [["void k<float>(int)", 100, 0, 40_000]] * 2
    _write(tmp_path / "t" / "run_kernel_trace.csv", hdr, rows)
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "kstats_by_launch.py"), str(tmp_path / "t"), str(out)],
                   check=True, capture_output=True)
    k = {x.get("mode"): x for x in json.loads(out.read_text())}
    assert k["upper mode"]["launches"] == 5 and k["upper mode"]["median_us"] == 7400.0
    assert k["lower mode"]["launches"] == 7
