"""scripts/prof_summary.py on a synthetic rocprofv3 kernel trace: per-(kernel, grid) statistics and
the back-to-back subset (launches that start within B2B_US of the previous one's end) that
bench.py reports beside its event time."""
import csv
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("prof_summary", os.path.join(ROOT, "scripts", "prof_summary.py"))
prof_summary = importlib.util.module_from_spec(spec)
spec.loader.exec_module(prof_summary)

FIELDS = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Thread_Id", "Dispatch_Id", "Kernel_Id", "Kernel_Name",
          "Correlation_Id", "Start_Timestamp", "End_Timestamp", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
          "Accum_VGPR_Count", "SGPR_Count", "Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z",
          "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]


def _trace(path, launches):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for i, (name, grid, start_ns, dur_ns) in enumerate(launches):
            w.writerow({k: 0 for k in FIELDS} | {"Kind": "KERNEL_DISPATCH", "Kernel_Name": name, "Grid_Size_X": grid,
                                                 "Start_Timestamp": start_ns, "End_Timestamp": start_ns + dur_ns,
                                                 "Dispatch_Id": i})


def test_back_to_back_subset(tmp_path):
    k = "void gpd::step_kernel_duo<double, 0, true>(double*, ...)"
    launches = [(k, 49152, 0, 6000)]                       # isolated (first)
    t = 6000 + 1500
    for _ in range(4):                                    # back to back: gaps of 1.5 us
        launches.append((k, 49152, t, 5000))
        t += 5000 + 1500
    t += 20000
    launches.append((k, 49152, t, 7000))                  # isolated again
    launches.append(("void other_kernel()", 256, t + 9000, 1000))
    d = tmp_path / "run" / "prof_bench"
    d.mkdir(parents=True)
    _trace(d / "bench_kernel_trace.csv", launches)
    out = tmp_path / "summary.md"
    prof_summary.main(str(tmp_path / "run"), str(out))
    s = json.load(open(str(out).replace(".md", ".json")))
    (row,) = [r for r in s["kernels"] if r["grid"] == 49152]
    assert row["kernel"] == "gpd::step_kernel_duo<double, 0, true>"
    assert row["launches"] == 6 and row["b2b_launches"] == 4
    assert row["b2b_median_us"] == 5.0 and row["min_us"] == 5.0
    assert abs(row["mean_us"] - (6 + 4 * 5 + 7) / 6) < 1e-12
    assert "other_kernel" not in json.dumps(s)             # only step kernels are summarised
