#!/usr/bin/env python3
"""Summarise rocprofv3 output (kernel trace + PMC passes) per step-kernel configuration.

    python scripts/prof_summary.py <round-dir-under-gpurun_out> <profiles/rN_summary.md>

Groups gpd::step_kernel dispatches by grid size (one 64-lane block per 64 drones, so
n_envs = Grid_Size_X for single-drone envs) and reports mean / median / min duration, and the
HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE passes with the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of wide coalesced reads -> x2;
WRITE_SIZE is exact for 16-B streaming stores).  Both counters are in KB (x1024).
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def kernel_groups(trace_csv, name="step_kernel"):
    g = defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        if name in r["Kernel_Name"]:
            g[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    return g


def pmc_groups(pmc_csv, counter, name="step_kernel"):
    g = defaultdict(list)
    for r in csv.DictReader(open(pmc_csv)):
        if name in r["Kernel_Name"] and r["Counter_Name"] == counter:
            g[int(r["Grid_Size"])].append(float(r["Counter_Value"]))
    return g


def main(rdir, out_md):
    lines = [f"# rocprofv3 summary — {os.path.basename(rdir.rstrip('/'))}", ""]
    summary = {"kernels": [], "pmc": [], "precision": os.environ.get("GPD_PROFILE_PRECISION", "f64")}
    for trace in sorted(glob.glob(os.path.join(rdir, "**", "*_kernel_trace.csv"), recursive=True)):
        lines += [f"## {os.path.relpath(trace, rdir)}", "", "| kernel | grid (lanes) | launches | mean us | median us | min us |",
                  "|---|---|---|---|---|---|"]
        for (k, grid), v in sorted(kernel_groups(trace).items(), key=lambda kv: kv[0][1]):
            short = k.split("(")[0].replace("void ", "")
            row = {"trace": os.path.relpath(trace, rdir), "kernel": short, "grid": grid, "launches": len(v),
                   "mean_us": statistics.mean(v), "median_us": statistics.median(v), "min_us": min(v)}
            summary["kernels"].append(row)
            lines.append(f"| `{short}` | {grid} | {len(v)} | {row['mean_us']:.2f} | {row['median_us']:.2f} | {row['min_us']:.2f} |")
        lines.append("")
    pmc = {}
    for f in sorted(glob.glob(os.path.join(rdir, "**", "*_counter_collection.csv"), recursive=True)):
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            for grid, v in pmc_groups(f, counter).items():
                pmc.setdefault(grid, {})[counter] = statistics.mean(v) * 1024.0
    if pmc:
        lines += ["## HBM traffic per step-kernel launch (PMC, separate passes)", "",
                  "| grid (lanes) | FETCH_SIZE raw MB | FETCH x2 (gfx950) MB | WRITE_SIZE MB | traffic MB |", "|---|---|---|---|---|"]
        for grid, c in sorted(pmc.items()):
            fr = c.get("FETCH_SIZE", float("nan"))
            wr = c.get("WRITE_SIZE", float("nan"))
            traffic = 2 * fr + wr
            summary["pmc"].append({"grid": grid, "fetch_raw_bytes": fr, "fetch_bytes": 2 * fr, "write_bytes": wr,
                                   "traffic_bytes": traffic})
            lines.append(f"| {grid} | {fr / 1e6:.3f} | {2 * fr / 1e6:.3f} | {wr / 1e6:.3f} | {traffic / 1e6:.3f} |")
        lines.append("")
    os.makedirs(os.path.dirname(os.path.abspath(out_md)), exist_ok=True)
    open(out_md, "w").write("\n".join(lines) + "\n")
    json.dump(summary, open(out_md.replace(".md", ".json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
