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
    """{(kernel, grid): [(duration us, started within B2B_US of the previous launch's end)]}"""
    rows = sorted((r for r in csv.DictReader(open(trace_csv)) if name in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    g = defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        b2b = prev_end is not None and (s - prev_end) / 1000.0 < B2B_US
        g[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(((e - s) / 1000.0, b2b))
        prev_end = e
    return g


# Launches that start within this many us of the previous one's end ran back to back, as in the
# graph-replayed timed region; the rest ran after an idle queue (the profiler makes most
# launches isolated: each one waits for the host), which adds a cold start to their duration.
B2B_US = 3.0


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
        lines += [f"## {os.path.relpath(trace, rdir)}", "",
                  "| kernel | grid (lanes) | launches | mean us | median us | min us | back-to-back launches | their median us |",
                  "|---|---|---|---|---|---|---|---|"]
        for (k, grid), dv in sorted(kernel_groups(trace).items(), key=lambda kv: kv[0][1]):
            short = k.split("(")[0].replace("void ", "")
            v = [d for d, _ in dv]
            b = [d for d, bb in dv if bb]
            row = {"trace": os.path.relpath(trace, rdir), "kernel": short, "grid": grid, "launches": len(v),
                   "mean_us": statistics.mean(v), "median_us": statistics.median(v), "min_us": min(v),
                   "b2b_launches": len(b), "b2b_median_us": statistics.median(b) if b else None}
            summary["kernels"].append(row)
            bm = f"{row['b2b_median_us']:.2f}" if b else "-"
            lines.append(f"| `{short}` | {grid} | {len(v)} | {row['mean_us']:.2f} | {row['median_us']:.2f} | "
                         f"{row['min_us']:.2f} | {len(b)} | {bm} |")
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
