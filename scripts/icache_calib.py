#!/usr/bin/env python3
"""I-cache calibration of the headline kernel from a `gpu_job.sh pmc_icache` run.

    python scripts/icache_calib.py gpurun_out/<tag> profiles/rN/icache

Reads the SQC I-cache pass (icache_main_1), the FETCH_SIZE pass (icache_main_2) and the
WRITE_SIZE pass (icache_main_3) of `scripts/prof_step.py --envs 4096 --steps 40`, takes the
per-launch medians of the io kernel, and writes calibration.json (read by bench.py's
instruction_fetch_bytes: misses x the FETCH_SIZE per miss of the round-3 ubench,
profiles/r3/icache/calibration.json) and README.md beside it."""
import csv
import json
import os
import statistics
import sys

KERNEL = "gpd::step_kernel_duo<double, 0, true>"
GRID = 49152


def per_launch(csv_path, counter):
    vals = {}
    for r in csv.DictReader(open(csv_path)):
        if "gpd::step_kernel_duo<double, 0, true>(" in r["Kernel_Name"] and int(r["Grid_Size"]) == GRID and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return statistics.median(vals.values()), len(vals)


def main(run, out):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    per_miss = json.load(open(os.path.join(root, "profiles", "r3", "icache", "calibration.json")))
    per_miss = per_miss["fetch_size_bytes_per_icache_miss"]
    p1 = os.path.join(run, "icache_main_1", "pmc_counter_collection.csv")
    hits, n = per_launch(p1, "SQC_ICACHE_HITS")
    miss, _ = per_launch(p1, "SQC_ICACHE_MISSES")
    dup, _ = per_launch(p1, "SQC_ICACHE_MISSES_DUPLICATE")
    fetch, _ = per_launch(os.path.join(run, "icache_main_2", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write, _ = per_launch(os.path.join(run, "icache_main_3", "pmc_counter_collection.csv"), "WRITE_SIZE")
    alg = 774 * 4096
    traffic = 2 * fetch * 1024 + write * 1024
    os.makedirs(out, exist_ok=True)
    cal = {"what": f"the io kernel's SQC I-cache misses per launch ({run}/icache_main_1, median of {n} launches) x "
                   "the round-3 calibration's FETCH_SIZE per miss (profiles/r3/icache/calibration.json)",
           "fetch_size_bytes_per_icache_miss": per_miss,
           "step_kernels": {KERNEL: {"grid": GRID, "icache_hits_per_launch": hits, "icache_misses_per_launch": miss,
                                     "icache_misses_duplicate_per_launch": dup,
                                     "instruction_fetch_size_bytes": miss * per_miss,
                                     "fetch_size_kb_per_launch": fetch, "write_size_kb_per_launch": write,
                                     "traffic_bytes": traffic, "alg_bytes": alg, "traffic_over_alg": traffic / alg}}}
    json.dump(cal, open(os.path.join(out, "calibration.json"), "w"), indent=1)
    with open(os.path.join(out, "README.md"), "w") as f:
        f.write(f"# Headline io kernel: I-cache and HBM counters (`scripts/gpu_job.sh pmc_icache`, run `{run}`)\n\n"
                f"`{KERNEL}` at 4096 envs, `scripts/prof_step.py --envs 4096 --steps 40`, one rocprofv3 `--pmc` pass\n"
                "per counter group (SQC I-cache; FETCH_SIZE; WRITE_SIZE), medians per launch "
                f"({n} launches):\n\n| counter | per launch |\n|---|---|\n"
                f"| SQC_ICACHE_HITS | {hits:,.0f} |\n| SQC_ICACHE_MISSES | {miss:,.0f} |\n"
                f"| SQC_ICACHE_MISSES_DUPLICATE | {dup:,.0f} |\n"
                f"| FETCH_SIZE | {fetch:,.0f} KB -> {2 * fetch / 1024:.3f} MB with the gfx950 x2 |\n"
                f"| WRITE_SIZE | {write / 1024:.3f} MB |\n\n"
                f"HBM traffic {traffic / 1e6:.3f} MB per launch against {alg / 1e6:.3f} MB algorithmic "
                f"({traffic / alg:.3f}); instruction fetch {miss * per_miss / 1e6:.3f} MB of it "
                f"({miss:,.0f} misses x {per_miss:.1f} B, profiles/r3/icache/calibration.json).\n")
    print(json.dumps(cal["step_kernels"][KERNEL], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
