#!/usr/bin/env python3
"""Table of scripts/pmc_itemize.sh: per launch shape, the step kernel's back-to-back median
duration and its HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, KB counters, MI355X_MICROARCH.md
§HBM), against the algorithmic bytes (774 B per drone-step, f64 RPM) and the necessary bytes
(+ ang_v 24, ring append 16, counters 8, - last action 32 B: DESIGN.md §7.1)."""
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import kernel_groups, pmc_groups  # noqa: E402


def main(rdir, envs=4096):
    alg = 774 * envs
    print(f"| shape | kernel us (b2b median) | fetch MB (x2) | write MB | traffic MB | traffic / alg ({alg / 1e6:.3f} MB) |")
    print("|---|---|---|---|---|---|")
    for d in sorted(glob.glob(os.path.join(rdir, "w*_p*"))):
        tr = glob.glob(os.path.join(d, "trace", "**", "*_kernel_trace.csv"), recursive=True)
        us = None
        if tr:
            g = kernel_groups(tr[0])
            b = [x for v in g.values() for x, bb in v if bb] or [x for v in g.values() for x, _ in v]
            us = statistics.median(b)
        vals = {}
        for c, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
            f = glob.glob(os.path.join(d, sub, "**", "*_counter_collection.csv"), recursive=True)
            if f:
                v = [x for vv in pmc_groups(f[0], c).values() for x in vv]
                vals[c] = statistics.mean(v) * 1024.0 if v else float("nan")
        fe, wr = 2 * vals.get("FETCH_SIZE", float("nan")), vals.get("WRITE_SIZE", float("nan"))
        print(f"| {os.path.basename(d)} | {us:.2f} | {fe / 1e6:.3f} | {wr / 1e6:.3f} | {(fe + wr) / 1e6:.3f} | "
              f"{(fe + wr) / alg:.3f} |" if us is not None else f"| {os.path.basename(d)} | - |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4096)
