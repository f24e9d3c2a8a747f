"""Digest of gpurun_out/ab/*.json (scripts/ab_libs.sh): kernel us per config for each build."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        r = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable:", e)
        continue
    sw = [round(s["kernel_us"], 1) for s in r.get("sweep", [])]
    oc = [round(o["kernel_us"], 2) for o in r.get("other_configs", [])]
    print(f"{os.path.basename(f):28s} bench {r['kernel_us']:.3f} us  step {r['ms_per_step'] * 1e3:.3f} us  sweep {sw}  other {oc}")
