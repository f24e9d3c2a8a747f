"""Profiling driver: bench.py's RL-rollout leg alone (one hipGraph of K x (policy MLP forward +
sample + gpd_step)), so that a rocprofv3 kernel trace holds the step kernel as an RL caller runs it,
with the policy's kernels between consecutive steps.  Usage:
    rocprofv3 --kernel-trace --stats -d OUT -o rollout --output-format csv -- python3 scripts/prof_rollout.py [--policy N]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--policy", type=int, default=0, help="gpd_config store_policy (0 = the library's choice)")
ap.add_argument("--precision", default="f64")
a = ap.parse_args()
r = bench.rollout_leg(torch.device("cuda:0"), a.precision, "rpm", a.envs, store_policy=a.policy)
print(json.dumps(r), flush=True)
