"""Large-N step time vs memory allocation history: the same 1M-env step measured (a) in a fresh
process, (b) after a 4M-env sim was created and closed, (c) after torch allocated and freed a 4 GB
tensor.  Picks apart whether the sim's own hipMalloc buffers or torch's output tensors land on
memory that streams slower (TLB fragment size / placement)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim  # noqa: E402

G = 16


def step_us(E, reps=8):
    sim = BatchedAviarySim(n_envs=E, task="hover", precision="f64", device="cuda:0")
    acts = [(torch.rand((E, 1, 4), device="cuda:0") * 2 - 1).contiguous() for _ in range(G)]
    g = sim.capture_graph(acts)
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    sim.close()
    del g, acts
    return 1000 * s.elapsed_time(e) / (reps * G)


mode = sys.argv[1]
if mode == "after4m":
    print("4M first:", round(step_us(1 << 22, 2), 1))
elif mode == "aftertensor":
    x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda:0")
    del x
elif mode == "emptycache":
    print("4M first:", round(step_us(1 << 22, 2), 1))
    torch.cuda.empty_cache()
print(mode, [round(step_us(1 << 20), 1) for _ in range(3)], flush=True)
