"""Probe: the fused rollout-policy kernel (libgpd_policy.so) alone - microseconds per launch over
back-to-back launches (HIP events), for the bench's shapes, split by what the call does:
deterministic forward, sampled forward, forward + the previous step's bootstrap, bootstrap only,
and torch's forward of the same networks beside it.
    python scripts/policy_probe.py [n_envs | sweep | graph]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ac(n_obs, n_act, dev):
    import torch.nn as nn

    def mlp(o):
        return nn.Sequential(nn.Linear(n_obs, 64), nn.Tanh(), nn.Linear(64, 64), nn.Tanh(), nn.Linear(64, o))

    class AC(nn.Module):
        def __init__(self):
            super().__init__()
            self.pi, self.vf = mlp(n_act), mlp(1)
            self.log_std = nn.Parameter(torch.zeros(n_act))
    return AC().to(dev)


def per_launch_us(fn, n=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / n


def graph_us(fn, k=64, reps=10):
    """per launch over hipGraph replays of k launches (no host launch cost)"""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(k):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / (reps * k)


def graphed():
    """The bench's shape (4096 rows, 72 -> 4) by graph replay: deterministic, sampled, sampled with
    the previous step's bootstrap (9 % truncated rows), bootstrap only."""
    from gym_pybullet_drones_routing_amd.policy import MlpPolicyKernel
    E, n_obs, n_act = 4096, 72, 4
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = ac(n_obs, n_act, dev)
    k = MlpPolicyKernel(m, seed=1)
    obs, tobs = torch.randn((E, n_obs), device=dev), torch.randn((E, n_obs), device=dev)
    act = torch.zeros((E, n_act), device=dev)
    bo, ba = torch.zeros((E, n_obs), device=dev), torch.zeros((E, n_act), device=dev)
    bl, bv = torch.zeros(E, device=dev), torch.zeros(E, device=dev)
    rew = torch.rand(E, device=dev)
    te = torch.zeros(E, dtype=torch.uint8, device=dev)
    tr = (torch.rand(E, device=dev) < 0.09).to(torch.uint8)
    br, bd = torch.zeros(E, device=dev), torch.zeros(E, device=dev)
    res = {
        "forward_det": graph_us(lambda: k.step(obs, act, bo, ba, bl, bv, deterministic=True)),
        "forward_sample": graph_us(lambda: k.step(obs, act, bo, ba, bl, bv)),
        "forward_sample_bootstrap": graph_us(lambda: k.step(obs, act, bo, ba, bl, bv, prev=(rew, te, tr, tobs),
                                                             buf_rew=br, buf_done=bd)),
        "bootstrap_only": graph_us(lambda: k.step(None, prev=(rew, te, tr, tobs), buf_rew=br, buf_done=bd)),
    }
    print(f"[policy-graph] {os.environ.get('GPD_POLICY_LIB', 'libgpd_policy.so')}: " +
          ", ".join(f"{a} {b:.2f} us" for a, b in res.items()), flush=True)


def main():
    from gym_pybullet_drones_routing_amd.policy import MlpPolicyKernel
    E = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 4096
    dev = torch.device("cuda:0")
    for n_obs, n_act in ((72, 4), (27, 1)):
        torch.manual_seed(0)
        m = ac(n_obs, n_act, dev)
        k = MlpPolicyKernel(m, seed=1)
        obs = torch.randn((E, n_obs), device=dev)
        tobs = torch.randn((E, n_obs), device=dev)
        act = torch.zeros((E, n_act), device=dev)
        bo, ba = torch.zeros((E, n_obs), device=dev), torch.zeros((E, n_act), device=dev)
        bl, bv = torch.zeros(E, device=dev), torch.zeros(E, device=dev)
        rew = torch.rand(E, device=dev)
        te = torch.zeros(E, dtype=torch.uint8, device=dev)
        tr = (torch.rand(E, device=dev) < 0.09).to(torch.uint8)
        br, bd = torch.zeros(E, device=dev), torch.zeros(E, device=dev)
        res = {
            "forward_det": per_launch_us(lambda: k.step(obs, act, bo, ba, bl, bv, deterministic=True)),
            "forward_sample": per_launch_us(lambda: k.step(obs, act, bo, ba, bl, bv)),
            "forward_sample_bootstrap": per_launch_us(lambda: k.step(obs, act, bo, ba, bl, bv, prev=(rew, te, tr, tobs),
                                                                     buf_rew=br, buf_done=bd)),
            "bootstrap_only": per_launch_us(lambda: k.step(None, prev=(rew, te, tr, tobs), buf_rew=br, buf_done=bd)),
            "critic_only": per_launch_us(lambda: k.step(obs, buf_val=bv)),
        }
        with torch.no_grad():
            res["torch_forward_actor_critic"] = per_launch_us(lambda: (m.pi(obs), m.vf(obs)))
        macs = E * 2 * (n_obs * 64 + 64 * 64 + 64 * (n_act + 1) / 2)
        print(f"[policy] E={E} n_obs={n_obs} n_act={n_act}: " +
              ", ".join(f"{a} {b:.2f} us" for a, b in res.items()) +
              f"; {macs / 1e6:.1f} M MACs -> {2 * macs / (res['forward_det'] * 1e-6) / 1e12:.2f} TFLOP/s", flush=True)


def sweep():
    """forward_det and critic_only against the batch size: a flat curve = fixed latency, a linear
    one = throughput."""
    from gym_pybullet_drones_routing_amd.policy import MlpPolicyKernel
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = ac(72, 4, dev)
    k = MlpPolicyKernel(m, seed=1)
    for E in (16, 256, 1024, 4096, 16384, 65536):
        obs = torch.randn((E, 72), device=dev)
        act = torch.zeros((E, 4), device=dev)
        bv = torch.zeros(E, device=dev)
        fd = per_launch_us(lambda: k.step(obs, act, None, None, None, bv, deterministic=True), 100)
        co = per_launch_us(lambda: k.step(obs, buf_val=bv), 100)
        print(f"[policy-sweep] E={E}: forward_det {fd:.2f} us, critic_only {co:.2f} us", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":
        sweep()
    elif len(sys.argv) > 1 and sys.argv[1] == "graph":
        with torch.no_grad():
            graphed()
    else:
        main()
