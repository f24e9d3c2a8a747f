"""Probe: RCCL collectives on one GPU (one-rank group) - eager cost per call through torch's
ProcessGroupNCCL and through the raw RCCL binding (gym_pybullet_drones_routing_amd/rccl.py), graph
capture of each, and the teardown after a capture.  Every stage prints; a stage that exceeds its
time box ends the process (os._exit) with a message instead of hanging the box.
    python scripts/rccl_probe.py [torch|raw|both]"""
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def boxed(name, seconds):
    ev = threading.Event()

    def watch():
        if not ev.wait(seconds):
            print(f"[probe] {name}: no return after {seconds} s - exiting", flush=True)
            os._exit(3)
    threading.Thread(target=watch, daemon=True).start()
    return ev


def timeit(fn, n=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / n


def graph_us(fn, k=32, reps=20):
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
    return g, 1000.0 * e0.elapsed_time(e1) / (reps * k), timeit(g.replay, 20) / k


def main(which):
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    ev = boxed("init_process_group", 60)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ev.set()
    n = 1_400_000
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    if which in ("torch", "both"):
        ev = boxed("torch eager", 60)
        us_ag = timeit(lambda: dist.all_gather_into_tensor(dst, src))
        us_a2a = timeit(lambda: dist.all_to_all_single(dst, src, [n], [n]))
        ev.set()
        print(f"[probe] torch PG eager: all_gather_into_tensor {us_ag:.1f} us, all_to_all_single {us_a2a:.1f} us "
              f"({n} B)", flush=True)
        ev = boxed("torch graph", 60)
        g, dev_us, host_us = graph_us(lambda: dist.all_gather_into_tensor(dst, src))
        ok = torch.equal(dst, src)
        ev.set()
        print(f"[probe] torch PG graph of 32 all_gathers: {dev_us:.1f} us per call (events), {host_us:.1f} us "
              f"(wall), correct {ok}", flush=True)
        ev = boxed("torch graph teardown", 30)
        del g
        torch.cuda.synchronize()
        ev.set()
        print("[probe] torch graph deleted", flush=True)
    if which in ("raw", "both"):
        from gym_pybullet_drones_routing_amd.rccl import RcclComm
        ev = boxed("raw init", 60)
        comm = RcclComm(dev)
        ev.set()
        print(f"[probe] raw RCCL comm up ({comm.lib_path})", flush=True)
        ev = boxed("raw eager", 60)
        us_ag = timeit(lambda: comm.all_gather(src, dst))
        us_g = timeit(lambda: comm.gather(src, dst, 0))
        ev.set()
        print(f"[probe] raw RCCL eager: all_gather {us_ag:.1f} us, gather (send/recv group) {us_g:.1f} us", flush=True)
        ev = boxed("raw graph", 60)
        dst.zero_()
        g, dev_us, host_us = graph_us(lambda: comm.all_gather(src, dst))
        ok = torch.equal(dst, src)
        g2, dev2, host2 = graph_us(lambda: comm.gather(src, dst, 0))
        ev.set()
        print(f"[probe] raw RCCL graph: all_gather {dev_us:.1f} us per call (events), {host_us:.1f} (wall), "
              f"correct {ok}; gather {dev2:.1f} / {host2:.1f} us", flush=True)
        ev = boxed("raw teardown", 30)
        del g, g2
        torch.cuda.synchronize()
        comm.destroy()
        ev.set()
        print("[probe] raw comm destroyed", flush=True)
    ev = boxed("destroy_process_group", 30)
    dist.destroy_process_group()
    ev.set()
    print("[probe] process group destroyed", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "both")
