"""Phase timing of step_kernel from the diagnostic build (GPD_LIB=.../libgpd_stamps.so).

Phases (lane 0 of every block, s_memtime shader clocks):
 0 entry -> 1 state/action loads consumed + first substep -> 2 all substeps ->
 3 task hooks / obs angles -> 4 history DMA landed -> 5 reset/terminal rows -> 6 tile written +
 barrier -> 7 tile copy-out issued."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPD_LIB"] = os.environ.get("GPD_STAMPS_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym_pybullet_drones_routing_amd", "libgpd_stamps.so")
import numpy as np, torch
from gym_pybullet_drones_routing_amd import _lib
from gym_pybullet_drones_routing_amd.sim import BatchedAviarySim
lib = _lib.load()
lib.gpd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
for prec in os.environ.get("STAMP_PRECS", "f64 f32").split():
    for E in [int(x) for x in os.environ.get("STAMP_ENVS", "4096 1048576").split()]:
        waves = int(os.environ.get("STAMP_WAVES", "0"))
        sim = BatchedAviarySim(n_envs=E, task="hover", precision=prec, device="cuda:0",
                               tuning={"step_waves": waves} if waves else None)
        scale = float(os.environ.get("ACT_SCALE", "1.0"))
        acts = [((torch.rand((E, 1, 4), device="cuda:0") * 2 - 1) * scale).contiguous() for _ in range(16)]
        g = sim.capture_graph(acts)
        for _ in range(4): g.replay()
        torch.cuda.synchronize()
        nb = min(65536, -(-sim.n_drones // sim.constants.drones_per_block))
        buf = np.zeros((nb, 24), np.uint64)
        assert lib.gpd_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), nb) == 0
        t = buf.astype(np.int64)
        order = [0, 10, 1, 2, 3, 4, 5, 6, 8, 9, 7]   # 10: loads landed; 8/9 inside the copy-out (after LDS reads, after stores)
        d = [(a, b, int(np.median(t[:, b] - t[:, a]))) for a, b in zip(order[:-1], order[1:])]
        tot = t[:, 7] - t[:, 0]
        print(f"{prec} E={E} lanes/block {sim.constants.lanes_per_block}: per-block phase cycles (median) " + " ".join(f"{a}->{b}:{c}" for a, b, c in d) +
              f" | total median {int(np.median(tot))} p90 {int(np.percentile(tot, 90))} max {int(tot.max())}", flush=True)
        slow = int(np.argmax(tot))
        print(f"    slowest block {slow}: " + " ".join(f"{a}->{b}:{int(t[slow, b] - t[slow, a])}"
                                                    for a, b in zip(order[:-1], order[1:])), flush=True)
        hist = np.percentile(tot, [10, 25, 50, 75, 90, 95, 99]).astype(int)
        print(f"    block total percentiles 10/25/50/75/90/95/99: {list(hist)}; blocks > median+1000: "
              f"{int((tot > np.median(tot) + 1000).sum())} of {len(tot)}", flush=True)
        # s_memrealtime (100 MHz, shared by the device): block start spread and first-start -> last-end span
        rs, re_ = t[:, 11], t[:, 12]
        if sim.constants.lanes_per_block >= 128 and t[:, 13].min() > 0:   # rate (two-wave) / io (three-wave) wave's end
            rw = t[:, 13] - rs
            print(f"    {'io' if sim.constants.lanes_per_block == 192 else 'rate'} wave ends {int(np.median(t[:, 13] - re_)) * 10} ns after the pose wave (median), "
                  f"duration median {int(np.median(rw)) * 10} ns", flush=True)
            re_ = np.maximum(re_, t[:, 13])
        if sim.constants.lanes_per_block == 192 and t[:, 17].min() > 0:
            io = t[:, 17:23]
            names = ["entry->B0 arrive", "B0 wait", "DMA issue + B1..B7", "vmcnt(0)", "stores", "final barrier wait"]
            dd = [int(np.median(t[:, 17] - t[:, 0]))] + [int(np.median(io[:, j + 1] - io[:, j])) for j in range(5)]
            print("    io wave (cycles, median): pose-entry->io-entry " + str(dd[0]) + " | " +
                  " ".join(f"{names[j + 1]}:{dd[j + 1]}" for j in range(5)) +
                  f" | io B0 arrive -> pose stamp1 {int(np.median(t[:, 1] - io[:, 0]))}"
                  f" | io final arrive vs pose stamp5 {int(np.median(io[:, 4] - t[:, 5]))}", flush=True)
        hw = t[:, 14:14 + sim.constants.lanes_per_block // 64]
        simd = (hw >> 4) & 3
        same = [(simd[:, a] == simd[:, b]).mean() for a in range(simd.shape[1]) for b in range(a + 1, simd.shape[1])]
        print(f"    SIMD of waves (first blocks): {simd[:6].tolist()}; fraction of blocks where a wave pair shares a SIMD: "
              f"{[round(float(x), 3) for x in same]}", flush=True)
        if rs.min() > 0:
            print(f"    realtime: start spread {(rs.max() - rs.min()) * 10} ns, block duration median "
                  f"{int(np.median(re_ - rs)) * 10} ns max {int((re_ - rs).max()) * 10} ns, span {(re_.max() - rs.min()) * 10} ns",
                  flush=True)
        sim.close()
