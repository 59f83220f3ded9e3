"""Diagnostic: the fixed cost around a timed region -- torch.cuda.synchronize on an idle device, and
one small k-sweep launch + synchronize -- with HIP's default wait mode or (--spin) hipDeviceScheduleSpin
set before torch initialises the device; then 20 / 200 C3 steps on two streams (bench.py's headline).
   python tools/sync_latency.py [--spin]"""
import ctypes
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def main():
    spin = "--spin" in sys.argv
    if spin:
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(1), flush=True)  # hipDeviceScheduleSpin
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table

    dev = torch.device("cuda", 0)
    torch.cuda.init()
    ctx = get_context(0)
    ctx.set_timing(False)
    model = bench.load_model()
    # the k-sweep streams first: with more streams than the process's hardware queues (GPU_MAX_HW_QUEUES,
    # 4 by default) two streams may share one, and a shared queue serialises their kernels
    ss = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    s = ss[0] if "--extra-stream" not in sys.argv else torch.cuda.Stream(dev)
    t = []
    for _ in range(2000):
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t.append(time.perf_counter() - t0)
    print(f"idle synchronize: median {statistics.median(t) * 1e6:.2f} us", flush=True)
    one = DeviceFleetTable(fleet_table(bench.build_fleets([0], 64), model), model, KS, 0.5, dev)
    for _ in range(20):
        one.launch(ctx, s.cuda_stream)
    torch.cuda.synchronize(dev)
    t = []
    for _ in range(500):
        t0 = time.perf_counter()
        one.launch(ctx, s.cuda_stream)
        torch.cuda.synchronize(dev)
        t.append(time.perf_counter() - t0)
    print(f"one-fleet launch + synchronize: median {statistics.median(t) * 1e6:.2f} us", flush=True)
    table = fleet_table(bench.build_fleets(range(4096), 64), model)
    dts = [DeviceFleetTable(table, model, KS, 0.5, dev) for _ in range(16)]
    for i in range(8):
        dts[i % 16].launch(ctx, ss[i % 2].cuda_stream)
    for steps in (20, 200, 20, 200):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            dts[i % 16].launch(ctx, ss[i % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        print(f"C3 steps {steps}: {(time.perf_counter() - t0) / steps * 1e6:.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
