"""A/B of path B (the pre-lowered CSR batch through halda_solve_batch_device[_settled]) on the C3 batch
(4096 M = 64 fleets x 9 k, host-lowered): per-launch device times (screen, k = 1 kernel, general kernel),
one stream (HIP events over K launches) and two streams (wall, K steps), with and without the settled
flags; a checksum of the results so that libraries can be compared. One JSON line per setting.

  HALDA_LIB=path/to/libhalda.so python tools/ab_pathb.py [--steps 20]
"""

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--fleets", type=int, default=4096)
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.batch import assemble, settled_instances
    from distilp_amd.solver.lower import lower_fleet

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    model = bench.load_model()
    fleets = bench.build_fleets(range(args.fleets), 64)
    batch, _ = assemble([lower_fleet(d, model, "4bit") for d in fleets], [KS] * len(fleets))
    copies = [bench.to_device(batch, torch, dev) for _ in range(2)]
    ptrs = [({f: t.data_ptr() for f, t in k.items()}, {f: t.data_ptr() for f, t in o.items()}) for k, o in copies]
    st = torch.from_numpy(settled_instances(batch)).to(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    lib = os.environ.get("HALDA_LIB", "default")
    for settled in (st.data_ptr(), None):
        def step(i, s):
            ctx.solve_device(ptrs[i % 2][0], batch, ptrs[i % 2][1], stream=s.cuda_stream, settled=settled)

        for i in range(4):
            step(i, streams[i % 2])
        torch.cuda.synchronize(dev)
        out = copies[0][1]
        chk = float(torch.where(out["status"] == 0, out["obj_lin"], torch.zeros_like(out["obj_lin"])).sum())
        ctx.set_timing(True)
        per = []
        for i in range(10):
            step(i, streams[0])
            torch.cuda.synchronize(dev)
            per.append(ctx.last_phase_ms())
        ctx.set_timing(False)
        phase = {k: statistics.mean(p[k] for p in per) for k in per[0]}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        one = []
        for _ in range(3):
            e0.record(streams[0])
            for i in range(args.steps):
                step(i, streams[0])
            e1.record(streams[0])
            torch.cuda.synchronize(dev)
            one.append(e0.elapsed_time(e1) / args.steps)
        two = []
        for _ in range(3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(args.steps):
                step(i, streams[i % 2])
            torch.cuda.synchronize(dev)
            two.append((time.perf_counter() - t0) / args.steps * 1e3)
        print(json.dumps({"lib": lib, "settled": settled is not None, "phase_ms": phase,
                          "one_stream_ms": statistics.median(one), "two_stream_ms": statistics.median(two),
                          "n_optimal": int((out["status"] == 0).sum()), "checksum": chk}), flush=True)


if __name__ == "__main__":
    main()
