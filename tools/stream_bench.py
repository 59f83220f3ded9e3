"""Config C5 (BASELINE.json configs[4]): real-time re-placement of a re-profiled fleet.

A base fleet (seed 0, M devices, llama_3_70b/online, L = 80, kv 4bit) is re-profiled
continuously: every instance multiplies each numeric device field by an independent
log-uniform factor in [0.9, 1.1]. Batches of B perturbed fleets go
through the whole k-sweep on the GPU (libhalda halda_solve_fleets: lowering, the 9 fixed-k
MILPs per fleet, argmin over k).

Reported (one JSON line):
  gpu_*        device-resident tables, back-to-back launches (lower + solve + pick), HIP events;
  e2e_*        end to end from the host: perturbation on the host (NumPy), PCIe in, k-sweep,
               PCIe out (halda_solve_fleets_host, synchronous, one batch at a time).
The exact solver needs no primal/dual warm start: what a re-profiled fleet reuses is its
structure (row pattern, sets) -- recomputed per instance here, since it costs nothing on the GPU.

  python tools/stream_bench.py [--M 64] [--batch 4096] [--iters 20]
"""

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def tiled(table, n):
    """n copies of a one-fleet table."""
    from dataclasses import replace

    from distilp_amd.solver.fleets import F64_FIELDS, BYTE_FIELDS

    M = table.n_devices
    upd = {f: np.tile(getattr(table, f), n) for f in ("os_class", "flags") + F64_FIELDS + BYTE_FIELDS}
    return replace(table, dev_off=np.arange(n + 1, dtype=np.int64) * M, **upd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()

    import torch

    from distilp_amd.common import DeviceProfile, ModelProfileSplit
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import (F64_FIELDS, BYTE_FIELDS, HaldaFleetResultC, _bind, _fleets_struct,
                                           fleet_table, model_struct, solve_table)
    from distilp_amd.synth import load_model_dict, synth_fleet

    model = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    base = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(0, args.M)]], model)
    rng = np.random.default_rng(10_000)
    B = args.batch
    big = tiled(base, B)

    # ---- GPU-resident: two device copies of a perturbed batch, launches back to back
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    lib = _bind(ctx.lib)
    stream = torch.cuda.Stream(dev)
    m = model_struct(model, 0.5)
    karr = np.asarray(KS, np.int32)
    bufs = []
    for _ in range(2):
        t = big.perturbed(rng)
        arrs = {f: torch.from_numpy(np.ascontiguousarray(getattr(t, f))).to(dev)
                for f in ("dev_off", "os_class", "flags") + F64_FIELDS + BYTE_FIELDS}
        outs = {"best_k": torch.empty(B, dtype=torch.int32, device=dev),
                "obj_value": torch.empty(B, dtype=torch.float64, device=dev),
                "w": torch.empty(t.n_devices, dtype=torch.int32, device=dev),
                "n": torch.empty(t.n_devices, dtype=torch.int32, device=dev)}
        fs = _fleets_struct(t, lambda f, a=arrs: a[f].data_ptr())
        r = HaldaFleetResultC(outs["best_k"].data_ptr(), outs["obj_value"].data_ptr(), outs["w"].data_ptr(),
                              outs["n"].data_ptr(), None, None, None, None)
        bufs.append((arrs, outs, fs, r, t))

    def launch(i):
        _, _, fs, r, _ = bufs[i % 2]
        rc = lib.halda_solve_fleets(ctx.ctx, ctypes.byref(m), ctypes.byref(fs), karr.ctypes.data, len(KS),
                                    ctypes.byref(r), ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0, rc

    for i in range(3):
        launch(i)
    torch.cuda.synchronize(dev)
    # spot check against the synchronous host API on the same perturbed batch
    arrs, outs, fs, r, t = bufs[0]
    launch(0)
    torch.cuda.synchronize(dev)
    ref = solve_table(t, model, KS, 0.5)
    assert np.array_equal(outs["best_k"].cpu().numpy(), ref.best_k)
    assert np.array_equal(outs["w"].cpu().numpy(), ref.w)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(args.iters):
        launch(i)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    gpu_ms = e0.elapsed_time(e1) / args.iters

    # ---- end to end: host perturbation + PCIe + k-sweep + PCIe, one batch at a time
    t0 = time.perf_counter()
    n_e2e = max(3, args.iters // 4)
    pert_s = 0.0
    for _ in range(n_e2e):
        tp = time.perf_counter()
        tb = big.perturbed(rng)
        pert_s += time.perf_counter() - tp
        solve_table(tb, model, KS, 0.5)
    e2e_s = (time.perf_counter() - t0) / n_e2e
    line = {
        "config": f"C5: re-profiled M={args.M} fleet (L=80, llama_3_70b/online, kv 4bit), fields x LU(0.9,1.1), "
                  f"batches of {B} fleets x {len(KS)} k",
        "gpu_ms_per_batch": gpu_ms,
        "gpu_fleets_per_s": B / (gpu_ms * 1e-3),
        "gpu_instances_per_s": B * len(KS) / (gpu_ms * 1e-3),
        "e2e_ms_per_batch": e2e_s * 1e3,
        "e2e_fleets_per_s": B / e2e_s,
        "e2e_instances_per_s": B * len(KS) / e2e_s,
        "host_perturb_ms_per_batch": pert_s / n_e2e * 1e3,
        "target_instances_per_s": 10_000,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
