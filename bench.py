"""Benchmark: HALDA MILP instances solved/s on MI355X (config C3 of BASELINE.json).

Workload per GPU and step: 4096 seeded synthetic fleets of M = 64 devices
(L = 80, model llama_3_70b/online, kv "4bit"), every fleet with all 9
k-candidates of L = 80 -> 36,864 fixed-k MILP instances, solved exactly by ONE
libhalda launch (halda_solve_batch_device) from inputs already resident in HBM.
Weak scaling: rank r solves its own 4096 fleets (seeds r*4096 ...). No
collective on the data path (fleets are independent); a barrier brackets the
timed region and the max time over ranks is reported.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Extra JSON fields: roofline (dominant kernel halda_solve_kernel vs HBM peak,
algorithmic bytes per launch defined in DESIGN.md §Measurement), cpu_baseline
(the oracle = reference lowering + scipy/HiGHS, timed on ONE host core on a
bounded sample of the same workload), feasible_instances_per_s, fleets_per_s,
time_to_optimal_ms (median end-to-end halda_solve of one M=64 fleet).
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
KS_L80 = [1, 2, 4, 5, 8, 10, 16, 20, 40]
METRIC = "HALDA MILP instances solved/sec (node), M=64 devs L=80; time-to-optimal"


def build_workload(rank: int, fleets: int, M: int, ks=None):
    from distilp_amd.common import DeviceProfile, ModelProfileSplit
    from distilp_amd.solver.batch import assemble
    from distilp_amd.solver.lower import lower_fleet
    from distilp_amd.synth import load_model_dict, load_templates, synth_fleet

    model = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    tpl = load_templates()
    lowered = []
    for s in range(rank * fleets, (rank + 1) * fleets):
        devs = [DeviceProfile.model_validate(d) for d in synth_fleet(s, M, tpl)]
        lowered.append(lower_fleet(devs, model, "4bit"))
    batch, refs = assemble(lowered, [list(ks or KS_L80)] * len(lowered))
    return model, lowered, batch, refs


def algorithmic_bytes(lowered, batch, refs):
    """Bytes each launch must move: {kernel name: bytes per launch}.

    A solved (surviving) instance: its fleet's CSR once (row_ptr + col_idx/val, which contains the
    equality row), its header (n_cols, n_rows, 3 offsets), c / col_lb / col_ub (8 B each) and
    integrality (1 B) per column (which contain the w bounds and c[C]), row_lb / row_ub per row,
    x out and the result scalars. A screened instance: its header, the equality row (two row_ptr
    entries, M col_idx/val, its row bounds), lb of its M w-columns, c[C] and the verdict byte,
    plus the result scalars when the screen settles it (M > W = L/k).
      halda_screen_kernel + halda_solve_k1_kernel (default): every instance's screen bytes, then
        the survivors' solve bytes;
      halda_screen_k1_kernel (HALDA_TWO_PASS=0, one wave per instance): settled instances' screen
        bytes + survivors' solve bytes + the verdict byte of every instance."""
    hdr, res = 4 + 4 + 8 + 8 + 8, 4 + 8 + 8 + 8 + 8
    solve, screen, fused = 0, 0, 0
    fleets_solved = set()
    for ref in refs:
        fl = lowered[ref.fleet]
        scr = hdr + 8 + 12 * fl.M + 16 + 8 * fl.M + 8 + 1
        screen += scr
        if ref.W - fl.M >= 0:
            if ref.fleet not in fleets_solved:
                fleets_solved.add(ref.fleet)
                solve += 4 * (fl.n_rows + 1) + 12 * fl.nnz
                fused += 4 * (fl.n_rows + 1) + 12 * fl.nnz
            one = hdr + 25 * fl.n_cols + 16 * fl.n_rows + 8 * fl.n_cols + res
            solve += one
            fused += one + 1
        else:
            screen += res
            fused += scr + res
    return {"halda_screen_k1_kernel": fused, "halda_screen_kernel": screen, "halda_solve_k1_kernel": solve}


def to_device(batch, torch, dev):
    fields = ("n_cols", "n_rows", "csr_off", "col_off", "row_off", "row_ptr", "col_idx", "val", "c", "col_lb",
              "col_ub", "row_lb", "row_ub", "integrality")
    keep = {f: torch.from_numpy(np.ascontiguousarray(getattr(batch, f))).to(dev) for f in fields}
    n = batch.n_inst
    out = {
        "status": torch.empty(n, dtype=torch.int32, device=dev),
        "x": torch.zeros(batch.total_cols, dtype=torch.float64, device=dev),
        "obj_lin": torch.empty(n, dtype=torch.float64, device=dev),
        "dual_bound": torch.empty(n, dtype=torch.float64, device=dev),
        "gap": torch.empty(n, dtype=torch.float64, device=dev),
        "nodes": torch.empty(n, dtype=torch.int64, device=dev),
    }
    return keep, out


def cpu_baseline_child(budget_s: float, M: int) -> None:
    """Runs in a child process pinned to one core: oracle (reference lowering + scipy HiGHS) on the
    same C3 fleets (seeds 0, 1, ...) until the time budget is used; prints one JSON line."""
    os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    from distilp_amd.common import DeviceProfile, ModelProfileSplit
    from distilp_amd.synth import load_model_dict, load_templates, synth_fleet
    from oracle import milp_oracle as mo

    model = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    tpl = load_templates()
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, M, tpl)] for s in range(512)]
    t0 = time.perf_counter()
    n_inst = n_fleets = 0
    while time.perf_counter() - t0 < budget_s and n_fleets < len(fleets):
        mo.halda_solve_oracle(fleets[n_fleets], model, k_candidates=KS_L80, mip_gap=1e-4, kv_bits="4bit",
                              solver="highs")
        n_fleets += 1
        n_inst += len(KS_L80)
    dt = time.perf_counter() - t0
    print(json.dumps({"instances": n_inst, "fleets": n_fleets, "seconds": dt}))


def run_cpu_baseline(budget_s: float, M: int):
    try:
        out = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--cpu-baseline-child",
                              "--cpu-budget", str(budget_s), "--M", str(M)],
                             capture_output=True, text=True, timeout=budget_s * 4 + 120, check=True)
        rec = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "instances/s", "cores": 1, "kind": "port", "sample": f"failed: {e}"}
    return {
        "value": rec["instances"] / rec["seconds"], "unit": "instances/s", "cores": 1, "kind": "port",
        "sample": (f"{rec['fleets']} C3 fleets (seeds 0..{rec['fleets'] - 1}) x 9 k = {rec['instances']} instances "
                   f"in {rec['seconds']:.1f} s; oracle/milp_oracle.py = reference lowering + scipy 1.15 HiGHS "
                   f"1.8.0 (the reference's arithmetic), pinned to 1 core"),
    }


def time_to_optimal(model, M: int, runs: int = 30):
    from distilp_amd.common import DeviceProfile
    from distilp_amd.solver import halda_solve
    from distilp_amd.synth import synth_fleet
    import contextlib
    import io

    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(0, M)]
    times = []
    for i in range(runs + 3):
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            halda_solve(devs, model, mip_gap=1e-4, plot=False, kv_bits="4bit")
        if i >= 3:
            times.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(times)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/*_pmc.json, written by tools/pmc_summary.py), or None when none covers this kernel."""
    cands = sorted((REPO / "profiles").glob("r*_pmc.json"))
    if not cands:
        return None
    try:
        rec = json.loads(cands[-1].read_text())
        return rec["kernels"][kernel]["hbm_bytes_per_launch"]
    except Exception:  # noqa: BLE001
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--fleets", type=int, default=4096, help="fleets per GPU per step")
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--copies", type=int, default=2, help="resident copies of the batch, used in turn")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ks", type=str, default="", help="diagnostic: comma-separated k-candidates instead of C3's")
    ap.add_argument("--cpu-baseline-child", action="store_true")
    args = ap.parse_args()
    if args.cpu_baseline_child:
        cpu_baseline_child(args.cpu_budget, args.M)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu_base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_base = run_cpu_baseline(args.cpu_budget, args.M)  # before any GPU work, in a child process

    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from distilp_amd.solver._libhalda import get_context

    t_setup = time.perf_counter()
    ks = [int(k) for k in args.ks.split(",")] if args.ks else None
    model, lowered, batch, refs = build_workload(rank, args.fleets, args.M, ks)
    # args.copies resident copies of the batch, used in turn: the bytes one step reads (~221 MB at C3)
    # times the copies exceed the 256 MiB Infinity Cache, so every step reads its inputs from HBM
    copies = [to_device(batch, torch, dev) for _ in range(args.copies)]
    keep, out = copies[0]
    ctx = get_context(local)
    stream = torch.cuda.Stream(dev)  # a real (non-null) stream: the kernels and the events share it
    cptrs = [({f: t.data_ptr() for f, t in k.items()}, {f: t.data_ptr() for f, t in o.items()}) for k, o in copies]
    turn = [0]
    setup_s = time.perf_counter() - t_setup

    def step():
        ptrs, optrs = cptrs[turn[0] % len(cptrs)]
        turn[0] += 1
        ctx.solve_device(ptrs, batch, optrs, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # sanity: statuses of this workload (k = 1 feasible, k > 1 infeasible when M > W)
    st = out["status"].cpu().numpy()
    n_opt, n_inf = int((st == 0).sum()), int((st == 2).sum())
    if n_opt + n_inf != batch.n_inst:
        raise RuntimeError(f"unexpected statuses: {np.unique(st, return_counts=True)}")

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ctx.set_timing(False)  # no per-launch instrumentation events inside the timed region
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    seq_ms = ev0.elapsed_time(ev1) / args.steps  # HIP events on the kernels' stream: whole launch sequence
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # per-launch device times (HIP events recorded by libhalda on the kernels' stream around each
    # launch), after the timed region; the dominant kernel is the longest of them
    ctx.set_timing(True)
    phases = []
    for _ in range(max(3, min(args.steps, 10))):
        step()
        torch.cuda.synchronize(dev)
        phases.append(ctx.last_phase_ms())
    phase_ms = {k: statistics.mean(p[k] for p in phases) for k in phases[0]}
    dom = max(phase_ms, key=phase_ms.get)

    total_inst = batch.n_inst * world * args.steps
    value = total_inst / elapsed
    alg_bytes = algorithmic_bytes(lowered, batch, refs)
    alg = alg_bytes.get(dom, batch.n_inst)  # the general kernel alone only scans the verdict bytes
    solve_ms = phase_ms[dom]
    achieved = alg / (solve_ms * 1e-3) / 1e9
    traffic = pmc_traffic(dom)
    if rank == 0:
        tto = time_to_optimal(model, args.M) if world == 1 else None
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "instances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded C3 fleets, distilp_amd/synth.py)",
            "config": {
                "workload": f"C3: {args.fleets} synthetic M={args.M} fleets x 9 k-candidates per GPU "
                            "(L=80, llama_3_70b/online, kv 4bit), one exact libhalda launch per step",
                "instances_per_step_per_gpu": batch.n_inst,
                "feasible_per_step_per_gpu": n_opt,
                "parallelism": f"dp{world} (fleets sharded, no collective on the data path)",
                "resident_copies": args.copies,
            },
            "feasible_instances_per_s": n_opt * world * args.steps / elapsed,
            "fleets_per_s": args.fleets * world * args.steps / elapsed,
            "time_to_optimal_ms": tto,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": dom,
                "kernel_ms": solve_ms,
                "algorithmic_bytes_per_launch": alg,
                "sequence_ms": seq_ms,
                "launch_ms": phase_ms,
                "algorithmic_bytes": alg_bytes,
            },
            "cpu_baseline": cpu_base,
            "setup_s": setup_s,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
