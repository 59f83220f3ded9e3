"""Benchmark: HALDA MILP instances solved/s on MI355X (config C3 of BASELINE.json).

Headline workload per GPU and step (weak scaling, the default): 4096 seeded synthetic fleets of M = 64
devices (L = 80, model llama_3_70b/online, kv "4bit"), each swept over all 9 k-candidates of L = 80 ->
36,864 fixed-k MILP instances, i.e. 4096 `halda_solve` k-sweeps. Every step takes the fleets' device-field
table (resident in HBM, 16 rotating copies > the Infinity Cache) through the whole reference path -- the
lowering of every (fleet, k) (halda_p_solver.py:59-338), the exact solves (:340-353) and the argmin over k
with the reference's tie rule (:391-414). The K timed steps are ONE group launch (halda_fleets_group_launch
-> halda_sweep_steps_kernel), bit-identical per batch to K launches (checked before timing).

The ONE JSON line (compact_line: <= 3.5 KB) carries beside the headline: the roofline of the headline's
launch (HBM and VALU issue), the CPU baseline (the oracle -- reference lowering + scipy / HiGHS 1.8.0 -- on
the host cores, pinned), the per-batch launches, latency mode, the C5 stream, the public batch API, the
milp() replacement on a pre-lowered CSR batch (solve_only), config C2 (4096 M = 16 fleets, k > 1 MILPs),
feasible-only instances/s and the time to optimal of one M = 64 halda_solve; DESIGN.md §5 defines each.
`--full-json PATH` writes the detailed record.

Multi-GPU: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run, before any GPU call in
this process) unless it already runs as one of them (WORLD_SIZE set, e.g. by the driver's own
torch.distributed.run); --gpus must equal the world size it sees and the node must have N GPUs, else it
exits with an error. Fleets are independent: no collective on the data path. Each rank times its own
region between a barrier and its device's synchronize; the max over ranks is reported (timed()).
"""

from __future__ import annotations

import argparse
import contextlib
import json
import math
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
# VALU-issue roof beside the HBM one: SIMD cycles per wave64 VALU instruction by type -- FP64
# add / mul / FMA 4 (16 FP64 lanes per cycle), FP64 transcendentals 8, every other VALU 2 (SIMD-32,
# MI355X_MICROARCH.md:54) -- on 1,024 SIMDs at <= 2.4 GHz. The counts per item are NOT constants here: they are
# read from the newest profiles/*_valu.json whose libhalda.so hash equals the library this process loads
# (tools/valu_stamp.py writes them from rocprofv3 SQ_INSTS_VALU and per-type SQ_INSTS_VALU_* passes); with no
# matching profile the VALU roof is reported as null.
VALU_CYCLES = {"fp64": 4, "trans_f64": 8, "other": 2}
N_SIMDS = 1024
CLOCK_GHZ = 2.4
KS_L80 = [1, 2, 4, 5, 8, 10, 16, 20, 40]
METRIC = "HALDA MILP instances solved/sec (node), M=64 devs L=80; time-to-optimal"
C3_FLEETS = 4096
MALL_BYTES = 256 << 20  # Infinity Cache: rotate enough resident copies that every step reads HBM


# ------------------------------------------------------------------ workload
def fleet_seeds(args, rank: int, world: int, strong: bool):
    if strong:
        from distilp_amd.distributed import shard_bounds

        lo, hi = shard_bounds(C3_FLEETS, rank, world)
        return list(range(lo, hi))
    return list(range(rank * args.fleets, (rank + 1) * args.fleets))


def build_fleets(seeds, M: int):
    from distilp_amd.common import DeviceProfile
    from distilp_amd.synth import load_templates, synth_fleet

    tpl = load_templates()
    return [[DeviceProfile.model_validate(d) for d in synth_fleet(s, M, tpl)] for s in seeds]


def load_model():
    from distilp_amd.common import ModelProfileSplit
    from distilp_amd.synth import load_model_dict

    return ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()


def build_workload(rank: int, fleets: int, M: int, ks=None):
    """(model, lowered fleets, CSR batch, refs) of rank `rank`'s weak-scaling fleets (diagnostic tools)."""
    from distilp_amd.solver.batch import assemble
    from distilp_amd.solver.lower import lower_fleet

    model = load_model()
    lowered = [lower_fleet(devs, model, "4bit") for devs in build_fleets(range(rank * fleets, (rank + 1) * fleets), M)]
    batch, refs = assemble(lowered, [list(ks or KS_L80)] * len(lowered))
    return model, lowered, batch, refs


# ------------------------------------------------------------------ algorithmic bytes
HDR = 4 + 4 + 8 + 8 + 8  # n_cols, n_rows, csr_off, col_off, row_off
RES = 4 + 8 + 8 + 8 + 8  # status, obj_lin, dual_bound, gap, nodes
DEV_FIELDS = 10 * 8 + 6 * 8 + 2  # FleetTable bytes per device (f64 x 10, int64 x 6, os_class, flags)


def algorithmic_bytes(lowered, refs, n_k: int, settled=None):
    """Bytes each launch must move, {kernel: bytes per launch}, for the lowered batch
    `lowered` (host lowering of the same fleets, one FleetMILP per fleet) and its instances `refs`.

    Solve (CSR) launches -- a solved (surviving) instance: its fleet's CSR once (row_ptr + col_idx/val,
    which contains the equality row), its header, c / col_lb / col_ub (8 B each) and integrality
    (1 B) per column, row_lb / row_ub per row, x out and the result scalars. A screened instance: its
    header, the equality row (two row_ptr entries, M col_idx/val, its row bounds), lb of its M
    w-columns, c[C] and the verdict byte, plus the result scalars when the screen settles it.
    k-sweep launches (halda_solve_fleets) -- lowering: the fleet's device fields in; out the CSR, the
    objective offsets and per instance its header plus, for W >= M, every column / row vector, for
    W < M (the screen settles it) the w bounds, the C column and the equality-row bounds; pick: per
    instance its status, per optimal instance its header, c and x, per fleet the offsets in and best k,
    obj_value and w / n out, obj_by_k / status when requested (not in the bench). `settled` (one flag per
    instance, halda_solve_batch_device_settled): a settled instance costs the screen its header, its flag,
    its verdict byte and the result scalars. halda_solve_k1_settled_kernel (a settled batch: no screen
    launch, the k = 1 kernel screens the unsettled instances on its way, whose screen reads are part of
    the solve's): the solve's bytes plus per instance its flag and verdict byte, and a settled instance's
    result scalars."""
    solve = screen = lower = pick = fused = 0
    fleets_seen, fleets_solved = set(), set()
    for i, ref in enumerate(refs):
        fl = lowered[ref.fleet]
        M, nc, nr = fl.M, fl.n_cols, fl.n_rows
        csr = 4 * (nr + 1) + 12 * fl.nnz
        scr = HDR + 1 + 1 if settled is not None and settled[i] else HDR + 8 + 12 * M + 16 + 8 * M + 8 + 1
        screen += scr
        fused += 2 + (RES if settled is not None and settled[i] else 0)
        if ref.fleet not in fleets_seen:
            fleets_seen.add(ref.fleet)
            lower += DEV_FIELDS * M + 8 + csr + 24
            pick += 24 + 4 + 8 + 8 * M
        lower += HDR
        pick += 4
        if ref.W - M >= 0:
            if ref.fleet not in fleets_solved:  # a solved fleet's CSR is read once per launch
                fleets_solved.add(ref.fleet)
                solve += csr
            one = HDR + 25 * nc + 16 * nr + 8 * nc + RES
            solve += one
            lower += 25 * nc + 16 * nr
            pick += HDR + 16 * nc
        else:
            screen += RES
            lower += 16 * M + 25 + 16
    # fused k-sweep (no CSR): device fields in, per fleet best k / obj_value / w / n out -- the first
    # launch (register or lane-segment kernel), or the table kernel when it runs the whole batch alone
    # (as the dominant launch it does; as the gated second launch it only redoes flagged fleets)
    sweep = sum(DEV_FIELDS * fl.M + 8 + 4 + 8 + 8 * fl.M for fl in lowered)
    return {"halda_screen_kernel": screen, "halda_solve_k1_kernel": solve, "halda_solve_k1_settled_kernel": solve + fused,
            "halda_lower_kernel": lower, "halda_pick_kernel": pick, "halda_sweep_kernel": sweep,
            "halda_sweep_seg_kernel": sweep, "halda_sweep_tables_kernel": sweep}


# ------------------------------------------------------------------ CPU baseline
def cpu_baseline_child(budget_s: float, M: int, core: int, first: int, count: int) -> None:
    """One pinned process: the oracle (reference lowering + scipy HiGHS) on C3 fleets first ..
    first+count-1 until the time budget is used; prints one JSON line."""
    os.sched_setaffinity(0, {core})
    from oracle import milp_oracle as mo

    model = load_model()
    fleets = build_fleets(range(first, first + count), M)
    t0 = time.perf_counter()
    n_inst = n_fleets = 0
    while time.perf_counter() - t0 < budget_s and n_fleets < len(fleets):
        mo.halda_solve_oracle(fleets[n_fleets], model, k_candidates=KS_L80, mip_gap=1e-4, kv_bits="4bit",
                              solver="highs")
        n_fleets += 1
        n_inst += len(KS_L80)
    print(json.dumps({"instances": n_inst, "fleets": n_fleets, "seconds": time.perf_counter() - t0}))


def usable_cores():
    """Cores this process may run on: its affinity set, capped by the cgroup CPU quota and by the CPU
    share the GPU box states in OMP_NUM_THREADS (there nproc shows the whole machine)."""
    cores = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    if quota is not None:
        cores = cores[:quota]
    share = os.environ.get("OMP_NUM_THREADS")  # the GPU box states the job's CPU share here (16)
    if share and share.isdigit() and int(share) > 0:
        cores = cores[:int(share)]
    return cores, quota


def run_cpu_baseline(budget_s: float, M: int):
    """All usable cores (one pinned oracle process each, disjoint fleets), then one core alone."""
    cores, quota = usable_cores()
    per = int(budget_s * 40) + 16  # fleets prepared per process (> budget_s of HiGHS work on one core)

    def spawn(core, first):
        return subprocess.Popen([sys.executable, str(Path(__file__).resolve()), "--cpu-baseline-child",
                                 "--cpu-budget", str(budget_s), "--M", str(M), "--cpu-core", str(core),
                                 "--cpu-first", str(first), "--cpu-count", str(per)],
                                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)

    def collect(procs):
        recs = []
        for p in procs:
            out, err = p.communicate(timeout=budget_s * 6 + 300)
            if p.returncode != 0:
                raise RuntimeError(f"cpu baseline child failed: {err[-400:]}")
            recs.append(json.loads(out.strip().splitlines()[-1]))
        return recs

    try:
        allc = collect([spawn(c, i * per) for i, c in enumerate(cores)])
        one = collect([spawn(cores[0], 0)])[0]
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "instances/s", "cores": len(cores), "kind": "port", "sample": f"failed: {e}"}
    inst = sum(r["instances"] for r in allc)
    secs = max(r["seconds"] for r in allc)
    return {
        "value": inst / secs, "unit": "instances/s", "cores": len(cores), "kind": "port",
        "nproc": os.cpu_count(), "cgroup_cpu_quota": quota,
        "one_core_value": one["instances"] / one["seconds"],
        "sample": (f"{len(cores)} pinned procs x ~{budget_s:.0f} s, own C3 fleets: {sum(r['fleets'] for r in allc)} "
                   f"fleets x 9 k in {secs:.1f} s; oracle/milp_oracle.py (reference lowering + HiGHS 1.8.0)"),
    }


# ------------------------------------------------------------------ GPU legs
HOST_ENQUEUE = {}  # per timed leg: host seconds to enqueue its K steps (before the final synchronize)


class Ranks:
    """The ranks of one bench job: `sync` waits for this rank's device, `barrier` / `max` / `min` are the
    collectives (no-ops at world 1). The reductions run on the device for RCCL, on the host for gloo."""

    def __init__(self, dist, world: int, sync, device=None):
        self.dist, self.world, self.sync, self.device = dist, world, sync, device

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if self.world == 1:
            return x
        import torch

        on = self.device if self.dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=on)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX if self.world > 1 else None)

    def min(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MIN if self.world > 1 else None)


def timed(step, steps, R: Ranks, tag=None, many=None, on_stream=None):
    """Seconds for `steps` steps, max over ranks. Every rank leaves a barrier, waits for its device, reads
    the clock, enqueues the steps, waits for its device and reads the clock again: its own elapsed time,
    taken BEFORE any collective, so neither the closing collective nor a late rank's barrier exit is
    inside the region; then the all-reduce MAX. `many`, when given, enqueues all steps in one call (one
    ctypes call); else step() runs `steps` times. `on_stream` = (torch, stream): HIP events recorded on
    that stream around the steps as well; returns (seconds, event ms of this rank) then."""
    R.barrier()
    R.sync()
    ev = None
    if on_stream is not None:
        torch_, stream = on_stream
        ev = (torch_.cuda.Event(enable_timing=True), torch_.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    if ev:
        ev[0].record(stream)
    if many is not None:
        many(steps)
    else:
        for _ in range(steps):
            step()
    if ev:
        ev[1].record(stream)
    if tag:
        HOST_ENQUEUE[tag] = time.perf_counter() - t0
    R.sync()
    elapsed = time.perf_counter() - t0
    elapsed = R.max(elapsed)
    if ev:
        return elapsed, ev[0].elapsed_time(ev[1])
    return elapsed


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


def lib_sha256() -> str:
    """sha256 of the libhalda.so this process loads (keys the VALU-count profiles to a build)."""
    import hashlib

    from distilp_amd.solver._libhalda import LIB_PATH

    return hashlib.sha256(Path(LIB_PATH).read_bytes()).hexdigest()


def valu_profile(kernel: str, workload: str):
    """{valu_per_wave, waves, ...} of `kernel` on `workload` ("c3" / "c2") from the newest
    profiles/*_valu.json (tools/valu_stamp.py) recorded for THIS libhalda.so build, else None."""
    sha = lib_sha256()
    for c in sorted((REPO / "profiles").glob("r*_valu.json"), reverse=True):
        try:
            j = json.loads(c.read_text())
            if j.get("libhalda_sha256") != sha:
                continue
            e = j["workloads"][workload][kernel]
            return dict(e, source=f"profiles/{c.name}")
        except Exception:  # noqa: BLE001
            continue
    return None


def valu_issue(vp, units: int, ms: float):
    """VALU-issue roof of a launch of `units` items (or waves, for a per-batch kernel profile) that took
    `ms`: the SIMD cycles its VALU instructions need at the peak clock over the SIMD cycles available.
    Priced by type from the build's per-type counters: FP64 add / mul / FMA at 4 cycles per wave64
    instruction (16 FP64 lanes per cycle per SIMD: 78.6 TF), FP64 transcendentals at 8, every other
    VALU at 2 (SIMD-32, MI355X_MICROARCH.md:54); `frac_all_at_4` prices every VALU at 4 (one wave alone
    per SIMD, or every uncounted op on the FP64 pipe), the bound this roof was quoted at before round 6."""
    if not vp:
        return {"frac": None, "why": "no profiles/*_valu.json recorded for this libhalda.so build"}
    per = vp["valu_per_wave"] * vp["waves"] / vp.get("items", vp["waves"])  # VALU per unit
    simd_cycles = N_SIMDS * CLOCK_GHZ * 1e9 * ms * 1e-3
    out = {"valu_per_item": per, "frac_all_at_4": per * units * 4 / simd_cycles,
           "wait_any_frac": vp.get("wait_any_frac"), "source": vp["source"]}
    t = vp.get("valu_types")
    if t:
        scale = vp["waves"] / vp.get("items", vp["waves"])
        fp64 = (t["add_f64"] + t["mul_f64"] + t["fma_f64"]) * scale
        trans = t["trans_f64"] * scale
        other = per - fp64 - trans
        out.update(fp64_per_item=fp64, fp64_trans_per_item=trans, other_per_item=other,
                   frac=(VALU_CYCLES["fp64"] * fp64 + VALU_CYCLES["trans_f64"] * trans + VALU_CYCLES["other"] * other)
                   * units / simd_cycles)
    else:
        out["frac"] = None
        out["why"] = "no per-type VALU pass for this build (profiles/run_round.sh)"
    return out


def roofline(phase_ms, alg_bytes, traffic_fn, one_launch_ms=None, workload="c3"):
    """Roofline of the dominant launch. phase_ms: per-launch device times (HIP events around each
    launch, one launch at a time). one_launch_ms: when every step is that one launch, its mean time
    from HIP events around K back-to-back launches on ONE stream (no per-launch instrumentation, no
    overlap with another batch). Two roofs are reported as peers: HBM (algorithmic bytes / kernel time /
    8 TB/s) and FP64-VALU issue (profiled VALU per wave x waves x 4 cycles / (1,024 SIMDs x 2.4 GHz x
    kernel time)); `bound` keeps the contract's vocabulary (the kernel's memory roof), `nearest_roof`
    names the larger fraction."""
    dom = max(phase_ms, key=phase_ms.get)
    alg = alg_bytes.get(dom)
    single = one_launch_ms is not None and single_launch_steps(phase_ms)
    ms = one_launch_ms if single else phase_ms[dom]
    achieved = alg / (ms * 1e-3) / 1e9 if alg else None
    frac = achieved / HBM_PEAK_GBS if achieved else None
    vp = valu_profile(dom, workload)
    valu = valu_issue(vp, vp["waves"] if vp else 0, ms)
    roofs = {"hbm": frac, "valu_issue": valu["frac"]}
    nearest = max((k for k, v in roofs.items() if v is not None), key=lambda k: roofs[k], default=None)
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": frac,
            "traffic": traffic_fn(dom), "kernel": dom, "kernel_ms": ms,
            "kernel_ms_from": ("HIP events around K back-to-back launches on one stream" if single
                               else "HIP events around each launch"),
            "algorithmic_bytes_per_launch": alg, "roofs": roofs, "nearest_roof": nearest, "valu_issue": valu,
            "launch_ms": phase_ms}


def group_roofline(launch_ms, steps, batch_bytes, n_fleets, single, kern="halda_sweep_steps_kernel",
                   workload="c3_steps"):
    """Roofline of the headline's launch as launched: ONE halda_sweep_steps_kernel launch of `steps`
    batches, algorithmic bytes = steps x one batch's, time = HIP events around that launch
    on its stream; HBM traffic and the VALU count from this build's rocprofv3 profiles (per launch of
    the same K). `single` (the per-batch kernel's own roofline, one launch per batch) is kept beside it."""
    alg = steps * batch_bytes
    achieved = alg / (launch_ms * 1e-3) / 1e9
    vp = valu_profile(kern, workload)
    valu = valu_issue(vp if vp and vp.get("items") else None, steps * n_fleets, launch_ms)
    per_batch = pmc_entry(kern, "hbm_bytes_per_batch")
    traffic = per_batch * steps if per_batch is not None else None  # HBM bytes scale with the batches
    roofs = {"hbm": achieved / HBM_PEAK_GBS, "valu_issue": valu["frac"]}
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic, "kernel": kern, "kernel_ms": launch_ms,
            "kernel_ms_from": "HIP events around one launch of K batches on its stream (median of 3)",
            "steps_per_launch": steps, "algorithmic_bytes_per_launch": alg, "algorithmic_bytes_per_batch": batch_bytes,
            "roofs": roofs, "nearest_roof": max((k for k, v in roofs.items() if v is not None), key=lambda k: roofs[k]),
            "valu_issue": valu, "single_batch_kernel": single}


def single_launch_steps(phase_ms):
    dom = max(phase_ms, key=phase_ms.get)
    return all(v < 1e-3 for k, v in phase_ms.items() if k != dom)


def sweep_bytes(table) -> int:
    """Algorithmic bytes of one fused k-sweep launch over `table`: per fleet its device
    fields (130 B per device) and dev_off (8 B) in; best k (4 B), obj_value (8 B) and w / n (8 B per
    device) out."""
    sizes = table.sizes()
    return int(sum(DEV_FIELDS * int(m) + 8 + 4 + 8 + 8 * int(m) for m in sizes))


def timed_events(step, steps, torch, dev, stream, many=None):
    """Device time per step of `steps` launches on `stream`, from HIP events recorded on that stream."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    e0.record(stream)
    if many is not None:
        many(steps)
    else:
        for _ in range(steps):
            step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / steps


def pmc_entry(kernel, field):
    """`field` of `kernel` in the newest committed rocprofv3 PMC summary (profiles/*_pmc.json, written by
    tools/pmc_summary.py) recorded for THIS libhalda.so build (its libhalda_sha256), or None when none
    covers this kernel and build."""
    sha = lib_sha256()
    for c in sorted((REPO / "profiles").glob("r*_pmc.json"), reverse=True):
        try:
            j = json.loads(c.read_text())
            if j.get("libhalda_sha256") != sha:
                continue
            return j["kernels"][kernel][field]
        except Exception:  # noqa: BLE001
            continue
    return None


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` (pmc_entry)."""
    return pmc_entry(kernel, "hbm_bytes_per_launch")


def time_to_optimal(model, M: int, runs: int = 100):
    """Median wall ms of one M = 64 halda_solve (Python call -> HALDAResult), and its parts, each the
    median of `runs` calls of that part alone (so they need not add up exactly): `pack` the C packer
    (DeviceProfile objects -> the fleet's field table), `gpu_call` the synchronous libhalda call
    (halda_solve_fleets_host: table across PCIe, the k-sweep kernel, results back) and the objective
    constants, `rest` the total's median minus those two (k list, per-k results with NumPy's c.x, the
    pick and HALDAResult). `gpu_call_copy_path`: the same call through explicit H2D / D2H copies instead
    of the kernel reading and writing pinned host memory (a second context, HALDA_HOST_PATH=copy)."""
    import contextlib
    import io

    from distilp_amd.solver import halda_solve
    from distilp_amd.solver._libhalda import HaldaContext
    from distilp_amd.solver.fleets import _bind, model_struct, pack_one, sweep_one

    devs = build_fleets([0], M)[0]

    def med(fn):
        ts = []
        for i in range(runs + 5):
            t0 = time.perf_counter()
            fn()
            if i >= 5:
                ts.append((time.perf_counter() - t0) * 1e3)
        return statistics.median(ts)

    def one():
        with contextlib.redirect_stdout(io.StringIO()):
            halda_solve(devs, model, mip_gap=1e-4, plot=False, kv_bits="4bit")

    total = med(one)
    ks = KS_L80
    pack = med(lambda: pack_one(devs, model, ks))
    ws = pack_one(devs, model, ks)
    call = med(lambda: sweep_one(ws, model, 0.5))
    parts = {"pack_ms": pack, "gpu_call_ms": call, "rest_ms": total - pack - call}
    import ctypes

    os.environ["HALDA_HOST_PATH"] = "copy"
    try:
        ctx2 = HaldaContext(0)
    finally:
        os.environ.pop("HALDA_HOST_PATH", None)
    lib = _bind(ctx2.lib)
    m = model_struct(model, 0.5)

    def copy_call():
        rc = lib.halda_solve_fleets_host(ctx2.ctx, ctypes.byref(m), ctypes.byref(ws.fs), ws.karr.ctypes.data,
                                         len(ws.ks), ctypes.byref(ws.res))
        if rc != 0:
            raise RuntimeError("copy-path call failed")

    parts["gpu_call_copy_path_ms"] = med(copy_call)
    ctx2.close()
    return total, parts


def batch_api(model, fleets, runs: int = 3):
    """The public throughput API end to end: halda_solve_batch on the C3 fleets (a list of 4096
    DeviceProfile lists -> 4096 HALDAResult): packing, ONE fused k-sweep (PCIe in / out), the host-formed
    objectives. Median wall time of `runs` calls; the answers checked against one halda_solve."""
    import contextlib
    import io

    from distilp_amd.solver import halda_solve, halda_solve_batch

    times = []
    out = None
    for _ in range(runs + 1):
        t0 = time.perf_counter()
        out = halda_solve_batch(fleets, model, mip_gap=1e-4, kv_bits="4bit")
        times.append((time.perf_counter() - t0) * 1e3)
    with contextlib.redirect_stdout(io.StringIO()):
        one = halda_solve(fleets[0], model, mip_gap=1e-4, plot=False, kv_bits="4bit")
    if (out[0].k, out[0].w, out[0].n, out[0].obj_value) != (one.k, one.w, one.n, one.obj_value):
        raise RuntimeError("halda_solve_batch disagrees with halda_solve")
    return {"ms": statistics.median(times[1:]), "fleets_per_s": len(fleets) / (statistics.median(times[1:]) * 1e-3)}


def c5_stream(model, M: int, batches: int = 8, B: int = C3_FLEETS):
    """Config C5 (BASELINE.json configs[4]) end to end from the host: a base fleet (seed 0) re-profiled
    per instance (every numeric device field x LU(0.9, 1.1), FleetTable.perturbed), batches of B
    instances through halda_solve_fleets_host (PCIe in, the k-sweep, PCIe out), one at a time.
    The re-profiled tables are the stream's input, made before the timed loop (the host RNG that stands in
    for new profiles arriving, `reprofile_ms` per batch, is no part of the solve)."""
    from dataclasses import replace

    from distilp_amd.solver.fleets import F64_FIELDS, BYTE_FIELDS, fleet_table, solve_table

    base = fleet_table(build_fleets([0], M), model)
    big = replace(base, dev_off=np.arange(B + 1, dtype=np.int64) * M,
                  **{f: np.tile(getattr(base, f), B) for f in ("os_class", "flags") + F64_FIELDS + BYTE_FIELDS})
    rng = np.random.default_rng(10_000)
    solve_table(big.perturbed(rng), model, KS_L80, 0.5)  # warm-up
    t0 = time.perf_counter()
    tabs = [big.perturbed(rng) for _ in range(batches)]
    t_in = (time.perf_counter() - t0) / batches
    t0 = time.perf_counter()
    for t in tabs:
        res = solve_table(t, model, KS_L80, 0.5)
        if not (res.best_k > 0).all():
            raise RuntimeError("C5: a re-profiled fleet without a feasible k")
    dt = (time.perf_counter() - t0) / batches
    return {"ms_per_batch": dt * 1e3, "fleets_per_s": B / dt, "instances_per_s": B * len(KS_L80) / dt,
            "reprofile_ms": t_in * 1e3}


def c2_leg(args, torch, dev, ctx, model, stream, srefs):
    """Config C2 (BASELINE.json configs[1]) as its own leg: 4096 synthetic M = 16 fleets x every k of
    L = 80 (k = 1, 2, 4, 5 feasible: the k > 1 MILPs of halda_p_solver.py:391-412 are solved here), one
    k-sweep per step from resident tables: the K steps as ONE group launch (the k-slot form:
    halda_sweep_kslot_steps_kernel + the gated table launch), beside it as K launches over two streams and
    over one stream; its own roofline from the per-batch k-slot launch time."""
    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup, PlanRotation, fleet_table

    M2 = 16
    table = fleet_table(build_fleets(range(C3_FLEETS), M2), model)
    n = max(2, min(32, math.ceil(2 * MALL_BYTES / max(DeviceFleetTable(table, model, KS_L80, 0.5, dev).nbytes(), 1))))
    # the timed steps return what a halda_solve returns per fleet (best k, obj_value, w, n), as the C3
    # headline does; the per-k statuses are read once from a probe copy
    tabs = [DeviceFleetTable(table, model, KS_L80, 0.5, dev) for _ in range(n)]
    probe = DeviceFleetTable(table, model, KS_L80, 0.5, dev, want_per_k=True)
    for t in tabs:
        t.plan(ctx)
    turn = [0]
    rot2, rot1 = PlanRotation(tabs, ctx, srefs), PlanRotation(tabs, ctx, [stream.cuda_stream])

    def many2(k):
        rot2.launch(turn[0], k)
        turn[0] += k

    def many1(k):
        rot1.launch(turn[0], k)
        turn[0] += k

    def step2():
        tabs[turn[0] % n].launch(ctx, srefs[turn[0] % len(srefs)])
        turn[0] += 1

    def step1():
        tabs[turn[0] % n].launch(ctx, stream.cuda_stream)
        turn[0] += 1

    ctx.set_timing(False)
    # warm every stream the leg uses with the leg's own launch (each stream's scratch slot is grown to
    # this batch here, not inside a timed region)
    for _ in range(max(2, args.warmup)):
        step1()
    for _ in range(2 * len(srefs)):
        step2()
    probe.launch(ctx, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    st = probe.out["status"].cpu().numpy()
    n_opt = int((st == 0).sum())
    if not np.array_equal(probe.out["best_k"].cpu().numpy(), tabs[0].out["best_k"].cpu().numpy()):
        raise RuntimeError("C2: the probe copy disagrees with the timed copies")
    bk = tabs[(turn[0] - 1) % n].out["best_k"].cpu().numpy()
    if not (bk > 0).all():
        raise RuntimeError("C2: a fleet without a feasible k")
    steps = args.steps
    alg = sweep_bytes(table)
    group = PlanGroup(tabs, ctx)

    def manyg(k):
        group.launch(turn[0], k, stream.cuda_stream)
        turn[0] += k

    manyg(steps)  # warm
    torch.cuda.synchronize(dev)
    R1 = Ranks(None, 1, lambda: torch.cuda.synchronize(dev))
    elg = timed(None, steps, R1, many=manyg)
    evg = statistics.median(timed_events(None, 1, torch, dev, stream, many=lambda _: manyg(steps)) for _ in range(3))
    el2 = timed(step2, steps, R1, many=many2)
    ev1 = timed_events(step1, steps, torch, dev, stream, many=many1)
    ctx.set_timing(True)
    per = []
    for _ in range(5):
        step1()
        torch.cuda.synchronize(dev)
        per.append(ctx.last_fleet_ms())
    ctx.set_timing(False)
    ph = {k: statistics.mean(p.get(k, 0.0) for p in per) for k in per[0]}
    inst = C3_FLEETS * len(KS_L80)
    return {
        "instances_per_step": inst, "feasible_per_step": n_opt,
        "ms_per_step": elg / steps * 1e3, "instances_per_s": inst * steps / elg,
        "ms_per_batch_events": evg / steps, "group_persistent": group.persistent,
        "ms_per_step_one_stream": ev1, "ms_per_step_two_streams": el2 / steps * 1e3,
        "steps": steps, "resident_copies": n,
        "roofline": group_roofline(evg, steps, alg, C3_FLEETS,
                                   roofline(ph, {k: alg for k in ph}, pmc_traffic,
                                            ev1 if single_launch_steps(ph) else None, workload="c2"),
                                   kern="halda_sweep_kslot_steps_kernel", workload="c2_steps"),
    }


@contextlib.contextmanager
def stdout_to_stderr():
    """File descriptor 1 sent to fd 2 for the block (native libraries that print to stdout: RCCL's banner,
    gloo's connection lines), so that the bench's stdout holds its JSON line alone."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def latency_leg(torch, dev, ctx, model, stream, runs: int = 50):
    """Latency mode (halda_p_solver.py:391-412 is the k loop it shards): the k-sweep of
    one C2 fleet and of 4096 C2 fleets through halda_solve_fleets_sharded over a real one-rank RCCL
    communicator (the three device all-reduces and the shard kernels included) against the plain
    sweep, and the same step sequence for 2 / 4 / 8 virtual ranks on this one GPU
    (halda_solve_fleets_sharded_emulated: every rank's sub-sweep runs here one after another and each
    all-reduce is a device reduction, so it prices the extra launches, not an 8-GPU latency). Per
    call: device ms from HIP events around `runs` back-to-back calls on one stream, and the wall ms
    of one synchronous call (enqueue -> results on the device, median)."""
    from distilp_amd.solver.fleets import (DeviceFleetTable, RcclComm, fleet_table, launch_sharded,
                                           launch_sharded_emulated)

    out = {}
    try:
        with stdout_to_stderr():  # RCCL prints its version banner on stdout: keep stdout the one JSON line
            comm = RcclComm(1, 0, RcclComm.unique_id(), dev.index or 0)
    except Exception as e:  # noqa: BLE001
        comm = None
        out["rccl_error"] = str(e)[:200]
    sref = stream.cuda_stream
    for name, n in (("one_fleet", 1), ("fleets_4096", C3_FLEETS)):
        table = fleet_table(build_fleets(range(50_000, 50_000 + n), 16), model)
        dt = DeviceFleetTable(table, model, KS_L80, 0.5, dev)
        ways = {"plain": lambda: dt.launch(ctx, sref)}
        if comm is not None:
            ways["rccl_world1"] = lambda: launch_sharded(dt, ctx, comm, sref)
        for w in (2, 4, 8):
            ways[f"emulated_world{w}"] = (lambda w=w: launch_sharded_emulated(dt, ctx, w, 0, sref))
        rec = {}
        for way, fn in ways.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize(dev)
            ev = timed_events(fn, runs, torch, dev, stream)
            walls = []
            for _ in range(min(runs, 30)):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize(dev)
                walls.append((time.perf_counter() - t0) * 1e3)
            rec[way] = {"device_ms_per_call": ev, "wall_ms_sync_call": statistics.median(walls)}
        # the critical path a rank of a real world-w node would have: the plain sweep of its own k's alone
        for w in (2, 4, 8):
            per_rank = []
            for r in range(w):
                sub = KS_L80[r::w]
                if not sub:
                    continue
                ds = DeviceFleetTable(table, model, sub, 0.5, dev)
                for _ in range(3):
                    ds.launch(ctx, sref)
                per_rank.append(timed_events(lambda: ds.launch(ctx, sref), runs, torch, dev, stream))
            rec[f"rank_subsweep_world{w}"] = {"max_device_ms": max(per_rank), "per_rank_device_ms": per_rank}
        out[name] = rec
    if comm is not None:
        comm.close()
    return out


def _g(x, n: int = 5):
    """x rounded to n significant digits (the compact line), None and non-floats unchanged."""
    return float(f"{x:.{n}g}") if isinstance(x, float) else x


def _pick(d, *keys, n: int = 5):
    return None if d is None else {k: _g(d.get(k), n) for k in keys if d.get(k) is not None}


def compact_line(full: dict) -> dict:
    """The ONE JSON line the bench prints (<= 3.5 KB, so a driver that keeps the last ~4 KB of stdout keeps
    all of it): the contract's keys first, then each leg's figures, the figures BASELINE's metric names
    last -- the C5 stream, the batch API, the milp() replacement, C2, feasible-only instances/s and the
    time to optimal. Every field is defined in DESIGN.md §5; `--full-json` writes the detailed record."""
    rf = full["roofline"]
    vi = rf.get("valu_issue") or {}
    sb = rf.get("single_batch_kernel") or {}
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup")}
    line["ms_per_step"] = _g(full["ms_per_step"], 6)
    line.update({k: full[k] for k in ("higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")})
    line["roofline"] = dict(
        {k: _g(rf.get(k)) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms",
                                     "steps_per_launch")},
        alg_bytes_per_launch=rf.get("algorithmic_bytes_per_launch"),
        valu_issue=_pick(vi, "frac", "frac_all_at_4", "valu_per_item", "fp64_per_item", "fp64_trans_per_item",
                         "other_per_item", "wait_any_frac", n=3),
        single_batch={"kernel": sb.get("kernel"), "kernel_ms": _g(sb.get("kernel_ms")), "frac": _g(sb.get("frac"), 3)})
    cb = full.get("cpu_baseline")
    line["cpu_baseline"] = None if cb is None else dict(
        _pick(cb, "value", "unit", "cores", "kind", "one_core_value", "nproc"), sample=cb.get("sample"))
    line["rank_launch_ms"] = _pick(full.get("rank_launch_ms"), "max", "min")
    line["weak_200"] = _pick(full.get("weak_200"), "ms_per_step", "instances_per_s")
    line["strong"] = _pick(full.get("strong"), "fleets_total", "ms_per_step", "instances_per_s")
    line["per_launch_ms_per_step"] = _g(full["per_launch"]["ms_per_step"])
    line["one_stream_ms_per_step"] = _g(full["one_stream"]["ms_per_step"])
    line["host_enqueue_ms_per_step"] = _g(full["host_enqueue_ms_per_step"], 3)
    lat = full.get("latency_mode")
    if lat:
        line["latency_mode_device_ms"] = {
            name: dict({way: _g(lat[name][way]["device_ms_per_call"], 4) for way in ("plain", "rccl_world1")
                        if way in lat[name]},
                       world8_rank_max=_g(lat[name]["rank_subsweep_world8"]["max_device_ms"], 4))
            for name in ("one_fleet", "fleets_4096") if name in lat}
    line["fleets_per_s"] = _g(full["fleets_per_s"])
    line["c5_stream"] = _pick(full.get("c5_stream"), "instances_per_s", "reprofile_ms", "ms_per_batch")
    line["batch_api"] = _pick(full.get("batch_api"), "fleets_per_s", "ms")
    so = full["solve_only"]
    line["solve_only"] = dict(
        _pick(so, "ms_per_step_one_stream", "ms_per_step_no_settled"),
        roofline=_pick(so["roofline"], "kernel", "kernel_ms", "traffic", "frac"), ms_per_step=_g(so["ms_per_step"]))
    c2 = full.get("c2")
    line["c2"] = None
    if c2:
        r2 = c2["roofline"]
        line["c2"] = dict(_pick(c2, "ms_per_batch_events", "ms_per_step_two_streams", "instances_per_s"),
                          roofline=dict(_pick(r2, "kernel_ms", "traffic"),
                                        valu_issue_frac=_g((r2.get("valu_issue") or {}).get("frac"), 3),
                                        frac=_g(r2.get("frac"))),
                          ms_per_step=_g(c2["ms_per_step"]))
    line["feasible_instances_per_s"] = _g(full["feasible_instances_per_s"])
    line["time_to_optimal_parts"] = _pick(full.get("time_to_optimal_parts"), "pack_ms", "gpu_call_ms", "rest_ms",
                                          "gpu_call_copy_path_ms", n=3)
    line["time_to_optimal_ms"] = _g(full.get("time_to_optimal_ms"))
    return line


def launch_ranks(args) -> int:
    """--gpus N from a plain `python bench.py`: start N ranks (one process per GPU) with
    torch.distributed.run before this process touches the GPU, relay their output and exit code."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--fleets", type=int, default=C3_FLEETS, help="fleets per GPU per step (weak scaling)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="headline: weak (fleets per GPU fixed) or strong (4096 fleets in total)")
    ap.add_argument("--streams", type=int, choices=(1, 2, 3, 4), default=2,
                    help="streams the k-sweep steps alternate over (1: every launch serialised, e.g. for "
                         "per-dispatch profiling)")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl", help=argparse.SUPPRESS)
    ap.add_argument("--share-gpu", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--copies", type=int, default=0, help="resident copies per leg (0: enough to exceed the MALL)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-tto", action="store_true")
    ap.add_argument("--no-c2", action="store_true", help="skip the config-2 leg (4096 M = 16 fleets)")
    ap.add_argument("--no-latency", action="store_true", help="skip the latency-mode leg")
    ap.add_argument("--ks", type=str, default="", help="diagnostic: comma-separated k-candidates instead of C3's")
    ap.add_argument("--full-json", type=str, default="",
                    help="also write the detailed record (every leg's figures, per-launch times) to this file")
    ap.add_argument("--cpu-baseline-child", action="store_true")
    ap.add_argument("--cpu-core", type=int, default=0)
    ap.add_argument("--cpu-first", type=int, default=0)
    ap.add_argument("--cpu-count", type=int, default=64)
    args = ap.parse_args()
    if args.cpu_baseline_child:
        cpu_baseline_child(args.cpu_budget, args.M, args.cpu_core, args.cpu_first, args.cpu_count)
        return 0

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return launch_ranks(args)
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        return 2

    cpu_base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_base = run_cpu_baseline(args.cpu_budget, args.M)  # before any GPU work, in child processes

    import torch
    import torch.distributed as dist

    n_dev = torch.cuda.device_count()
    if args.share_gpu:  # diagnostic: every rank on GPU 0 (exercises the multi-rank path on a 1-GPU box)
        local = 0
    elif n_dev < world or local >= n_dev:
        print(f"bench.py: --gpus {args.gpus} needs {world} GPUs on this node, {n_dev} visible", file=sys.stderr)
        return 2
    rccl_world = 1
    torch.cuda.set_device(local)  # before the process group: its barriers run on this rank's GPU
    dev = torch.device("cuda", local)
    if world > 1:
        with stdout_to_stderr():
            if args.backend == "nccl":
                dist.init_process_group("nccl", init_method="env://", device_id=dev)
            else:
                dist.init_process_group("gloo", init_method="env://")
            dist.barrier()  # the backends connect (and print) on first use
        rccl_world = dist.get_world_size()
        if rccl_world != args.gpus:
            print(f"bench.py: RCCL world size {rccl_world} != --gpus {args.gpus}", file=sys.stderr)
            return 2

    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.batch import assemble, settled_instances
    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup, PlanRotation, fleet_table
    from distilp_amd.solver.lower import lower_fleet

    t_setup = time.perf_counter()
    ks = [int(k) for k in args.ks.split(",")] if args.ks else KS_L80
    model = load_model()
    strong_head = args.scaling == "strong"
    seeds = fleet_seeds(args, rank, world, strong_head)
    fleets = build_fleets(seeds, args.M)
    table = fleet_table(fleets, model)
    ctx = get_context(local)
    stream = torch.cuda.Stream(dev)
    sref = stream.cuda_stream
    # the k-sweep steps alternate between two streams: consecutive batches are independent (own
    # tables and results), so one batch's field loads overlap the previous batch's compute tail
    extra = [torch.cuda.Stream(dev) for _ in range(args.streams - 1)]
    srefs = [sref] + [x.cuda_stream for x in extra]

    # ---- headline: the k-sweep from resident device-field tables (rotating copies > the MALL)
    tbytes = DeviceFleetTable(table, model, ks, 0.5, dev).nbytes()
    n_sw = args.copies or max(2, min(32, math.ceil(2 * MALL_BYTES / max(tbytes, 1))))
    sweeps = [DeviceFleetTable(table, model, ks, 0.5, dev) for _ in range(n_sw)]
    turn = [0, 0]  # per leg: which resident copy the next step reads

    def sweep_step():
        sweeps[turn[0] % n_sw].launch(ctx, srefs[turn[0] % len(srefs)])
        turn[0] += 1

    def sweep_step_one_stream():
        sweeps[turn[0] % n_sw].launch(ctx, sref)
        turn[0] += 1

    # the timed regions enqueue their steps from C (the same launches, the same rotation over the
    # resident copies and streams as the step functions above)
    rot2, rot1, group = None, None, None

    def sweep_group(k):
        # the headline: K batches (copy (turn + t) % n_sw each) in ONE launch on one stream
        # (halda_fleets_group_launch: one wave per (batch, fleet) item)
        group.launch(turn[0], k, sref)
        turn[0] += k

    def sweep_many(k):
        rot2.launch(turn[0], k)
        turn[0] += k

    def sweep_many_one_stream(k):
        rot1.launch(turn[0], k)
        turn[0] += k

    # ---- solve-only leg: the same fleets lowered on the host, CSR batch resident in HBM
    lowered = [lower_fleet(devs, model, "4bit") for devs in fleets]
    batch, refs = assemble(lowered, [ks] * len(lowered))
    n_so = args.copies or 2
    copies = [to_device(batch, torch, dev) for _ in range(n_so)]
    cptrs = [({f: t.data_ptr() for f, t in k.items()}, {f: t.data_ptr() for f, t in o.items()}) for k, o in copies]
    # the lowering's own verdicts: the bound-infeasible k's (M > W = L / k), computed with the lowering
    # (set-up, like the CSR) and handed to halda_solve_batch_device_settled, which then reads none of
    # their rows; every step still writes all results
    settled = settled_instances(batch)
    settled_dev = torch.from_numpy(settled).to(dev)
    hint = [settled_dev.data_ptr()]

    def solve_step():
        # consecutive batches alternate over the streams too (per-stream scratch: the next batch's
        # screen overlaps the previous batch's k = 1 solves)
        ptrs, optrs = cptrs[turn[1] % n_so]
        ctx.solve_device(ptrs, batch, optrs, stream=srefs[turn[1] % len(srefs)], settled=hint[0])
        turn[1] += 1

    def solve_step_one_stream():
        ptrs, optrs = cptrs[turn[1] % n_so]
        turn[1] += 1
        ctx.solve_device(ptrs, batch, optrs, stream=sref, settled=hint[0])

    setup_s = time.perf_counter() - t_setup

    # prepared launches (halda_fleets_plan_create) are set-up, not steps
    for t in sweeps:
        t.plan(ctx)
    rot2, rot1 = PlanRotation(sweeps, ctx, srefs), PlanRotation(sweeps, ctx, [sref])
    group = PlanGroup(sweeps, ctx)
    # warm-up and sanity: the sweep's per-fleet answers equal the solve-only leg's k = 1 solves (at least
    # one warm-up step per stream, so that no stream meets its first launch inside a timed region)
    for _ in range(max(args.warmup, len(srefs))):
        sweep_step()
        solve_step()
    torch.cuda.synchronize(dev)
    st = copies[(turn[1] - 1) % n_so][1]["status"].cpu().numpy()
    n_opt, n_inf = int((st == 0).sum()), int((st == 2).sum())
    if n_opt + n_inf != batch.n_inst:
        raise RuntimeError(f"unexpected statuses: {np.unique(st, return_counts=True)}")
    bk = sweeps[0].out["best_k"].cpu().numpy()
    if not (bk > 0).all():
        raise RuntimeError("a fleet without a feasible k in the sweep")
    # the group launch leaves every copy's results bit-identical to its own per-batch launch (checked on
    # the first copy; every group launch in this process has K steps, so a kernel trace averages alike)
    ref = {k: v.cpu().numpy().copy() for k, v in sweeps[0].out.items()}
    for v in sweeps[0].out.values():
        v.zero_()
    torch.cuda.synchronize(dev)  # the zeroing (torch's stream) before the launch on sref
    turn[0] = 0
    sweep_group(args.steps)
    torch.cuda.synchronize(dev)
    for k, v in sweeps[0].out.items():
        if not np.array_equal(v.cpu().numpy(), ref[k]):
            raise RuntimeError(f"group launch: {k} differs from the per-batch launch")

    ctx.set_timing(False)  # no per-launch instrumentation events inside the timed regions
    # the headline's own warm-up right before its timed region: W untimed steps as one group launch (the
    # checks above left the GPU idle for milliseconds of host work)
    sweep_group(max(args.warmup, 1))
    torch.cuda.synchronize(dev)
    R = Ranks(dist, world, lambda: torch.cuda.synchronize(dev), dev)
    el_sweep = timed(None, args.steps, R, tag="headline", many=sweep_group)
    # each rank's device time of its group launch: HIP events on its stream around the same region run
    # once more right after (events recorded inside the headline region would put two host-side event
    # records in front of its one launch: ~0.4 us per step at K = 20)
    _, ev_head = timed(None, args.steps, R, many=sweep_group, on_stream=(torch, stream))
    rank_launch_ms = {"max": R.max(ev_head), "min": R.min(ev_head)}
    el_200 = None
    if world > 1:  # beside the driver's K: a 200-step weak-scaling region (one launch of 200 batches)
        sweep_group(max(args.warmup, 1))
        el_200 = timed(None, 200, R, many=sweep_group)
    if os.environ.get("HALDA_BENCH_REPEAT"):  # diagnostic: the same region again, timings on stderr
        again, evs = [], []
        for _ in range(int(os.environ["HALDA_BENCH_REPEAT"])):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            e0.record(stream)
            sweep_group(args.steps)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            again.append(time.perf_counter() - t0)
            evs.append(e0.elapsed_time(e1) * 1e-3)
        print(f"bench: headline region {el_sweep * 1e6:.1f} us, repeated (wall, events): "
              f"{[(round(a * 1e6, 1), round(b * 1e6, 1)) for a, b in zip(again, evs)]}", file=sys.stderr)
    el_sweep2 = timed(sweep_step, args.steps, R, tag="per_launch", many=sweep_many)
    el_sweep1 = timed(sweep_step_one_stream, args.steps, R, many=sweep_many_one_stream)
    sweep_ev_ms = timed_events(sweep_step_one_stream, args.steps, torch, dev, stream, many=sweep_many_one_stream)
    # the group launch's own device time (HIP events on its stream around the one launch of K batches)
    group_ms = statistics.median(timed_events(None, 1, torch, dev, stream, many=lambda _: sweep_group(args.steps))
                                 for _ in range(3))
    el_solve = timed(solve_step, args.steps, R)
    el_solve1 = timed(solve_step_one_stream, args.steps, R)
    hint[0] = None  # the same legs without the settled flags: the screen proves every verdict itself
    el_solve_ns = timed(solve_step, args.steps, R)
    el_solve1_ns = timed(solve_step_one_stream, args.steps, R)
    hint[0] = settled_dev.data_ptr()
    el_strong = None
    if world > 1 and not strong_head:
        s_seeds = fleet_seeds(args, rank, world, True)
        s_table = fleet_table(build_fleets(s_seeds, args.M), model)
        n_st = max(2, min(32, math.ceil(2 * MALL_BYTES / max(DeviceFleetTable(s_table, model, ks, 0.5, dev).nbytes(), 1))))
        s_sweeps = [DeviceFleetTable(s_table, model, ks, 0.5, dev) for _ in range(n_st)]
        for t in s_sweeps:
            t.plan(ctx)
        sturn = [0]

        def strong_step():
            s_sweeps[sturn[0] % n_st].launch(ctx, srefs[sturn[0] % len(srefs)])
            sturn[0] += 1

        srot = PlanRotation(s_sweeps, ctx, srefs)

        def strong_many(k):
            srot.launch(sturn[0], k)
            sturn[0] += k

        for _ in range(max(args.warmup, len(srefs))):
            strong_step()
        el_strong = timed(strong_step, args.steps, R, many=strong_many)

    # per-launch device times (HIP events recorded by libhalda on the kernels' stream), after the
    # timed regions; the dominant launch of each leg is the longest
    ctx.set_timing(True)
    fl_ms, so_ms = [], []
    for _ in range(max(3, min(args.steps, 10))):
        sweep_step()
        torch.cuda.synchronize(dev)
        fl_ms.append(ctx.last_fleet_ms())
        solve_step()
        torch.cuda.synchronize(dev)
        so_ms.append(ctx.last_phase_ms())
    fl_mean = {k: statistics.mean(p.get(k, 0.0) for p in fl_ms) for k in fl_ms[0]}
    so_mean = {k: statistics.mean(p[k] for p in so_ms) for k in so_ms[0]}
    alg = algorithmic_bytes(lowered, refs, len(ks))
    alg_so = algorithmic_bytes(lowered, refs, len(ks), settled)

    inst_rank = len(fleets) * len(ks)
    total = inst_rank * world * args.steps if not strong_head else C3_FLEETS * len(ks) * args.steps
    value = total / el_sweep
    n_fleets_total = (len(fleets) * world if not strong_head else C3_FLEETS) * args.steps
    c2 = lat = None
    if world == 1 and not args.no_c2:
        c2 = c2_leg(args, torch, dev, ctx, model, stream, srefs)
        lat = None if args.no_latency else latency_leg(torch, dev, ctx, model, stream)
    if rank == 0:
        tto, tto_parts = time_to_optimal(model, args.M) if (world == 1 and not args.no_tto) else (None, None)
        c5 = c5_stream(model, args.M) if (world == 1 and not args.no_tto) else None
        bapi = batch_api(model, fleets) if (world == 1 and not args.no_tto) else None
        full = {
            "metric": METRIC,
            "value": value,
            "unit": "instances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el_sweep / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded C3 fleets, distilp_amd/synth.py)",
            "config": {
                "workload": (f"C3: {len(fleets) if not strong_head else C3_FLEETS} M={args.M} fleets x {len(ks)} k "
                             f"per {'GPU' if not strong_head else 'node'} (L=80, llama_3_70b/online, kv 4bit), one "
                             "k-sweep per step from HBM-resident tables"),
                "instances_per_step_per_gpu": inst_rank,
                "feasible_per_step_per_gpu": n_opt,
                "parallelism": f"dp{world}",
                "rccl_world_size": rccl_world,
                "resident_copies": n_sw,
            },
            "roofline": group_roofline(group_ms, args.steps, alg["halda_sweep_kernel"], len(fleets),
                                       roofline(fl_mean, alg, pmc_traffic, sweep_ev_ms)),
            "cpu_baseline": cpu_base,
            "launch": {"persistent": group.persistent, "launches_per_region": 1 if group.persistent else args.steps},
            "rank_launch_ms": rank_launch_ms,
            "weak_200": None if el_200 is None else {"ms_per_step": el_200 / 200 * 1e3,
                                                      "instances_per_s": inst_rank * world * 200 / el_200},
            "per_launch": {"ms_per_step": el_sweep2 / args.steps * 1e3, "instances_per_s": total / el_sweep2,
                           "host_enqueue_ms_per_step": HOST_ENQUEUE["per_launch"] / args.steps * 1e3,
                           "streams": args.streams},
            "one_stream": {"ms_per_step": el_sweep1 / args.steps * 1e3, "instances_per_s": total / el_sweep1},
            "host_enqueue_ms_per_step": HOST_ENQUEUE["headline"] / args.steps * 1e3,
            "strong": None if el_strong is None else {
                "fleets_total": C3_FLEETS, "ms_per_step": el_strong / args.steps * 1e3,
                "instances_per_s": C3_FLEETS * len(ks) * args.steps / el_strong,
            },
            "latency_mode": lat,
            "setup_s": setup_s,
            "fleets_per_s": n_fleets_total / el_sweep,
            "c5_stream": c5,
            "solve_only": {
                "instances_per_s": inst_rank * world * args.steps / el_solve,
                "ms_per_step": el_solve / args.steps * 1e3,
                "ms_per_step_one_stream": el_solve1 / args.steps * 1e3,
                "ms_per_step_no_settled": el_solve_ns / args.steps * 1e3,
                "ms_per_step_one_stream_no_settled": el_solve1_ns / args.steps * 1e3,
                "settled_per_step": int(settled.sum()),
                "streams": len(srefs),
                "resident_copies": n_so,
                "roofline": roofline(so_mean, alg_so, pmc_traffic),
            },
            "c2": c2,
            "batch_api": bapi,
            "feasible_instances_per_s": value * n_opt / batch.n_inst,
            "time_to_optimal_parts": tto_parts,
            "time_to_optimal_ms": tto,
        }
        if args.full_json:
            Path(args.full_json).parent.mkdir(parents=True, exist_ok=True)
            Path(args.full_json).write_text(json.dumps(full, indent=1) + "\n")
        print(json.dumps(compact_line(full)), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
