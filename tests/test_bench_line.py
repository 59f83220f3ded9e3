"""bench.py's host logic on CPU: the compact JSON line (its size and key order, so a driver that keeps the
last ~4 KB of stdout keeps all of it) and the multi-rank timing of timed() over gloo (each rank's region
ends at its own device synchronize; the closing collective is outside it)."""

import json
import os
import socket
import time

import torch.multiprocessing as mp

from .conftest import REPO


def _f(i):  # a full-precision float, as the legs produce them
    return (i + 1) / 3.0 * 10 ** (i % 7)


def _full(world=1):
    """A detailed record with every key bench.main() fills, full-precision floats everywhere."""
    roof = {"bound": "hbm", "achieved": _f(1), "peak": 8000.0, "unit": "GB/s", "frac": _f(2) / 1e3, "traffic": _f(3) * 1e6,
            "kernel": "halda_sweep_steps_kernel", "kernel_ms": _f(4), "kernel_ms_from": "x" * 80, "steps_per_launch": 20,
            "algorithmic_bytes_per_launch": 725155840, "algorithmic_bytes_per_batch": 36257792,
            "roofs": {"hbm": _f(5), "valu_issue": _f(6)}, "nearest_roof": "hbm",
            "valu_issue": {"frac": _f(7), "frac_all_at_4": _f(8), "valu_per_item": _f(9), "fp64_per_item": _f(10),
                           "fp64_trans_per_item": _f(11), "other_per_item": _f(12), "wait_any_frac": _f(13),
                           "source": "profiles/r06_valu.json"},
            "single_batch_kernel": {"kernel": "halda_sweep_kernel", "kernel_ms": _f(14), "frac": _f(15),
                                    "launch_ms": {"halda_sweep_kernel": _f(16)}}}
    lat = {name: {"plain": {"device_ms_per_call": _f(20), "wall_ms_sync_call": _f(21)},
                  "rccl_world1": {"device_ms_per_call": _f(22), "wall_ms_sync_call": _f(23)},
                  **{f"emulated_world{w}": {"device_ms_per_call": _f(24), "wall_ms_sync_call": _f(25)} for w in (2, 4, 8)},
                  **{f"rank_subsweep_world{w}": {"max_device_ms": _f(26), "per_rank_device_ms": [_f(27)] * w}
                     for w in (2, 4, 8)}}
           for name in ("one_fleet", "fleets_4096")}
    return {
        "metric": "HALDA MILP instances solved/sec (node), M=64 devs L=80; time-to-optimal", "value": _f(30) * 1e9,
        "unit": "instances/s", "n_gpus": world, "steps": 20, "warmup": 5, "ms_per_step": _f(31) / 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded C3 fleets, distilp_amd/synth.py)",
        "config": {"workload": "C3: 4096 M=64 fleets x 9 k per GPU (L=80, llama_3_70b/online, kv 4bit), one k-sweep "
                               "per step from HBM-resident tables", "instances_per_step_per_gpu": 36864,
                   "feasible_per_step_per_gpu": 4096, "parallelism": f"dp{world}", "rccl_world_size": world,
                   "resident_copies": 16},
        "roofline": roof,
        "cpu_baseline": {"value": _f(40), "unit": "instances/s", "cores": 16, "kind": "port", "nproc": 256,
                         "cgroup_cpu_quota": 16, "one_core_value": _f(41),
                         "sample": "16 pinned procs x ~12 s, own C3 fleets: 5496 fleets x 9 k in 12.3 s; "
                                   "oracle/milp_oracle.py (reference lowering + HiGHS 1.8.0)"} if world == 1 else None,
        "launch": {"persistent": True, "launches_per_region": 1},
        "rank_launch_ms": {"max": _f(42), "min": _f(43)},
        "weak_200": {"ms_per_step": _f(44), "instances_per_s": _f(45)} if world > 1 else None,
        "per_launch": {"ms_per_step": _f(46), "instances_per_s": _f(47), "host_enqueue_ms_per_step": _f(48), "streams": 2},
        "one_stream": {"ms_per_step": _f(49), "instances_per_s": _f(50)},
        "host_enqueue_ms_per_step": _f(51),
        "strong": {"fleets_total": 4096, "ms_per_step": _f(52), "instances_per_s": _f(53)} if world > 1 else None,
        "latency_mode": lat if world == 1 else None,
        "setup_s": _f(54), "fleets_per_s": _f(55),
        "c5_stream": {"ms_per_batch": _f(56), "fleets_per_s": _f(57), "instances_per_s": _f(58),
                      "reprofile_ms": _f(59)} if world == 1 else None,
        "solve_only": {"instances_per_s": _f(60), "ms_per_step": _f(61), "ms_per_step_one_stream": _f(62),
                       "ms_per_step_no_settled": _f(63), "ms_per_step_one_stream_no_settled": _f(64),
                       "settled_per_step": 32768, "streams": 2, "resident_copies": 2, "roofline": dict(roof)},
        "c2": {"instances_per_step": 36864, "feasible_per_step": 12000, "ms_per_step": _f(70), "instances_per_s": _f(71),
               "ms_per_batch_events": _f(72), "group_persistent": True, "ms_per_step_one_stream": _f(73),
               "ms_per_step_two_streams": _f(74), "steps": 20, "resident_copies": 32, "roofline": dict(roof)}
        if world == 1 else None,
        "batch_api": {"ms": _f(75), "fleets_per_s": _f(76)} if world == 1 else None,
        "feasible_instances_per_s": _f(77),
        "time_to_optimal_parts": {"pack_ms": _f(78), "gpu_call_ms": _f(79), "rest_ms": _f(80),
                                  "gpu_call_copy_path_ms": _f(81)} if world == 1 else None,
        "time_to_optimal_ms": _f(82) if world == 1 else None,
    }


def test_compact_line_fits_and_ends_with_the_metric_figures():
    import bench

    for world in (1, 8):
        line = bench.compact_line(_full(world))
        text = json.dumps(line)
        assert len(text) <= 3500, (world, len(text))
        keys = list(line)
        # the contract's keys lead, in the contract's order
        assert keys[:13] == ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                             "scaling", "vs_baseline", "dtype", "data", "config"]
        assert "roofline" in line and "cpu_baseline" in line
        # BASELINE's metric figures close the line (time to optimal last)
        assert keys[-8:] == ["fleets_per_s", "c5_stream", "batch_api", "solve_only", "c2", "feasible_instances_per_s",
                             "time_to_optimal_parts", "time_to_optimal_ms"]
        assert line["value"] == _full(world)["value"]  # the headline keeps full precision
    one = bench.compact_line(_full(1))
    assert one["c2"]["roofline"]["frac"] is not None and one["c2"]["ms_per_step"] is not None
    assert list(one["c2"])[-1] == "ms_per_step" and list(one["solve_only"])[-1] == "ms_per_step"
    assert one["roofline"]["valu_issue"]["fp64_per_item"] is not None
    assert one["time_to_optimal_parts"]["pack_ms"] is not None
    assert list(one["c5_stream"])[-1] == "ms_per_batch" and one["c5_stream"]["reprofile_ms"] is not None
    eight = bench.compact_line(_full(8))
    assert eight["weak_200"]["ms_per_step"] is not None and eight["config"]["rccl_world_size"] == 8


def test_valu_issue_prices_fp64_apart():
    import bench

    vp = {"valu_per_wave": 100.0, "waves": 10, "items": 10, "source": "x", "wait_any_frac": 0.3,
          "valu_types": {"add_f64": 10.0, "mul_f64": 5.0, "fma_f64": 5.0, "trans_f64": 1.0, "int32": 30.0,
                         "int64": 0.0, "cvt": 4.0}}
    # 1,024 SIMDs at 2.4 GHz for 1 ms
    cyc = bench.N_SIMDS * bench.CLOCK_GHZ * 1e6
    v = bench.valu_issue(vp, units=int(cyc // 1000), ms=1.0)
    units = int(cyc // 1000)
    assert abs(v["frac"] - (20 * 4 + 1 * 8 + 79 * 2) * units / cyc) < 1e-12
    assert abs(v["frac_all_at_4"] - 100 * 4 * units / cyc) < 1e-12
    assert v["fp64_per_item"] == 20.0 and v["other_per_item"] == 79.0
    assert bench.valu_issue(None, 1, 1.0)["frac"] is None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _SlowBarrier:
    """torch.distributed with a barrier that makes rank 1 arrive `delay` s late: a late rank (or a slow
    collective) at either barrier must not land inside any rank's timed region."""

    def __init__(self, dist, rank, delay):
        self._d, self._rank, self._delay = dist, rank, delay

    def barrier(self):
        if self._rank == 1:
            time.sleep(self._delay)
        self._d.barrier()

    def __getattr__(self, name):
        return getattr(self._d, name)


def _timed_worker(rank, world, port, outdir):
    import sys

    sys.path.insert(0, str(REPO))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        R = bench.Ranks(_SlowBarrier(dist, rank, 0.4), world, sync=lambda: None)
        step_s = 0.01 if rank == 0 else 0.05  # rank 1's steps are the slow ones
        el = bench.timed(lambda: time.sleep(step_s), 4, R)
        with open(os.path.join(outdir, f"t{rank}.json"), "w") as f:
            json.dump({"elapsed": el, "max": R.max(float(rank)), "min": R.min(float(rank))}, f)
    finally:
        dist.destroy_process_group()


def test_timed_excludes_barriers_and_takes_the_max_over_ranks(tmp_path):
    port = _free_port()
    mp.start_processes(_timed_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r = [json.loads((tmp_path / f"t{i}.json").read_text()) for i in range(2)]
    # both ranks report the slow rank's region (4 x 50 ms), never the 0.4 s barrier delay
    for x in r:
        assert 0.2 <= x["elapsed"] < 0.35, x
        assert x["max"] == 1.0 and x["min"] == 0.0
    assert r[0]["elapsed"] == r[1]["elapsed"]
