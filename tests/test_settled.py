"""The caller's settled instances (batch.settled_instances, the host side of
halda_solve_batch_device_settled): every instance it marks is one the reference's milp() reports
infeasible (res.success == False, halda_p_solver.py:369-436; checked against the reference-run synthetic
goldens), it marks every bound-infeasible k (M > W = L / k), and it refuses instances the screen would
not call infeasible (a malformed equality row, NaN bounds that prove nothing)."""

import numpy as np

from distilp_amd.solver.batch import assemble, settled_instances
from distilp_amd.solver.lower import lower_fleet

from .helpers import synth_devices


def test_settled_instances_are_reference_infeasible(synth_golden, llama_online_model):
    n_set = 0
    for M, G in sorted(synth_golden.items()):
        for fleet in G["fleets"]:
            devs = synth_devices(M, fleet["seed"], fleet["devices"])
            ks = [rec["k"] for rec in fleet["per_k"]]
            batch, refs = assemble([lower_fleet(devs, llama_online_model)], [ks])
            st = settled_instances(batch)
            for rec, ref, s in zip(fleet["per_k"], refs, st):
                if s:
                    assert not rec["success"], (M, fleet["seed"], rec["k"])
                assert bool(s) == (M > ref.W), (M, fleet["seed"], rec["k"])
            n_set += int(st.sum())
    assert n_set > 0


def test_settled_instances_refuse_what_the_screen_would_not_settle(llama_online_model):
    devs = synth_devices(16, 0)
    batch, refs = assemble([lower_fleet(devs, llama_online_model)], [[1, 8, 16]])
    assert settled_instances(batch).tolist() == [0, 1, 1]
    # a malformed equality row (shared by the fleet's instances): UNSUPPORTED on the GPU, never settled
    bad = assemble([lower_fleet(devs, llama_online_model)], [[1, 8, 16]])[0]
    bad.val = bad.val.copy()
    eq = int(bad.row_ptr[bad.csr_off[1] + bad.n_rows[1] - 1])
    bad.val[eq + 3] = 2.0
    assert not settled_instances(bad).any()
    # NaN bounds count 0: with every w bound NaN, nothing is proved
    nan = assemble([lower_fleet(devs, llama_online_model)], [[1, 8, 16]])[0]
    nan.col_lb = nan.col_lb.copy()
    for i in range(nan.n_inst):
        nan.col_lb[nan.col_off[i]:nan.col_off[i] + 16] = np.nan
    assert not settled_instances(nan).any()
    # a negative bound is infeasible by itself, even at k = 1
    neg = assemble([lower_fleet(devs, llama_online_model)], [[1]])[0]
    neg.col_lb = neg.col_lb.copy()
    neg.col_lb[neg.col_off[0] + 5] = -1.0
    assert settled_instances(neg).tolist() == [1]
