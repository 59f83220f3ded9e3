import sys; sys.path.insert(0,'/root/repo')
import numpy as np
from distilp_amd.common import DeviceProfile, ModelProfileSplit
from distilp_amd.synth import load_model_dict, synth_fleet
from distilp_amd.solver.lower import lower_fleet
from distilp_amd.solver.batch import assemble
from distilp_amd.solver._libhalda import get_context
from oracle import milp_oracle as mo
model = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
for M, seed in [(6,3),(16,1),(64,2)]:
    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(seed, M)]
    fl = lower_fleet(devs, model, "4bit")
    for k in [1, 2]:
        batch, refs = assemble([fl], [[k]])
        p = mo.lower_dense(devs, model, k, 0.5)
        i = [j for j in range(M) if p["ub"][M + j] > 0][0]
        for lbv in [0.0, 3.0]:
            b2 = batch
            b2.col_lb = batch.col_lb.copy(); b2.col_lb[refs[0].col_off + M + i] = lbv
            p["lb"] = p["lb"].copy(); p["lb"][M + i] = lbv
            res = get_context(0).solve(b2)
            st, xo, v1, v2, _ = mo.exact_solve(p)
            print(M, seed, k, lbv, "gpu", int(res.status[0]), float(res.obj_lin[0]), "oracle", st, v1, flush=True)
