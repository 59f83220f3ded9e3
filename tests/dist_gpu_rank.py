"""One rank of tests/test_gpu_distributed.py (started as a subprocess): both multi-GPU modes of
distilp_amd.distributed with the real libhalda engine on cuda:0, gloo collectives; writes its
results as JSON.   python tests/dist_gpu_rank.py RANK WORLD PORT OUTDIR"""

import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def main():
    rank, world, port, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import torch.distributed as dist

    from distilp_amd.common import ModelProfileSplit
    from distilp_amd.distributed import halda_solve_batch_distributed, halda_solve_distributed
    from distilp_amd.solver import halda_solve
    from distilp_amd.synth import load_model_dict
    from tests.helpers import fixture_fleet, synth_devices

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {"single": {}, "batch": {}, "single_of_batch": {}}
        for folder, kv in (("llama_3_70b/online", "4bit"), ("hermes_70b", "4bit"), ("llama_3_70b/online", "8bit")):
            devs, model = fixture_fleet(folder)
            r = halda_solve_distributed(devs, model, mip_gap=1e-4, kv_bits=kv, device=0)
            out["single"][f"{folder}|{kv}"] = r.model_dump()
        m2 = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
        for M in (4, 16, 64):
            fleets = [synth_devices(M, s) for s in range(20 if M < 64 else 8)]
            res = halda_solve_batch_distributed(fleets, m2, mip_gap=1e-4, kv_bits="4bit", device=0)
            out["batch"][str(M)] = [o.model_dump() for o in res]
            # the same fleets one at a time through halda_solve (the objective must be the same bits)
            out["single_of_batch"][str(M)] = [
                halda_solve(devs, m2, mip_gap=1e-4, plot=False, kv_bits="4bit", device=0).model_dump()
                for devs in fleets]
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
