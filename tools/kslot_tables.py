"""Diagnostic: dump the k = 2 tables (G, H per device and layer count) the k-slot kernel builds for
the C2 fleets, from a -DHALDA_STAMPS -DHALDA_STAMPS_DUMP build (make -C distilp_amd/csrc dump), to
gpurun_out/c2_tables.npz (offline study of the threshold scan).
  HALDA_LIB=build/variants/libhalda_dump.so python tools/kslot_tables.py"""
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def main():
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context, load_library
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    stream = torch.cuda.Stream(dev)
    model = bench.load_model()
    nf, M = 4096, 16
    table = fleet_table(bench.build_fleets(range(nf), M), model)
    dt = DeviceFleetTable(table, model, KS, 0.5, dev, want_per_k=True)
    dt.launch(ctx, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    lib = load_library()
    buf = np.zeros(4096 * 16 * 32 * 2)
    lib.halda_debug_dump.argtypes = [ctypes.c_void_p]
    lib.halda_debug_dump(buf.ctypes.data)
    t = buf.reshape(4096, 16, 32, 2)[:nf, :M, :25]
    out = Path("gpurun_out")
    out.mkdir(exist_ok=True)
    np.savez_compressed(out / "c2_tables.npz", G=t[..., 0], H=t[..., 1],
                        obj_by_k=dt.out["obj_by_k"].cpu().numpy().reshape(nf, len(KS)),
                        best_k=dt.out["best_k"].cpu().numpy(), w=dt.out["w"].cpu().numpy())
    print("dumped", t.shape, np.isfinite(t[..., 0]).mean())


if __name__ == "__main__":
    main()
