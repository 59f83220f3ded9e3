"""Diagnostic: does torch's bundled HIP runtime still see the GPU after libhalda (linked against
/opt/rocm's runtime) has initialised HIP in the same process?  python tools/probe_runtime_order.py [lib|torch]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
first = sys.argv[1] if len(sys.argv) > 1 else "lib"
if first == "lib":
    from distilp_amd.solver._libhalda import get_context

    get_context(0)
    print("libhalda context ok")
import torch

print("torch device_count", torch.cuda.device_count(), "available", torch.cuda.is_available())
x = torch.ones(4, device="cuda")
print("torch tensor on", x.device, float(x.sum()))
if first != "lib":
    from distilp_amd.solver._libhalda import get_context

    get_context(0)
    print("libhalda context ok")
