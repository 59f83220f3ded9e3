"""Static instruction histogram of one kernel in a hipcc -S output (development aid).
   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude --cuda-device-only -S \
       -o /tmp/h.s distilp_amd/csrc/halda.hip && python tools/isa_hist.py /tmp/h.s halda_sweep_kernel"""
import re
import sys
from collections import Counter


def main(path, kernel, top=25):
    L = open(path).read().splitlines()
    st = next(i for i, l in enumerate(L) if re.match(rf"^_Z\w*{kernel}\w*:", l))
    ops = Counter()
    for l in L[st:]:
        t = l.strip()
        if t.startswith("s_endpgm"):
            break
        if t and not t.startswith((";", ".")):
            ops[t.split()[0]] += 1
    kinds = Counter()
    for op, n in ops.items():
        kinds["valu_f64" if op.startswith("v_") and "f64" in op else "valu" if op.startswith("v_") else
              "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "vmem"] += n
    print(kernel, "total", sum(ops.values()), dict(kinds))
    for op, n in ops.most_common(top):
        print(f"  {op:28s} {n}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:]))
