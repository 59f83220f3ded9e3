"""Static instruction mix of the solve kernel between PHASE_MARK comments.

Development aid: build an asm file whose HALDA_STAMP(k) sites are replaced by
`asm volatile("; PHASE_MARK k")`, then
    python tools/asm_regions.py /tmp/hm.s [kernel name, default solve_kernel]
(-DHALDA_MARKS builds such a listing of the fused sweep's HALDA_SSTAMP sites) prints, per region, the VALU / SALU / LDS / VMEM instruction counts and the
number of branch labels (loop bodies are counted once)."""
import re
import sys
from collections import Counter


def main(path, kernel="solve_kernel"):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z.*{kernel}.*:", l))
    region, stats = "pre", {}
    for l in lines[start:]:
        m = re.search(r"PHASE_MARK (\d+)", l)
        if m:
            region = "after" + m.group(1)
            continue
        t = l.strip()
        if t.startswith("s_endpgm"):
            break
        c = stats.setdefault(region, Counter())
        if re.match(r"^\.LBB", t):
            c["labels"] += 1
        op = t.split()[0] if t and not t.startswith((";", ".")) else ""
        if not op:
            continue
        kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
                "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
        c[kind] += 1
        if op.startswith("v_") and "f64" in op:
            c["valu_f64"] += 1
        if op.startswith("v_cvt"):
            c["cvt"] += 1
    for r, c in stats.items():
        print(f"{r:8s}", dict(c))


if __name__ == "__main__":
    main(*sys.argv[1:])
