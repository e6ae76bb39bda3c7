#!/usr/bin/env python3
"""Per-kernel ISA statistics of one librsd HIP source (device-only compile, gfx950).

    python tools/isa_stats.py csrc/svao.hip [--flags "..."] [--match svao_pass1]

Compiles the file with the Makefile's HIP flags (plus --flags) to gfx950 assembly and prints, per
kernel whose symbol contains --match: instructions (by class: VALU / SALU / VMEM / SMEM / LDS /
branch), VGPRs, SGPRs, scratch and occupancy.  Used to check an instruction-count change before a
GPU run (no GPU needed)."""
import argparse
import re
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parents[1] / "ray-traced-stochastic-depth-map_amd"
BASE = ["-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-munsafe-fp-atomics"]


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--flags", default="")
    ap.add_argument("--match", default="")
    ap.add_argument("--dump", default=None, help="write the assembly here")
    a = ap.parse_args()
    src = Path(a.src)
    if not src.is_absolute():
        src = (PKG / src) if (PKG / src).exists() else src.resolve()
    cmd = ["/opt/rocm/bin/hipcc", *BASE, *a.flags.split(), "--cuda-device-only", "-S", "-o", "-", str(src)]
    asm = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    if a.dump:
        Path(a.dump).write_text(asm)
    kernels = {}
    cur = None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+|[A-Za-z_]\w*):\s*(;.*)?$", line)
        if m and not line.startswith("."):
            name = m.group(1)
            cur = kernels.setdefault(name, {"insts": {}, "meta": {}}) if a.match in name else None
            continue
        if cur is None:
            continue
        s = line.strip()
        if s.startswith(".Lfunc_end") or s.startswith(".section"):
            cur = None
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            mm = re.match(r";\s*(NumVgprs|NumSgprs|ScratchSize|Occupancy|NumAgprs|TotalNumVgprs):\s*(\d+)", s)
            if mm:
                cur["meta"][mm.group(1)] = int(mm.group(2))
            continue
        op = s.split()[0]
        c = classify(op)
        cur["insts"][c] = cur["insts"].get(c, 0) + 1
    # metadata comments follow the function end: second pass
    for name in kernels:
        i = asm.find(name + ":")
        j = asm.find(".Lfunc_end", i)
        tail = asm[j:j + 4000]
        for key in ("NumVgprs", "NumSgprs", "ScratchSize", "Occupancy"):
            mm = re.search(r";\s*" + key + r":\s*(\d+)", tail)
            if mm:
                kernels[name]["meta"][key] = int(mm.group(1))
    for name, k in kernels.items():
        if not k["insts"]:
            continue
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        tot = sum(k["insts"].values())
        print(f"{dem}\n  total {tot}  " + "  ".join(f"{c} {n}" for c, n in sorted(k["insts"].items())) +
              "  |  " + "  ".join(f"{c} {n}" for c, n in k["meta"].items()))


if __name__ == "__main__":
    sys.exit(main())
