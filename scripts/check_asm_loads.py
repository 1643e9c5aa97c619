"""Static check for the one hazard of inline-asm global loads (loads hipcc
does not track): a destination register read, copied or overwritten before
the counted `s_waitcnt vmcnt(N)` that retires its load.  hipcc treats an asm
output as written at ;;#ASMEND, so under register pressure or across a loop
back edge it may copy or reuse the register while the data is in flight
(a register ring of such loads did exactly that in a stage-2 FJLT draft:
hundreds of hazards, wrong sums).

The scan walks each kernel's ISA in order, keeps the issue-ordered queue of
vector-memory operations (vmcnt retires all but the newest N), and flags any
instruction that names a register of a not-yet-retired asm load.  Straight-
line order only: a use reached through a back edge with a different queue
state is still flagged the first time the linear walk meets it.

usage: python scripts/check_asm_loads.py [src.hip ...]   (default: every
source under libskylark_amd/_native/src with an inline-asm global load)
exit status 1 when any kernel has a hazard."""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "libskylark_amd", "_native", "src")
INC = os.path.join(ROOT, "libskylark_amd", "_native", "include")
VMEM = ("global_", "buffer_", "flat_load", "flat_store", "scratch_")


def _regs(tok: str) -> set:
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def scan(asm: str) -> dict:
    """{kernel symbol: hazard count} for every kernel in one .s file."""
    out = {}
    for name in re.findall(r"^(_Z\S+):", asm, re.M):
        i = asm.index(name + ":")
        j = asm.find(".Lfunc_end", i)
        body = asm[i:j if j > 0 else len(asm)]
        lines = [l.strip() for l in body.split("\n")
                 if l.strip() and (not l.strip().startswith(";") or l.strip().startswith(";;#ASM"))]
        q, inasm, hz = [], False, 0
        for l in lines:
            if l.startswith(";;#ASMSTART"):
                inasm = True
                continue
            if l.startswith(";;#ASMEND"):
                inasm = False
                continue
            m = re.search(r"vmcnt\((\d+)\)", l)
            if l.startswith("s_waitcnt") and m:
                n = int(m.group(1))
                q = q[len(q) - n:] if n < len(q) else q
                continue
            if l.startswith(".") or l.endswith(":"):
                continue
            op, toks = l.split()[0], [t.strip(",") for t in l.split()[1:]]
            pend = set().union(*q) if q else set()
            if op.startswith(VMEM):
                load = "load" in op and "lds" not in op
                if any(_regs(t) & pend for t in (toks[1:] if load else toks)):
                    hz += 1
                q.append(_regs(toks[0]) if (load and inasm and toks) else set())
                continue
            if any(_regs(t) & pend for t in toks):
                hz += 1
        if "k_" in name:
            out[name] = hz
    return out


def main(argv):
    srcs = argv or [p for p in sorted(glob.glob(os.path.join(SRC, "*.hip")))
                    if re.search(r'asm volatile\("global_load_dword', open(p).read())]
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for p in srcs:
            base = os.path.splitext(os.path.basename(p))[0]
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", INC,
                            "--save-temps", "-c", p, "-o", os.path.join(td, base + ".o")], cwd=td, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            s = open(os.path.join(td, base + "-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
            res = scan(s)
            nb = sum(1 for v in res.values() if v)
            bad += nb
            print(f"{base}: {len(res)} kernels, {nb} with asm-load hazards")
            for k, v in res.items():
                if v:
                    print(f"  {k[:90]}: {v}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
