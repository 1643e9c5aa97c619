"""Static ISA check of the inline-asm global loads (scripts/check_asm_loads.py):
no kernel reads, copies or overwrites an asm load's destination register
before the counted vmcnt that retires it.  Host-only (hipcc cross-compiles
gfx950); the checker itself is validated on a known-bad register ring."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="needs hipcc")


def test_asm_loaded_registers_are_never_touched_in_flight():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_asm_loads.py")], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 with asm-load hazards" in r.stdout


def test_checker_flags_a_ring_copied_across_the_back_edge():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import check_asm_loads as c
    # a destination copied (v_mov) before the wait that retires its load
    bad = """_Zk_bad:
;;#ASMSTART
global_load_dwordx2 v[4:5], v[0:1], off
;;#ASMEND
v_mov_b32_e32 v8, v4
s_waitcnt vmcnt(0)
.Lfunc_end0:
"""
    good = bad.replace("v_mov_b32_e32 v8, v4\ns_waitcnt vmcnt(0)", "s_waitcnt vmcnt(0)\nv_mov_b32_e32 v8, v4")
    assert c.scan(bad) == {"_Zk_bad": 1}
    assert c.scan(good) == {"_Zk_bad": 0}
