"""LSRN sketch-panel GEMM only (2e4 x 1e4 x 26816 bf16, f32 out): ours vs
hipBLASLt, for kernel traces / counters of the two (no other work)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from benchmarks.bench_gemm_nt import case  # noqa: E402

if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "lsrn"
    if which == "lsrn":
        case("lsrn_panel", 20000, 10000, 26816)
    else:
        case("square", 8192, 8192, 8192)
