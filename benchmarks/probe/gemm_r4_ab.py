"""Same-box A/B of gemm_nt.hip builds (the round-4 build 51e1f5f vs the
current source, both as standalone libraries: benchmarks/probe/gemm_*.so)
on the square 8192^3 and LSRN panel shapes, three interleaved rounds."""
import os
import sys

here = os.path.dirname(os.path.abspath(__file__))
os.environ["GEMM_AB_LIBS"] = f"r4:{here}/gemm_r4.so,cur:{here}/gemm_cur.so"
sys.path.insert(0, os.path.dirname(os.path.dirname(here)))
from benchmarks.bench_gemm_nt import case  # noqa: E402

if __name__ == "__main__":
    for _ in range(3):
        case("square", 8192, 8192, 8192)
        case("lsrn_panel", 20000, 10000, 26816)
