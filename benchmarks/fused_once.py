"""Run the fused tall-skinny pass N times (for rocprofv3 --pmc counter runs).
usage: fused_once.py [flags=0|3|4] [reps=20] [lda=1000] [gram=1|0]
(gram=0 with flags=3 is the randSVD inter-pass variant; flags=4 is the final
pass: Y stored, fp64 in-pass Gram)"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ctypes as C  # noqa: E402

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng, tallskinny  # noqa: E402,F401


def main():
    flags = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ld = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    gram = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    m, n, k = 1_000_000, 1000, 40
    dev = torch.device("cuda")
    lib = _lib.require()
    buf = torch.empty(m, ld, dtype=torch.bfloat16, device=dev)
    rng.fill_random(buf, D.Normal(), 1, 0, ir=ld, ic=1)
    A = buf[:, :n]
    Zt = (torch.randn(k, n, device=dev) / 30).to(torch.bfloat16)
    W = torch.empty(n, k, device=dev)
    final = flags == 4
    G = torch.empty(k, k, device=dev, dtype=torch.float64 if final else torch.float32)
    Y = torch.empty(m, k, device=dev) if final else None
    ws = torch.empty(int(lib.sl_tsk_fused_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(reps):
        _lib.call("sl_tsk_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W), _lib.ptr(G) if gram else None,
                  _lib.ptr(Y) if final else None, k if final else 0, _lib.ptr(ws), flags, st)
    torch.cuda.synchronize()
    print("ok", flags, reps, ld)


if __name__ == "__main__":
    main()
