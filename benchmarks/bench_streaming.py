"""Out-of-core sketching throughput: a host-resident f32 matrix (default
4e6 x 1000 = 16 GB) sketched through one MI355X by sketch.streaming, vs the
bare pinned H2D copy of the same bytes (the PCIe bound).

usage: python benchmarks/bench_streaming.py [--rows 4e6] [--cols 1000] [--S 256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=4e6)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--S", type=int, default=256)
    a = ap.parse_args()
    import libskylark_amd as sk
    m, n = int(a.rows), a.cols
    dev = torch.device("cuda")
    A = torch.empty(m, n, dtype=torch.float32)
    for r0 in range(0, m, 1 << 20):
        A[r0:r0 + (1 << 20)].normal_()
    Ap = A.pin_memory()
    nbytes = A.numel() * 4
    # bare H2D bound (pinned, 1 GiB chunks)
    buf = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    flat = Ap.view(-1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for o in range(0, flat.numel(), buf.numel()):
        w = min(buf.numel(), flat.numel() - o)
        buf[:w].copy_(flat[o:o + w], non_blocking=True)
    torch.cuda.synchronize()
    h2d = time.perf_counter() - t
    rows = [{"what": "pinned H2D copy", "s": round(h2d, 4), "GBps": round(nbytes / h2d / 1e9, 2)}]
    for name, T, dim in [("JLT columnwise", sk.sketch.JLT(m, a.S, context=sk.Context(1)), 0),
                         ("CWT columnwise", sk.sketch.CWT(m, 4 * a.S, context=sk.Context(2)), 0),
                         ("GaussianRFT rowwise", sk.sketch.GaussianRFT(n, 4 * a.S, sigma=10.0,
                                                                       context=sk.Context(3)), 1)]:
        for src, label in [(A, "pageable"), (Ap, "pinned")]:
            torch.cuda.synchronize()
            t = time.perf_counter()
            out = T.apply_streamed(src, dim, device=dev)
            torch.cuda.synchronize()
            s = time.perf_counter() - t
            rows.append({"what": f"{name} ({label} host A)", "s": round(s, 4), "GBps": round(nbytes / s / 1e9, 2),
                         "out_shape": list(out.shape)})
            del out
    for r in rows:
        r.update({"rows": m, "cols": n, "bytes": nbytes})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
