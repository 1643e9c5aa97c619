"""Probe the device Jacobi eigensolver: sweeps and time per call."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from libskylark_amd.ops import small_la as SL

dev = torch.device("cuda")
for name, X in [("gauss1000x40", torch.randn(1000, 40, dtype=torch.float64)),
                ("clustered", torch.randn(100000, 40, dtype=torch.float64)),
                ("graded", torch.randn(1000, 40, dtype=torch.float64) * torch.logspace(0, -6, 40, dtype=torch.float64))]:
    C = (X.t() @ X).to(dev)
    sw = torch.zeros(1, dtype=torch.int32, device=dev)
    out = SL.sym_eig_topr(C, 20, sweeps=sw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        SL.sym_eig_topr(C, 20, out=out, sweeps=sw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20 * 1e6
    ref = torch.linalg.eigvalsh(C.cpu()).flip(0)[:20]
    err = ((out[40 * 20:].cpu() - ref).abs() / ref.abs()).max().item()
    print(f"{name}: sweeps={int(sw.item())} time={dt:.1f}us max_rel_err={err:.2e}")
