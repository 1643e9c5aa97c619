"""A/B of the BlockADMM block Gram Z^T Z (1e6 x 1024, bf16 cache / f32) forms,
and the block's (Z^T Z + I)^-1 in f64.  usage: python benchmarks/probe/gram_ab.py"""
import json
import time

import torch


def tm(f, it=5):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


dev = torch.device("cuda")
ni, sj = 1_000_000, 1024
Z = (torch.randn(ni, sj, device=dev) * 0.03).to(torch.bfloat16)
Zf = Z.float()
ref = (Zf.double().t() @ Zf.double())
res = {}
res["mm_bf16_out_f32"] = tm(lambda: torch.mm(Z.t(), Z, out_dtype=torch.float32))
for b in (8, 16, 32, 64):
    Zb = Z.view(b, ni // b, sj)
    try:
        f = lambda: torch.bmm(Zb.transpose(1, 2), Zb, out_dtype=torch.float32).sum(0)
        res[f"bmm{b}_bf16_out_f32"] = tm(f)
        err = float((f().double() - ref).abs().max() / ref.abs().max())
        res[f"bmm{b}_relerr"] = err
    except Exception as e:  # noqa: BLE001
        res[f"bmm{b}_bf16_out_f32"] = str(e)[:120]
    Zfb = Zf.view(b, ni // b, sj)
    res[f"bmm{b}_f32"] = tm(lambda: torch.bmm(Zfb.transpose(1, 2), Zfb).sum(0))
res["mm_f32"] = tm(lambda: Zf.t() @ Zf)
C = ref.clone()
C.diagonal().add_(1.0)
res["chol_inv_f64"] = tm(lambda: torch.cholesky_inverse(torch.linalg.cholesky(C)))
Cf = C.float()
res["chol_inv_f32"] = tm(lambda: torch.cholesky_inverse(torch.linalg.cholesky(Cf)))
res["inv_f64_solve"] = tm(lambda: torch.linalg.inv(C))
print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))
