"""Phase stamps of the core eigensolver at K = 40 (probe kernel, s_memtime
cycles at the shader clock): tridiagonalisation, multisection, twisted
vectors, MGS, residual check, back-transform.  Graded 40 x 40 SPD input,
top 21 eigenvalues / 20 vectors, as the randSVD's final core."""
import ctypes as C
import glob
import json
import os

import torch

dev = torch.device("cuda")
g = torch.Generator().manual_seed(2)
k, r = 40, 20
Q, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
lamd = 1e4 * 0.8 ** torch.arange(k, dtype=torch.float64)
Cm = ((Q * lamd) @ Q.t()).to(dev).contiguous()
for so in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe_*.so"))):
  lib = C.CDLL(so)
  lib.probe_eig.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
  out = torch.zeros(r + k * r, dtype=torch.float64, device=dev)
  ts = torch.zeros(16, dtype=torch.int64, device=dev)
  s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
  runs = []
  for it in range(20):
      lib.probe_eig(C.c_void_p(Cm.data_ptr()), k, r, C.c_void_p(out.data_ptr()), C.c_void_p(ts.data_ptr()), s)
      torch.cuda.synchronize()
      t = ts.cpu().tolist()
      runs.append(t)
  names = ["tridiag", "scale", "multisection", "twisted", "mgs", "residual", "backtransform", "tail"]
  order = [(0, 7), (7, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 8)]
  med = {}
  for nm, (a, b) in zip(names, order):
      v = sorted(rr[b] - rr[a] for rr in runs[2:])
      med[nm] = v[len(v) // 2]
  err = float((out[:r] - lamd[:r].to(dev)).abs().max() / lamd[0])
  print(json.dumps({"variant": os.path.basename(so), "cycles_median": med, "flags": runs[-1][9], "lam_err_rel": err}))
