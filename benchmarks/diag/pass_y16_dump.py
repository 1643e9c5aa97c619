"""Diagnostic: block 0's y16 image as written by the y waves and as read by W wave KT."""
import ctypes as C
import sys

import torch

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
from libskylark_amd.ops import _lib
_lib.require()
_lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
_lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
dev = torch.device("cuda")
for (m, n, k) in [(16, 512, 20), (16, 1000, 40)]:
    g = torch.Generator(device=dev).manual_seed(1)
    A = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
    Zt = torch.randn(k, n, device=dev, generator=g).to(torch.bfloat16)
    ws = torch.zeros(int(_lib.require().sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    dbg = torch.zeros(65536, dtype=torch.uint8, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    _lib.call("sl_rsvd_pass", vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k, vp(ws.data_ptr()),
              vp(dbg.data_ptr()), k, 0, 4 << 6, st)
    torch.cuda.synchronize()
    KT = (k + 15) // 16
    KP = 16 * KT
    hi = dbg[:KP * 32].view(torch.bfloat16).view(KP, 16)     # [col][row]
    lo = dbg[4096:4096 + KP * 32].view(torch.bfloat16).view(KP, 16)
    yw = (hi.float() + lo.float()).t()                        # 16 x KP
    y = (A.double() @ Zt.double().t()).float()
    acc = dbg[16384:16384 + KP * 4 * 16].view(torch.float32).view(KP, 4, 4)   # [col][g4][e]
    acc = acc.reshape(KP, 16).t()
    print(f"n={n} k={k}: written-y err {float((yw[:, :k] - y).abs().max()):.3e}  acc err {float((acc[:, :k] - y).abs().max()):.3e} |y| {float(y.abs().max()):.2e}")
    # W wave's reads: per t, lane l = (g4, i16): 8 bf16 = rows rb..rb+7 of part (g4 & 1), col 16 t + i16
    rd = dbg[8192:8192 + KT * 64 * 16].view(torch.bfloat16).view(KT, 64, 8).float()
    bad = 0
    for t in range(KT):
        for l in range(64):
            g4, i16 = l >> 4, l & 15
            rb = 8 * (g4 >> 1)
            src = (hi if (g4 & 1) == 0 else lo)[16 * t + i16, rb:rb + 8].float()
            if not torch.equal(src, rd[t, l]):
                bad += 1
                if bad <= 4:
                    print("  mismatch t", t, "lane", l, src.tolist(), rd[t, l].tolist())
    print(f"  read-vs-written mismatches: {bad} of {KT * 64}")
    sys.stdout.flush()


# LDS slot image + Z fragments as step 1 saw them (y wave 0, block 0)
def swz(row):
    return ((row << 1) & 15) ^ (((row >> 3) & 1) * 9)


for (m, n, k) in [(16, 512, 20), (16, 1000, 40)]:
    g = torch.Generator(device=dev).manual_seed(1)
    A = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
    Zt = torch.randn(k, n, device=dev, generator=g).to(torch.bfloat16)
    ws = torch.zeros(int(_lib.require().sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    dbg = torch.zeros(65536 + 32768, dtype=torch.uint8, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    _lib.call("sl_rsvd_pass", vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k, vp(ws.data_ptr()),
              vp(dbg.data_ptr()), k, 0, 4 << 6, st)
    torch.cuda.synchronize()
    img = dbg[65536:].view(torch.int16).view(8, 16, 16, 8).cpu()     # [region][row][slot][8]
    Ah = A.view(torch.int16).cpu()
    bad = 0
    for r in range(8):
        if 128 * r >= n:
            continue
        for row in range(16):
            for sl in range(16):
                ch = sl ^ swz(row)
                col = 128 * r + 8 * ch
                col = col if col + 8 <= n else n - 8
                if not torch.equal(img[r, row, sl], Ah[row, col:col + 8]):
                    bad += 1
    KS = 32 if n > 512 else 16
    zf = dbg[32768:32768 + KS * 64 * 16].view(torch.int16).view(KS, 64, 8).cpu()
    Zh = Zt.view(torch.int16).cpu()
    zbad = 0
    for ks in range(KS):
        for l in range(64):
            g4, i16 = l >> 4, l & 15
            kk = 32 * ks + 8 * g4
            ref = Zh[i16, kk:kk + 8] if (i16 < k and kk + 8 <= n) else torch.zeros(8, dtype=torch.int16)
            if not torch.equal(zf[ks, l], ref):
                zbad += 1
    print(f"n={n}: LDS slot mismatched 16-B chunks {bad}, zf mismatched fragments {zbad}")
    sys.stdout.flush()
