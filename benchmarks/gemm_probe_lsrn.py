"""hipBLASLt bf16 GEMM throughput for the LSRN sketch panel shapes (probe)."""
import time, torch
d = torch.device("cuda")
def tm(fn, it=10):
    fn(); torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it
t, n, p = 20000, 5000, 13300
P = torch.randn(t, p, device=d).bfloat16(); H = torch.randn(p, n, device=d).bfloat16()
out = torch.zeros(t, n, device=d)
fl = 2 * t * n * p
for name, fn, f in [
    ("addmm_f32out_beta1", lambda: torch.addmm(out, P, H, out_dtype=torch.float32, out=out), fl),
    ("mm_f32out", lambda: torch.mm(P, H, out_dtype=torch.float32), fl),
    ("mm_bf16out", lambda: torch.mm(P, H), fl),
    ("mm_Ht_layout", lambda: torch.mm(P, H.t().contiguous().t(), out_dtype=torch.float32), fl),
    ("sq8192_bf16", lambda: torch.mm(P[:8192, :8192], H[:8192, :5000].repeat(1, 2)[:, :8192].contiguous()), 2 * 8192**3),
]:
    try:
        s = tm(fn)
        print(f"{name}: {s*1e3:.3f} ms  {f/s/1e12:.0f} TFLOP/s", flush=True)
    except Exception as e:
        print(name, "failed", e)
P2 = torch.cat([P, P], 1); H2 = torch.cat([H, H], 0)
s = tm(lambda: torch.addmm(out, P2, H2, out_dtype=torch.float32, out=out))
print(f"kstack_2p: {s*1e3:.3f} ms  {2*fl/s/1e12:.0f} TFLOP/s")
Pt = P.t().contiguous()
s = tm(lambda: torch.addmm(out, Pt.t(), H, out_dtype=torch.float32, out=out))
print(f"addmm_Pcolmajor: {s*1e3:.3f} ms  {fl/s/1e12:.0f} TFLOP/s")
