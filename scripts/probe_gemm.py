import torch, time
d = torch.device("cuda")
print("allow_tf32", torch.backends.cuda.matmul.allow_tf32, getattr(torch.backends.cuda.matmul, "fp32_precision", None))
print("preferred blas", torch.backends.cuda.preferred_blas_library())
a = torch.randn(4096, 1000, device=d); b = torch.randn(1000, 40, device=d)
r = (a.double() @ b.double())
for lib in ["cublaslt", "cublas"]:
    try:
        torch.backends.cuda.preferred_blas_library(lib)
        c = a @ b
        print(lib, "fp32 rel err", ((c.double() - r).abs().max() / r.abs().max()).item())
    except Exception as e:
        print(lib, "err", e)
try:
    x = torch.mm(a.bfloat16(), b.bfloat16(), out_dtype=torch.float32)
    print("out_dtype ok", x.dtype)
except Exception as e:
    print("out_dtype unsupported", type(e).__name__, e)
# small linear algebra timing on GPU vs CPU
W = torch.randn(1000, 40, dtype=torch.float64, device=d)
for name, fn in [("qr", lambda X: torch.linalg.qr(X)), ("svd", lambda X: torch.linalg.svd(X, full_matrices=False)), ("chol", lambda X: torch.linalg.cholesky_ex(X.t() @ X))]:
    fn(W); torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): fn(W)
    torch.cuda.synchronize(); g = (time.perf_counter() - t) / 10
    Wc = W.cpu(); fn(Wc); t = time.perf_counter()
    for _ in range(10): fn(Wc)
    c = (time.perf_counter() - t) / 10
    print(f"{name}: gpu {g*1e6:.0f}us cpu {c*1e6:.0f}us")
t = time.perf_counter()
for _ in range(20): W.cpu(); 
print("d2h 320KB", (time.perf_counter() - t) / 20 * 1e6, "us")
