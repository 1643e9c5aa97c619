import sys, os, time, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from libskylark_amd.ops import tallskinny as T, rng
from libskylark_amd.base import distributions as D
dev = torch.device("cuda")
m, n, k = 1_000_000, 1000, 40
A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
Z = torch.randn(n, k, device=dev) / 30
def tm(f, it=20):
    f(); torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): f()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it * 1e6
a = tm(lambda: T.fused_pass(A, Z, keep_y=True, gram=True, exact=True, gram64=True))
b = tm(lambda: T.fused_pass(A, Z, keep_y=True, gram=False, exact=True))
_, _, Y = T.fused_pass(A, Z, keep_y=True, gram=False, exact=True)
c = tm(lambda: T.gram64(Y))
print(f"final+G64 {a:.1f} us | final no-G {b:.1f} us | gram64(Y) {c:.1f} us | split {b + c:.1f} us")
