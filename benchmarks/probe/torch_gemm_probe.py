import torch, time, json
dev = torch.device("cuda")
def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / reps
for dt, m, n in ((torch.float32, 1_000_000, 1000), (torch.float64, 200_000, 5000)):
    A = torch.randn(m, n, device=dev, dtype=dt)
    for k in (40, 128):
        Z = torch.randn(n, k, device=dev, dtype=dt)
        Y = torch.randn(m, k, device=dev, dtype=dt)
        a = t(lambda: A @ Z)
        b = t(lambda: A.t() @ Y)
        gb = m * n * A.element_size() / 1e9
        print(json.dumps({"dtype": str(dt), "m": m, "n": n, "k": k, "AZ_ms": round(a, 3), "AZ_TBps": round(gb / a, 2),
                          "AtY_ms": round(b, 3), "AtY_TBps": round(gb / b, 2)}), flush=True)
    del A
    torch.cuda.empty_cache()
