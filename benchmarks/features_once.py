"""Drive the fused feature GEMM a few times (PMC / trace target).
usage: python benchmarks/features_once.py [rows] [dim] [S] [dtype f32|bf16] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from libskylark_amd.ops import fused as F  # noqa: E402


def main():
    m = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    dt = torch.bfloat16 if (len(sys.argv) > 4 and sys.argv[4] == "bf16") else torch.float32
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    dev = torch.device("cuda")
    A = torch.rand(m, d, device=dev).to(dt)
    W = F.SplitW(torch.randn(S, d, device=dev) / 10)
    sh = torch.rand(S, device=dev) * 6.28
    for _ in range(reps):
        Z = F.feature_gemm(A, W, 1, shifts=sh, outscale=0.02, epi=F.EPI_COS)
    torch.cuda.synchronize()
    print("ok", tuple(Z.shape))


if __name__ == "__main__":
    main()
