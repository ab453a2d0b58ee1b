"""tony_amd MFMA GEMMs vs hipBLASLt (torch.matmul) on the conv-shaped problems of Inception-v3 (bs128).

NT (forward / dgrad of 1x1 convs): C[M,N] = A[M,K] B[N,K]^T ; TN (wgrad): C[N1,N2] = A[M,N1]^T B[M,N2].
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tony_amd.ops.gemm import gemm_nt, gemm_tn  # noqa: E402

NT = [(156800, 64, 192), (156800, 352, 192), (156800, 192, 352), (36992, 768, 768), (36992, 192, 768),
      (36992, 768, 192), (8192, 1280, 1280), (8192, 2048, 1280), (682112, 80, 64), (156800, 64, 64)]
TN = [(156800, 352, 192), (36992, 768, 768), (36992, 192, 768), (8192, 1280, 1280), (682112, 80, 64)]


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    print("| NT M,N,K | tony ms (TF/s) | hipBLASLt ms (TF/s) |")
    print("|---|---|---|")
    for m, n, k in NT:
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
        f = 2.0 * m * n * k
        t1 = t(lambda: gemm_nt(a, b))
        t2 = t(lambda: a @ b.t())
        print(f"| {m},{n},{k} | {t1:.3f} ({f / t1 / 1e9:.0f}) | {t2:.3f} ({f / t2 / 1e9:.0f}) |")
    print("\n| TN M,N1,N2 | tony ms (TF/s) | hipBLASLt ms (TF/s) |")
    print("|---|---|---|")
    for m, n1, n2 in TN:
        a = torch.randn(m, n1, device=dev, dtype=torch.bfloat16)
        b = torch.randn(m, n2, device=dev, dtype=torch.bfloat16)
        f = 2.0 * m * n1 * n2
        t1 = t(lambda: gemm_tn(a, b))
        t2 = t(lambda: a.t() @ b)
        print(f"| {m},{n1},{n2} | {t1:.3f} ({f / t1 / 1e9:.0f}) | {t2:.3f} ({f / t2 / 1e9:.0f}) |")


if __name__ == "__main__":
    main()
