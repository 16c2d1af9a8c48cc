"""What the vendor GEMM (torch.mm -> hipBLASLt) reaches on the 3x3 convolutions' GEMM shapes at
the 64x64 level (N=32, 128->128): forward / input-grad as [131072 x 1152] x [1152 x 128], weight-grad
as [128 x 131072] x [131072 x 1152]. Explicit im2col operands (not counted); bf16, fp32 accumulate.
A ceiling reference for the halo kernels (38.65 GFLOP per launch)."""
import torch


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    d = "cuda"
    bf = torch.bfloat16
    M, K, N = 131072, 1152, 128
    a = torch.randn(M, K, device=d, dtype=bf)
    b = torch.randn(K, N, device=d, dtype=bf)
    fl = 2.0 * M * K * N
    us = t(lambda: torch.mm(a, b))
    print(f"fwd   [{M}x{K}]x[{K}x{N}]: {us:7.1f} us  {fl / us / 1e6:7.1f} TF/s")
    g = torch.randn(N, M, device=d, dtype=bf)
    us = t(lambda: torch.mm(g, a))
    print(f"wgrad [{N}x{M}]x[{M}x{K}]: {us:7.1f} us  {fl / us / 1e6:7.1f} TF/s")
    a2 = torch.randn(M, 256, device=d, dtype=bf)
    b2 = torch.randn(256, 128, device=d, dtype=bf)
    us = t(lambda: torch.mm(a2, b2))
    print(f"1x1   [{M}x256]x[256x128]: {us:7.1f} us  {(M * 256 + M * 128) * 2 / us / 1e3:7.0f} GB/s")


if __name__ == "__main__":
    main()
