"""Which hipBLASLt kernel torch.matmul picks for the step's NT GEMM shapes (for study of its
schedule with llvm-objdump), and its time per launch.  rocprofv3 --kernel-trace --stats -- python tools/blaslt_probe.py"""
import torch

torch.backends.cuda.matmul.allow_tf32 = False
for (M, N, K) in [(4096, 4096, 4096), (4800, 12288, 4096), (4800, 4096, 11008)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b.T
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(20):
        c = a @ b.T
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / 20
    print(f"M{M} N{N} K{K}: {us:.1f} us  {2 * M * N * K / us / 1e6:.0f} TFLOP/s", flush=True)
