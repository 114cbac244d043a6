"""Profiling target: the workload kernels at benchmark shapes (run under rocprofv3)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from headlamp_intel_gpu_plugin_amd.ops import workload  # noqa: E402

dev = torch.device("cuda", 0)
for size in (4096, 8192):
    a = (torch.rand(size, size, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(size, size, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty_like(a)
    for variant in ("tile256", "tile256_dma"):
        for _ in range(10):
            workload.gemm_bf16_nt(a, b, out=c, variant=variant)
    ref = torch.empty_like(a)
    for _ in range(10):
        torch.matmul(a, b.T, out=ref)  # hipBLASLt reference point
torch.cuda.synchronize()
n = 512 * 1024 * 1024 // 4
x = torch.rand(n, device=dev)
y = torch.rand(n, device=dev)
z = torch.empty_like(x)
for _ in range(10):
    workload.stream_triad(x, y, 0.5, out=z)
torch.cuda.synchronize()
print("gemm 8192:", round(workload.time_gemm(8192, 10), 1), "TF; triad:", round(workload.time_triad(2048, 10), 2), "TB/s")
