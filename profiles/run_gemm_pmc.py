"""PMC target: each GEMM variant 5x at 8192^3 (uniform random operands), run under rocprofv3 --pmc."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from headlamp_intel_gpu_plugin_amd.ops import workload  # noqa: E402

dev = torch.device("cuda", 0)
size = 8192
a = (torch.rand(size, size, device=dev) * 2 - 1).to(torch.bfloat16)
b = (torch.rand(size, size, device=dev) * 2 - 1).to(torch.bfloat16)
c = torch.empty_like(a)
for variant in ("tile128", "tile256", "tile256_dma"):
    for _ in range(5):
        workload.gemm_bf16_nt(a, b, out=c, variant=variant)
torch.cuda.synchronize()
x = torch.rand(256 * 1024 * 1024, device=dev)
y = torch.rand_like(x)
z = torch.empty_like(x)
for _ in range(5):
    workload.stream_triad(x, y, 0.5, out=z)
torch.cuda.synchronize()
print("done")
