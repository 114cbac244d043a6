"""A/B the gemm_bf16_nt kernel variants in one process (guide §5.4 rule 24).

    python tools/gemm_ab.py [--sizes 4096 8192] [--iters 20] [--out gpurun_out/gemm_ab.json]

Times every variant at each size³ on uniform random [-1, 1) bf16 operands
(zero-filled operands read high: guide §5.4 rule 25) next to torch.matmul
(hipBLASLt) as the library reference, and prints one JSON document.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from headlamp_intel_gpu_plugin_amd.ops import workload  # noqa: E402


def time_torch(size, iters):
    a = (torch.rand(size, size, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(size, size, device="cuda") * 2 - 1).to(torch.bfloat16)
    for _ in range(3):
        a @ b.T
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        a @ b.T
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / 1e3)
    ts.sort()
    return workload.gemm_tflops(size, size, size, ts[len(ts) // 2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[2048, 4096, 8192])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    rows = []
    for size in args.sizes:
        r = {"size": size}
        for v in ("tile128", "tile256", "tile256_dma", "auto"):
            r[v] = round(workload.time_gemm(size=size, iters=args.iters, variant=v), 1)
        r["torch_hipblaslt"] = round(time_torch(size, args.iters), 1)
        rows.append(r)
        print(json.dumps(r), flush=True)
    doc = {"unit": "TFLOP/s (median)", "operands": "uniform random [-1,1) bf16", "device": torch.cuda.get_device_name(0),
           "rows": rows}
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
