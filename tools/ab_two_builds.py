"""Same-process A/B of builds of the `_workload` module (guide §5.4 rule 24).

    python tools/ab_two_builds.py OTHER.so [OTHER2.so ...] [--sizes 4096 8192] [--iters 20] [--rounds 3]

Loads the in-tree build ("new") and every given build (named after its
directory) side by side, then times the 8-phase GEMM (variant tile256_dma)
of each, interleaved round by round on the same uniform random [-1, 1)
operands, and prints the medians (TFLOP/s) and whether all outputs agree.
"""
import argparse
import importlib.machinery
import importlib.util
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    loader = importlib.machinery.ExtensionFileLoader("_workload", path)
    spec = importlib.util.spec_from_file_location("_workload", path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules.pop("_workload", None)
    return mod


def time_one(mod, a, b, c, size, iters):
    stream = torch.cuda.current_stream().cuda_stream
    args = (a.data_ptr(), b.data_ptr(), c.data_ptr(), size, size, size, stream, 3)
    for _ in range(3):
        mod.gemm_bf16_nt(*args)
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        mod.gemm_bf16_nt(*args)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / 1e3)
    return 2.0 * size ** 3 / statistics.median(ts) / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("builds", nargs="+")
    ap.add_argument("--sizes", type=int, nargs="+", default=[4096, 8192])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    mods = {"new": load(os.path.join(ROOT, "headlamp_intel_gpu_plugin_amd", "ops", "_workload.so"))}
    for path in args.builds:
        name = os.path.basename(os.path.dirname(os.path.abspath(path)))
        mods["old" if name == "prev" else name] = load(path)
    for size in args.sizes:
        a = (torch.rand(size, size, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(size, size, device="cuda") * 2 - 1).to(torch.bfloat16)
        outs = {k: torch.empty_like(a) for k in mods}
        tf = {k: [] for k in mods}
        for _ in range(args.rounds):
            for k, m in mods.items():
                tf[k].append(time_one(m, a, b, outs[k], size, args.iters))
        same = all(torch.equal(outs["new"], o) for o in outs.values())
        print(json.dumps({"size": size, **{k: round(statistics.median(v), 1) for k, v in tf.items()},
                          "rounds": {k: [round(x, 1) for x in v] for k, v in tf.items()}, "bitwise_equal": same}),
              flush=True)


if __name__ == "__main__":
    main()
