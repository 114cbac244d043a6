"""How long does torch.cuda.synchronize() take while a Burner keeps the GPU busy?"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from headlamp_intel_gpu_plugin_amd.ops.workload import Burner  # noqa: E402

for gi in (0, 4, 16):
    b = Burner(device=0, size=4096, gemms=4, triad_mb=512, graph_iters=gi).start()
    time.sleep(1.0)
    ts = []
    for _ in range(8):
        t = time.perf_counter()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
        time.sleep(0.05)
    paused = []
    for _ in range(8):
        t = time.perf_counter()
        b.pause()
        torch.cuda.synchronize()
        b.resume()
        paused.append((time.perf_counter() - t) * 1e3)
        time.sleep(0.05)
    it0 = b.iterations
    time.sleep(1.0)
    rate = b.iterations - it0
    b.stop()
    print(f"graph_iters={gi} mode={b.mode} iters/s={rate} sync ms: " + " ".join(f"{x:.1f}" for x in ts)
          + " | paused sync ms: " + " ".join(f"{x:.1f}" for x in paused), flush=True)
