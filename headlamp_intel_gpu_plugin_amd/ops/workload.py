"""MI355X workload kernels (native: ops/kernels/workload.hip) with torch tensors.

* :func:`gemm_bf16_nt` — ``C = A @ B.T`` on MFMA (bf16 in, fp32 accumulate, bf16 out)
* :func:`stream_triad` — ``c = a + s * b`` (fp32, HBM-bound)
* :class:`Burner` — runs a GEMM + triad mix on a side stream for a target
  duration: the synthetic "GPU pod" whose power / HBM / activity the
  exporter reports.

Shapes are validated on the host before any launch (the kernels assume full
tiles and 16-byte alignment); there is no PyTorch fallback.
"""
from __future__ import annotations

import threading
from typing import Optional

import torch

from . import load_native

_mod = None


def native():
    global _mod
    if _mod is None:
        _mod = load_native("_workload")
    return _mod


def tile():
    return native().tile()


def _stream_handle(stream: Optional[torch.cuda.Stream], device) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


#: Kernel variants of gemm_bf16_nt (see kernels/workload.hip): picked by shape
#: by default; forcing one is for tests and A/B timing.
GEMM_VARIANTS = {"auto": 0, "tile128": 1, "tile256": 2, "tile256_dma": 3}


def gemm_bf16_nt(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
                 stream: Optional[torch.cuda.Stream] = None, variant: str = "auto") -> torch.Tensor:
    """C[M,N] = A[M,K] @ B[N,K]^T with M,N multiples of 128 and K of 64.

    ``variant`` forces one kernel: ``tile256`` needs M,N multiples of 256 and
    ``tile256_dma`` (the 8-phase LDS-DMA kernel) additionally K a multiple of 128.
    """
    if variant not in GEMM_VARIANTS:
        raise ValueError(f"unknown variant {variant!r}; one of {sorted(GEMM_VARIANTS)}")
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("gemm_bf16_nt expects bfloat16 inputs")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"shape mismatch: A{tuple(a.shape)} B{tuple(b.shape)} (need A[M,K], B[N,K])")
    if not (a.is_cuda and b.is_cuda) or a.device != b.device:
        raise ValueError("A and B must be on the same GPU")
    bm, bn, bk = tile()
    m, k = a.shape
    n = b.shape[0]
    if m % bm or n % bn or k % bk:
        raise ValueError(f"gemm_bf16_nt needs M%{bm}==0, N%{bn}==0, K%{bk}==0 (got {m}x{n}x{k})")
    a = a.contiguous()
    b = b.contiguous()
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    elif out.shape != (m, n) or out.dtype != torch.bfloat16 or not out.is_contiguous() or out.device != a.device:
        raise ValueError("out must be a contiguous bfloat16 [M,N] tensor on A's device")
    native().gemm_bf16_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, _stream_handle(stream, a.device),
                          GEMM_VARIANTS[variant])
    return out


def stream_triad(a: torch.Tensor, b: torch.Tensor, s: float, out: Optional[torch.Tensor] = None,
                 stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """out = a + s * b over contiguous float32 vectors whose length is a multiple of 4."""
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError("stream_triad expects float32")
    if a.shape != b.shape or not a.is_contiguous() or not b.is_contiguous():
        raise ValueError("a and b must be contiguous and the same shape")
    n = a.numel()
    if n % 4:
        raise ValueError("length must be a multiple of 4")
    if out is None:
        out = torch.empty_like(a)
    native().stream_triad(a.data_ptr(), b.data_ptr(), out.data_ptr(), n, float(s), _stream_handle(stream, a.device))
    return out


class Burner:
    """Keeps one GPU busy with a training-like mix until stopped.

    Each iteration runs ``gemms`` MFMA GEMMs of ``size``³ then one HBM triad
    over ``triad_mb`` MB on its own stream. With ``graph_iters > 0`` that many
    iterations are captured once into a HIP graph and replayed, so the host
    thread wakes once per replay instead of launching every kernel from
    Python. The default is eager launches: on this ROCm stack a device-wide
    ``torch.cuda.synchronize()`` takes ~0.4-2 s once a graph has been replayed
    on the device, even with the device idle (tools/diag/sync_vs_burner.py,
    profiles/r1_diag_graph_sync.md), and the benchmark's timed region is
    bracketed by exactly that call. Callers keep the launch rate low with
    larger kernels instead (bench.py: 2 × 8192³ GEMMs + triad per iteration).
    """

    def __init__(self, device: int = 0, size: int = 4096, gemms: int = 4, triad_mb: int = 1024,
                 graph_iters: int = 0):
        self.device = torch.device("cuda", device)
        self.size = size
        self.gemms = gemms
        self.triad_n = (triad_mb * 1024 * 1024 // 4) // 4 * 4
        self.graph_iters = graph_iters
        self.mode = "pending"  # "graph" once capture succeeded, "eager" if graphs are disabled
        self._stop = threading.Event()
        self._pause = threading.Event()
        self._idle = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.iterations = 0
        self.error: Optional[BaseException] = None

    def _run(self) -> None:
        try:
            torch.cuda.set_device(self.device)
            g = torch.Generator(device=self.device).manual_seed(0)
            a = torch.randn(self.size, self.size, device=self.device, dtype=torch.bfloat16, generator=g)
            b = torch.randn(self.size, self.size, device=self.device, dtype=torch.bfloat16, generator=g)
            c = torch.empty_like(a)
            x = torch.rand(self.triad_n, device=self.device, generator=g)
            y = torch.rand(self.triad_n, device=self.device, generator=g)
            z = torch.empty_like(x)
            stream = torch.cuda.Stream(self.device)

            def one_iteration():
                for _ in range(self.gemms):
                    gemm_bf16_nt(a, b, out=c, stream=stream)
                stream_triad(x, y, 0.5, out=z, stream=stream)

            with torch.cuda.stream(stream):
                one_iteration()  # warm-up outside capture (sets kernel attributes once)
            stream.synchronize()
            if self.graph_iters > 0:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=stream):
                    for _ in range(self.graph_iters):
                        one_iteration()
                self.mode = "graph"
                while not self._stop.is_set():
                    if self._pause.is_set():
                        self._hold()
                        continue
                    graph.replay()
                    stream.synchronize()
                    self.iterations += self.graph_iters
            else:
                self.mode = "eager"
                while not self._stop.is_set():
                    if self._pause.is_set():
                        self._hold()
                        continue
                    with torch.cuda.stream(stream):
                        one_iteration()
                    stream.synchronize()
                    self.iterations += 1
        except BaseException as e:  # surfaced by stop()
            self.error = e
        finally:
            self._idle.set()

    def _hold(self) -> None:
        self._idle.set()
        while self._pause.is_set() and not self._stop.is_set():
            self._stop.wait(0.001)
        self._idle.clear()

    def pause(self, timeout: float = 10.0) -> None:
        """Stop issuing work and wait until the in-flight iteration finished
        (a device-wide synchronize then only waits for the caller's work)."""
        if self._thread is None or not self._thread.is_alive():
            return
        self._pause.set()
        self._idle.wait(timeout)

    def resume(self) -> None:
        self._pause.clear()

    def start(self) -> "Burner":
        self._thread = threading.Thread(target=self._run, daemon=True, name="gpu-burner")
        self._thread.start()
        return self

    def stop(self, timeout: float = 30.0) -> int:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout)
        if self.error:
            raise RuntimeError(f"burner failed: {self.error}") from self.error
        return self.iterations

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def gemm_tflops(m: int, n: int, k: int, seconds: float) -> float:
    return 2.0 * m * n * k / seconds / 1e12


def time_gemm(size: int = 8192, iters: int = 20, device: int = 0, variant: str = "auto") -> float:
    """Median TFLOP/s of gemm_bf16_nt at size³ (uniform random operands)."""
    dev = torch.device("cuda", device)
    a = (torch.rand(size, size, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(size, size, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty_like(a)
    for _ in range(3):
        gemm_bf16_nt(a, b, out=c, variant=variant)
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        gemm_bf16_nt(a, b, out=c, variant=variant)
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e) / 1e3)
    times.sort()
    return gemm_tflops(size, size, size, times[len(times) // 2])


def time_triad(mb: int = 2048, iters: int = 20, device: int = 0) -> float:
    """Median TB/s of stream_triad over ``mb`` MB per vector (3 streams of traffic)."""
    dev = torch.device("cuda", device)
    n = (mb * 1024 * 1024 // 4) // 4 * 4
    x = torch.rand(n, device=dev)
    y = torch.rand(n, device=dev)
    z = torch.empty_like(x)
    for _ in range(3):
        stream_triad(x, y, 0.5, out=z)
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        stream_triad(x, y, 0.5, out=z)
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e) / 1e3)
    times.sort()
    return 3 * n * 4 / times[len(times) // 2] / 1e12

