"""GPU tests for the native code (run on an MI355X with ``pytest -m gpu``).

Kernel numerics are checked against a plain PyTorch fp32 reference of the same
op. The probe is checked against the MI355X facts the plugin assumes
(gfx950, 256 CUs, wave64, 288 GB HBM).
"""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

from headlamp_intel_gpu_plugin_amd.ops import probe, workload  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    return torch.device("cuda", 0)


# ---------------------------------------------------------------------------
# probe
# ---------------------------------------------------------------------------

def test_probe_sees_devices(dev):
    assert probe.available()
    assert probe.device_count() >= 1


def test_probe_device_is_mi355x(dev):
    info = probe.device_info(0)
    assert info["arch"].startswith("gfx950"), info
    assert info["wavefront"] == 64
    assert info["compute_units"] == 256, info
    assert 280e9 < info["hbm_bytes"] <= 288 * 2**30, info  # 288 GiB
    assert info["lds_per_cu"] >= 64 * 1024
    assert len(info["bdf"]) >= 12 and info["bdf"].count(":") == 2


def test_probe_sample_reads_sysfs(dev):
    s = probe.sample(0)
    present = {k for k, v in s.items() if v is not None}
    # At least the HBM and activity counters are world-readable on amdgpu.
    assert present & {"vram_total_b", "vram_used_b", "gfx_busy_pct", "power_w"}, s
    if s["vram_total_b"] is not None:
        assert s["vram_total_b"] > 250e9
    if s["power_w"] is not None:
        assert 10 < s["power_w"] < 2000


def test_probe_render_metrics_parses(dev):
    text = probe.render_metrics("node-x")
    rows = probe.parse_exposition(text)
    names = {n for n, _, _ in rows}
    assert "gpu_total_vram" in names
    for n, labels, v in rows:
        assert labels["hostname"] == "node-x"
        assert int(labels["gpu_id"]) < probe.device_count()


def test_probe_topology_links(dev):
    topo = probe.topology()
    n = probe.device_count()
    assert len(topo) == n * (n - 1)
    for k, v in topo.items():
        # On an 8×MI355X node every peer is one xGMI hop away.
        assert v["type"] in ("XGMI", "PCIE", "OTHER", "UNKNOWN")


def test_probe_bad_index_raises(dev):
    with pytest.raises(IndexError):
        probe.sample(probe.device_count())


# ---------------------------------------------------------------------------
# workload kernels vs fp32 PyTorch reference
# ---------------------------------------------------------------------------

def _ref(a, b):
    return a.float() @ b.float().T


@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (256, 384, 192), (1024, 512, 2048), (384, 1152, 64),
                                   # ≥128 tiles of 256² → the 8-wave 256×256 kernel
                                   (2048, 4096, 320), (4096, 2048, 64)])
def test_gemm_matches_fp32_reference(dev, m, n, k):
    g = torch.Generator(device=dev).manual_seed(m * 7 + n + k)
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
    b = torch.randn(n, k, device=dev, dtype=torch.bfloat16, generator=g)
    c = workload.gemm_bf16_nt(a, b)
    ref = _ref(a, b)
    # Output is rounded to bf16 (8 mantissa bits): relative 2^-8 of the magnitude.
    tol = ref.abs().clamp_min(1.0) * 2 ** -7
    assert ((c.float() - ref).abs() <= tol).all(), (c.float() - ref).abs().max().item()


def test_gemm_identity_with_asymmetric_b(dev):
    # A = I catches a transposed C-write only with an asymmetric B (guide §3).
    n = 128
    a = torch.eye(n, device=dev, dtype=torch.bfloat16)
    bvals = torch.arange(n * n, device=dev, dtype=torch.float32).reshape(n, n) % 97 - 48
    b = bvals.to(torch.bfloat16)
    a_k = torch.zeros(n, 128, device=dev, dtype=torch.bfloat16)
    a_k[:, :n] = a
    b_k = torch.zeros(n, 128, device=dev, dtype=torch.bfloat16)
    b_k[:, :n] = b
    c = workload.gemm_bf16_nt(a_k, b_k)
    # C = I @ B^T = B^T exactly (small integers are exact in bf16).
    assert torch.equal(c.float(), bvals.T.contiguous())


@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (4096, 2048, 128)])
def test_gemm_multi_tile_exact_integers(dev, m, n, k):
    # |sum| <= 2*1*k <= 256: exact in bf16, so any indexing error shows up exactly.
    a = (torch.arange(m * k, device=dev) % 5 - 2).reshape(m, k).to(torch.bfloat16)
    b = ((torch.arange(n * k, device=dev) * 7) % 3 - 1).reshape(n, k).to(torch.bfloat16)
    c = workload.gemm_bf16_nt(a, b)
    assert torch.equal(c.float(), _ref(a, b))


def test_gemm_big_tile_identity_asymmetric(dev):
    # A = I (padded to 4096 rows) with an asymmetric B through the 256² kernel.
    m, n, k = 4096, 2048, 256
    a = torch.zeros(m, k, device=dev, dtype=torch.bfloat16)
    a[:k, :k] = torch.eye(k, device=dev, dtype=torch.bfloat16)
    bvals = (torch.arange(n * k, device=dev, dtype=torch.float32).reshape(n, k) % 61) - 30
    c = workload.gemm_bf16_nt(a, bvals.to(torch.bfloat16))
    assert torch.equal(c[:k].float(), bvals.T[:k].contiguous())
    assert torch.count_nonzero(c[k:]) == 0


# Every kernel variant forced on shapes that exercise its edges: one block,
# one loop iteration (K=128 for the 8-phase kernel), odd tile counts, M != N.
VARIANT_SHAPES = {
    "tile128": [(128, 128, 64), (384, 640, 192), (1024, 512, 1024)],
    "tile256": [(256, 256, 64), (512, 768, 320), (2048, 1024, 1024)],
    "tile256_dma": [(256, 256, 128), (256, 512, 384), (768, 512, 256), (2048, 1024, 1024), (1280, 2304, 640)],
}


@pytest.mark.parametrize("variant,m,n,k", [(v, *shape) for v, shapes in VARIANT_SHAPES.items() for shape in shapes])
def test_gemm_variant_exact_integers(dev, variant, m, n, k):
    a = (torch.arange(m * k, device=dev) % 5 - 2).reshape(m, k).to(torch.bfloat16)
    b = ((torch.arange(n * k, device=dev) * 7 + 3) % 3 - 1).reshape(n, k).to(torch.bfloat16)
    c = workload.gemm_bf16_nt(a, b, variant=variant)
    assert torch.equal(c.float(), _ref(a, b)), (c.float() - _ref(a, b)).abs().max().item()


@pytest.mark.parametrize("variant", ["tile256", "tile256_dma"])
def test_gemm_variant_identity_asymmetric(dev, variant):
    # A = I with an asymmetric B: a transposed store or a swapped half-tile shows up exactly.
    m, n, k = 512, 768, 256
    a = torch.zeros(m, k, device=dev, dtype=torch.bfloat16)
    a[:k, :k] = torch.eye(k, device=dev, dtype=torch.bfloat16)
    bvals = (torch.arange(n * k, device=dev, dtype=torch.float32).reshape(n, k) % 61) - 30
    c = workload.gemm_bf16_nt(a, bvals.to(torch.bfloat16), variant=variant)
    assert torch.equal(c[:k].float(), bvals.T[:k].contiguous())
    assert torch.count_nonzero(c[k:]) == 0


def test_gemm_dma_kernel_repeatable_random(dev):
    # LDS-DMA ordering bugs show up as rare wrong tiles: compare 30 launches
    # at two sizes against one fp32 reference each, bit for bit across runs.
    for m, n, k in [(4096, 4096, 1024), (2048, 3072, 2048)]:
        g = torch.Generator(device=dev).manual_seed(m + n + k)
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=g)
        b = torch.randn(n, k, device=dev, dtype=torch.bfloat16, generator=g)
        ref = _ref(a, b)
        first = workload.gemm_bf16_nt(a, b, variant="tile256_dma")
        tol = ref.abs().clamp_min(1.0) * 2 ** -7
        assert ((first.float() - ref).abs() <= tol).all()
        for _ in range(29):
            again = workload.gemm_bf16_nt(a, b, variant="tile256_dma")
            assert torch.equal(again, first)


def test_gemm_variant_rejects_unfit_shapes(dev):
    a = torch.randn(256, 192, device=dev, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        workload.gemm_bf16_nt(a, a, variant="tile256_dma")  # K % 128 != 0
    with pytest.raises(ValueError):
        workload.gemm_bf16_nt(a, a, variant="nope")


def test_gemm_misaligned_output(dev):
    # The 8-phase kernel's packed epilogue stores 16 B per lane: a C that is
    # contiguous but not 16-B aligned is refused by that variant and routed
    # to a 2-byte-store kernel by `auto`, with the same result.
    g = torch.Generator(device=dev).manual_seed(7)
    a = torch.randn(2048, 256, device=dev, dtype=torch.bfloat16, generator=g)
    b = torch.randn(4096, 256, device=dev, dtype=torch.bfloat16, generator=g)
    buf = torch.empty(2048 * 4096 + 1, device=dev, dtype=torch.bfloat16)
    out = buf[1:].view(2048, 4096)  # 2-byte offset
    with pytest.raises(RuntimeError):
        workload.gemm_bf16_nt(a, b, out=out, variant="tile256_dma")
    workload.gemm_bf16_nt(a, b, out=out)
    assert torch.equal(out, workload.gemm_bf16_nt(a, b, variant="tile256"))


def test_gemm_variants_throughput(dev):
    # A/B in one process (guide §5.4 rule 24): the kernel the default dispatch
    # picks at this shape (8-phase LDS-DMA) must beat the other two, and `auto`
    # must be that kernel (same speed within clock noise).
    tf = {v: workload.time_gemm(size=8192, iters=10, variant=v) for v in ("tile128", "tile256", "tile256_dma", "auto")}
    print("gemm 8192^3 TFLOP/s: " + ", ".join(f"{v} {t:.0f}" for v, t in tf.items()))
    assert tf["tile256_dma"] > 1.1 * max(tf["tile128"], tf["tile256"]), tf
    assert tf["auto"] > 1.05 * max(tf["tile128"], tf["tile256"]), tf


def test_gemm_respects_stream(dev):
    a = torch.randn(512, 256, device=dev, dtype=torch.bfloat16)
    b = torch.randn(512, 256, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        c = workload.gemm_bf16_nt(a, b, stream=s)
    s.synchronize()
    assert torch.allclose(c.float(), _ref(a, b), rtol=2e-2, atol=2e-1)


def test_gemm_rejects_partial_tiles(dev):
    a = torch.randn(100, 64, device=dev, dtype=torch.bfloat16)
    b = torch.randn(128, 64, device=dev, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        workload.gemm_bf16_nt(a, b)


def test_triad_matches_reference(dev):
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.rand(3 * 1024 * 1024 + 4, device=dev, generator=g)
    y = torch.rand(3 * 1024 * 1024 + 4, device=dev, generator=g)
    z = workload.stream_triad(x, y, -1.75)
    torch.testing.assert_close(z, x + -1.75 * y)


def test_gemm_throughput_floor(dev):
    tf = workload.time_gemm(size=8192, iters=10)
    print(f"gemm_bf16_nt 8192^3: {tf:.0f} TFLOP/s")
    assert tf > 200, tf  # dense bf16 peak 2500; floor catches a broken (non-MFMA) path


def test_triad_bandwidth_floor(dev):
    tb = workload.time_triad(mb=2048, iters=10)
    print(f"stream_triad: {tb:.2f} TB/s")
    assert tb > 2.5, tb


def test_burner_runs_and_loads_gpu(dev):
    with workload.Burner(device=0, size=2048, gemms=2, triad_mb=64) as b:
        time.sleep(1.5)
        busy = probe.sample(0)["gfx_busy_pct"]
        # Paused between iterations, a device-wide synchronize only waits for
        # the caller's own work (bench.py brackets its timed region so).
        b.pause()
        n = b.iterations
        t = time.perf_counter()
        torch.cuda.synchronize()
        assert time.perf_counter() - t < 0.2
        time.sleep(0.1)
        assert b.iterations == n  # nothing issued while paused
        b.resume()
        time.sleep(0.3)
    assert b.mode == "eager" and b.iterations > n
    if busy is not None:
        assert busy >= 0
    with workload.Burner(device=0, size=1024, gemms=1, triad_mb=16, graph_iters=4) as g:
        time.sleep(0.5)
    assert g.mode == "graph" and g.iterations >= 4  # the mix also replays as one captured HIP graph


def test_native_kernels_replay_in_a_hip_graph(dev):
    # The extension launches on the caller's stream, so it is capturable.
    a = torch.randn(512, 256, device=dev, dtype=torch.bfloat16)
    b = torch.randn(768, 256, device=dev, dtype=torch.bfloat16)
    c = torch.empty(512, 768, device=dev, dtype=torch.bfloat16)
    x = torch.rand(1 << 16, device=dev)
    y = torch.rand(1 << 16, device=dev)
    z = torch.empty_like(x)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        workload.gemm_bf16_nt(a, b, out=c, stream=s)
        workload.stream_triad(x, y, 2.0, out=z, stream=s)
    s.synchronize()
    eager_c, eager_z = c.clone(), z.clone()
    c.zero_()
    z.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        workload.gemm_bf16_nt(a, b, out=c, stream=s)
        workload.stream_triad(x, y, 2.0, out=z, stream=s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(c, eager_c) and torch.equal(z, eager_z)
