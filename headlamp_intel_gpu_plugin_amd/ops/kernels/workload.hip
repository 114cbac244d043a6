// GPU workload kernels for the synthetic cluster's GPU pods (gfx950 / CDNA4).
//
// The plugin observes MI355X nodes; to validate that path end to end on a
// real GPU (exporter → Prometheus → Metrics page), the benchmark's "pods"
// must actually load the device the way training jobs do: matrix cores and
// HBM. Two kernels, written for CDNA4 directly:
//
//   gemm_bf16_nt  C[M,N] = A[M,K] · B[N,K]ᵀ, bf16 in, fp32 accumulate on
//                 MFMA (v_mfma_f32_16x16x32_bf16), bf16 out (RNE).
//                 Two instantiations of one template:
//                   256×256×64 tile, 8 wave64s as 2×4, each wave a 128×64
//                   sub-tile (8×4 MFMA tiles), 144 KiB of LDS → 1 block/CU —
//                   used when M and N are multiples of 256;
//                   128×128×64 tile, 4 wave64s as 2×2 (64×64 each), 72 KiB.
//                 A/B staged global→LDS with 16-byte vector loads into a double
//                 buffer (one barrier per K-step: tile k+1 is fetched into
//                 registers while tile k is consumed, then written to the
//                 other buffer); LDS rows padded to 144 B so the 16 lanes of a
//                 ds_read_b128 group hit 16 distinct 4-bank slots; each MFMA
//                 cluster runs at s_setprio 1 (keeps hipcc from moving MFMAs
//                 into the load phase, guide T5); bijective XCD-aware block
//                 remap + 8-row tile grouping so blocks sharing an XCD's L2
//                 work on neighbouring tiles. Measured on MI355X (random
//                 [-1,1) operands, tools/microbench/gemm_variants.hip):
//                 256² tile 1177 TFLOP/s at 8192³, 1025 at 4096³; 128² tile
//                 888–950 at 8192³.
//   stream_triad  c = a + s·b over fp32, 16-byte accesses, one pass with 4
//                 vectors per thread and non-temporal stores: 5.78 TB/s.
//
// Both are bounds-safe by construction: the host wrappers reject shapes the
// tiling does not cover (see ops/workload.py), and every launch is checked.
//
// Python binding: CPython C API module `_workload` (bottom of file), taking
// device pointers as integers and the caller's HIP stream, so it composes
// with PyTorch tensors and streams without a torch C++ dependency.

#include <Python.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// Staging registers use a clang vector type: arrays of HIP's struct-based
// uint4 are kept in scratch memory by hipcc, vector-typed arrays are not.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int LDS_STRIDE = BK + 8;  // bf16 elements per LDS row (144 B)

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

// Bijective remap: blocks b and b+8 run on the same XCD (round-robin dispatch),
// so give each XCD-group a contiguous range of tile ids (guide §5, "XCD swizzle
// must be bijective").
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig % 8;
  const int q = nwg / 8;
  const int r = nwg % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

template <int BM, int BN, int WM, int WN>
struct GemmTile {
  static constexpr int kThreads = WM * WN * 64;
  static constexpr int kTm = BM / WM / 16;  // MFMA tiles per wave along M
  static constexpr int kTn = BN / WN / 16;  // … along N
  static constexpr int kCa = BM * BK * 2 / 16 / kThreads;  // 16-B chunks per thread, A
  static constexpr int kCb = BN * BK * 2 / 16 / kThreads;  // … B
  static constexpr int kRowStep = kThreads / 8;            // rows covered by one chunk pass
  static constexpr size_t kLds = 2 * (BM + BN) * LDS_STRIDE * sizeof(uint16_t);
  static_assert(kCa * kThreads * 16 == BM * BK * 2 && kCb * kThreads * 16 == BN * BK * 2, "tile/thread mismatch");
};

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void gemm_bf16_nt(const uint16_t* __restrict__ A,
                                                             const uint16_t* __restrict__ B,
                                                             uint16_t* __restrict__ C, int M, int N, int K) {
  using T = GemmTile<BM, BN, WM, WN>;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];  // [2][A rows | B rows][LDS_STRIDE]

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int wg = xcd_remap(static_cast<int>(blockIdx.x), tiles_m * tiles_n);
  // Group 8 tile-rows so consecutive ids share B tiles in L2.
  const int span = 8 * tiles_n;
  const int first_m = (wg / span) * 8;
  const int rows_in_group = min(8, tiles_m - first_m);
  const int m0 = (first_m + (wg % span) % rows_in_group) * BM;
  const int n0 = ((wg % span) / rows_in_group) * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / WN;
  const int wc = wave % WN;

  // Chunk p of this thread: row srow + p*kRowStep, 16-byte column scol.
  const int srow = tid >> 3;
  const int scol = (tid & 7) * 8;
  const uint16_t* ga = A + static_cast<size_t>(m0 + srow) * K + scol;
  const uint16_t* gb = B + static_cast<size_t>(n0 + srow) * K + scol;
  const size_t gstep = static_cast<size_t>(T::kRowStep) * K;
  u32x4 ra[T::kCa], rb[T::kCb];

  f32x4 acc[T::kTm][T::kTn];
#pragma unroll
  for (int i = 0; i < T::kTm; ++i)
#pragma unroll
    for (int j = 0; j < T::kTn; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define GEMM_LOAD(k0)                                                                                   \
  {                                                                                                     \
    _Pragma("unroll") for (int p = 0; p < T::kCa; ++p) ra[p] = *reinterpret_cast<const u32x4*>(ga + p * gstep + (k0)); \
    _Pragma("unroll") for (int p = 0; p < T::kCb; ++p) rb[p] = *reinterpret_cast<const u32x4*>(gb + p * gstep + (k0)); \
  }
#define GEMM_STORE(buf)                                                                                 \
  {                                                                                                     \
    uint16_t* la_ = lds + (buf) * (BM + BN) * LDS_STRIDE + srow * LDS_STRIDE + scol;                    \
    uint16_t* lb_ = la_ + BM * LDS_STRIDE;                                                              \
    _Pragma("unroll") for (int p = 0; p < T::kCa; ++p)                                                  \
      *reinterpret_cast<u32x4*>(la_ + p * T::kRowStep * LDS_STRIDE) = ra[p];                            \
    _Pragma("unroll") for (int p = 0; p < T::kCb; ++p)                                                  \
      *reinterpret_cast<u32x4*>(lb_ + p * T::kRowStep * LDS_STRIDE) = rb[p];                            \
  }

  const int nk = K / BK;
  GEMM_LOAD(0)
  GEMM_STORE(0)
  __syncthreads();

  // v_mfma_f32_16x16x32_bf16 fragments: lane l holds A[row l&15][k 8(l>>4)..+7]
  // and B[k 8(l>>4)..+7][col l&15].
  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  const int arow = wr * (BM / WM) + frow;
  const int brow = wc * (BN / WN) + frow;

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) GEMM_LOAD((kt + 1) * BK)  // in flight while this tile is consumed

    const uint16_t* la = lds + buf * (BM + BN) * LDS_STRIDE;
    const uint16_t* lb = la + BM * LDS_STRIDE;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[T::kTm], bfr[T::kTn];
#pragma unroll
      for (int i = 0; i < T::kTm; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(la + (arow + i * 16) * LDS_STRIDE + kk + fk);
#pragma unroll
      for (int j = 0; j < T::kTn; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + (brow + j * 16) * LDS_STRIDE + kk + fk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < T::kTm; ++i)
#pragma unroll
        for (int j = 0; j < T::kTn; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }

    // The other buffer was last read before the previous barrier.
    if (kt + 1 < nk) GEMM_STORE(buf ^ 1)
    __syncthreads();
  }
#undef GEMM_LOAD
#undef GEMM_STORE

  // Epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r.
  const int ccol = lane & 15;
  const int crow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < T::kTm; ++i)
#pragma unroll
    for (int j = 0; j < T::kTn; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * (BM / WM) + i * 16 + crow + r;
        const int col = n0 + wc * (BN / WN) + j * 16 + ccol;
        C[static_cast<size_t>(row) * N + col] = f32_to_bf16_rne(acc[i][j][r]);
      }
}

// One pass, no grid-stride loop: each thread moves TRIAD_U 16-byte vectors,
// all loads issued before any store (memory-level parallelism), and the
// result is written non-temporally so it does not evict the operands from
// L2 / Infinity Cache. Measured on MI355X (2 GiB per vector): 5.78 TB/s vs
// 4.6–5.3 TB/s for grid-stride variants (tools/microbench/triad_variants.hip).
constexpr int TRIAD_U = 4;
typedef float vf4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_triad(const vf4* __restrict__ a, const vf4* __restrict__ b,
                                                    vf4* __restrict__ c, float s, size_t n4) {
  const size_t base = static_cast<size_t>(blockIdx.x) * (256 * TRIAD_U) + threadIdx.x;
  vf4 x[TRIAD_U], y[TRIAD_U];
#pragma unroll
  for (int u = 0; u < TRIAD_U; ++u) {
    const size_t i = base + static_cast<size_t>(u) * 256;
    if (i < n4) {
      x[u] = a[i];
      y[u] = b[i];
    }
  }
#pragma unroll
  for (int u = 0; u < TRIAD_U; ++u) {
    const size_t i = base + static_cast<size_t>(u) * 256;
    if (i < n4) __builtin_nontemporal_store(x[u] + s * y[u], &c[i]);
  }
}

using Big = GemmTile<256, 256, 2, 4>;
using Small = GemmTile<128, 128, 2, 2>;
bool g_big_attr = false;
bool g_small_attr = false;

template <int BM, int BN, int WM, int WN>
const char* launch_tile(const void* a, const void* b, void* c, int m, int n, int k, hipStream_t stream, bool* attr) {
  using T = GemmTile<BM, BN, WM, WN>;
  auto kernel = gemm_bf16_nt<BM, BN, WM, WN>;
  if (!*attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(T::kLds)) != hipSuccess)
      return "gemm_bf16_nt: cannot reserve LDS";
    *attr = true;
  }
  const int blocks = (m / BM) * (n / BN);
  hipLaunchKernelGGL(kernel, dim3(blocks), dim3(T::kThreads), T::kLds, stream, static_cast<const uint16_t*>(a),
                     static_cast<const uint16_t*>(b), static_cast<uint16_t*>(c), m, n, k);
  hipError_t err = hipGetLastError();
  return err == hipSuccess ? nullptr : hipGetErrorString(err);
}

const char* launch_gemm(const void* a, const void* b, void* c, int m, int n, int k, hipStream_t stream) {
  if (m <= 0 || n <= 0 || k <= 0 || m % 128 || n % 128 || k % BK) return "gemm_bf16_nt: M,N must be multiples of 128 and K of 64";
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) return "gemm_bf16_nt: A and B must be 16-byte aligned";
  // The 256² tile needs ≥ one block per CU to beat the 128² tile (256 CUs).
  if (m % 256 == 0 && n % 256 == 0 && (m / 256) * (n / 256) >= 128)
    return launch_tile<256, 256, 2, 4>(a, b, c, m, n, k, stream, &g_big_attr);
  return launch_tile<128, 128, 2, 2>(a, b, c, m, n, k, stream, &g_small_attr);
}

const char* launch_triad(const void* a, const void* b, void* c, size_t n, float s, hipStream_t stream) {
  if (n == 0 || n % 4) return "stream_triad: length must be a positive multiple of 4";
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15)
    return "stream_triad: buffers must be 16-byte aligned";
  const size_t n4 = n / 4;
  const size_t per_block = 256 * TRIAD_U;
  const size_t blocks = (n4 + per_block - 1) / per_block;
  if (blocks > 0x7fffffffu) return "stream_triad: vector too long for one pass";
  hipLaunchKernelGGL(stream_triad, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                     static_cast<const vf4*>(a), static_cast<const vf4*>(b), static_cast<vf4*>(c), s, n4);
  hipError_t err = hipGetLastError();
  return err == hipSuccess ? nullptr : hipGetErrorString(err);
}

// ---------------------------------------------------------------------------
// Python binding
// ---------------------------------------------------------------------------

PyObject* py_gemm(PyObject*, PyObject* args) {
  unsigned long long a, b, c, stream;
  int m, n, k;
  if (!PyArg_ParseTuple(args, "KKKiiiK", &a, &b, &c, &m, &n, &k, &stream)) return nullptr;
  const char* err = launch_gemm(reinterpret_cast<void*>(a), reinterpret_cast<void*>(b), reinterpret_cast<void*>(c), m,
                                n, k, reinterpret_cast<hipStream_t>(stream));
  if (err) {
    PyErr_SetString(PyExc_RuntimeError, err);
    return nullptr;
  }
  Py_RETURN_NONE;
}

PyObject* py_triad(PyObject*, PyObject* args) {
  unsigned long long a, b, c, n, stream;
  double s;
  if (!PyArg_ParseTuple(args, "KKKKdK", &a, &b, &c, &n, &s, &stream)) return nullptr;
  const char* err = launch_triad(reinterpret_cast<void*>(a), reinterpret_cast<void*>(b), reinterpret_cast<void*>(c),
                                 static_cast<size_t>(n), static_cast<float>(s), reinterpret_cast<hipStream_t>(stream));
  if (err) {
    PyErr_SetString(PyExc_RuntimeError, err);
    return nullptr;
  }
  Py_RETURN_NONE;
}

PyObject* py_tile(PyObject*, PyObject*) { return Py_BuildValue("(iii)", 128, 128, BK); }

PyMethodDef kMethods[] = {
    {"gemm_bf16_nt", py_gemm, METH_VARARGS, "gemm_bf16_nt(a, b, c, M, N, K, stream): C = A @ B^T (bf16, fp32 acc)."},
    {"stream_triad", py_triad, METH_VARARGS, "stream_triad(a, b, c, n, s, stream): c = a + s*b (fp32)."},
    {"tile", py_tile, METH_NOARGS, "(BM, BN, BK) of the GEMM tiling."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_workload", "MI355X workload kernels (MFMA GEMM, HBM triad).", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__workload(void) { return PyModule_Create(&kModule); }
