// GPU workload kernels for the synthetic cluster's GPU pods (gfx950 / CDNA4).
//
// The plugin observes MI355X nodes; to validate that path end to end on a
// real GPU (exporter → Prometheus → Metrics page), the benchmark's "pods"
// must actually load the device the way training jobs do: matrix cores and
// HBM. Two kernels, written for CDNA4 directly:
//
//   gemm_bf16_nt  C[M,N] = A[M,K] · B[N,K]ᵀ, bf16 in, fp32 accumulate on
//                 MFMA (v_mfma_f32_16x16x32_bf16), bf16 out (RNE).
//                 128×128×64 block tile, 4 wave64s as 2×2, each wave a 64×64
//                 sub-tile = 4×4 MFMA tiles; A/B staged global→LDS with
//                 16-byte vector loads into a double buffer (one barrier per
//                 K-step: tile k+1 is fetched into registers while tile k is
//                 consumed, then written to the other buffer); LDS rows padded
//                 to 144 B so the 16 lanes of a ds_read_b128 group hit 16
//                 distinct 4-bank slots; bijective XCD-aware block remap so
//                 blocks that share an XCD's L2 work on neighbouring tiles.
//   stream_triad  c = a + s·b over fp32 with 16-byte accesses, grid-stride —
//                 the HBM-bound half of a training step.
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

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 64;
constexpr int THREADS = 256;              // 4 wave64
constexpr int LDS_STRIDE = BK + 8;        // bf16 elements per LDS row (144 B)
constexpr int TILE_ELEMS = BM * LDS_STRIDE;
constexpr int CHUNKS = (BM * BK * 2) / 16 / THREADS;  // 16-B chunks per thread per operand (= 4)

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

__global__ __launch_bounds__(THREADS) void gemm_bf16_nt(const uint16_t* __restrict__ A,
                                                           const uint16_t* __restrict__ B,
                                                           uint16_t* __restrict__ C, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];  // [2][A|B][BM][LDS_STRIDE]

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(static_cast<int>(blockIdx.x), nwg);
  // Group 8 tile-rows together so consecutive ids share B tiles in L2.
  constexpr int GROUP = 8;
  const int group_span = GROUP * tiles_n;
  const int group = wg / group_span;
  const int first_m = group * GROUP;
  const int rows_in_group = min(GROUP, tiles_m - first_m);
  const int tm = first_m + (wg % group_span) % rows_in_group;
  const int tn = (wg % group_span) / rows_in_group;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1;  // wave row (0..1) → 64 rows
  const int wc = wave & 1;   // wave col (0..1) → 64 cols

  // Global → register staging: chunk c = p*THREADS + tid covers row c/8 and
  // 16-B column c%8. Eight named registers rather than an array indexed in
  // a loop: hipcc otherwise keeps the staging array in scratch memory.
  uint4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
  const int srow = tid >> 3;         // row of chunk p=0; chunk p adds p*32 rows
  const int scol = (tid & 7) * 8;
  const uint16_t* ga = A + static_cast<size_t>(m0 + srow) * K + scol;
  const uint16_t* gb = B + static_cast<size_t>(n0 + srow) * K + scol;
  const size_t rstep = static_cast<size_t>(THREADS / 8) * K;  // 32 rows
#define GEMM_LOAD_TILE(k0)                                              \
  {                                                                     \
    ra0 = *reinterpret_cast<const uint4*>(ga + (k0));                   \
    ra1 = *reinterpret_cast<const uint4*>(ga + rstep + (k0));           \
    ra2 = *reinterpret_cast<const uint4*>(ga + 2 * rstep + (k0));       \
    ra3 = *reinterpret_cast<const uint4*>(ga + 3 * rstep + (k0));       \
    rb0 = *reinterpret_cast<const uint4*>(gb + (k0));                   \
    rb1 = *reinterpret_cast<const uint4*>(gb + rstep + (k0));           \
    rb2 = *reinterpret_cast<const uint4*>(gb + 2 * rstep + (k0));       \
    rb3 = *reinterpret_cast<const uint4*>(gb + 3 * rstep + (k0));       \
  }
  const int sofs = srow * LDS_STRIDE + scol;
  constexpr int lstep = (THREADS / 8) * LDS_STRIDE;
#define GEMM_STORE_TILE(buf)                                            \
  {                                                                     \
    uint16_t* la_ = lds + (buf) * 2 * TILE_ELEMS + sofs;                \
    uint16_t* lb_ = la_ + TILE_ELEMS;                                   \
    *reinterpret_cast<uint4*>(la_) = ra0;                               \
    *reinterpret_cast<uint4*>(la_ + lstep) = ra1;                       \
    *reinterpret_cast<uint4*>(la_ + 2 * lstep) = ra2;                   \
    *reinterpret_cast<uint4*>(la_ + 3 * lstep) = ra3;                   \
    *reinterpret_cast<uint4*>(lb_) = rb0;                               \
    *reinterpret_cast<uint4*>(lb_ + lstep) = rb1;                       \
    *reinterpret_cast<uint4*>(lb_ + 2 * lstep) = rb2;                   \
    *reinterpret_cast<uint4*>(lb_ + 3 * lstep) = rb3;                   \
  }
  static_assert(CHUNKS == 4, "staging code assumes 4 chunks per thread per operand");

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  GEMM_LOAD_TILE(0)
  GEMM_STORE_TILE(0)
  __syncthreads();

  // Fragment coordinates for v_mfma_f32_16x16x32_bf16: lane l holds
  // A[row l&15][k 8(l>>4)..+7] and B[k 8(l>>4)..+7][col l&15].
  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      GEMM_LOAD_TILE((kt + 1) * BK)  // in flight while we compute
    }

    const uint16_t* la = lds + buf * 2 * TILE_ELEMS;
    const uint16_t* lb = la + TILE_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const bf16x8*>(la + (wr * 64 + i * 16 + frow) * LDS_STRIDE + kk + fk);
        bfr[i] = *reinterpret_cast<const bf16x8*>(lb + (wc * 64 + i * 16 + frow) * LDS_STRIDE + kk + fk);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }

    if (kt + 1 < nk) GEMM_STORE_TILE(buf ^ 1)  // buffer last read before the previous barrier
    __syncthreads();
  }

  // Epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r.
  const int ccol = lane & 15;
  const int crow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 64 + i * 16 + crow + r;
        const int col = n0 + wc * 64 + j * 16 + ccol;
        C[static_cast<size_t>(row) * N + col] = f32_to_bf16_rne(acc[i][j][r]);
      }
#undef GEMM_LOAD_TILE
#undef GEMM_STORE_TILE
}

__global__ __launch_bounds__(256) void stream_triad(const float4* __restrict__ a, const float4* __restrict__ b,
                                                    float4* __restrict__ c, float s, size_t n4) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 x = a[i];
    const float4 y = b[i];
    c[i] = make_float4(x.x + s * y.x, x.y + s * y.y, x.z + s * y.z, x.w + s * y.w);
  }
}

constexpr size_t kGemmLds = 2 * 2 * TILE_ELEMS * sizeof(uint16_t);

bool g_attr_set = false;

const char* launch_gemm(const void* a, const void* b, void* c, int m, int n, int k, hipStream_t stream) {
  if (m <= 0 || n <= 0 || k <= 0 || m % BM || n % BN || k % BK) return "gemm_bf16_nt: M,N must be multiples of 128 and K of 64";
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) return "gemm_bf16_nt: A and B must be 16-byte aligned";
  if (!g_attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_bf16_nt), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(kGemmLds)) != hipSuccess)
      return "gemm_bf16_nt: cannot reserve LDS";
    g_attr_set = true;
  }
  const int blocks = (m / BM) * (n / BN);
  hipLaunchKernelGGL(gemm_bf16_nt, dim3(blocks), dim3(THREADS), kGemmLds, stream, static_cast<const uint16_t*>(a),
                     static_cast<const uint16_t*>(b), static_cast<uint16_t*>(c), m, n, k);
  hipError_t err = hipGetLastError();
  return err == hipSuccess ? nullptr : hipGetErrorString(err);
}

const char* launch_triad(const void* a, const void* b, void* c, size_t n, float s, hipStream_t stream) {
  if (n == 0 || n % 4) return "stream_triad: length must be a positive multiple of 4";
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15)
    return "stream_triad: buffers must be 16-byte aligned";
  const size_t n4 = n / 4;
  // Enough waves to cover HBM latency on all 256 CUs without a huge tail.
  size_t blocks = (n4 + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(stream_triad, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                     static_cast<const float4*>(a), static_cast<const float4*>(b), static_cast<float4*>(c), s, n4);
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

PyObject* py_tile(PyObject*, PyObject*) { return Py_BuildValue("(iii)", BM, BN, BK); }

PyMethodDef kMethods[] = {
    {"gemm_bf16_nt", py_gemm, METH_VARARGS, "gemm_bf16_nt(a, b, c, M, N, K, stream): C = A @ B^T (bf16, fp32 acc)."},
    {"stream_triad", py_triad, METH_VARARGS, "stream_triad(a, b, c, n, s, stream): c = a + s*b (fp32)."},
    {"tile", py_tile, METH_NOARGS, "(BM, BN, BK) of the GEMM tiling."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_workload", "MI355X workload kernels (MFMA GEMM, HBM triad).", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__workload(void) { return PyModule_Create(&kModule); }
