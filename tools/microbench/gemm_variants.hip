// Micro-benchmark: bf16 MFMA GEMM tile-shape variants on gfx950 (standalone; not shipped).
// C[M,N] = A[M,K] · B[N,K]^T, register-staged double-buffered LDS, one barrier per K-step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <int BM, int BN, int WM, int WN, bool PRIO>
__global__ __launch_bounds__(WM * WN * 64) void gemm(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                   uint16_t* __restrict__ C, int M, int N, int K) {
  constexpr int BK = 64, LS = BK + 8, T = WM * WN * 64;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // MFMA tiles per wave
  constexpr int CA = BM * BK * 2 / 16 / T, CB = BN * BK * 2 / 16 / T;  // 16-B chunks per thread
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int span = 8 * tiles_n, grp = wg / span, first = grp * 8, rows = min(8, tiles_m - first);
  const int m0 = (first + (wg % span) % rows) * BM, n0 = ((wg % span) / rows) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave / WN, wc = wave % WN;
  u32x4 ra[CA], rb[CB];
  const int srow = tid >> 3, scol = (tid & 7) * 8;
  constexpr int RSTEP = T / 8;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  const int nk = K / BK;
  {
#pragma unroll
    for (int p = 0; p < CA; ++p) ra[p] = *(const u32x4*)(A + (size_t)(m0 + srow + p * RSTEP) * K + 0 + scol);
#pragma unroll
    for (int p = 0; p < CB; ++p) rb[p] = *(const u32x4*)(B + (size_t)(n0 + srow + p * RSTEP) * K + 0 + scol);
    {
      uint16_t* la_ = lds + 0 * (BM + BN) * LS;
      uint16_t* lb_ = la_ + BM * LS;
#pragma unroll
      for (int p = 0; p < CA; ++p) *(u32x4*)(la_ + (srow + p * RSTEP) * LS + scol) = ra[p];
#pragma unroll
      for (int p = 0; p < CB; ++p) *(u32x4*)(lb_ + (srow + p * RSTEP) * LS + scol) = rb[p];
    }
  }
  __syncthreads();
  const int frow = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      const int k1 = (kt + 1) * BK;
#pragma unroll
    for (int p = 0; p < CA; ++p) ra[p] = *(const u32x4*)(A + (size_t)(m0 + srow + p * RSTEP) * K + k1 + scol);
#pragma unroll
    for (int p = 0; p < CB; ++p) rb[p] = *(const u32x4*)(B + (size_t)(n0 + srow + p * RSTEP) * K + k1 + scol);
    }
    const uint16_t* la = lds + buf * (BM + BN) * LS;
    const uint16_t* lb = la + BM * LS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *(const bf16x8*)(la + (wr * (BM / WM) + i * 16 + frow) * LS + kk + fk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8*)(lb + (wc * (BN / WN) + j * 16 + frow) * LS + kk + fk);
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
    }
    if (kt + 1 < nk) {
      const int nb = buf ^ 1;
    {
      uint16_t* la_ = lds + nb * (BM + BN) * LS;
      uint16_t* lb_ = la_ + BM * LS;
#pragma unroll
      for (int p = 0; p < CA; ++p) *(u32x4*)(la_ + (srow + p * RSTEP) * LS + scol) = ra[p];
#pragma unroll
      for (int p = 0; p < CB; ++p) *(u32x4*)(lb_ + (srow + p * RSTEP) * LS + scol) = rb[p];
    }
    }
    __syncthreads();
  }
  const int ccol = lane & 15, crow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(size_t)(m0 + wr * (BM / WM) + i * 16 + crow + r) * N + n0 + wc * (BN / WN) + j * 16 + ccol] = f2bf(acc[i][j][r]);
}

template <int BM, int BN, int WM, int WN, bool PRIO>
double bench(const char* name, const uint16_t* a, const uint16_t* b, uint16_t* c, int S) {
  constexpr size_t lds = 2 * (BM + BN) * (64 + 8) * 2;
  auto k = gemm<BM, BN, WM, WN, PRIO>;
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    printf("%s: LDS %zu too large\n", name, lds);
    return 0;
  }
  const int blocks = (S / BM) * (S / BN);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(WM * WN * 64), lds, 0, a, b, c, S, S, S);
  std::vector<float> t;
  for (int it = 0; it < 10; ++it) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(WM * WN * 64), lds, 0, a, b, c, S, S, S);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  double tf = 2.0 * S * S * (double)S / (t[t.size() / 2] * 1e-3) / 1e12;
  printf("%-28s S=%5d  %7.1f TFLOP/s  (lds %zu B)\n", name, S, tf, lds);
  return tf;
}

__global__ void fill(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    float f = ((x & 0xffff) / 32768.0f) - 1.0f;
    p[i] = f2bf(f);
  }
}

int main() {
  for (int S : {4096, 8192}) {
    size_t n = (size_t)S * S;
    uint16_t *a, *b, *c;
    if (hipMalloc(&a, n * 2) || hipMalloc(&b, n * 2) || hipMalloc(&c, n * 2)) return 1;
    hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, a, n, 1u);
    hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, b, n, 2u);
    (void)hipDeviceSynchronize();
    bench<128, 128, 2, 2, false>("128x128 w2x2 (shipped)", a, b, c, S);
    bench<128, 128, 2, 2, true>("128x128 w2x2 prio", a, b, c, S);
    bench<128, 256, 2, 4, false>("128x256 w2x4", a, b, c, S);
    bench<128, 256, 2, 4, true>("128x256 w2x4 prio", a, b, c, S);
    bench<256, 128, 4, 2, false>("256x128 w4x2", a, b, c, S);
    bench<256, 256, 2, 4, false>("256x256 w2x4", a, b, c, S);
    bench<256, 256, 2, 4, true>("256x256 w2x4 prio", a, b, c, S);
    bench<128, 128, 2, 2, false>("128x128 w2x2 (again)", a, b, c, S);
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(c);
  }
  return 0;
}
