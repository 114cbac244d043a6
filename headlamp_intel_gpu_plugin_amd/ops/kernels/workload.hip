// GPU workload kernels for the synthetic cluster's GPU pods (gfx950 / CDNA4).
//
// The plugin observes MI355X nodes; to validate that path end to end on a
// real GPU (exporter → Prometheus → Metrics page), the benchmark's "pods"
// must actually load the device the way training jobs do: matrix cores and
// HBM. Two kernels, written for CDNA4 directly:
//
//   gemm_bf16_nt  C[M,N] = A[M,K] · B[N,K]ᵀ, bf16 in, fp32 accumulate on
//                 MFMA (v_mfma_f32_16x16x32_bf16), bf16 out (RNE). Three
//                 kernels, picked by shape (or forced with `variant`):
//                   gemm_bf16_nt_8ph — 256×256×64 tile, 8 wave64s, operands
//                   staged by LDS-DMA (global_load_lds_dwordx4) with a
//                   source-side XOR swizzle, 8-phase ping-pong schedule with
//                   three half-tiles in flight (design notes above the
//                   kernel), and a packed epilogue (operands swapped in
//                   the MFMA so each lane holds a row segment, cvt_pk +
//                   permlane16_swap → 16-byte stores). Used when
//                   M,N % 256 == 0, K % 128 == 0 and the grid has ≥ 128
//                   blocks: 1566 TFLOP/s at 8192³ on random operands
//                   (profiles/r1_gemm_ab_latest.json);
//                   gemm_bf16_nt<256,256,2,4> — same tile, register-staged
//                   double buffer (1121 TFLOP/s), for K % 128 == 64;
//                   gemm_bf16_nt<128,128,2,2> — 4 waves, 64×64 per wave,
//                   for shapes the 256² tiles do not cover or fill.
//                 The register-staged kernels fetch tile k+1 into registers
//                 while tile k is consumed, write it to the other LDS buffer
//                 (128-B rows, XOR-swizzled 16-B chunks: conflict-free
//                 ds_read_b128), one barrier per K-step. All three run each MFMA cluster at
//                 s_setprio 1 and use a bijective XCD-aware block remap with
//                 tile-row grouping (8 rows; 4 in the 8-phase kernel, where
//                 the A/B measured it fastest) so blocks sharing an XCD's L2 work on
//                 neighbouring tiles.
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
// LDS rows are 128 B (no padding). 16-byte chunk c of row r is stored at
// chunk c ^ (r & 7): the 16 lanes of each ds_read_b128 lane group then hit
// 16 distinct 16-byte slots (the 144-B padded layout measured 33-37 % of LDS
// cycles in bank conflicts, profiles/r1_pmc_kernels.md).
constexpr int LDS_STRIDE = BK;

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// Two floats → packed bf16 (lo in bits 0-15), round-to-nearest-even: one
// v_cvt_pk_bf16_f32 on gfx950.
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
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
  const int sswz = ((tid & 7) ^ (srow & 7)) * 8;  // swizzled LDS column of this thread's chunk
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
    uint16_t* la_ = lds + (buf) * (BM + BN) * LDS_STRIDE + srow * LDS_STRIDE + sswz;                    \
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
  const int fswz = frow & 7;  // every fragment row ≡ frow (mod 16)
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
        af[i] = *reinterpret_cast<const bf16x8*>(la + (arow + i * 16) * LDS_STRIDE + ((((kk + fk) >> 3) ^ fswz) << 3));
#pragma unroll
      for (int j = 0; j < T::kTn; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + (brow + j * 16) * LDS_STRIDE + ((((kk + fk) >> 3) ^ fswz) << 3));
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

// ---------------------------------------------------------------------------
// gemm_bf16_nt_8ph: 256×256×64 tile, LDS-DMA staging, 8-phase ping-pong.
//
// Same C = A·Bᵀ contract as gemm_bf16_nt, restructured around what gfx950
// rewards at one 512-thread block per CU (cdna_hip_programming.md §5, "The
// 256² 8-phase template"):
//   * operands go global → LDS with global_load_lds_dwordx4 (no VGPR staging,
//     no ds_write pass); the LDS image is lane-linear, so the bank swizzle is
//     applied to the per-lane SOURCE address and undone on the ds_read:
//     16-byte chunk c of row r lives at chunk c ^ (r & 7), which makes every
//     ds_read_b128 lane group hit 16 distinct 16-byte slots (conflict-free);
//   * LDS holds two K-tiles (128 KiB), each as four 16 KiB half-tiles:
//     A0/A1 = the first/second 64-row subtile of both wave rows, B0/B1 = the
//     first/second 32-column subtile of all four wave columns. A phase
//     computes one 64×32 quadrant of each wave's 128×64 output (16 MFMAs)
//     and issues one half-tile of prefetch, so 8 phases cover 2 K-tiles;
//   * three half-tiles stay in flight across barriers: a counted
//     `s_waitcnt vmcnt(6)` at phases 4 and 8 (never 0 in the loop) and raw
//     s_barrier instead of __syncthreads (whose fence would drain vmcnt);
//   * the two wave rows run one barrier apart (wave row 1 takes an extra
//     barrier up front, row 0 one at the end), so on each SIMD one wave
//     issues ds_reads while its partner runs MFMAs.
// Staging order (half-tile written → phase), chosen so every buffer is
// rewritten only after all its readers retired their ds_reads (B reads are
// retired before the phase's first barrier by lgkmcnt(8)) and read only after
// a vmcnt wait plus a barrier:
//   even buffer (read phases 1-3): B0@2 A0@3 B1@4 A1@5 (next even K-tile)
//   odd  buffer (read phases 5-7): B0@6 A0@7 B1@8 A1@1 (next odd K-tile)
// Staging past the last K-tile reloads the last tile into a buffer that is
// never read again, keeping every wave's vmcnt arithmetic identical.
// ---------------------------------------------------------------------------

constexpr int P8_THREADS = 512;
// Tile-rows per L2 group of the block → tile map. Same-process A/B on one
// MI355X (tools/build_variants.py + tools/ab_two_builds.py, 7 rounds, random
// operands, TFLOP/s at 4096³ / 8192³ / 16384³): 1 → 1429 / 1421 / 1341,
// 2 → 1430 / 1511 / 1340, 4 → 1452 / 1546 / 1513, 8 → 1439 / 1544 / 1490,
// 16 → 1428 / 1486 / — (profiles/r1_gemm_group_ab.md).
#ifndef P8_GROUP
#define P8_GROUP 4
#endif
constexpr int P8_HALF = 128 * 128;       // bytes per half-tile (128 rows × 64 bf16)
constexpr int P8_BUF = 4 * P8_HALF;      // one K-tile: A0 A1 B0 B1
constexpr int P8_LDS = 2 * P8_BUF;       // 128 KiB
enum { kA0 = 0, kA1 = 1, kB0 = 2, kB1 = 3 };

// Row of the 256-row operand tile held by LDS row `r` (0..127) of half-tile `kind`.
__device__ __forceinline__ int p8_src_row(int kind, int r) {
  return kind < 2 ? (r >> 6) * 128 + (kind & 1) * 64 + (r & 63)   // A: wave row r/64, subtile kind
                  : (r >> 5) * 64 + (kind & 1) * 32 + (r & 31);   // B: wave col r/32, subtile kind-2
}

__global__ __launch_bounds__(P8_THREADS) void gemm_bf16_nt_8ph(const uint16_t* __restrict__ A,
                                                              const uint16_t* __restrict__ B,
                                                              uint16_t* __restrict__ C, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

  const int tiles_m = M / 256;
  const int tiles_n = N / 256;
  const int wg = xcd_remap(static_cast<int>(blockIdx.x), tiles_m * tiles_n);
  const int span = P8_GROUP * tiles_n;
  const int first_m = (wg / span) * P8_GROUP;
  const int rows_in_group = min(P8_GROUP, tiles_m - first_m);
  const int m0 = (first_m + (wg % span) % rows_in_group) * 256;
  const int n0 = ((wg % span) / rows_in_group) * 256;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2;  // 2 wave rows × 4 wave columns
  const int wc = wave & 3;
  const int nk = K / 64;

  // Staging: this wave writes LDS rows [16·wave, 16·wave+16) of every
  // half-tile with two 1 KiB glds; lane l covers row 16·wave + 8s + l/8,
  // physical chunk l%8, loaded from logical chunk (l%8) ^ (row & 7).
  uint32_t src_off[4][2];  // element offset of this lane's 16 B at k = 0
#pragma unroll
  for (int kind = 0; kind < 4; ++kind)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r = wave * 16 + s * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ (r & 7);
      const int grow = (kind < 2 ? m0 : n0) + p8_src_row(kind, r);
      src_off[kind][s] = static_cast<uint32_t>(grow) * static_cast<uint32_t>(K) + chunk * 8;
    }

#define P8_STAGE(kind, buf, ktile)                                                                         \
  {                                                                                                        \
    const int kt_ = min((ktile), nk - 1);                                                                  \
    const uint16_t* base_ = (kind) < 2 ? A : B;                                                            \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                                        \
      __builtin_amdgcn_global_load_lds(                                                                    \
          (__attribute__((address_space(1))) void*)(base_ + src_off[kind][s] + kt_ * 64),                  \
          (__attribute__((address_space(3))) void*)(                                                       \
              smem + (buf) * P8_BUF + (kind) * P8_HALF + (wave * 16 + s * 8) * 128),                        \
          16, 0, 0);                                                                                       \
    }                                                                                                      \
  }

  // Fragment reads: lane l takes row l&15 of a 16-row group, k-chunk
  // (l>>4) + 4·ks, through the same XOR (row & 7 == frow & 7).
  const int frow = lane & 15;
  const int rd0 = (((lane >> 4)) ^ (frow & 7)) * 16;  // byte offset of ks = 0; ks = 1 is rd0 ^ 64
  const int a_row = wr * 64 + frow;                    // LDS row within an A half-tile
  const int b_row = wc * 32 + frow;                    // … within a B half-tile

  bf16x8 af[8];     // A fragments of one 64-row subtile: [mt*2 + ks]
  bf16x8 bq[2][4];  // B fragments of both 32-col subtiles: [nh][nt*2 + ks]
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define P8_READ_A(buf, mh)                                                                                 \
  {                                                                                                        \
    const unsigned char* h_ = smem + (buf) * P8_BUF + (mh) * P8_HALF;                                       \
    _Pragma("unroll") for (int mt = 0; mt < 4; ++mt) {                                                     \
      const unsigned char* row_ = h_ + (a_row + mt * 16) * 128;                                            \
      af[mt * 2 + 0] = *reinterpret_cast<const bf16x8*>(row_ + rd0);                                       \
      af[mt * 2 + 1] = *reinterpret_cast<const bf16x8*>(row_ + (rd0 ^ 64));                                \
    }                                                                                                      \
  }
#define P8_READ_B(buf, nh)                                                                                 \
  {                                                                                                        \
    const unsigned char* h_ = smem + (buf) * P8_BUF + (2 + (nh)) * P8_HALF;                                 \
    _Pragma("unroll") for (int nt = 0; nt < 2; ++nt) {                                                     \
      const unsigned char* row_ = h_ + (b_row + nt * 16) * 128;                                            \
      bq[nh][nt * 2 + 0] = *reinterpret_cast<const bf16x8*>(row_ + rd0);                                   \
      bq[nh][nt * 2 + 1] = *reinterpret_cast<const bf16x8*>(row_ + (rd0 ^ 64));                            \
    }                                                                                                      \
  }
// Operands enter the MFMA as (B, A): the product is the 16×16 tile of Cᵀ,
// whose C/D layout puts FOUR CONSECUTIVE COLUMNS of one C row in each lane
// (row m = lane&15, columns 4(lane>>4)..+3) — what the packed epilogue
// below stores. Same fragments, same products, same accumulation.
#define P8_MFMA(mh, nh)                                                                                    \
  {                                                                                                        \
    __builtin_amdgcn_s_setprio(1);                                                                         \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                                       \
    _Pragma("unroll") for (int mt = 0; mt < 4; ++mt)                                                       \
    _Pragma("unroll") for (int nt = 0; nt < 2; ++nt)                                                       \
      acc[(mh) * 4 + mt][(nh) * 2 + nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                         \
          bq[nh][nt * 2 + ks], af[mt * 2 + ks], acc[(mh) * 4 + mt][(nh) * 2 + nt], 0, 0, 0);               \
    __builtin_amdgcn_s_setprio(0);                                                                         \
  }
#define P8_SYNC_MFMA(mh, nh)                                                                               \
  __builtin_amdgcn_s_barrier();                                                                            \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
  __builtin_amdgcn_sched_barrier(0);                                                                       \
  P8_MFMA(mh, nh)                                                                                          \
  __builtin_amdgcn_s_barrier();

  // Prologue: K-tile 0 → even buffer, then B0 A0 B1 of K-tile 1 → odd buffer;
  // vmcnt(6) leaves those three half-tiles in flight and retires K-tile 0.
  P8_STAGE(kB0, 0, 0) P8_STAGE(kA0, 0, 0) P8_STAGE(kB1, 0, 0) P8_STAGE(kA1, 0, 0)
  P8_STAGE(kB0, 1, 1) P8_STAGE(kA0, 1, 1) P8_STAGE(kB1, 1, 1)
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier

  for (int it = 0; it < nk / 2; ++it) {
    const int kt = 2 * it;
    // ---- even buffer: K-tile kt ----
    P8_READ_B(0, 0)
    __builtin_amdgcn_sched_barrier(0);
    P8_READ_A(0, 0)
    P8_STAGE(kA1, 1, kt + 1)
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // retire the 4 B reads before the barrier
    P8_SYNC_MFMA(0, 0)
    P8_READ_B(0, 1)
    P8_STAGE(kB0, 0, kt + 2)
    P8_SYNC_MFMA(0, 1)
    P8_READ_A(0, 1)
    P8_STAGE(kA0, 0, kt + 2)
    P8_SYNC_MFMA(1, 1)
    P8_STAGE(kB1, 0, kt + 2)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // odd buffer (K-tile kt+1) complete
    P8_SYNC_MFMA(1, 0)
    // ---- odd buffer: K-tile kt+1 ----
    P8_READ_B(1, 0)
    __builtin_amdgcn_sched_barrier(0);
    P8_READ_A(1, 0)
    P8_STAGE(kA1, 0, kt + 2)
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    P8_SYNC_MFMA(0, 0)
    P8_READ_B(1, 1)
    P8_STAGE(kB0, 1, kt + 3)
    P8_SYNC_MFMA(0, 1)
    P8_READ_A(1, 1)
    P8_STAGE(kA0, 1, kt + 3)
    P8_SYNC_MFMA(1, 1)
    P8_STAGE(kB1, 1, kt + 3)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // even buffer (K-tile kt+2) complete
    P8_SYNC_MFMA(1, 0)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the block
  if (wr == 0) __builtin_amdgcn_s_barrier();        // balance the stagger barrier
#undef P8_STAGE
#undef P8_READ_A
#undef P8_READ_B
#undef P8_MFMA
#undef P8_SYNC_MFMA

  // Epilogue (guide T21): acc[i][j] holds C[row][4g..4g+3] of its 16×16 tile,
  // g = lane>>4. Pack to bf16 pairs, then one v_permlane16_swap per dword
  // between the two 16-column tiles of a 32-column subtile (j = 2p, 2p+1)
  // leaves each lane 8 CONSECUTIVE columns: lane group g holds columns
  // 16(g&1) + 8(g>>1) .. +7 — one 16-byte store where the plain layout
  // needed sixteen 2-byte ones (the store tail is issue-bound).
  const int g = lane >> 4;
  const int col16 = (g & 1) * 16 + (g >> 1) * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + (lane & 15);
    uint16_t* crow = C + static_cast<size_t>(row) * N + n0 + wc * 64 + col16;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t a0 = pack_bf16x2(acc[i][2 * p][0], acc[i][2 * p][1]);
      uint32_t a1 = pack_bf16x2(acc[i][2 * p][2], acc[i][2 * p][3]);
      uint32_t b0 = pack_bf16x2(acc[i][2 * p + 1][0], acc[i][2 * p + 1][1]);
      uint32_t b1 = pack_bf16x2(acc[i][2 * p + 1][2], acc[i][2 * p + 1][3]);
      // Odd 16-lane rows of the first operand swap with even rows of the second.
      const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
      *reinterpret_cast<u32x4*>(crow + p * 32) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    }
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
bool g_8ph_attr = false;

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

const char* launch_8ph(const void* a, const void* b, void* c, int m, int n, int k, hipStream_t stream) {
  if (!g_8ph_attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_bf16_nt_8ph), hipFuncAttributeMaxDynamicSharedMemorySize,
                            P8_LDS) != hipSuccess)
      return "gemm_bf16_nt_8ph: cannot reserve LDS";
    g_8ph_attr = true;
  }
  hipLaunchKernelGGL(gemm_bf16_nt_8ph, dim3((m / 256) * (n / 256)), dim3(P8_THREADS), P8_LDS, stream,
                     static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), static_cast<uint16_t*>(c), m, n,
                     k);
  hipError_t err = hipGetLastError();
  return err == hipSuccess ? nullptr : hipGetErrorString(err);
}

// Kernel variants: 0 = pick by shape, 1 = 128² register-staged, 2 = 256²
// register-staged, 3 = 256² 8-phase LDS-DMA.
enum { kAuto = 0, kTile128 = 1, kTile256 = 2, kTile256Dma = 3 };

bool fits_8ph(const void* c, int m, int n, int k) {
  // 32-bit per-lane source offsets: every element index must fit in uint32;
  // the packed epilogue stores 16 bytes per lane, so C must be 16-B aligned.
  return m % 256 == 0 && n % 256 == 0 && k % 128 == 0 && (reinterpret_cast<uintptr_t>(c) & 15) == 0 &&
         static_cast<uint64_t>(m) * k < (1ull << 32) && static_cast<uint64_t>(n) * k < (1ull << 32);
}

const char* launch_gemm(const void* a, const void* b, void* c, int m, int n, int k, hipStream_t stream,
                        int variant = kAuto) {
  if (m <= 0 || n <= 0 || k <= 0 || m % 128 || n % 128 || k % BK) return "gemm_bf16_nt: M,N must be multiples of 128 and K of 64";
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) return "gemm_bf16_nt: A and B must be 16-byte aligned";
  const bool big = m % 256 == 0 && n % 256 == 0;
  switch (variant) {
    case kTile128:
      return launch_tile<128, 128, 2, 2>(a, b, c, m, n, k, stream, &g_small_attr);
    case kTile256:
      if (!big) return "gemm_bf16_nt: the 256x256 tile needs M,N multiples of 256";
      return launch_tile<256, 256, 2, 4>(a, b, c, m, n, k, stream, &g_big_attr);
    case kTile256Dma:
      if (!fits_8ph(c, m, n, k))
        return "gemm_bf16_nt: the 8-phase tile needs M,N multiples of 256, K of 128, M*K and N*K < 2^32, C 16-byte aligned";
      return launch_8ph(a, b, c, m, n, k, stream);
    case kAuto:
      break;
    default:
      return "gemm_bf16_nt: unknown variant";
  }
  // The 256² tiles need ≥ one block per CU to beat the 128² tile (256 CUs).
  if (big && (m / 256) * (n / 256) >= 128) {
    if (fits_8ph(c, m, n, k)) return launch_8ph(a, b, c, m, n, k, stream);
    return launch_tile<256, 256, 2, 4>(a, b, c, m, n, k, stream, &g_big_attr);
  }
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
  int m, n, k, variant = kAuto;
  if (!PyArg_ParseTuple(args, "KKKiiiK|i", &a, &b, &c, &m, &n, &k, &stream, &variant)) return nullptr;
  const char* err = launch_gemm(reinterpret_cast<void*>(a), reinterpret_cast<void*>(b), reinterpret_cast<void*>(c), m,
                                n, k, reinterpret_cast<hipStream_t>(stream), variant);
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
    {"gemm_bf16_nt", py_gemm, METH_VARARGS,
     "gemm_bf16_nt(a, b, c, M, N, K, stream, variant=0): C = A @ B^T (bf16, fp32 acc); variant 0 auto, "
     "1 128x128, 2 256x256 register-staged, 3 256x256 8-phase LDS-DMA."},
    {"stream_triad", py_triad, METH_VARARGS, "stream_triad(a, b, c, n, s, stream): c = a + s*b (fp32)."},
    {"tile", py_tile, METH_NOARGS, "(BM, BN, BK) of the GEMM tiling."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_workload", "MI355X workload kernels (MFMA GEMM, HBM triad).", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__workload(void) { return PyModule_Create(&kModule); }
