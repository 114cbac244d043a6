// Micro-benchmark: HBM triad variants on gfx950 (standalone; not shipped).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef float vf4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// V0: current shipped kernel (grid-stride, 1 float4 per iteration)
__global__ __launch_bounds__(256) void v0(const float4* __restrict__ a, const float4* __restrict__ b, float4* __restrict__ c, float s, size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 x = a[i], y = b[i];
    c[i] = make_float4(x.x + s * y.x, x.y + s * y.y, x.z + s * y.z, x.w + s * y.w);
  }
}

// V1: U float4 per thread per iteration, loads batched before stores; optional nontemporal store
template <int U, bool NT>
__global__ __launch_bounds__(256) void v1(const float4* __restrict__ a, const float4* __restrict__ b, float4* __restrict__ c, float s, size_t n4) {
  const size_t tile = (size_t)blockDim.x * U;
  const size_t stride = (size_t)gridDim.x * tile;
  for (size_t base = (size_t)blockIdx.x * tile + threadIdx.x; base < n4; base += stride) {
    float4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + (size_t)u * blockDim.x;
      if (i < n4) { x[u] = a[i]; y[u] = b[i]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + (size_t)u * blockDim.x;
      if (i < n4) {
        vf4 r = {x[u].x + s * y[u].x, x[u].y + s * y[u].y, x[u].z + s * y[u].z, x[u].w + s * y[u].w};
        if (NT) __builtin_nontemporal_store(r, reinterpret_cast<vf4*>(&c[i])); else *reinterpret_cast<vf4*>(&c[i]) = r;
      }
    }
  }
}

template <typename K>
float run(K kernel, int blocks, const float4* a, const float4* b, float4* c, size_t n4) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, 0, a, b, c, 0.5f, n4);
  std::vector<float> t;
  for (int it = 0; it < 15; ++it) {
    hipEventRecord(e0); hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, 0, a, b, c, 0.5f, n4); hipEventRecord(e1);
    hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return 3.0f * n4 * 16 / (t[t.size() / 2] * 1e-3f) / 1e12f;
}

int main() {
  const size_t n = 512ull * 1024 * 1024 / 4 * 4;  // 512M floats → 2 GiB per vector
  const size_t n4 = n / 4;
  float4 *a, *b, *c;
  CHECK(hipMalloc(&a, n * 4)); CHECK(hipMalloc(&b, n * 4)); CHECK(hipMalloc(&c, n * 4));
  CHECK(hipMemset(a, 0, n * 4)); CHECK(hipMemset(b, 0, n * 4));
  int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (int g : grids) printf("v0      blocks=%6d  %.2f TB/s\n", g, run(v0, g, a, b, c, n4));
  for (int g : grids) printf("v1<2>   blocks=%6d  %.2f TB/s\n", g, run(v1<2, false>, g, a, b, c, n4));
  for (int g : grids) printf("v1<4>   blocks=%6d  %.2f TB/s\n", g, run(v1<4, false>, g, a, b, c, n4));
  for (int g : grids) printf("v1<4>nt blocks=%6d  %.2f TB/s\n", g, run(v1<4, true>, g, a, b, c, n4));
  for (int g : grids) printf("v1<8>nt blocks=%6d  %.2f TB/s\n", g, run(v1<8, true>, g, a, b, c, n4));
  // one-pass (no grid stride): each thread exactly U chunks
  printf("v1<4>nt exact      %.2f TB/s\n", run(v1<4, true>, (int)((n4 + 1023) / 1024), a, b, c, n4));
  printf("v1<2>nt exact      %.2f TB/s\n", run(v1<2, true>, (int)((n4 + 511) / 512), a, b, c, n4));
  return 0;
}
