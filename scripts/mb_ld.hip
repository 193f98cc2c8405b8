// Micro-benchmark (round 5): why does the histogram pass's load phase (32-B rows + a 4-B wY per row) run at half the
// streaming rate? Loads only, 11M rows, 2 lanes per row (16 B of bins each), variants of the wY load and of LDS use.
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_ld.hip -o scripts/mb_ld.bin && ./scripts/mb_ld.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

// YM 0: no wY; 1: every lane loads its row's wY (4 B); 2: only even lanes load wY; 3: wY as float4 per 4 rows (lane
// r % 4 == 0 of ... every lane loads the 16-B quad of its row group); LDS: dynamic LDS bytes requested (occupancy)
template <int YM, int U>
__global__ __launch_bounds__(1024) void k_ld(const uint4* __restrict__ bins, const float* __restrict__ y, int N,
                                             unsigned* __restrict__ out) {
  extern __shared__ unsigned smem[];
  const int t = threadIdx.x, h = t & 1, r = t >> 1;
  constexpr int RPB = 512;
  const int per = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(N, r0 + per);
  unsigned acc = 0;
  for (int base = r0; base < r1; base += RPB * U) {
    uint4 b[U];
    float yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = min(base + u * RPB + r, r1 - 1);
      b[u] = bins[(size_t)row * 2 + h];
      if (YM == 1) yv[u] = y[row];
      if (YM == 2) yv[u] = h == 0 ? y[row] : 0.f;
      if (YM == 3) yv[u] = reinterpret_cast<const float4*>(y)[row >> 2].x;
      if (YM == 0) yv[u] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += b[u].x ^ b[u].y ^ b[u].z ^ b[u].w ^ __float_as_uint(yv[u]);
  }
  if (acc == 0x12345678u) out[0] = acc + smem[0];
}

template <typename Fn>
static float best_of(Fn fn) {
  hipEvent_t a, e;
  hipEventCreate(&a); hipEventCreate(&e);
  fn();
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
  float best = 1e9;
  for (int r = 0; r < 9; ++r) {
    hipEventRecord(a);
    fn();
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, a, e);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const int N = 11000000;
  uint4* b; float* y; unsigned* out;
  hipMalloc(&b, (size_t)N * 32); hipMalloc(&y, (size_t)N * 4 + 64); hipMalloc(&out, 4);
  hipMemset(b, 1, (size_t)N * 32); hipMemset(y, 0, (size_t)N * 4);
#define R(YM, U, LDS, G)                                                                                        \
  {                                                                                                           \
    const float ms = best_of([&]() { hipLaunchKernelGGL((k_ld<YM, U>), dim3(G), dim3(1024), LDS, 0, b, y, N, out); }); \
    printf("ym %d U %d lds %6d grid %4d  %7.4f ms  %5.2f TB/s (bins only)\n", YM, U, LDS, G, ms,                \
           (double)N * 32 / ms / 1e9);                                                                        \
  }
  R(0, 2, 0, 256) R(0, 4, 0, 256) R(0, 2, 65664, 256) R(1, 2, 0, 256) R(1, 4, 0, 256) R(1, 2, 65664, 256)
  R(2, 2, 0, 256) R(3, 2, 0, 256) R(0, 2, 0, 512) R(1, 2, 0, 512) R(1, 2, 0, 1024) R(0, 2, 0, 1024)
  return 0;
}
