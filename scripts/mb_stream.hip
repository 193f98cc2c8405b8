// Micro-benchmark (round 5): streaming-read recipes on gfx950 for the tree passes (how many bytes in flight per
// CU does a 352-MB read need to approach HBM speed?).
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_stream.hip -o scripts/mb_stream.bin && ./scripts/mb_stream.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>

// contiguous chunk per block, U independent 16-B loads per lane per round
template <int U, int BLK>
__global__ __launch_bounds__(BLK) void k_chunk(const uint4* __restrict__ a, long long n16, unsigned* __restrict__ out) {
  const long long per = (n16 + gridDim.x - 1) / gridDim.x;
  const long long b0 = blockIdx.x * per, b1 = b0 + per < n16 ? b0 + per : n16;
  unsigned acc = 0;
  for (long long base = b0; base < b1; base += (long long)U * BLK) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      long long i = base + k * BLK + threadIdx.x;
      i = i < b1 ? i : b1 - 1;
      v[k] = a[i];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// grid-stride, U loads per lane per round
template <int U, int BLK>
__global__ __launch_bounds__(BLK) void k_stride(const uint4* __restrict__ a, long long n16, unsigned* __restrict__ out) {
  unsigned acc = 0;
  const long long step = (long long)gridDim.x * BLK * U;
  for (long long base = (long long)blockIdx.x * BLK * U; base < n16; base += step) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      long long i = base + k * BLK + threadIdx.x;
      i = i < n16 ? i : n16 - 1;
      v[k] = a[i];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// 8 planes of M uint4 each (word-planar bins, 4 rows per uint4): lane = 8 * i + j reads plane j, quad (base + i);
// plus the 16-B y quad of those rows (shared by the 8 plane lanes). Contiguous chunk of quads per block.
template <int U, int BLK>
__global__ __launch_bounds__(BLK) void k_planes(const uint4* __restrict__ a, const uint4* __restrict__ y, long long M, int P,
                                                unsigned* __restrict__ out) {
  const long long per = (M + gridDim.x - 1) / gridDim.x;
  const long long q0 = blockIdx.x * per, q1 = q0 + per < M ? q0 + per : M;
  const int j = threadIdx.x & 7, i = threadIdx.x >> 3;
  constexpr int QPR = BLK / 8;
  unsigned acc = 0;
  const int jj = j < P ? j : P - 1;
  for (long long base = q0; base < q1; base += (long long)U * QPR) {
    uint4 v[U], w[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      long long q = base + k * QPR + i;
      q = q < q1 ? q : q1 - 1;
      v[k] = a[(size_t)jj * M + q];
      w[k] = y[q];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w ^ w[k].x;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
static float best_of(F fn) {
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
  const long long bytes = 11000000LL * 32;
  const long long n16 = bytes / 16;
  uint4* a; uint4* y; unsigned* out;
  hipMalloc(&a, bytes + 4096); hipMalloc(&y, 11000000LL * 4 + 64); hipMalloc(&out, 4);
  hipMemset(a, 1, bytes); hipMemset(y, 2, 11000000LL * 4);
  const double gb = bytes / 1e9;
#define RUN(KER, U, BLK, G, LABEL)                                                                              \
  {                                                                                                           \
    const float ms = best_of([&]() { hipLaunchKernelGGL((KER<U, BLK>), dim3(G), dim3(BLK), 0, 0, a, n16, out); }); \
    printf("%-8s U %d blk %4d grid %5d  %7.4f ms  %5.2f TB/s  (%3d KB in flight/CU at 1 blk/CU)\n", LABEL, U, BLK, G, \
           ms, gb / ms, U * BLK * 16 / 1024);                                                                 \
  }
  for (int g : {256, 512, 1024, 2048}) {
    RUN(k_chunk, 1, 1024, g, "chunk") RUN(k_chunk, 2, 1024, g, "chunk") RUN(k_chunk, 4, 1024, g, "chunk")
    RUN(k_chunk, 8, 1024, g, "chunk") RUN(k_chunk, 4, 512, g, "chunk") RUN(k_chunk, 8, 256, g, "chunk")
  }
  for (int g : {1024, 2048, 4096, 8192}) {
    RUN(k_stride, 1, 256, g, "stride") RUN(k_stride, 4, 256, g, "stride") RUN(k_stride, 8, 256, g, "stride")
    RUN(k_stride, 4, 1024, g / 4, "stride")
  }
  const long long M = 11000000LL / 4;
  const int P = 7;
  const double gbp = (double)M * 16 * (P + 1) / 1e9;
  for (int g : {256, 512, 1024}) {
    for (int u : {1, 2, 4, 8}) {
      float ms = 0;
      if (u == 1) ms = best_of([&]() { hipLaunchKernelGGL((k_planes<1, 1024>), dim3(g), dim3(1024), 0, 0, a, y, M, P, out); });
      if (u == 2) ms = best_of([&]() { hipLaunchKernelGGL((k_planes<2, 1024>), dim3(g), dim3(1024), 0, 0, a, y, M, P, out); });
      if (u == 4) ms = best_of([&]() { hipLaunchKernelGGL((k_planes<4, 1024>), dim3(g), dim3(1024), 0, 0, a, y, M, P, out); });
      if (u == 8) ms = best_of([&]() { hipLaunchKernelGGL((k_planes<8, 1024>), dim3(g), dim3(1024), 0, 0, a, y, M, P, out); });
      printf("planes7  U %d blk 1024 grid %5d  %7.4f ms  %5.2f TB/s (bins + y)\n", u, g, ms, gbp / ms);
    }
  }
  return 0;
}
