// Micro-benchmark: LDS histogram update throughput on gfx950 for different update primitives.
// hipcc --offload-arch=gfx950 -O3 mb_lds_atomic.hip -o mb && ./mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define NB 256
#define FT 28
#define BLK 512

template <int MODE>
__global__ __launch_bounds__(BLK) void kern(const uint8_t* __restrict__ bins, const float2* __restrict__ aux, int N,
                                            float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  for (int i = threadIdx.x; i < FT * 514; i += BLK) sm[i] = 0.f;
  __syncthreads();
  const int g = threadIdx.x >> 3, j = threadIdx.x & 7;
  const unsigned* b32 = (const unsigned*)bins;
  const int rows_per_block = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(N, r0 + rows_per_block);
  for (int base = r0; base < r1; base += 64 * 8) {
    unsigned wd[8];
    float2 ab[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = base + g + u * 64;
      const bool v = row < r1;
      wd[u] = (v && j < 7) ? b32[(size_t)row * 7 + j] : 0u;
      ab[u] = v ? aux[row] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (base + g + u * 64 >= r1 || j >= 7) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int f = j * 4 + k;
        const int bin = (wd[u] >> (8 * k)) & 0xFF;
        float* p = sm + f * 514 + bin;
        if (MODE == 0) { p[0] += ab[u].x; p[257] += ab[u].y; }                                  // racy, no atomic
        if (MODE == 1) { atomicAdd(p, ab[u].x); atomicAdd(p + 257, ab[u].y); }                  // ds_add_f32 x2
        if (MODE == 2) { atomicAdd((unsigned*)p, 1u); atomicAdd((unsigned*)p + 257, (unsigned)(int)(ab[u].y * 65536.f)); }  // ds_add_u32 x2
        if (MODE == 3) {                                                                      // one ds_add_u64 (packed)
          unsigned long long* q = (unsigned long long*)(sm) + f * 257 + bin;
          atomicAdd(q, (1ull << 40) + (unsigned long long)(long long)(ab[u].y * 65536.f));
        }
        if (MODE == 4) { atomicAdd(p, ab[u].x); }                                               // ds_add_f32 x1
        if (MODE == 5) {
          __hip_atomic_fetch_add(p, ab[u].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(p + 257, ab[u].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  }
  __syncthreads();
  float s = 0.f;
  for (int i = threadIdx.x; i < FT * 514; i += BLK) s += sm[i];
  atomicAdd(out, s);
}

template <int MODE>
float run(const uint8_t* bins, const float2* aux, int N, float* out, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  size_t lds = FT * 514 * 4 + 1024;
  if (MODE == 3) lds = FT * 257 * 8 + 1024;
  hipLaunchKernelGGL(kern<MODE>, dim3(grid), dim3(BLK), lds, 0, bins, aux, N, out);
  hipDeviceSynchronize();
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(a);
    hipLaunchKernelGGL(kern<MODE>, dim3(grid), dim3(BLK), lds, 0, bins, aux, N, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const int N = 11000000;
  std::vector<uint8_t> hb((size_t)N * 28);
  uint32_t s = 12345;
  for (auto& x : hb) { s = s * 1664525u + 1013904223u; x = (uint8_t)((s >> 24) % 255); }
  std::vector<float2> ha(N);
  for (int i = 0; i < N; ++i) ha[i] = make_float2(1.f, ((i * 7) % 100) / 100.f - 0.5f);
  uint8_t* db; float2* da; float* dout;
  hipMalloc(&db, hb.size()); hipMalloc(&da, N * sizeof(float2)); hipMalloc(&dout, 4);
  hipMemcpy(db, hb.data(), hb.size(), hipMemcpyHostToDevice);
  hipMemcpy(da, ha.data(), N * sizeof(float2), hipMemcpyHostToDevice);
  const char* names[] = {"plain LDS RMW (racy)", "ds_add_f32 x2 (atomicAdd)", "ds_add_u32 x2", "ds_add_u64 x1 packed",
                         "ds_add_f32 x1", "ds_add_f32 x2 relaxed/workgroup"};
  for (int grid : {256, 512}) {
    printf("grid %d\n", grid);
    printf("  %-34s %8.3f ms\n", names[0], run<0>(db, da, N, dout, grid));
    printf("  %-34s %8.3f ms\n", names[1], run<1>(db, da, N, dout, grid));
    printf("  %-34s %8.3f ms\n", names[2], run<2>(db, da, N, dout, grid));
    printf("  %-34s %8.3f ms\n", names[3], run<3>(db, da, N, dout, grid));
    printf("  %-34s %8.3f ms\n", names[4], run<4>(db, da, N, dout, grid));
    printf("  %-34s %8.3f ms\n", names[5], run<5>(db, da, N, dout, grid));
  }
  return 0;
}
