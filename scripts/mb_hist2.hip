// Micro-benchmark: which LDS update primitive bounds the tree-histogram pass on gfx950?
// One pass over N rows x 32 B (28 features + pad, random bins) + one fp32 value per row, production
// geometry of k_hist_build (8 lanes per row, 4 features per lane, [bin][FTILE] bank-spread layout).
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_hist2.hip -o /tmp/mb_hist2 && /tmp/mb_hist2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>

#define FTILE 32
#define HPLANE (256 * FTILE + 16)
#define LPR 8
#define UNR 8

__device__ __forceinline__ int fslot(int fl) { return (fl & 16) | ((fl + ((fl >> 4) << 1)) & 15); }

// MODE 0: ds_add_u64 (packed count|value)   1: ds_add_u32 (value only)   2: 2x ds_add_u32
//      3: ds_add_f32                         4: racy u64 read-modify-write  5: no LDS update (loads + VALU)
//      6: ds_add_u32 + ds_add_u32 into a half-width (u16x2-packed) count plane
template <int MODE, int BLK>
__global__ __launch_bounds__(BLK) void kern(const unsigned* __restrict__ bins32, const float* __restrict__ val,
                                            int N, int F, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  constexpr int RPI = BLK / LPR;
  const int nent = (MODE == 0 || MODE == 4 || MODE == 2 || MODE == 6) ? HPLANE : HPLANE / 2 + 8;
  for (int i = threadIdx.x; i < nent; i += BLK) sm[i] = 0ull;
  __syncthreads();
  const int g = threadIdx.x / LPR, j = threadIdx.x % LPR;
  const int W = 8;
  const int rot = g & 1;
  int off[4], sh[4];
  unsigned vmask = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = (k + rot) & 3;
    off[k] = fslot(j * 4 + kk);
    sh[k] = 8 * kk;
    if (j * 4 + kk < F) vmask |= 0xFFu << (8 * kk);
  }
  const int per = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(N, r0 + per);
  unsigned long long acc = 0;
  unsigned* S32 = (unsigned*)sm;
  float* SF = (float*)sm;
  for (int base = r0; base < r1; base += RPI * UNR) {
    unsigned wd[UNR];
    float v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const size_t row = (size_t)min(base + g + u * RPI, r1 - 1);
      wd[u] = bins32[row * W + j];
      v[u] = val[row];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (base + g + u * RPI >= r1 || vmask == 0u) continue;
      const long long q = ((long long)1 << 48) + (long long)__float2int_rz(v[u] * 1073741824.f);
      const unsigned q32 = (unsigned)__float2int_rz(v[u] * 65536.f);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!((vmask >> sh[k]) & 1u)) continue;
        const unsigned bin = (wd[u] >> sh[k]) & 0xFFu;
        const int e = bin * FTILE + off[k];
        if (MODE == 0) atomicAdd(sm + e, (unsigned long long)q);
        if (MODE == 1) atomicAdd(S32 + e, q32);
        if (MODE == 2) { atomicAdd(S32 + e, q32); atomicAdd(S32 + HPLANE + e, 1u); }
        if (MODE == 3) atomicAdd(SF + e, v[u]);
        if (MODE == 4) sm[e] += (unsigned long long)q;
        if (MODE == 5) acc += (unsigned long long)q ^ (unsigned long long)e;
        if (MODE == 6) { atomicAdd(S32 + e, q32); atomicAdd(S32 + HPLANE + (e >> 1), (e & 1) ? 65536u : 1u); }
      }
    }
  }
  __syncthreads();
  unsigned long long s = acc;
  for (int i = threadIdx.x; i < nent; i += BLK) s += sm[i];
  atomicAdd(out, s);
}

template <int MODE, int BLK>
float run(const unsigned* b, const float* v, int N, int F, unsigned long long* out, int grid, int lds_kb_extra = 0) {
  hipEvent_t a, e;
  hipEventCreate(&a); hipEventCreate(&e);
  size_t lds = (MODE == 0 || MODE == 4 || MODE == 2 || MODE == 6) ? HPLANE * 8 : (HPLANE / 2 + 8) * 8;
  lds += lds_kb_extra * 1024;
  hipMemset(out, 0, 8);
  hipLaunchKernelGGL((kern<MODE, BLK>), dim3(grid), dim3(BLK), lds, 0, b, v, N, F, out);
  hipError_t rc = hipDeviceSynchronize();
  unsigned long long chk = 0;
  hipMemcpy(&chk, out, 8, hipMemcpyDeviceToHost);
  printf("[mode %d checksum %llx] ", MODE, chk);
  if (rc != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(rc)); exit(1); }
  float best = 1e9;
  for (int r = 0; r < 7; ++r) {
    hipEventRecord(a);
    hipLaunchKernelGGL((kern<MODE, BLK>), dim3(grid), dim3(BLK), lds, 0, b, v, N, F, out);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, a, e);
    if (ms < best) best = ms;
  }
  return best;
}


// 2 lanes per row: each lane loads 16 B (half a row: 16 features) with one dwordx4; the wave covers 32 rows
// per load. MODE 7: instruction i adds feature 16h + 4(i>>2) + ((i+R)&3) (uniform word, rotated byte:
// 2-way bank conflict); MODE 8: feature 16h + ((i+R)&15) (conflict-free, per-lane word select);
// MODE 9: loads only.
template <int MODE, int BLK>
__global__ __launch_bounds__(BLK) void kern2(const uint4* __restrict__ bins, const float* __restrict__ val,
                                             int N, int F, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  constexpr int RPI = BLK / 2;
  for (int i = threadIdx.x; i < HPLANE; i += BLK) sm[i] = 0ull;
  __syncthreads();
  const int t = threadIdx.x, h = t & 1, R = (t >> 1) & 15;
  int off[16];
  unsigned vm = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int f = MODE == 7 ? 16 * h + 4 * (i >> 2) + ((i + R) & 3) : 16 * h + ((i + R) & 15);
    off[i] = fslot(f);
    if (f < F) vm |= 1u << i;
  }
  const int per = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(N, r0 + per);
  unsigned long long acc = 0;
  for (int base = r0; base < r1; base += RPI * 4) {
    uint4 q[4];
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t row = (size_t)min(base + (t >> 1) + u * RPI, r1 - 1);
      q[u] = bins[row * 2 + h];
      v[u] = val[row];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (base + (t >> 1) + u * RPI >= r1) continue;
      if (MODE == 9) { acc += q[u].x ^ q[u].y ^ q[u].z ^ q[u].w ^ __float_as_uint(v[u]); continue; }
      const unsigned long long qa = ((unsigned long long)1 << 48) + (unsigned long long)(long long)__float2int_rz(v[u] * 1073741824.f);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (!((vm >> i) & 1u)) continue;
        unsigned w;
        int sh;
        if (MODE == 7) {
          w = (i >> 2) == 0 ? q[u].x : (i >> 2) == 1 ? q[u].y : (i >> 2) == 2 ? q[u].z : q[u].w;
          sh = 8 * ((i + R) & 3);
        } else {
          const int wi = ((i + R) >> 2) & 3;
          w = q[u].x;
          w = wi == 1 ? q[u].y : w;
          w = wi == 2 ? q[u].z : w;
          w = wi == 3 ? q[u].w : w;
          sh = 8 * ((i + R) & 3);
        }
        const unsigned bin = (w >> sh) & 0xFFu;
        atomicAdd(sm + bin * FTILE + off[i], qa);
      }
    }
  }
  __syncthreads();
  unsigned long long s = acc;
  for (int i = threadIdx.x; i < HPLANE; i += BLK) s += sm[i];
  atomicAdd(out, s);
}

// loads only, production layout (one dword per lane + the row value)
template <int BLK>
__global__ __launch_bounds__(BLK) void kern_ld(const unsigned* __restrict__ bins32, const float* __restrict__ val,
                                               int N, unsigned long long* __restrict__ out) {
  constexpr int RPI = BLK / LPR;
  const int g = threadIdx.x / LPR, j = threadIdx.x % LPR;
  const int per = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(N, r0 + per);
  unsigned long long acc = 0;
  for (int base = r0; base < r1; base += RPI * UNR) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const size_t row = (size_t)min(base + g + u * RPI, r1 - 1);
      acc += bins32[row * 8 + j] ^ __float_as_uint(val[row]);
    }
  }
  atomicAdd(out, acc);
}

template <int MODE, int BLK>
float run2(const unsigned* b, const float* v, int N, int F, unsigned long long* out, int grid) {
  hipEvent_t a, e;
  hipEventCreate(&a); hipEventCreate(&e);
  size_t lds = HPLANE * 8;
  auto launch = [&]() {
    if (MODE == 10) hipLaunchKernelGGL((kern_ld<BLK>), dim3(grid), dim3(BLK), 0, 0, b, v, N, out);
    else hipLaunchKernelGGL((kern2<MODE, BLK>), dim3(grid), dim3(BLK), lds, 0, (const uint4*)b, v, N, F, out);
  };
  hipMemset(out, 0, 8);
  launch();
  hipError_t rc = hipDeviceSynchronize();
  unsigned long long chk = 0;
  hipMemcpy(&chk, out, 8, hipMemcpyDeviceToHost);
  printf("[mode %d checksum %llx] ", MODE, chk);
  if (rc != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(rc)); exit(1); }
  float best = 1e9;
  for (int r = 0; r < 7; ++r) {
    hipEventRecord(a);
    launch();
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, a, e);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const int N = 11000000, F = 28;
  std::vector<unsigned> hb((size_t)N * 8);
  uint32_t s = 12345;
  for (auto& x : hb) {
    unsigned w = 0;
    for (int k = 0; k < 4; ++k) { s = s * 1664525u + 1013904223u; w |= ((s >> 24) % 255u) << (8 * k); }
    x = w;
  }
  std::vector<float> hv(N);
  for (int i = 0; i < N; ++i) hv[i] = ((i * 7) % 100) / 100.f - 0.5f;
  unsigned* db; float* dv; unsigned long long* dout;
  hipMalloc(&db, hb.size() * 4); hipMalloc(&dv, N * 4); hipMalloc(&dout, 8);
  hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dv, hv.data(), N * 4, hipMemcpyHostToDevice);
  const double upd = (double)N * F;
  const char* names[] = {"ds_add_u64 packed", "ds_add_u32 value", "2x ds_add_u32", "ds_add_f32", "racy u64 RMW",
                         "no LDS update", "u32 value + u16x2 count"};
#define ROW(M, B, G, X)                                                                                     \
  {                                                                                                         \
    float ms = run<M, B>(db, dv, N, F, dout, G, X);                                                         \
    printf("%-26s blk %4d grid %4d lds+%3dKB  %7.3f ms  %6.2f Gupd/s  %5.2f TB/s\n", names[M], B, G, X, ms, \
           upd / ms / 1e6, (double)N * 36 / ms / 1e9);                                                      \
  }
  for (int g : {256, 512}) {
    ROW(0, 1024, g, 0) ROW(1, 1024, g, 0) ROW(2, 1024, g, 0) ROW(3, 1024, g, 0) ROW(4, 1024, g, 0)
    ROW(5, 1024, g, 0) ROW(6, 1024, g, 0)
  }
  // occupancy: 512-thread blocks, 2..4 per CU
  ROW(0, 512, 512, 0) ROW(0, 512, 1024, 0) ROW(1, 512, 512, 0) ROW(1, 512, 1024, 0) ROW(1, 256, 2048, 0)
  ROW(0, 1024, 256, 80)   // force one block per CU
  const char* n2[] = {"2 lanes/row dwordx4 2-way", "2 lanes/row dwordx4 cfree", "2 lanes/row loads only", "1 dword/lane loads only"};
#define ROW2(M, B, G)                                                                                  \
  {                                                                                                    \
    float ms = run2<M, B>(db, dv, N, F, dout, G);                                                      \
    printf("%-26s blk %4d grid %4d          %7.3f ms  %6.2f Gupd/s  %5.2f TB/s\n", n2[M - 7], B, G, ms,  \
           upd / ms / 1e6, (double)N * 36 / ms / 1e9);                                                 \
  }
  for (int g : {256, 512}) { ROW2(7, 1024, g) ROW2(8, 1024, g) ROW2(9, 1024, g) ROW2(10, 1024, g) }
  ROW2(7, 512, 512) ROW2(8, 512, 512) ROW2(9, 512, 512) ROW2(10, 512, 512) ROW2(10, 256, 2048) ROW2(9, 256, 2048)
  return 0;
}
