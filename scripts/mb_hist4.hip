// Micro-benchmark (round 5): a histogram pass over row-major 32-B rows (28 features + pad) + one fp32 wY per row,
// 11M rows, fixed-point packed ds_add_u64 into the bank-spread [bin][32 slot] LDS layout. Variants:
//   V1  2 lanes per row: one dwordx4 of bins (16 features) + the row's wY per lane; the 16 bytes are rotated once per
//       row by a lane-constant byte count R (alignbyte + word select), so step s adds feature 16h + ((s + R) & 15)
//       with a compile-time byte index and a precomputed slot offset: 16 atomics per 16-B load, conflict-free.
//   V8  the production geometry (8 lanes per row, one dword each) for comparison.
//  MODE 0 atomics, 1 loads only. PF: software prefetch of the next batch before this batch's atomics.
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_hist4.hip -o scripts/mb_hist4.bin && ./scripts/mb_hist4.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>

#define FTILE 32
#define HPLANE (256 * FTILE + 16)

__device__ __forceinline__ int fslot(int fl) { return (fl & 16) | ((fl + ((fl >> 4) << 1)) & 15); }

template <int MODE, int BLK, int U, bool PF>
__global__ __launch_bounds__(BLK) void k_v1(const uint4* __restrict__ bins /*[N][2]*/, const float* __restrict__ y, int N,
                                            int F, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  for (int i = threadIdx.x; i < HPLANE; i += BLK) sm[i] = 0ull;
  __syncthreads();
  constexpr int RPB = BLK / 2;                   // rows per block round
  const int t = threadIdx.x, h = t & 1, r = (t >> 1);
  const int R = r & 7;                           // byte rotation: 8 rows of a 16-lane group -> 8 distinct
  unsigned off[16];
  unsigned vmask = 0;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int f = 16 * h + ((s + R) & 15);
    off[s] = (unsigned)fslot(f) * 8u;
    if (f < F) vmask |= 1u << s;
  }
  const int per = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(N, r0 + per);
  char* H = (char*)sm;
  unsigned long long acc = 0;
  uint4 b[U];
  float yv[U];
  auto load = [&](int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = min(base + u * RPB + r, r1 - 1);
      b[u] = bins[(size_t)row * 2 + h];
      yv[u] = y[row];
    }
  };
  if (r0 < r1) load(r0);
  for (int base = r0; base < r1; base += RPB * U) {
    uint4 cb[U];
    float cy[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { cb[u] = b[u]; cy[u] = yv[u]; }
    if (PF && base + RPB * U < r1) load(base + RPB * U);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + u * RPB + r >= r1) continue;
      if (MODE == 1) { acc += cb[u].x ^ cb[u].y ^ cb[u].z ^ cb[u].w ^ __float_as_uint(cy[u]); continue; }
      // rotate the 16 bytes by R: words by R >> 2 (0 or 1), then bytes by R & 3
      const bool q = R >= 4;
      const unsigned w0 = q ? cb[u].y : cb[u].x, w1 = q ? cb[u].z : cb[u].y, w2 = q ? cb[u].w : cb[u].z,
                     w3 = q ? cb[u].x : cb[u].w;
      const int bs = R & 3;
      const unsigned v[4] = {__builtin_amdgcn_alignbyte(w1, w0, bs), __builtin_amdgcn_alignbyte(w2, w1, bs),
                             __builtin_amdgcn_alignbyte(w3, w2, bs), __builtin_amdgcn_alignbyte(w0, w3, bs)};
      const long long qa = (1ll << 48) + (long long)(int)(cy[u] * 1073741824.f);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (!((vmask >> s) & 1u)) continue;
        atomicAdd((unsigned long long*)(H + ((__builtin_amdgcn_ubfe(v[s >> 2], 8 * (s & 3), 8) << 8) + off[s])),
                  (unsigned long long)qa);
      }
    }
    if (!PF && base + RPB * U < r1) load(base + RPB * U);
  }
  __syncthreads();
  unsigned long long tt = acc;
  for (int i = threadIdx.x; i < HPLANE; i += BLK) tt += sm[i];
  for (int o = 32; o > 0; o >>= 1) tt += __shfl_xor(tt, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out + (blockIdx.x & 63) * 8, tt);   // no same-address storm
}

// production geometry: 8 lanes per row, one dword each (4 features), rotated by row parity
template <int MODE, int BLK, int U>
__global__ __launch_bounds__(BLK) void k_v8(const unsigned* __restrict__ bins32, const float* __restrict__ y, int N, int F,
                                            unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  for (int i = threadIdx.x; i < HPLANE; i += BLK) sm[i] = 0ull;
  __syncthreads();
  constexpr int RPB = BLK / 8;
  const int g = threadIdx.x >> 3, j = threadIdx.x & 7, rot = g & 1;
  unsigned off[4], sh[4];
  bool live = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = (k + rot) & 3;
    off[k] = (unsigned)fslot(j * 4 + kk) * 8u;
    sh[k] = 8 * kk;
    if (j * 4 + kk < F) live = true;
  }
  const int per = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(N, r0 + per);
  char* H = (char*)sm;
  unsigned long long acc = 0;
  for (int base = r0; base < r1; base += RPB * U) {
    unsigned w[U];
    float yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = min(base + u * RPB + g, r1 - 1);
      w[u] = bins32[(size_t)row * 8 + j];
      yv[u] = y[row];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + u * RPB + g >= r1) continue;
      if (MODE == 1) { acc += w[u] ^ __float_as_uint(yv[u]); continue; }
      if (!live) continue;
      const long long qa = (1ll << 48) + (long long)(int)(yv[u] * 1073741824.f);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        atomicAdd((unsigned long long*)(H + ((__builtin_amdgcn_ubfe(w[u], sh[k], 8) << 8) + off[k])),
                  (unsigned long long)qa);
    }
  }
  __syncthreads();
  unsigned long long tt = acc;
  for (int i = threadIdx.x; i < HPLANE; i += BLK) tt += sm[i];
  for (int o = 32; o > 0; o >>= 1) tt += __shfl_xor(tt, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out + (blockIdx.x & 63) * 8, tt);   // no same-address storm
}

static int g_copy = 0;   // which copy of the data the next launch reads (cold runs rotate over NCOPY copies)
#define NCOPY 4
template <typename Fn>
static float best_of(Fn fn, unsigned long long* out, unsigned long long* chk) {
  hipEvent_t a, e;
  hipEventCreate(&a); hipEventCreate(&e);
  hipMemset(out, 0, 8 * 64 * 8);
  fn();
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
  unsigned long long h[512];
  hipMemcpy(h, out, 8 * 512, hipMemcpyDeviceToHost);
  *chk = 0;
  for (int i = 0; i < 64; ++i) *chk += h[i * 8];
  float best = 1e9;
  for (int r = 0; r < 9; ++r) {
    g_copy = (g_copy + 1) % NCOPY;
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
  const int N = 11000000, F = 28;
  std::vector<unsigned> hb((size_t)N * 8);
  uint32_t s = 12345;
  for (size_t i = 0; i < hb.size(); ++i) {
    unsigned w = 0;
    for (int k = 0; k < 4; ++k) {
      s = s * 1664525u + 1013904223u;
      const int f = (int)(i % 8) * 4 + k;
      w |= (f < F ? ((s >> 24) % 255u) : 0u) << (8 * k);
    }
    hb[i] = w;
  }
  std::vector<float> hy(N);
  for (int i = 0; i < N; ++i) hy[i] = ((i * 7) % 100) / 100.f - 0.5f;
  unsigned* dbs[NCOPY]; float* dys[NCOPY]; unsigned long long* dout;
  for (int c = 0; c < NCOPY; ++c) {
    hipMalloc(&dbs[c], hb.size() * 4); hipMalloc(&dys[c], N * 4);
    hipMemcpy(dbs[c], hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dys[c], hy.data(), N * 4, hipMemcpyHostToDevice);
  }
  hipMalloc(&dout, 8 * 64 * 8);
#define db dbs[g_copy]
#define dy dys[g_copy]
  const size_t lds = HPLANE * 8;
  const double upd = (double)N * F;
  unsigned long long chk = 0;
#define V1(MODE, BLK, U, PF, G)                                                                                 \
  {                                                                                                           \
    const float ms = best_of([&]() { hipLaunchKernelGGL((k_v1<MODE, BLK, U, PF>), dim3(G), dim3(BLK), lds, 0,    \
                                                        (const uint4*)db, dy, N, F, dout); }, dout, &chk);   \
    printf("V1 mode %d blk %4d U %d pf %d grid %4d  %7.4f ms  %6.1f Gupd/s  chk %llx\n", MODE, BLK, U, (int)PF, G, ms,  \
           upd / ms / 1e6, chk);                                                                              \
  }
#define V8(MODE, BLK, U, G)                                                                                     \
  {                                                                                                           \
    const float ms = best_of([&]() { hipLaunchKernelGGL((k_v8<MODE, BLK, U>), dim3(G), dim3(BLK), lds, 0, db, dy, N, F, \
                                                        dout); }, dout, &chk);                               \
    printf("V8 mode %d blk %4d U %d      grid %4d  %7.4f ms  %6.1f Gupd/s  chk %llx\n", MODE, BLK, U, G, ms,        \
           upd / ms / 1e6, chk);                                                                              \
  }
  V8(0, 1024, 8, 256) V8(1, 1024, 8, 256)
  V1(1, 1024, 2, false, 256) V1(1, 1024, 4, false, 256)
  V1(0, 1024, 1, false, 256) V1(0, 1024, 2, false, 256) V1(0, 1024, 4, false, 256)
  V1(0, 1024, 1, true, 256) V1(0, 1024, 2, true, 256)
  V1(0, 512, 2, false, 512) V1(0, 512, 4, false, 512) V1(0, 512, 2, true, 512)
  V1(0, 1024, 2, false, 512) V1(0, 1024, 2, true, 512)
  V1(1, 512, 2, false, 512)
  return 0;
}
