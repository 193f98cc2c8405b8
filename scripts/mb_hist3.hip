// Micro-benchmark (round 5): what bounds a tree-histogram pass on gfx950 once the row loads are wide?
//  A. pure LDS atomic throughput (addresses precomputed in registers, conflict-free): u64 / u32, all lanes,
//     half / quarter of the lanes active.
//  B. word-planar bins (plane p = features 4p..4p+3 of every row, [N] uint32), one lane = (4 consecutive rows,
//     one plane): ONE dwordx4 of bins + ONE dwordx4 of wY per 16 atomics; optional per-row node-id filter.
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_hist3.hip -o scripts/mb_hist3.bin && ./scripts/mb_hist3.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>

#define FTILE 32
#define HPLANE (256 * FTILE + 16)

__device__ __forceinline__ int fslot(int fl) { return (fl & 16) | ((fl + ((fl >> 4) << 1)) & 15); }

// A: ITERS rounds of 16 atomics per lane. ACT: active-lane pattern (1 all, 2 even lanes, 4 every 4th lane)
template <int MODE, int ACT>
__global__ __launch_bounds__(1024) void k_atom(int iters, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  for (int i = threadIdx.x; i < HPLANE; i += blockDim.x) sm[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  unsigned addr[16];
  unsigned s = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    s = s * 1664525u + 1013904223u;
    const unsigned bin = (s >> 24);
    const int f = ((lane & 15) + k) & 31;          // 16 lanes of a group: 16 distinct features
    addr[k] = (bin * FTILE + fslot(f)) * (MODE == 0 ? 8u : 4u);
  }
  const bool act = (lane % ACT) == 0;
  char* H = (char*)sm;
  for (int it = 0; it < iters; ++it) {
    if (act) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (MODE == 0) atomicAdd((unsigned long long*)(H + addr[k]), (unsigned long long)(it + 1));
        else atomicAdd((unsigned*)(H + addr[k]), (unsigned)(it + 1));
      }
    }
  }
  __syncthreads();
  unsigned long long t = 0;
  for (int i = threadIdx.x; i < HPLANE; i += blockDim.x) t += sm[i];
  atomicAdd(out, t);
}

// B: planar histogram. MODE 0: atomics, 1: loads only, 2: atomics for rows with nid & 1 (filter), 3: filter +
// loads only. BLK threads, grid G.
template <int MODE, int BLK>
__global__ __launch_bounds__(BLK) void k_planar(const uint4* __restrict__ planes /*[P][N/4]*/, const float4* __restrict__ y4,
                                                const unsigned* __restrict__ nid4 /*[N/4] 4 node bytes*/, int N, int P,
                                                unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  for (int i = threadIdx.x; i < HPLANE; i += BLK) sm[i] = 0ull;
  __syncthreads();
  const int NG = N / 4;                      // row groups (N multiple of 4 here)
  const int per = (NG + gridDim.x - 1) / gridDim.x;
  const int g0 = blockIdx.x * per, g1 = min(NG, g0 + per);
  const int units = (g1 - g0) * P;
  char* H = (char*)sm;
  unsigned long long acc = 0;
  constexpr int U = 2;                       // units per lane in flight
  for (int ub = 0; ub < units; ub += BLK * U) {
    uint4 b[U];
    float4 y[U];
    unsigned nd[U];
    int pp[U], rg[U];
    bool ok[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int u = ub + k * BLK + threadIdx.x;
      ok[k] = u < units;
      const int uc = ok[k] ? u : 0;
      rg[k] = uc / P;
      pp[k] = uc - rg[k] * P;
      const int g = g0 + rg[k];
      b[k] = planes[(size_t)pp[k] * NG + g];
      y[k] = y4[g];
      nd[k] = (MODE >= 2) ? nid4[g] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (!ok[k]) continue;
      if (MODE == 1 || MODE == 3) {
        acc += b[k].x ^ b[k].y ^ b[k].z ^ b[k].w ^ __float_as_uint(y[k].x + y[k].y + y[k].z + y[k].w) ^ nd[k];
        continue;
      }
      // lane's 4 feature slots, rotated by the row group so the lanes of one plane hit distinct features
      const int rot = rg[k] & 3;
      unsigned off[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) off[j] = (unsigned)fslot(pp[k] * 4 + ((j + rot) & 3)) * 8u;
      const unsigned wv[4] = {b[k].x, b[k].y, b[k].z, b[k].w};
      const float yv[4] = {y[k].x, y[k].y, y[k].z, y[k].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (MODE == 2 && !((nd[k] >> (8 * r)) & 1u)) continue;
        const long long q = (1ll << 48) + (long long)(int)(yv[r] * 1073741824.f);
        const unsigned w = __builtin_amdgcn_alignbyte(wv[r], wv[r], rot);   // byte j of w = byte (j + rot) & 3
#pragma unroll
        for (int j = 0; j < 4; ++j)
          atomicAdd((unsigned long long*)(H + ((__builtin_amdgcn_ubfe(w, 8 * j, 8) << 8) + off[j])),
                    (unsigned long long)q);
      }
    }
  }
  __syncthreads();
  unsigned long long t = acc;
  for (int i = threadIdx.x; i < HPLANE; i += BLK) t += sm[i];
  atomicAdd(out, t);
}

static float best_of(void (*fn)(void*), void* ctx) {
  hipEvent_t a, e;
  hipEventCreate(&a); hipEventCreate(&e);
  fn(ctx);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
  float best = 1e9;
  for (int r = 0; r < 7; ++r) {
    hipEventRecord(a);
    fn(ctx);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, a, e);
    if (ms < best) best = ms;
  }
  return best;
}

struct Ctx { const uint4* pl; const float4* y; const unsigned* nid; int N, P, grid, iters; unsigned long long* out; };

template <int MODE, int ACT> static void run_atom(void* c) {
  Ctx* x = (Ctx*)c;
  hipLaunchKernelGGL((k_atom<MODE, ACT>), dim3(x->grid), dim3(1024), HPLANE * 8, 0, x->iters, x->out);
}
template <int MODE, int BLK> static void run_planar(void* c) {
  Ctx* x = (Ctx*)c;
  hipLaunchKernelGGL((k_planar<MODE, BLK>), dim3(x->grid), dim3(BLK), HPLANE * 8, 0, x->pl, x->y, x->nid, x->N, x->P,
                     x->out);
}

int main() {
  const int N = 11000000, P = 7;
  std::vector<unsigned> hb((size_t)N * P);
  uint32_t s = 12345;
  for (auto& x : hb) {
    unsigned w = 0;
    for (int k = 0; k < 4; ++k) { s = s * 1664525u + 1013904223u; w |= ((s >> 24) % 255u) << (8 * k); }
    x = w;
  }
  std::vector<float> hy(N);
  for (int i = 0; i < N; ++i) hy[i] = ((i * 7) % 100) / 100.f - 0.5f;
  std::vector<unsigned char> hn(N);
  for (int i = 0; i < N; ++i) { s = s * 1664525u + 1013904223u; hn[i] = ((s >> 20) % 10u) < 4u ? 1 : 0; }   // 40 %
  unsigned* db; float* dy; unsigned char* dn; unsigned long long* dout;
  hipMalloc(&db, hb.size() * 4); hipMalloc(&dy, N * 4); hipMalloc(&dn, N); hipMalloc(&dout, 8);
  hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dy, hy.data(), N * 4, hipMemcpyHostToDevice);
  hipMemcpy(dn, hn.data(), N, hipMemcpyHostToDevice);
  Ctx c{(const uint4*)db, (const float4*)dy, (const unsigned*)dn, N, P, 256, 2000, dout};
  const double upd = (double)N * P * 4;
  // A: pure atomics
  {
    const double n_at = 256.0 * 1024 * 2000 * 16;
    struct { const char* name; void (*fn)(void*); double frac; } rows[] = {
        {"u64 all lanes", run_atom<0, 1>, 1.0}, {"u64 half lanes", run_atom<0, 2>, 0.5},
        {"u64 quarter lanes", run_atom<0, 4>, 0.25}, {"u32 all lanes", run_atom<1, 1>, 1.0},
        {"u32 half lanes", run_atom<1, 2>, 0.5}};
    for (auto& r : rows) {
      const float ms = best_of(r.fn, &c);
      const double wave_instr_per_cu = n_at / 64.0 / 256.0;
      printf("A %-20s %8.3f ms  %7.1f G lane-atomics/s  %6.2f cycles/wave-instr/CU @2.4GHz\n", r.name, ms,
             n_at * r.frac / ms / 1e6, ms * 1e-3 * 2.4e9 / wave_instr_per_cu);
    }
  }
  // B: planar histograms
  for (int g : {256, 512}) {
    c.grid = g;
    struct { const char* name; void (*fn)(void*); } rows[] = {
        {"planar atomics b1024", run_planar<0, 1024>}, {"planar loads b1024", run_planar<1, 1024>},
        {"planar filt40 b1024", run_planar<2, 1024>}, {"planar filt ld b1024", run_planar<3, 1024>},
        {"planar atomics b512", run_planar<0, 512>}, {"planar loads b512", run_planar<1, 512>}};
    for (auto& r : rows) {
      if (g == 512 && r.fn == (void (*)(void*))run_planar<0, 512>) {}
      const float ms = best_of(r.fn, &c);
      printf("B %-22s grid %4d %8.3f ms  %7.1f Gupd/s  %5.2f TB/s (32 B/row)\n", r.name, g, ms, upd / ms / 1e6,
             (double)N * 32 / ms / 1e9);
    }
  }
  return 0;
}
