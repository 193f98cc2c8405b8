// K-Means Lloyd iteration on f32-input MFMA (reference: h2o-algos/src/main/java/hex/kmeans/KMeans.java,
// LloydsIterationTask: closest center per row + per-center sums / counts, reduced over chunks).
//
// One pass over the rows does both halves of the Lloyd step as matrix products on the matrix cores:
//
//  1. distance GEMM   S[c][row] = ||c||^2 - 2 c.x  (v_mfma_f32_16x16x4_f32, exact f32 fma chains)
//     A = 16 centers x 4 dims of C (registers for the whole launch), B = 4 dims x 16 rows of Xᵀ
//     (LDS). The 16x16 result leaves row = lane&15 and centers 4*(lane>>4)+r in the lane's 4
//     accumulator registers: the argmin over centers is 4 in-lane compares plus two cross-lane steps
//     (xor 16, xor 32), ties -> smaller center index like the reference's strict '<' scan. The same
//     B-operand values give ||x||^2 (partial sums per lane, the same two steps).
//     MEASURED (r3): the former orientation (D[row][center]) needed a 4-step butterfly per row and 8
//     broadcasts per 4 rows: ~80 ds_bpermute per 16 rows, which made the kernel LDS-pipe bound.
//  2. centroid GEMM   T[c][d] += sum_rows onehot(assign)[c][row] * w * X[row][d]
//     A = 16 centers x 4 rows (the one-hot of the rows' argmins, built from the step-1 registers by
//     lane shuffles), B = 4 rows x 16 dims of X (coalesced 64-byte row segments); a constant-1
//     column appended at dim P gives the weighted counts in the same accumulators.
//
// Each wave walks 16-row tiles (grid-stride) and keeps its sums in AGPR/VGPR accumulators; at the
// end it writes one [KT*16][PT*16] fp32 slab (no atomics). The host sums the slabs in fp64.
// Rows are read once (X: 4*P bytes/row) -> the launch streams at HBM rate.
// MEASURED r5 (10M x 20, k = 10): two 64-row tiles in flight per wave (register double buffer, 3 waves / SIMD)
// 322.7 us vs 318.0 us with one — the kernel is not bound by outstanding HBM reads; not kept
// (scripts/experiments/kmeans_double_buffer.diff, profiles/r5_kmeans_db_kernel_stats.md).
// MEASURED r5: the 64-row tile in phases over its four 16-row sub-tiles (distance MFMAs of different sub-tiles
// interleaved, one store branch per tile) with the row weight moved into the one-hot A operand and the counts'
// constant column kept in LDS (the B operand is read with no per-element VALU): 318.0 -> 286.6 us per Lloyd
// kernel, 0.352 -> 0.321 ms per iteration end to end (profiles/r5_kmeans_phased_kernel_stats.md).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>
#include <stdlib.h>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bfly_min_idx(float v, int& idx, int mask) {
  const float ov = __shfl_xor(v, mask, 64);
  const int oi = __shfl_xor(idx, mask, 64);
  if (ov < v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  return v;
}

// KT = center tiles of 16 (K <= 16*KT), PS = max dim steps of 4 (P <= 4*PS), PT = dim tiles of 16
// for the sums (P+1 <= 16*PT). Each wave stages 64 rows (4 MFMA row tiles) of X in its own LDS
// slice with coalesced loads (16-B vectors when P % 4 == 0): every row is read from HBM exactly
// once and both GEMMs take their operands from LDS (row stride P+1 keeps the strided A-operand
// reads of the distance GEMM on distinct banks).
#define KM_ROWS 64
// LDS row stride of a wave's slice: the smallest stride >= P + 1 that is 17 mod 32, so the distance GEMM's
// B-operand reads (lanes c16 x q, address c16 * Pp + q) and the centroid GEMM's row reads (q * Pp + c16) of
// each 32-lane half fall on (nearly) distinct banks — P + 1 = 21 left 25 % of the LDS-active cycles in bank
// conflicts (PMC, profiles/r3_session2_kmeans_c31.md). Kept only while three 4-wave blocks still fit a CU's
// LDS (the VGPR-bound occupancy).
#ifndef KM_VEC
#define KM_VEC 0
#endif
// KM_VEC: stride P + 8 or P + 4 with stride / 4 odd — rows 16-byte aligned (one ds_write_b128 per staged float4 group
// instead of four ds_write_b32) and the distance GEMM's reads (c16 * Pp + 4 s + q: c16 * Pp / 4 distinct mod 16)
// still on 64 distinct banks. MEASURED (r4, 10M x 20, k = 10, same box): 0.3965 / 0.3984 vs 0.3977 / 0.4001 ms per
// Lloyd step — the staging stores are not the limit; kept off. Again after the r5 phased tile: 284.3 vs 285.6 us.
// occ4: the 4-waves-per-SIMD variant (k_lloyd_mfma4) keeps the unpadded stride P + 1 unless the bank-spreading one
// still fits four 4-wave blocks in a CU's LDS (stride <= 38).
__host__ __device__ inline int km_stride(int P, bool occ4 = false) {
#if KM_VEC
  // > P: column P of every row holds the centroid GEMM's constant 1 (the counts), see the staging loop
  return ((P / 4) & 1) ? P + 8 : P + 4;
#else
  int pp = P + 1;
  const int adj = pp + ((17 - pp % 32) + 32) % 32;
  return adj <= (occ4 ? 38 : 52) ? adj : pp;
#endif
}
template <int KT, int PS, int PT, int G, bool OCC4>
__device__ __forceinline__ void lloyd_body(const float* __restrict__ X, int64_t N, int P, const float* __restrict__ C,
                                           int K, const float* __restrict__ w, int* __restrict__ assign,
                                           float* __restrict__ mind, float* __restrict__ slabs) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int q = lane >> 4;          // 0..3
  const int c16 = lane & 15;        // 0..15
  const int Pp = km_stride(P, OCC4);
  float* xs = lds + (size_t)wv * KM_ROWS * Pp;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + wv;
  const int64_t n_waves = (int64_t)gridDim.x * 4;
  const int ps = (P + 3) >> 2;

  // centers as the A operand of the distance MFMA: ca[t][s] = C[t*16 + c16][4s + q];
  // csq[t][r] = ||C[t*16 + 4q + r]||^2 for the D layout (FLT_MAX for padding centers)
  float ca[KT][PS];
  float csq[KT][4];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int c = t * 16 + c16;
#pragma unroll
    for (int s = 0; s < PS; ++s) {
      const int d = 4 * s + q;
      ca[t][s] = (c < K && d < P) ? C[(int64_t)c * P + d] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cr = t * 16 + 4 * q + r;
      float s2 = 0.f;
      if (cr < K)
        for (int d = 0; d < P; ++d) { const float v = C[(int64_t)cr * P + d]; s2 = fmaf(v, v, s2); }
      csq[t][r] = cr < K ? s2 : FLT_MAX;
    }
  }

  f32x4 acc[KT][PT];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int u = 0; u < PT; ++u) acc[t][u] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // P % 4 == 0 (the host pads the design matrix): the lane's float4 groups e4 = lane + 64 i, i < PS
  // (64 P / 4 <= 64 PS), are loaded with one dwordx4 each
  float* wsl = lds + (size_t)4 * KM_ROWS * Pp + wv * KM_ROWS;   // per-wave row weights of the tile
  // Software pipeline: the NEXT tile's rows (and weights) are loaded into registers while the current
  // tile is computed from LDS. MEASURED (r2): the former load -> wait -> LDS-write loop per 64-row tile
  // exposed one HBM round trip per float4 group (781 us per Lloyd step on 10M x 20 = ~1 TB/s).
  float4 pf[PS];
  float pwt = 0.f;
  auto issue = [&](int64_t rs) {
    const int nr = (int)((N - rs) < KM_ROWS ? (N - rs) : KM_ROWS);
    const int nel = nr * P;
    const float4* s4 = reinterpret_cast<const float4*>(X + rs * P);
#pragma unroll
    for (int i = 0; i < PS; ++i) {
      const int e4 = lane + 64 * i;
      pf[i] = 4 * e4 < nel ? s4[e4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    pwt = lane < nr ? (w ? w[rs + lane] : 1.f) : 0.f;
  };
  // LDS destinations of the lane's groups are the same for every tile: computed once (no per-tile
  // integer division by the runtime P); the 4 elements of a group share a row
  int doff[PS];
#pragma unroll
  for (int i = 0; i < PS; ++i) {
    const int e = 4 * (lane + 64 * i);
    const int r = e / P, c = e - r * P;
    doff[i] = e < KM_ROWS * P ? r * Pp + c : -1;
  }
  xs[lane * Pp + P] = 1.f;   // column P of each of the 64 rows (never staged over): the centroid GEMM's counts
  if (wave_g * KM_ROWS < N) issue(wave_g * KM_ROWS);
  for (int64_t r0 = wave_g * KM_ROWS; r0 < N; r0 += n_waves * KM_ROWS) {
    const int nrows = (int)((N - r0) < KM_ROWS ? (N - r0) : KM_ROWS);
    // ---- the prefetched tile -> this wave's LDS slice (row stride P+1; tail rows are zeros)
#pragma unroll
    for (int i = 0; i < PS; ++i) {
      if (doff[i] >= 0) {
        float* dst = xs + doff[i];
#if KM_VEC
        *reinterpret_cast<float4*>(dst) = pf[i];
#else
        dst[0] = pf[i].x; dst[1] = pf[i].y; dst[2] = pf[i].z; dst[3] = pf[i].w;
#endif
      }
    }
    wsl[lane] = pwt;
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's own LDS writes (vmcnt untouched)
    __builtin_amdgcn_wave_barrier();
    {
      const int64_t nx = r0 + n_waves * KM_ROWS;
      if (nx < N) issue(nx);                 // next tile's loads stay in flight during the compute below
    }
    // The 64-row tile in phases, each over the 4 16-row sub-tiles, so independent MFMA chains / shuffles of
    // different sub-tiles interleave (the former per-sub-tile order serialised distance -> argmin -> shuffle ->
    // centroid chains; the stores' divergent branch split the schedule once per sub-tile).
    // G sub-tiles per phase group (registers: G x KT distance tiles live at once)
#pragma unroll
    for (int g0 = 0; g0 < KM_ROWS / 16; g0 += G) {
    // ---- 1. distance GEMM: B[k = dim 4s+q][j = row c16]; the same values give ||x||^2
    f32x4 d[G][KT];
    float xq[G];
#pragma unroll
    for (int tr = 0; tr < G; ++tr) {
      xq[tr] = 0.f;
#pragma unroll
      for (int t = 0; t < KT; ++t) d[tr][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < PS; ++s) {
      if (s < ps) {
#pragma unroll
        for (int tr = 0; tr < G; ++tr) {
          const float xb = xs[((g0 + tr) * 16 + c16) * Pp + 4 * s + q];   // P % 4 == 0: a real (or padding-zero) dim
          xq[tr] = fmaf(xb, xb, xq[tr]);
#pragma unroll
          for (int t = 0; t < KT; ++t) d[tr][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[t][s], xb, d[tr][t], 0, 0, 0);
        }
      }
    }
    // ---- argmin over the centers (ties -> smaller index), then ||x||^2 across the lane quarters
    int bidx[G];
    float best[G];
#pragma unroll
    for (int tr = 0; tr < G; ++tr) {
      best[tr] = FLT_MAX;
      bidx[tr] = 0x7fffffff;
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sc = csq[t][r] - 2.f * d[tr][t][r];
          const int ci = t * 16 + 4 * q + r;              // increasing: strict '<' keeps the smaller index
          if (sc < best[tr]) { best[tr] = sc; bidx[tr] = ci; }
        }
    }
#pragma unroll
    for (int tr = 0; tr < G; ++tr) best[tr] = bfly_min_idx(best[tr], bidx[tr], 16);
#pragma unroll
    for (int tr = 0; tr < G; ++tr) best[tr] = bfly_min_idx(best[tr], bidx[tr], 32);
#pragma unroll
    for (int tr = 0; tr < G; ++tr) xq[tr] += __shfl_xor(xq[tr], 16, 64);
#pragma unroll
    for (int tr = 0; tr < G; ++tr) xq[tr] += __shfl_xor(xq[tr], 32, 64);
    if (q == 0) {                                      // every lane of column c16 holds row tr*16 + c16's result
#pragma unroll
      for (int tr = 0; tr < G; ++tr) {
        const int rrow = (g0 + tr) * 16 + c16;
        if (rrow < nrows) {
          if (assign) assign[r0 + rrow] = bidx[tr];  // (null: the Lloyd loop does not read assignments)
          mind[r0 + rrow] = fmaxf(xq[tr] + best[tr], 0.f);
        }
      }
    }
    // ---- 2. centroid GEMM in steps of 4 rows: A[i = center][k = row 4j+q] = onehot * row weight, B[k = row][j =
    // dim] read straight from the slice, whose column P holds 1.0 (the weighted counts) — no per-element VALU
#pragma unroll
    for (int tr = 0; tr < G; ++tr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rt = (g0 + tr) * 16 + 4 * j + q;                // row within the 64-row slice (zero-weight tail rows)
        const int my_a = __shfl(bidx[tr], 4 * j + q, 64);
        const float ww = wsl[rt];
        const float* xr = xs + rt * Pp;
#pragma unroll
        for (int u = 0; u < PT; ++u) {
          const int dd = u * 16 + c16;
          const float bv = dd <= P ? xr[dd] : 0.f;
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            const float av = (my_a == t * 16 + c16) ? ww : 0.f;
            acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t][u], 0, 0, 0);
          }
        }
      }
    }
    }
    __builtin_amdgcn_wave_barrier();   // the slice is rewritten by the next iteration's loads
  }
  // ---- per-BLOCK slab: [KT*16 centers][PT*16 dims], D layout row = 4q + r (center), col = c16 (dim). The four
  // waves' accumulators are summed through LDS (the staging slices are free now), so the host-side fp64 reduction
  // reads one slab per block instead of four (MEASURED r5: the torch slab sum was ~40 us of a 454 us iteration)
  constexpr int SL = KT * 16 * PT * 16;
  float* red = lds;                                   // one slab (SL <= the staging slices, see km_stride)
  for (int src = 1; src < 4; ++src) {
    __syncthreads();
    if (wv == src) {
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int u = 0; u < PT; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[(t * 16 + 4 * q + r) * (PT * 16) + u * 16 + c16] = acc[t][u][r];
    }
    __syncthreads();
    if (wv == 0) {
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int u = 0; u < PT; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][u][r] += red[(t * 16 + 4 * q + r) * (PT * 16) + u * 16 + c16];
    }
  }
  if (wv != 0) return;
  float* out = slabs + (int64_t)blockIdx.x * SL;
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int u = 0; u < PT; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(t * 16 + 4 * q + r) * (PT * 16) + u * 16 + c16] = acc[t][u][r];
}

#define KM_ARGS const float* __restrict__ X, int64_t N, int P, const float* __restrict__ C, int K, \
                const float* __restrict__ w, int* __restrict__ assign, float* __restrict__ mind, float* __restrict__ slabs
template <int KT, int PS, int PT>
__global__ __launch_bounds__(256) void k_lloyd_mfma(KM_ARGS) {
  lloyd_body<KT, PS, PT, (KT == 1 ? 4 : (KT == 2 ? 2 : 1)), false>(X, N, P, C, K, w, assign, mind, slabs);
}
// 4 waves / SIMD: phase groups of 2 sub-tiles (G = 4 needs more than 128 VGPRs) and the unpadded LDS stride.
// MEASURED r5 (10M x 20, k = 10; scripts/gpu_r5_c27.sh): 287.7 us (3 waves, G = 4, stride 49) -> 258.8 us.
#ifndef KM_W4
#define KM_W4 4         // A/B: waves per SIMD of the high-occupancy variant (5 with G = 1 spills: 253 -> 329 us)
#endif
#ifndef KM_G4
#define KM_G4 2         // A/B: its phase-group size (K <= 16)
#endif
template <int KT, int PS, int PT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KM_W4, KM_W4))) void k_lloyd_mfma4(KM_ARGS) {
  lloyd_body<KT, PS, PT, (KT == 1 ? KM_G4 : 1), true>(X, N, P, C, K, w, assign, mind, slabs);
}
#undef KM_ARGS
// shapes whose 4-wave variant compiles without spills (-Rpass-analysis=kernel-resource-usage)
__host__ __device__ constexpr bool km_occ4(int KT, int PS, int PT) {
  return KT == 1 && PS <= 6 && PT <= 2;
}
static bool km_occ4_enabled() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("H2O_KM_OCC4"); v = (e && e[0] == '0') ? 0 : 1; }
  return v == 1;
}
template <int KT, int PS, int PT>
static bool km_use4() { return km_occ4(KT, PS, PT) && km_occ4_enabled(); }

template <int KT, int PS, int PT>
hipError_t km_occ(int* per, int P) {
  const bool o4 = km_use4<KT, PS, PT>();
  const size_t lds = ((size_t)4 * KM_ROWS * km_stride(P, o4) + 4 * KM_ROWS) * sizeof(float);
  if constexpr (km_occ4(KT, PS, PT)) {
    if (o4) return hipOccupancyMaxActiveBlocksPerMultiprocessor(per, k_lloyd_mfma4<KT, PS, PT>, 256, lds);
  }
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per, k_lloyd_mfma<KT, PS, PT>, 256, lds);
}

template <int KT, int PS, int PT>
int launch(const float* X, long long N, int P, const float* C, int K, const float* w, int* assign, float* mind,
           float* slabs, int grid, hipStream_t s) {
  const bool o4 = km_use4<KT, PS, PT>();
  const size_t lds = ((size_t)4 * KM_ROWS * km_stride(P, o4) + 4 * KM_ROWS) * sizeof(float);   // 4 slices + 4 x 64 weights
  if constexpr (km_occ4(KT, PS, PT)) {
    if (o4) {
      hipLaunchKernelGGL((k_lloyd_mfma4<KT, PS, PT>), dim3(grid), dim3(256), lds, s, X, (int64_t)N, P, C, K, w, assign,
                         mind, slabs);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_lloyd_mfma<KT, PS, PT>), dim3(grid), dim3(256), lds, s, X, (int64_t)N, P, C, K, w, assign,
                     mind, slabs);
  return (int)hipGetLastError();
}

// The rest of a Lloyd iteration in one launch (KMeans.java: new centers = sums / counts, empty clusters keep their
// center for the re-seed, convergence = the largest center move): tot = the fp64 sum of the per-block slabs
// ([.][ldt], count in column P). Replaces ~6 small torch launches per iteration.
__global__ __launch_bounds__(256) void k_kmeans_update(const double* __restrict__ tot, int ldt, int K, int P,
                                                       const float* __restrict__ C, float* __restrict__ newC,
                                                       double* __restrict__ cnt_out, double* __restrict__ flags) {
  __shared__ float smax[4];
  __shared__ int sempty[4];
  float mx = 0.f;
  int empty = 0;
  for (int i = threadIdx.x; i < K * P; i += 256) {
    const int c = i / P, d = i - c * P;
    const double cnt = tot[(int64_t)c * ldt + P];
    const float v = cnt > 0.0 ? (float)(tot[(int64_t)c * ldt + d] / fmax(cnt, 1e-300)) : C[i];
    newC[i] = v;
    mx = fmaxf(mx, fabsf(v - C[i]));
  }
  for (int c = threadIdx.x; c < K; c += 256) {
    const double cnt = tot[(int64_t)c * ldt + P];
    cnt_out[c] = cnt;
    empty += cnt == 0.0 ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    empty += __shfl_xor(empty, o, 64);
  }
  if ((threadIdx.x & 63) == 0) { smax[threadIdx.x >> 6] = mx; sempty[threadIdx.x >> 6] = empty; }
  __syncthreads();
  if (threadIdx.x == 0) {
    flags[0] = (double)(sempty[0] + sempty[1] + sempty[2] + sempty[3]);
    flags[1] = (double)fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
  }
}

}  // namespace

extern "C" {

int h2o_kmeans_update(const double* tot, int ldt, int K, int P, const float* C, float* newC, double* cnt,
                      double* flags, hipStream_t s) {
  if (K < 1 || P < 1 || ldt < P + 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_kmeans_update, dim3(1), dim3(256), 0, s, tot, ldt, K, P, C, newC, cnt, flags);
  return (int)hipGetLastError();
}

// Shape class the MFMA Lloyd kernel supports (0 = not supported: caller falls back).
// Returns KT*100 + PS*10... encoded as (KT, PS, PT) via out[3].
int h2o_kmeans_mfma_shape(int K, int P, int* out) {
  if (K < 1 || P < 1 || K > 64 || P > 64) return 0;
  const int KT = K <= 16 ? 1 : (K <= 32 ? 2 : 4);
  // float4 groups per lane >= P / 4 (MEASURED r5: a PS = 5 shape for P = 20 saved 2 VGPRs, 263 vs 253-259 us: not kept)
  const int PS = P <= 16 ? 4 : (P <= 24 ? 6 : (P <= 32 ? 8 : 16));
  const int PT = (P + 1 + 15) / 16;
  out[0] = KT; out[1] = PS; out[2] = PT;
  return 1;
}

// Grid that fills the GPU exactly once: CUs x resident blocks per CU of this shape's kernel. Every block
// grid-strides over the rows with an equal share, so a grid above one resident round (the former fixed 1024
// blocks at 3 resident blocks per CU = 768) ran a second, one-third-full round of equal length.
int h2o_kmeans_mfma_grid(int K, int P) {
  int sh[3];
  if (!h2o_kmeans_mfma_shape(K, P, sh)) return 0;
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const int KT = sh[0], PS = sh[1], PT = sh[2];
  hipError_t e = hipErrorInvalidValue;
#define O(kt, ps, pt) if (KT == kt && PS == ps && PT == pt) e = km_occ<kt, ps, pt>(&per, P)
  O(1, 4, 1); O(1, 4, 2); O(1, 6, 2); O(1, 8, 2); O(1, 8, 3); O(1, 16, 3); O(1, 16, 4); O(1, 16, 5);
  O(2, 4, 1); O(2, 4, 2); O(2, 6, 2); O(2, 8, 2); O(2, 8, 3); O(2, 16, 3); O(2, 16, 4); O(2, 16, 5);
  O(4, 4, 1); O(4, 4, 2); O(4, 6, 2); O(4, 8, 2); O(4, 8, 3); O(4, 16, 3); O(4, 16, 4); O(4, 16, 5);
#undef O
  if (e != hipSuccess || per < 1) per = 1;
  return cus * per;
}

// slabs: [grid][KT*16][PT*16] fp32 (one per block; caller allocates with the shape from h2o_kmeans_mfma_shape)
int h2o_kmeans_mfma(const float* X, long long N, int P, const float* C, int K, const float* w, int* assign,
                    float* mind, float* slabs, int grid, hipStream_t s) {
  int sh[3];
  if (!h2o_kmeans_mfma_shape(K, P, sh) || N <= 0 || grid <= 0 || (P & 3)) return (int)hipErrorInvalidValue;
  const int KT = sh[0], PS = sh[1], PT = sh[2];
#define L(kt, ps, pt) if (KT == kt && PS == ps && PT == pt) return launch<kt, ps, pt>(X, N, P, C, K, w, assign, mind, slabs, grid, s)
  L(1, 4, 1); L(1, 4, 2); L(1, 6, 2); L(1, 8, 2); L(1, 8, 3); L(1, 16, 3); L(1, 16, 4); L(1, 16, 5);
  L(2, 4, 1); L(2, 4, 2); L(2, 6, 2); L(2, 8, 2); L(2, 8, 3); L(2, 16, 3); L(2, 16, 4); L(2, 16, 5);
  L(4, 4, 1); L(4, 4, 2); L(4, 6, 2); L(4, 8, 2); L(4, 8, 3); L(4, 16, 3); L(4, 16, 4); L(4, 16, 5);
#undef L
  return (int)hipErrorInvalidValue;
}

}  // extern "C"
