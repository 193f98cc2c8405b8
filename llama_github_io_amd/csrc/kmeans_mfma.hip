// K-Means Lloyd iteration on f32-input MFMA (reference: h2o-algos/src/main/java/hex/kmeans/KMeans.java,
// LloydsIterationTask: closest center per row + per-center sums / counts, reduced over chunks).
//
// One pass over the rows does both halves of the Lloyd step as matrix products on the matrix cores:
//
//  1. distance GEMM   S[row][c] = ||c||^2 - 2 x.c  (v_mfma_f32_16x16x4_f32, exact f32 fma chains)
//     A = 16 rows x 4 dims of X, B = 4 dims x 16 centers (Cᵀ, held in registers for the whole
//     launch). The 16x16 result leaves center c = lane&15 and rows 4*(lane>>4)+r in the lane's 4
//     accumulator registers, so the argmin over centers is a 4-step butterfly inside each 16-lane
//     group (ties -> smaller center index, like the reference's strict '<' scan).
//  2. centroid GEMM   T[c][d] += sum_rows onehot(assign)[c][row] * w * X[row][d]
//     A = 16 centers x 4 rows (the one-hot of the rows' argmins, built from the step-1 registers by
//     lane shuffles), B = 4 rows x 16 dims of X (coalesced 64-byte row segments); a constant-1
//     column appended at dim P gives the weighted counts in the same accumulators.
//
// Each wave walks 16-row tiles (grid-stride) and keeps its sums in AGPR/VGPR accumulators; at the
// end it writes one [KT*16][PT*16] fp32 slab (no atomics). The host sums the slabs in fp64.
// Rows are read once (X: 4*P bytes/row) -> the launch streams at HBM rate.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

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
template <int KT, int PS, int PT>
__global__ __launch_bounds__(256) void k_lloyd_mfma(const float* __restrict__ X, int64_t N, int P,
                                                    const float* __restrict__ C, int K,
                                                    const float* __restrict__ w, int* __restrict__ assign,
                                                    float* __restrict__ mind, float* __restrict__ slabs) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int q = lane >> 4;          // 0..3
  const int c16 = lane & 15;        // 0..15
  const int Pp = P + 1;
  float* xs = lds + (size_t)wv * KM_ROWS * Pp;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + wv;
  const int64_t n_waves = (int64_t)gridDim.x * 4;
  const int ps = (P + 3) >> 2;

  // centers as the B operand of the distance MFMA: cb[t][s] = C[t*16 + c16][4s + q]
  float cb[KT][PS];
  float csq[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int c = t * 16 + c16;
    float s2 = 0.f;
#pragma unroll
    for (int s = 0; s < PS; ++s) {
      const int d = 4 * s + q;
      cb[t][s] = (c < K && d < P) ? C[(int64_t)c * P + d] : 0.f;
    }
    if (c < K) {
      for (int d = 0; d < P; ++d) { const float v = C[(int64_t)c * P + d]; s2 = fmaf(v, v, s2); }
    }
    csq[t] = (c < K) ? s2 : FLT_MAX;
  }

  f32x4 acc[KT][PT];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int u = 0; u < PT; ++u) acc[t][u] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const bool vec4 = (P & 3) == 0;
  for (int64_t r0 = wave_g * KM_ROWS; r0 < N; r0 += n_waves * KM_ROWS) {
    const int nrows = (int)((N - r0) < KM_ROWS ? (N - r0) : KM_ROWS);
    const int nel = nrows * P;
    const float* src = X + r0 * P;
    // ---- stage 64 rows into this wave's LDS slice (row stride P+1), zero the tail rows
    if (vec4) {
      const float4* s4 = reinterpret_cast<const float4*>(src);
      for (int e4 = lane; e4 < (KM_ROWS * P) / 4; e4 += 64) {
        const int e = e4 * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < nel) v = s4[e4];
        const int r = e / P, c = e - r * P;       // P % 4 == 0: the 4 elements share a row
        float* dst = xs + r * Pp + c;
        dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
      }
    } else {
      for (int e = lane; e < KM_ROWS * P; e += 64) {
        const int r = e / P, c = e - r * P;
        xs[r * Pp + c] = e < nel ? src[e] : 0.f;
      }
    }
    __builtin_amdgcn_s_waitcnt(0);   // wave-private slice: the wave's own LDS writes are visible after this
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int tr = 0; tr < KM_ROWS / 16; ++tr) {
      const float* xt = xs + tr * 16 * Pp;
      // ---- 1. distance GEMM: A[i = row c16][k = dim 4s+q]
      f32x4 d[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) d[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < PS; ++s) {
        if (s < ps) {
          const int dd = 4 * s + q;
          const float a = dd < P ? xt[c16 * Pp + dd] : 0.f;
#pragma unroll
          for (int t = 0; t < KT; ++t) d[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, cb[t][s], d[t], 0, 0, 0);
        }
      }
      float best[4];
      int bidx[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        best[r] = FLT_MAX;
        bidx[r] = 0x7fffffff;
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const float sc = csq[t] - 2.f * d[t][r];
          const int ci = t * 16 + c16;
          if (ci < K && (sc < best[r] || (sc == best[r] && ci < bidx[r]))) { best[r] = sc; bidx[r] = ci; }
        }
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) best[r] = bfly_min_idx(best[r], bidx[r], m);
      }
      // ---- 2. centroid GEMM over the 16 rows in 4 steps of 4 rows (k = row 4j + q of the tile)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int a0 = __shfl(bidx[0], j * 16, 64), a1 = __shfl(bidx[1], j * 16, 64);
        const int a2 = __shfl(bidx[2], j * 16, 64), a3 = __shfl(bidx[3], j * 16, 64);
        const float b0 = __shfl(best[0], j * 16, 64), b1 = __shfl(best[1], j * 16, 64);
        const float b2 = __shfl(best[2], j * 16, 64), b3 = __shfl(best[3], j * 16, 64);
        const int my_a = q == 0 ? a0 : (q == 1 ? a1 : (q == 2 ? a2 : a3));
        const float my_b = q == 0 ? b0 : (q == 1 ? b1 : (q == 2 ? b2 : b3));
        const int rt = tr * 16 + 4 * j + q;          // row within the 64-row slice
        const int64_t rb = r0 + rt;
        const bool rok = rt < nrows;
        const float ww = rok ? (w ? w[rb] : 1.f) : 0.f;
        const float* xr = xs + rt * Pp;
        float xq = 0.f;
#pragma unroll
        for (int u = 0; u < PT; ++u) {
          const int dd = u * 16 + c16;
          const float xv = dd < P ? xr[dd] : 0.f;
          xq = fmaf(xv, xv, xq);
          const float bv = dd < P ? ww * xv : (dd == P ? ww : 0.f);
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            const float av = (my_a == t * 16 + c16) ? 1.f : 0.f;
            acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t][u], 0, 0, 0);
          }
        }
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) xq += __shfl_xor(xq, m, 64);
        if (rok && c16 == 0) {
          assign[rb] = my_a;
          mind[rb] = fmaxf(xq + my_b, 0.f);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();   // the slice is rewritten by the next iteration's loads
  }
  // ---- per-wave slab: [KT*16 centers][PT*16 dims], D layout row = 4q + r (center), col = c16 (dim)
  float* out = slabs + wave_g * (int64_t)(KT * 16) * (PT * 16);
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int u = 0; u < PT; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(t * 16 + 4 * q + r) * (PT * 16) + u * 16 + c16] = acc[t][u][r];
}

template <int KT, int PS, int PT>
int launch(const float* X, long long N, int P, const float* C, int K, const float* w, int* assign, float* mind,
           float* slabs, int grid, hipStream_t s) {
  const size_t lds = (size_t)4 * KM_ROWS * (P + 1) * sizeof(float);
  hipLaunchKernelGGL((k_lloyd_mfma<KT, PS, PT>), dim3(grid), dim3(256), lds, s, X, (int64_t)N, P, C, K, w, assign,
                     mind, slabs);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// Shape class the MFMA Lloyd kernel supports (0 = not supported: caller falls back).
// Returns KT*100 + PS*10... encoded as (KT, PS, PT) via out[3].
int h2o_kmeans_mfma_shape(int K, int P, int* out) {
  if (K < 1 || P < 1 || K > 64 || P > 64) return 0;
  const int KT = K <= 16 ? 1 : (K <= 32 ? 2 : 4);
  const int PS = P <= 16 ? 4 : (P <= 32 ? 8 : 16);
  const int PT = (P + 1 + 15) / 16;
  out[0] = KT; out[1] = PS; out[2] = PT;
  return 1;
}

// slabs: [grid*4][KT*16][PT*16] fp32 (caller allocates with the shape from h2o_kmeans_mfma_shape)
int h2o_kmeans_mfma(const float* X, long long N, int P, const float* C, int K, const float* w, int* assign,
                    float* mind, float* slabs, int grid, hipStream_t s) {
  int sh[3];
  if (!h2o_kmeans_mfma_shape(K, P, sh) || N <= 0 || grid <= 0) return (int)hipErrorInvalidValue;
  const int KT = sh[0], PS = sh[1], PT = sh[2];
#define L(kt, ps, pt) if (KT == kt && PS == ps && PT == pt) return launch<kt, ps, pt>(X, N, P, C, K, w, assign, mind, slabs, grid, s)
  L(1, 4, 1); L(1, 4, 2); L(1, 8, 2); L(1, 8, 3); L(1, 16, 3); L(1, 16, 4); L(1, 16, 5);
  L(2, 4, 1); L(2, 4, 2); L(2, 8, 2); L(2, 8, 3); L(2, 16, 3); L(2, 16, 4); L(2, 16, 5);
  L(4, 4, 1); L(4, 4, 2); L(4, 8, 2); L(4, 8, 3); L(4, 16, 3); L(4, 16, 4); L(4, 16, 5);
#undef L
  return (int)hipErrorInvalidValue;
}

}  // extern "C"
