// Weighted Gram matrix G = Zᵀ·diag(w)·Z on f32-input MFMA (GLM IRLSM GramTask, PCA GramSVD,
// covariance for Aggregator/KMeans init), optionally with one extra column u appended to Z (the
// augmented Gram [Z u]ᵀ W [Z u] carries the IRLS right-hand side Zᵀ W u in its last column, so one pass
// over Z replaces the Gram + Xᵀv pair of GLMIterationTask).
//
// Reference: h2o-algos/src/main/java/hex/gram/Gram.java (GramTask.map: per-row rank-1 updates in
// fp64, reduced over chunks) and hex/glm/GLMTask.java (GLMIterationTask). MI355X design:
//  * one wave per (64x64 tile pair ti <= tj, row slice): no LDS, no barriers. v_mfma_f32_32x32x2_f32
//    takes A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31], i.e. lane l loads column (l&31) of row
//    2kk + (l>>5): one coalesced 128-byte read per half wave per 32 columns, straight into the MFMA
//    operand registers. A diagonal tile is 3 MFMAs per row pair (the lower-left 32x32 block is the
//    transpose of the upper-right one), an off-diagonal tile 4.
//  * UNRG row pairs are loaded before their MFMAs (UNRG x 2-4 loads in flight per lane); many waves
//    per SIMD (no LDS limit on occupancy) hide the HBM latency that the LDS-staged version (4 waves
//    per 64 KiB of LDS, 2 blocks per CU) exposed: 10M x 51 took ~3 ms, 6x its MFMA bound.
//  * every wave writes its own fp32 slab; the slabs are summed in fp64 on the stream (deterministic,
//    no float atomics; fp32 runs stay short: rows per slice ~ N / S).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TILE = 64;
#ifndef GRAM_UNRG
#define GRAM_UNRG 8
#endif
constexpr int UNRG = GRAM_UNRG;      // row pairs in flight per lane

__device__ __forceinline__ float zload(const float* __restrict__ Z, int64_t ldz, const float* __restrict__ u,
                                       int64_t r, bool ok, int c, int P) {
  if (!ok) return 0.f;
  if (c < P) return Z[r * ldz + c];
  return (u != nullptr && c == P) ? u[r] : 0.f;
}

__global__ __launch_bounds__(64) void k_gram(const float* __restrict__ Z, int64_t ldz, const float* __restrict__ w,
                                             const float* __restrict__ u, int64_t N, int P, int nT,
                                             int64_t rows_per_split, float* __restrict__ slabs, int Ppad) {
  int pair = blockIdx.x;
  int ti = 0;
  while (pair >= nT - ti) { pair -= nT - ti; ++ti; }
  const int tj = ti + pair;
  const int i0 = ti * TILE, j0 = tj * TILE;
  const bool diag = ti == tj;
  const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r_end = min(N, r_begin + rows_per_split);
  const int lane = threadIdx.x;
  const int c = lane & 31, kh = lane >> 5;
  f32x16 a00, a01, a10, a11;
#pragma unroll
  for (int k = 0; k < 16; ++k) { a00[k] = 0.f; a01[k] = 0.f; a10[k] = 0.f; a11[k] = 0.f; }
  for (int64_t base = r_begin; base < r_end; base += 2 * UNRG) {
    float x0[UNRG], x1[UNRG], y0[UNRG], y1[UNRG], ww[UNRG];
#pragma unroll
    for (int q = 0; q < UNRG; ++q) {
      const int64_t r = base + 2 * q + kh;
      const bool ok = r < r_end;
      const int64_t rc = ok ? r : r_begin;
      ww[q] = ok ? (w ? w[rc] : 1.f) : 0.f;
      x0[q] = zload(Z, ldz, u, rc, ok, i0 + c, P);
      x1[q] = zload(Z, ldz, u, rc, ok, i0 + 32 + c, P);
      if (!diag) {
        y0[q] = zload(Z, ldz, u, rc, ok, j0 + c, P);
        y1[q] = zload(Z, ldz, u, rc, ok, j0 + 32 + c, P);
      }
    }
#pragma unroll
    for (int q = 0; q < UNRG; ++q) {
      const float b0 = diag ? x0[q] : y0[q], b1 = diag ? x1[q] : y1[q];
      const float wa0 = ww[q] * x0[q], wa1 = ww[q] * x1[q];
      a00 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa0, b0, a00, 0, 0, 0);
      a01 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa0, b1, a01, 0, 0, 0);
      a11 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa1, b1, a11, 0, 0, 0);
      if (!diag) a10 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa1, b0, a10, 0, 0, 0);
    }
  }
  // epilogue: D[row = (k&3) + 8*(k>>2) + 4*(lane>>5)][col = lane&31] per 32x32 quadrant
  float* out = slabs + (size_t)blockIdx.y * Ppad * Ppad;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rr = (k & 3) + 8 * (k >> 2) + 4 * kh;
    out[(size_t)(i0 + rr) * Ppad + j0 + c] = a00[k];
    out[(size_t)(i0 + rr) * Ppad + j0 + 32 + c] = a01[k];
    out[(size_t)(i0 + 32 + rr) * Ppad + j0 + 32 + c] = a11[k];
    if (diag) out[(size_t)(i0 + 32 + c) * Ppad + j0 + rr] = a01[k];     // lower-left = upper-rightᵀ
    else out[(size_t)(i0 + 32 + rr) * Ppad + j0 + c] = a10[k];
  }
}

// Xᵀ·v for a row-major [N, P] matrix and one or more right-hand sides (GLM XᵀWz): v is [N, R]
// row-major, out slabs [S, P, R] (fp32 per slice, summed in fp64 by the caller).
__global__ __launch_bounds__(256) void k_xtv(const float* __restrict__ Z, int64_t ldz, const float* __restrict__ v,
                                             int R, int64_t N, int P, int64_t rows_per_split,
                                             float* __restrict__ slabs) {
  const int p = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rq = threadIdx.x >> 6;  // 4 row phases
  const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
  int64_t r_end = r_begin + rows_per_split;
  if (r_end > N) r_end = N;
  __shared__ float red[4][64][8];
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (p < P) {
    int64_t r = r_begin + rq;
    // 4 rows per step, their loads issued before the accumulation (one load in flight per lane before)
    for (; r + 12 < r_end; r += 16) {
      float z[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) z[u] = Z[(r + 4 * u) * ldz + p];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        for (int q = 0; q < R && q < 8; ++q) acc[q] += z[u] * v[(r + 4 * u) * R + q];
    }
    for (; r < r_end; r += 4) {
      const float z = Z[r * ldz + p];
      for (int q = 0; q < R && q < 8; ++q) acc[q] += z * v[r * R + q];
    }
  }
  for (int q = 0; q < 8; ++q) red[rq][threadIdx.x & 63][q] = acc[q];
  __syncthreads();
  if (rq == 0 && p < P) {
    for (int q = 0; q < R && q < 8; ++q) {
      const float s = red[0][threadIdx.x & 63][q] + red[1][threadIdx.x & 63][q] + red[2][threadIdx.x & 63][q] +
                      red[3][threadIdx.x & 63][q];
      slabs[((size_t)blockIdx.y * P + p) * R + q] = s;
    }
  }
}

}  // namespace

// eta = Z @ B (+ off): Z [N, P] fp32 row-major, B [P, R] fp64 (R <= 8), eta [N, R] fp64 — the GLM linear
// predictor without an fp64 copy of Z (GLMIterationTask's per-row x·beta). A block owns TR consecutive rows,
// i.e. one contiguous TR*P-float span of Z: it is pulled into LDS with 16-byte loads (every lane of every
// load instruction reading consecutive bytes, all issued before the first use), then each thread
// accumulates one row's dot products in fp64 from LDS (row stride P words: odd P is bank-conflict free)
// and writes eta once. MEASURED: column-tiled / half-wave-per-row variants read the 204-byte rows of a
// 10M x 51 Z at 1.1-1.45 TB/s (several partial cache lines per load instruction).
#define ZB_THREADS 256
// IRLS epilogue of the z.beta pass (R == 1; GLMIterationTask's per-row working weight and response): with wi set,
// the row's mu = linkinv(eta), g'(mu) and V(mu) give wi = w / max(V g'^2, 1e-30) and zi = eta - off + (y - mu) g'
// as fp32 (the Gram pass's inputs) instead of eta — the ~12 fp64 elementwise launches of the torch chain become
// this epilogue. fam: 0 gaussian, 1 binomial / quasibinomial / fractionalbinomial, 2 poisson, 3 gamma;
// link: 0 identity, 1 logit, 2 log, 3 inverse (the clamps of glm.Family).
struct IrlsOut {
  int fam, link;
  const double* y;
  const double* w;
  float* wi;
  float* zi;
};
__device__ __forceinline__ void irls_eval(int fam, int link, double e, double o, double y, double w, float& wi,
                                          float& zi) {
  double mu, gp;
  switch (link) {
    case 1: {
      mu = 1.0 / (1.0 + exp(-e));
      const double m = fmin(fmax(mu, 1e-10), 1.0 - 1e-10);
      gp = 1.0 / (m * (1.0 - m));
      break;
    }
    case 2: mu = exp(fmin(e, 700.0)); gp = 1.0 / fmax(mu, 1e-10); break;
    case 3: {
      const double s = e + 1e-300;
      const double ee = fabs(e) < 1e-10 ? 1e-10 * (double)((s > 0.0) - (s < 0.0)) : e;
      mu = 1.0 / ee;
      gp = -1.0 / fmax(mu * mu, 1e-20);
      break;
    }
    default: mu = e; gp = 1.0;
  }
  double var;
  switch (fam) {
    case 1: { const double m = fmin(fmax(mu, 1e-10), 1.0 - 1e-10); var = m * (1.0 - m); break; }
    case 2: var = fmax(mu, 1e-10); break;
    case 3: var = fmax(mu * mu, 1e-20); break;
    default: var = 1.0;
  }
  wi = (float)(w / fmax(var * gp * gp, 1e-30));
  zi = (float)(e - o + (y - mu) * gp);
}
__device__ __forceinline__ void irls_row(const IrlsOut& io, int64_t row, double e, double o) {
  irls_eval(io.fam, io.link, e, o, io.y[row], io.w[row], io.wi[row], io.zi[row]);
}

// The IRLS pass fused into the Gram pass, for designs whose augmented rows fit one 64-column tile
// (P + 1 <= 64: a wave already holds whole rows of Z for k_gram's diagonal tile). Per batch of 16 rows each
// lane has the fp64 partial x.beta of its 2 columns for 8 row slots; a butterfly reduce-scatter over the
// 32 lanes of a row half (xor 16 / 8 / 4 keep half the slots each, xor 2 / 1 finish) leaves lane l with
// the full eta of slot (l >> 2) & 7 — 9 fp64 shuffles instead of 40, and one exp per lane instead of 8.
// That lane evaluates irls_eval for its row; wi and zi go back to the slot's 32 lanes by 16 fp32
// shuffles, zi lands in column P (the u column), and the MFMAs of k_gram's diagonal tile follow. The
// separate k_zbeta IRLS pass (a second full read of Z plus wi / zi round trips) disappears.
__global__ __launch_bounds__(64) void k_gram_irls(const float* __restrict__ Z, int64_t ldz,
                                                  const double* __restrict__ beta, const double* __restrict__ off,
                                                  IrlsOut io, int64_t N, int P, int64_t rows_per_split,
                                                  float* __restrict__ slabs) {
  const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r_end = min(N, r_begin + rows_per_split);
  const int lane = threadIdx.x;
  const int c = lane & 31, kh = lane >> 5;
  const int s_me = (lane >> 2) & 7;
  const int b4 = (lane >> 4) & 1, b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1;
  const double be0 = c < P ? beta[c] : 0.0, be1 = 32 + c < P ? beta[32 + c] : 0.0;
  f32x16 a00, a01, a11;
#pragma unroll
  for (int k = 0; k < 16; ++k) { a00[k] = 0.f; a01[k] = 0.f; a11[k] = 0.f; }
  for (int64_t base = r_begin; base < r_end; base += 16) {
    float x0[8], x1[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int64_t r = base + 2 * q + kh;
      const bool ok = r < r_end;
      x0[q] = ok && c < P ? Z[r * ldz + c] : 0.f;
      x1[q] = ok && 32 + c < P ? Z[r * ldz + 32 + c] : 0.f;
    }
    const int64_t rm = base + 2 * s_me + kh;
    const bool okm = rm < r_end;
    const int64_t rmc = okm ? rm : r_begin;
    const double ym = io.y[rmc], wm = io.w[rmc], om = off ? off[rmc] : 0.0;
    double p[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) p[q] = (double)x0[q] * be0 + (double)x1[q] * be1;
    double p4[4], p2[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) p4[i] = (b4 ? p[4 + i] : p[i]) + __shfl_xor(b4 ? p[i] : p[4 + i], 16, 64);
#pragma unroll
    for (int i = 0; i < 2; ++i) p2[i] = (b3 ? p4[2 + i] : p4[i]) + __shfl_xor(b3 ? p4[i] : p4[2 + i], 8, 64);
    double e = (b2 ? p2[1] : p2[0]) + __shfl_xor(b2 ? p2[0] : p2[1], 4, 64);
    e += __shfl_xor(e, 2, 64);
    e += __shfl_xor(e, 1, 64);
    float wim = 0.f, zim = 0.f;
    if (okm) irls_eval(io.fam, io.link, e + om, om, ym, wm, wim, zim);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int src = (kh << 5) | (q << 2);
      const float wq = __shfl(wim, src, 64), zq = __shfl(zim, src, 64);
      if (c == P) x0[q] = zq;
      if (32 + c == P) x1[q] = zq;
      const float wa0 = wq * x0[q], wa1 = wq * x1[q];
      a00 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa0, x0[q], a00, 0, 0, 0);
      a01 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa0, x1[q], a01, 0, 0, 0);
      a11 = __builtin_amdgcn_mfma_f32_32x32x2f32(wa1, x1[q], a11, 0, 0, 0);
    }
  }
  float* out = slabs + (size_t)blockIdx.y * TILE * TILE;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rr = (k & 3) + 8 * (k >> 2) + 4 * kh;
    out[(size_t)rr * TILE + c] = a00[k];
    out[(size_t)rr * TILE + 32 + c] = a01[k];
    out[(size_t)(32 + rr) * TILE + 32 + c] = a11[k];
    out[(size_t)(32 + c) * TILE + rr] = a01[k];
  }
}
#ifndef ZB_LDS_FLOATS
#define ZB_LDS_FLOATS 12288    // 48 KiB of Z per block
#endif
__global__ __launch_bounds__(ZB_THREADS) void k_zbeta(const float* __restrict__ Z, int64_t ldz,
                                                      const double* __restrict__ B, int R, int64_t N, int P, int TR,
                                                      const double* __restrict__ off, double* __restrict__ eta,
                                                      IrlsOut io) {
  __shared__ __attribute__((aligned(16))) float tile[ZB_LDS_FLOATS];
  __shared__ double bt[1024];                            // B when P * R <= 1024, else read from global
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * TR;
  if (r0 >= N) return;
  const int nr = (int)min((int64_t)TR, N - r0);
  const bool bl = P * R <= 1024;
  if (bl)
    for (int i = t; i < P * R; i += ZB_THREADS) bt[i] = B[i];
  const int64_t n = (int64_t)nr * P;
  const float* src = Z + r0 * ldz;
  if (ldz == P && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
    const int n4 = (int)(n >> 2);
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(tile);
    // every 16-byte load of the span is issued before the first LDS store (12 in flight per lane; a
    // load -> store loop waited on each one)
    constexpr int ZU = ZB_LDS_FLOATS / 4 / ZB_THREADS;
    float4 v[ZU];
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      const int i = t + u * ZB_THREADS;
      v[u] = i < n4 ? s4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      const int i = t + u * ZB_THREADS;
      if (i < n4) d4[i] = v[u];
    }
    for (int i = 4 * n4 + t; i < n; i += ZB_THREADS) tile[i] = src[i];
  } else {
    for (int i = t; i < n; i += ZB_THREADS) {
      const int rr = i / P, cc = i - rr * P;
      tile[i] = src[(int64_t)rr * ldz + cc];
    }
  }
  __syncthreads();
  if (t >= nr) return;
  const float* zr = tile + t * P;
  double acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.0;
  if (R == 1) {
    for (int c = 0; c < P; ++c) acc[0] += (double)zr[c] * (bl ? bt[c] : B[c]);
  } else {
    for (int c = 0; c < P; ++c) {
      const double z = (double)zr[c];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < R) acc[k] += z * (bl ? bt[c * R + k] : B[(int64_t)c * R + k]);
    }
  }
  const int64_t row = r0 + t;
  const double o = off ? off[row] : 0.0;
  if (io.wi) {
    irls_row(io, row, acc[0] + o, o);
    return;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < R) eta[row * R + k] = acc[k] + o;
}

// very wide designs (P > 12288, e.g. one-hot of huge factors): one wave per row, lanes stride the columns,
// fp64 wave reduction
__global__ __launch_bounds__(256) void k_zbeta_wide(const float* __restrict__ Z, int64_t ldz,
                                                   const double* __restrict__ B, int R, int64_t N, int P,
                                                   const double* __restrict__ off, double* __restrict__ eta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= N) return;
  const float* zr = Z + row * ldz;
  for (int k = 0; k < R; ++k) {
    double a = 0.0;
    for (int c = lane; c < P; c += 64) a += (double)zr[c] * B[(int64_t)c * R + k];
    for (int sh = 32; sh >= 1; sh >>= 1) a += __shfl_xor(a, sh, 64);
    if (lane == 0) eta[row * R + k] = a + (off ? off[row] : 0.0);
  }
}

extern "C" {

// slabs: fp32 [S, Ppad, Ppad], Ppad = ceil(P/64)*64 (caller zero-fills nothing: every upper tile is written)
// u (nullable): the extra column P of the augmented matrix (Ppad > P required then)
int h2o_gram(const float* Z, long long ldz, const float* w, const float* u, long long N, int P, int S, float* slabs,
             int Ppad, hipStream_t stream) {
  if (P <= 0 || N < 0 || S <= 0 || Ppad % TILE != 0 || Ppad < P + (u ? 1 : 0)) return (int)hipErrorInvalidValue;
  const int nT = Ppad / TILE;
  const long long rps = ((N + S - 1) / S + 1) / 2 * 2;
  dim3 grid(nT * (nT + 1) / 2, S);
  hipLaunchKernelGGL(k_gram, grid, dim3(64), 0, stream, Z, (int64_t)ldz, w, u, (int64_t)N, P, nT, (int64_t)rps,
                     slabs, Ppad);
  return (int)hipGetLastError();
}

int h2o_xtv(const float* Z, long long ldz, const float* v, int R, long long N, int P, int S, float* slabs,
            hipStream_t stream) {
  if (R < 1 || R > 8 || P <= 0 || S <= 0) return (int)hipErrorInvalidValue;
  const long long rps = (N + S - 1) / S;
  dim3 grid((P + 63) / 64, S);
  hipLaunchKernelGGL(k_xtv, grid, dim3(256), 0, stream, Z, (int64_t)ldz, v, R, (int64_t)N, P, (int64_t)rps, slabs);
  return (int)hipGetLastError();
}

int h2o_zbeta(const float* Z, long long ldz, const double* B, int R, long long N, int P, const double* off,
              double* eta, hipStream_t stream) {
  if (R < 1 || R > 8 || N <= 0) return N <= 0 ? 0 : (int)hipErrorInvalidValue;
  if (P <= 0 || ldz < P) return (int)hipErrorInvalidValue;
  // rows per block: the LDS span (<= 48 KiB), at most one per thread, a multiple of 4 (16-byte spans)
  int TR = ZB_LDS_FLOATS / P;
  if (TR > ZB_THREADS) TR = ZB_THREADS;
  TR &= ~3;
  if (TR < 1) TR = 1;
  if ((long long)TR * P > ZB_LDS_FLOATS) {
    hipLaunchKernelGGL(k_zbeta_wide, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, stream, Z, (int64_t)ldz, B, R,
                       (int64_t)N, P, off, eta);
    return (int)hipGetLastError();
  }
  const long long grid = (N + TR - 1) / TR;
  hipLaunchKernelGGL(k_zbeta, dim3((unsigned)grid), dim3(ZB_THREADS), 0, stream, Z, (int64_t)ldz, B, R, (int64_t)N, P,
                     TR, off, eta, IrlsOut{0, 0, nullptr, nullptr, nullptr, nullptr});
  return (int)hipGetLastError();
}

// The IRLS pass (see IrlsOut): wi / zi fp32 [N] from Z [N, P] fp32, beta fp64 [P], off / y / w fp64 [N]. Designs
// whose rows do not fit the LDS span (P > ZB_LDS_FLOATS / 4) are refused (the caller keeps the torch chain).
int h2o_irls_wz(const float* Z, long long ldz, const double* B, long long N, int P, const double* off,
                const double* y, const double* w, int fam, int link, float* wi, float* zi, hipStream_t stream) {
  if (N <= 0) return 0;
  if (P <= 0 || ldz < P || fam < 0 || fam > 3 || link < 0 || link > 3) return (int)hipErrorInvalidValue;
  int TR = ZB_LDS_FLOATS / P;
  if (TR > ZB_THREADS) TR = ZB_THREADS;
  TR &= ~3;
  if (TR < 4) return (int)hipErrorInvalidValue;
  const long long grid = (N + TR - 1) / TR;
  hipLaunchKernelGGL(k_zbeta, dim3((unsigned)grid), dim3(ZB_THREADS), 0, stream, Z, (int64_t)ldz, B, 1, (int64_t)N, P,
                     TR, off, (double*)nullptr, IrlsOut{fam, link, y, w, wi, zi});
  return (int)hipGetLastError();
}

// Fused IRLS + augmented Gram (k_gram_irls): slabs fp32 [S, 64, 64] of [Z zi]ᵀ diag(wi) [Z zi] with wi / zi
// evaluated in the pass (beta fp64 [P], off / y / w fp64 [N]); P + 1 <= 64 only.
int h2o_gram_irls(const float* Z, long long ldz, const double* B, long long N, int P, const double* off,
                  const double* y, const double* w, int fam, int link, int S, float* slabs, hipStream_t stream) {
  if (N <= 0) return 0;
  if (P <= 0 || P + 1 > TILE || ldz < P || S <= 0 || fam < 0 || fam > 3 || link < 0 || link > 3)
    return (int)hipErrorInvalidValue;
  const long long rps = ((N + S - 1) / S + 1) / 2 * 2;
  hipLaunchKernelGGL(k_gram_irls, dim3(1, S), dim3(64), 0, stream, Z, (int64_t)ldz, B, off,
                     IrlsOut{fam, link, y, w, nullptr, nullptr}, (int64_t)N, P, (int64_t)rps, slabs);
  return (int)hipGetLastError();
}

}  // extern "C"
