// Weighted Gram matrix G = Zᵀ·diag(w)·Z on f32-input MFMA (GLM IRLSM GramTask, PCA GramSVD,
// covariance for Aggregator/KMeans init).
//
// Reference: h2o-algos/src/main/java/hex/gram/Gram.java (GramTask.map: per-row rank-1 updates in
// fp64, reduced over chunks) and hex/glm/GLMTask.java (GLMIterationTask). MI355X design:
//  * 256-thread workgroup (4 waves, 2x2) owns one 64x64 output tile (ti <= tj: only the upper
//    triangle of tiles is computed, the host mirrors it) and one contiguous slice of rows.
//  * Rows stream through LDS in 64-row stages (double-buffered via a register prefetch of the
//    next stage): As[r][i] = w[r]·Z[r][i0+i], Bs[r][j] = Z[r][j0+j].
//  * Each wave issues v_mfma_f32_32x32x2_f32 (exact f32 products, k-ordered fma chain) over the
//    stage: lane l feeds A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31], i.e. two rows per MFMA.
//  * Every row slice writes its own fp32 slab; the slabs are summed in fp64 on the host stream
//    (deterministic, no float atomics; keeps fp32 accumulation runs short: rows/slice ≈ N/S).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TILE = 64;
constexpr int BK = 64;       // rows per LDS stage
constexpr int THREADS = 256;

__global__ __launch_bounds__(THREADS) void k_gram(const float* __restrict__ Z, int64_t ldz, const float* __restrict__ w,
                                                  int64_t N, int P, int nT, int64_t rows_per_split,
                                                  float* __restrict__ slabs, int Ppad) {
  // tile pair from blockIdx.x over the upper triangle
  int pair = blockIdx.x;
  int ti = 0;
  while (pair >= nT - ti) { pair -= nT - ti; ++ti; }
  const int tj = ti + pair;
  const int i0 = ti * TILE, j0 = tj * TILE;
  const int split = blockIdx.y;
  const int64_t r_begin = (int64_t)split * rows_per_split;
  int64_t r_end = r_begin + rows_per_split;
  if (r_end > N) r_end = N;

  __shared__ float As[2][BK][TILE];
  __shared__ float Bs[2][BK][TILE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wy = wave >> 1, wx = wave & 1;
  const int col = tid & 63;        // load column within the tile
  const int rsub = tid >> 6;       // 0..3: row phase for loads
  const bool diag = (ti == tj);

  f32x16 acc;
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;

  float ra[BK / 4], rb[BK / 4];
  auto load_stage = [&](int64_t r0) {
#pragma unroll
    for (int m = 0; m < BK / 4; ++m) {
      const int64_t r = r0 + rsub + 4 * m;
      float a = 0.f, b = 0.f;
      if (r < r_end) {
        const float ww = w ? w[r] : 1.f;
        const float* zr = Z + r * ldz;
        const float zi = (i0 + col < P) ? zr[i0 + col] : 0.f;
        a = ww * zi;
        b = diag ? zi : ((j0 + col < P) ? zr[j0 + col] : 0.f);
      }
      ra[m] = a; rb[m] = b;
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int m = 0; m < BK / 4; ++m) {
      As[buf][rsub + 4 * m][col] = ra[m];
      Bs[buf][rsub + 4 * m][col] = rb[m];
    }
  };

  int buf = 0;
  if (r_begin < r_end) {
    load_stage(r_begin);
    store_stage(0);
  }
  __syncthreads();
  for (int64_t r0 = r_begin; r0 < r_end; r0 += BK) {
    const bool more = r0 + BK < r_end;
    if (more) load_stage(r0 + BK);  // global loads in flight while the MFMAs run
    const int ai = 32 * wy + (lane & 31);
    const int bj = 32 * wx + (lane & 31);
    const int kh = lane >> 5;
#pragma unroll 8
    for (int kk = 0; kk < BK / 2; ++kk) {
      const float a = As[buf][2 * kk + kh][ai];
      const float b = Bs[buf][2 * kk + kh][bj];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    if (more) store_stage(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // epilogue: C/D map col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  float* out = slabs + (size_t)split * Ppad * Ppad;
  const int oc = j0 + 32 * wx + (lane & 31);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int orow = i0 + 32 * wy + (k & 3) + 8 * (k >> 2) + 4 * (lane >> 5);
    out[(size_t)orow * Ppad + oc] = acc[k];
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
    for (int64_t r = r_begin + rq; r < r_end; r += 4) {
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
// predictor without an fp64 copy of Z (GLMIterationTask's per-row x·beta). 256 rows per block; 32-column
// tiles staged through LDS with coalesced loads (row stride padded to 33 floats: conflict-free column reads),
// one row per thread, fp64 accumulation.
#define ZB_ROWS 256
#define ZB_COLS 32
__global__ __launch_bounds__(ZB_ROWS) void k_zbeta(const float* __restrict__ Z, int64_t ldz, const double* __restrict__ B,
                                                   int R, int64_t N, int P, const double* __restrict__ off,
                                                   double* __restrict__ eta) {
  __shared__ float tile[ZB_ROWS * (ZB_COLS + 1)];
  __shared__ double bt[ZB_COLS * 8];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * ZB_ROWS;
  double acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.0;
  for (int c0 = 0; c0 < P; c0 += ZB_COLS) {
    const int nc = min(ZB_COLS, P - c0);
    for (int i = t; i < ZB_ROWS * ZB_COLS; i += ZB_ROWS) {
      const int rr = i / ZB_COLS, cc = i - rr * ZB_COLS;
      const int64_t row = r0 + rr;
      tile[rr * (ZB_COLS + 1) + cc] = (row < N && cc < nc) ? Z[row * ldz + c0 + cc] : 0.f;
    }
    for (int i = t; i < ZB_COLS * R; i += ZB_ROWS) {
      const int cc = i / R, k = i - cc * R;
      bt[cc * 8 + k] = cc < nc ? B[(int64_t)(c0 + cc) * R + k] : 0.0;
    }
    __syncthreads();
    for (int cc = 0; cc < nc; ++cc) {
      const double z = (double)tile[t * (ZB_COLS + 1) + cc];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < R) acc[k] += z * bt[cc * 8 + k];
    }
    __syncthreads();
  }
  const int64_t row = r0 + t;
  if (row < N) {
    const double o = off ? off[row] : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < R) eta[row * R + k] = acc[k] + o;
  }
}

extern "C" {

// slabs: fp32 [S, Ppad, Ppad], Ppad = ceil(P/64)*64 (caller zero-fills nothing: every upper tile is written)
int h2o_gram(const float* Z, long long ldz, const float* w, long long N, int P, int S, float* slabs, int Ppad,
             hipStream_t stream) {
  if (P <= 0 || N < 0 || S <= 0 || Ppad % TILE != 0 || Ppad < P) return (int)hipErrorInvalidValue;
  const int nT = Ppad / TILE;
  const long long rps = ((N + S - 1) / S + BK - 1) / BK * BK;
  dim3 grid(nT * (nT + 1) / 2, S);
  hipLaunchKernelGGL(k_gram, grid, dim3(THREADS), 0, stream, Z, (int64_t)ldz, w, (int64_t)N, P, nT, (int64_t)rps,
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
  const long long grid = (N + ZB_ROWS - 1) / ZB_ROWS;
  hipLaunchKernelGGL(k_zbeta, dim3((unsigned)grid), dim3(ZB_ROWS), 0, stream, Z, (int64_t)ldz, B, R, (int64_t)N, P, off,
                     eta);
  return (int)hipGetLastError();
}

}  // extern "C"
