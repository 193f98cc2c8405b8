// DeepLearning layer epilogues (reference: h2o-algos/src/main/java/hex/deeplearning/Neurons.java —
// fprop: bias add + activation (+ input/hidden dropout); bprop: dE/dnet = dE/dout * act'(net)).
//
// The GEMMs themselves go to hipBLASLt through torch; these kernels fuse everything elementwise
// around them so each layer touches its activation tensor once per direction:
//   fwd: out = act(x + b) * mask/keep   (mask from a counter-based hash of (seed, element): no RNG
//        state, reproducible, regenerated in bwd instead of stored)
//   bwd: gx = gout * mask/keep * act'(.)  and the bias gradient column sums (LDS tree + one fp32
//        atomic per column per workgroup).
// Activations: 0 linear, 1 Rectifier (ReLU), 2 Tanh, 3 ExpRectifier (ELU).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return (uint32_t)x;
}

__device__ __forceinline__ float act_f(int a, float v) {
  switch (a) {
    case 1: return v > 0.f ? v : 0.f;
    case 2: return tanhf(v);
    case 3: return v > 0.f ? v : expm1f(v);
    default: return v;
  }
}

// derivative expressed through the activation OUTPUT y (what bwd keeps)
__device__ __forceinline__ float dact_from_y(int a, float y) {
  switch (a) {
    case 1: return y > 0.f ? 1.f : 0.f;
    case 2: return 1.f - y * y;
    case 3: return y > 0.f ? 1.f : y + 1.f;
    default: return 1.f;
  }
}

// T = float or bf16 activations (bf16: GEMM outputs feed the epilogue and the next GEMM directly, no
// fp32 round trip); bias, math and the bias gradient stay fp32.
__device__ __forceinline__ float ld(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float ld(const __hip_bfloat16* p, int64_t i) { return __bfloat162float(p[i]); }
__device__ __forceinline__ void st(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st(__hip_bfloat16* p, int64_t i, float v) { p[i] = __float2bfloat16(v); }

template <typename T>
__global__ __launch_bounds__(256) void k_bias_act_fwd(const T* __restrict__ x, const float* __restrict__ b,
                                                      T* __restrict__ y, int64_t rows, int cols, int act,
                                                      float drop, uint64_t seed, const uint64_t* __restrict__ seed_dev) {
  if (seed_dev) seed ^= *seed_dev * 0x9E3779B97F4A7C15ULL;   // per-step offset read on device (graph replays)
  const int64_t n = rows * (int64_t)cols;
  const float keep = 1.f - drop;
  const uint32_t thr = (uint32_t)(drop * 4294967296.0);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % cols);
    float v = act_f(act, ld(x, i) + (b ? b[c] : 0.f));
    if (drop > 0.f) v = (hash32(seed ^ (uint64_t)i * 0x9E3779B97F4A7C15ULL) < thr) ? 0.f : v / keep;
    st(y, i, v);
  }
}

// gx[i] = gy[i] * mask * act'(y); db[c] += sum_r gx[r, c]
template <typename T>
__global__ __launch_bounds__(256) void k_bias_act_bwd(const T* __restrict__ gy, const T* __restrict__ y,
                                                      T* __restrict__ gx, float* __restrict__ db, int64_t rows,
                                                      int cols, int act, float drop, uint64_t seed, int rows_per_block,
                                                      const uint64_t* __restrict__ seed_dev) {
  if (seed_dev) seed ^= *seed_dev * 0x9E3779B97F4A7C15ULL;
  // block handles a [rows_per_block x 64] column stripe: thread (ty, tx) with tx = column lane
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int64_t rbeg = (int64_t)blockIdx.y * rows_per_block;
  int64_t rend = rbeg + rows_per_block;
  if (rend > rows) rend = rows;
  const float keep = 1.f - drop;
  const uint32_t thr = (uint32_t)(drop * 4294967296.0);
  float acc = 0.f;
  if (c < cols) {
    for (int64_t r = rbeg + ty; r < rend; r += 4) {
      const int64_t i = r * cols + c;
      float yy = ld(y, i);
      float g = ld(gy, i);
      if (drop > 0.f) {
        const bool dropped = hash32(seed ^ (uint64_t)i * 0x9E3779B97F4A7C15ULL) < thr;
        g = dropped ? 0.f : g / keep;
        yy = dropped ? 0.f : yy * keep;  // stored y was scaled by 1/keep
      }
      const float v = g * dact_from_y(act, yy);
      st(gx, i, v);
      acc += v;
    }
  }
  __shared__ float red[4][64];
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && c < cols && db) atomicAdd(&db[c], red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx]);
}

// ADADELTA (Neurons.java: rho, epsilon) fused over the FLAT parameter buffer of the whole network:
// one launch updates every weight and bias (the per-tensor torch version is ~36 launches per step).
// L1/L2 apply to weights only: elements [0, n_decay) are the weight matrices, the rest biases.
// Transposed weight copy the fused DL step's backward pass reads (ops/dl.py): layer l's [n_out][n_in] block at
// w_off[l] is also written as [n_in][n_out] (bf16 or fp32), so no separate transpose launch follows the update.
struct WTMap {
  void* wt;
  int f32, L;
  long long w_off[7];
  int n_in[6], n_out[6];
  // the weight gradients straight from the fused step's split partials (dl_kernels.hip k_dl_wgrad): element
  // (r, c) of layer l sums partial[tile(l, r / 64, c / 64)][s][(r % 64) * 64 + c % 64] over the S splits, times
  // the batch's 1 / sum(w) at wpart[inv_off] (the separate split-sum launch and the g round trip are skipped)
  const float* wpart;
  int S, pad_;
  long long inv_off;
  int tile_start[7], tiles_j[6];
};

__global__ __launch_bounds__(256) void k_adadelta(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ eg2, float* __restrict__ edx2, int64_t n,
                                                  int64_t n_decay, float rho, float eps, float l1, float l2,
                                                  __hip_bfloat16* __restrict__ shadow, WTMap tm) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float pi = p[i];
    // layer, row and column of a weight (the split-partial read and the transposed write)
    int l = 0;
    int64_t r = 0, c = 0;
    if ((tm.wt || tm.wpart) && i < n_decay) {
      while (l + 1 < tm.L && i >= tm.w_off[l + 1]) ++l;
      const int64_t o = i - tm.w_off[l];
      r = o / tm.n_in[l];
      c = o - r * tm.n_in[l];
    }
    float gi;
    if (tm.wpart && i < n_decay) {
      const int64_t b = tm.tile_start[l] + (r >> 6) * tm.tiles_j[l] + (c >> 6);
      const float* ps = tm.wpart + b * tm.S * 4096 + ((r & 63) << 6) + (c & 63);
      float t = 0.f;
      for (int s2 = 0; s2 < tm.S; ++s2) t += ps[(int64_t)s2 * 4096];
      gi = t * tm.wpart[tm.inv_off];
    } else {
      gi = g[i];
    }
    if (i < n_decay) gi += l2 * pi + (pi > 0.f ? l1 : (pi < 0.f ? -l1 : 0.f));
    const float e = rho * eg2[i] + (1.f - rho) * gi * gi;
    const float d = -sqrtf(edx2[i] + eps) / sqrtf(e + eps) * gi;
    eg2[i] = e;
    edx2[i] = rho * edx2[i] + (1.f - rho) * d * d;
    p[i] = pi + d;
    if (shadow && i < n_decay) shadow[i] = __float2bfloat16(pi + d);   // bf16 weights for the next GEMMs
    if (tm.wt && i < n_decay) {
      const int64_t t = tm.w_off[l] + c * tm.n_out[l] + r;
      if (tm.f32) ((float*)tm.wt)[t] = pi + d;
      else ((__hip_bfloat16*)tm.wt)[t] = __float2bfloat16(pi + d);
    }
  }
}

// The same update with the transposed copy: one workgroup per 8-row strip of a 64 x 64 weight tile (the
// k_dl_wgrad tiling; 8 strips per tile so a [784, 200, 200, 2] network spreads over ~580 workgroups),
// trailing workgroups take the biases. The flat per-element kernel above writes the transpose with a stride of
// n_out elements (one cache line per weight); here the updated strip goes through LDS and both copies are written
// along their contiguous axis (the transposed one in 16-element runs).
// MEASURED (r6, 10M x 784 [200,200] bf16, 4096-row steps): one workgroup per whole tile (74 workgroups, 16
// elements x S split partials per thread) took 54.7 us per step against 8.6 for the flat kernel; end to end
// (scripts/gpu_r6_wave.sh, two runs each) 8-row strips 58.4 / 57.8M samples/s, 16-row 56.7 / 55.8, flat 57.5 / 57.4.

__device__ __forceinline__ float adadelta_one(float pi, float gi, float* eg2, float* edx2, int64_t i, bool decay,
                                              float rho, float eps, float l1, float l2) {
  if (decay) gi += l2 * pi + (pi > 0.f ? l1 : (pi < 0.f ? -l1 : 0.f));
  const float e = rho * eg2[i] + (1.f - rho) * gi * gi;
  const float d = -sqrtf(edx2[i] + eps) / sqrtf(e + eps) * gi;
  eg2[i] = e;
  edx2[i] = rho * edx2[i] + (1.f - rho) * d * d;
  return pi + d;
}

template <int AD_STRIP>
__global__ __launch_bounds__(256) void k_adadelta_tiles(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ eg2, float* __restrict__ edx2, int64_t n,
                                                        int64_t n_decay, float rho, float eps, float l1, float l2,
                                                        __hip_bfloat16* __restrict__ shadow, WTMap tm) {
  __shared__ float tile[AD_STRIP][65];
  constexpr int NS = 64 / AD_STRIP;
  const int nst = tm.tile_start[tm.L] * NS;
  if ((int)blockIdx.x >= nst) {                     // biases: plain elementwise
    const int64_t i = n_decay + (int64_t)(blockIdx.x - nst) * 256 + threadIdx.x;
    if (i < n) p[i] = adadelta_one(p[i], g[i], eg2, edx2, i, false, rho, eps, l1, l2);
    return;
  }
  const int b = blockIdx.x / NS, strip = blockIdx.x % NS;
  int l = 0;
  while (l + 1 < tm.L && b >= tm.tile_start[l + 1]) ++l;
  const int t = b - tm.tile_start[l];
  const int r0 = (t / tm.tiles_j[l]) * 64 + strip * AD_STRIP, c0 = (t % tm.tiles_j[l]) * 64;
  const int nin = tm.n_in[l], nout = tm.n_out[l];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = c0 + tx;
  const float* ps = tm.wpart ? tm.wpart + (int64_t)b * tm.S * 4096 + strip * AD_STRIP * 64 : nullptr;
  float gs[AD_STRIP / 4];
#pragma unroll
  for (int k = 0; k < AD_STRIP / 4; ++k) gs[k] = 0.f;
  if (ps) {                                         // all split partials of the thread's rows in flight together
    for (int s2 = 0; s2 < tm.S; ++s2)
#pragma unroll
      for (int k = 0; k < AD_STRIP / 4; ++k) gs[k] += ps[(int64_t)s2 * 4096 + (ty + 4 * k) * 64 + tx];
  }
  const float inv = tm.wpart ? tm.wpart[tm.inv_off] : 0.f;
#pragma unroll
  for (int k = 0; k < AD_STRIP / 4; ++k) {
    const int rr = ty + 4 * k, r = r0 + rr;
    if (r >= nout || c >= nin) continue;
    const int64_t i = tm.w_off[l] + (int64_t)r * nin + c;
    const float gi = ps ? gs[k] * inv : g[i];
    const float v = adadelta_one(p[i], gi, eg2, edx2, i, true, rho, eps, l1, l2);
    p[i] = v;
    if (shadow) shadow[i] = __float2bfloat16(v);
    tile[rr][tx] = v;
  }
  __syncthreads();
  // transposed: WT[c][r]; thread -> (column cc of the strip's 64, row run of 16): lanes 0-15 one column
  const int rr = threadIdx.x & (AD_STRIP - 1);
  const int r = r0 + rr;
  for (int cc = threadIdx.x / AD_STRIP; cc < 64; cc += 256 / AD_STRIP) {
    const int c2 = c0 + cc;
    if (r >= nout || c2 >= nin) continue;
    const int64_t o = tm.w_off[l] + (int64_t)c2 * nout + r;
    if (tm.f32) ((float*)tm.wt)[o] = tile[rr][cc];
    else ((__hip_bfloat16*)tm.wt)[o] = __float2bfloat16(tile[rr][cc]);
  }
}

// Output layer of the explicit MLP step: per row, softmax cross-entropy (K classes) or squared error (K = 1,
// regression) gradient w.r.t. the logits, dO = (softmax(o) - onehot(y)) * w * inv  |  (o - y) * w * inv,
// written as T (the dtype of the following GEMMs) and the output-bias gradient Σ_rows dO accumulated
// with one fp32 atomic per (row, class). inv = 1 / Σw (single process) or 1 (data-parallel sum).
template <typename T>
__global__ __launch_bounds__(256) void k_out_grad(const T* __restrict__ logits, const long long* __restrict__ ycls,
                                                  const float* __restrict__ yreg, const float* __restrict__ w,
                                                  const float* __restrict__ inv, int64_t rows, int K,
                                                  T* __restrict__ dO, float* __restrict__ db) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float s = w[r] * inv[0];
  const T* o = logits + r * K;
  if (ycls) {
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, ld(o, k));
    float z = 0.f;
    for (int k = 0; k < K; ++k) z += __expf(ld(o, k) - mx);
    const float iz = 1.f / z;
    const long long c = ycls[r];
    for (int k = 0; k < K; ++k) {
      const float g = (__expf(ld(o, k) - mx) * iz - (k == c ? 1.f : 0.f)) * s;
      st(dO, r * K + k, g);
      if (g != 0.f) atomicAdd(db + k, g);
    }
  } else {
    const float g = (ld(o, 0) - yreg[r]) * s;
    st(dO, r, g);
    if (g != 0.f) atomicAdd(db, g);
  }
}

// ---- DataInfo (Expander) numeric columns: feature-major raw X [F, N] fp32 -> row-major design Z [N, P]
// Per-feature weighted moments in one pass (NaN skipped): out[j] = {Σw, Σw·x, Σw·x²} (fp64). grid (blocks
// over rows, features); each block reduces its row range in fp64 and adds once per feature.
__global__ __launch_bounds__(256) void k_num_stats(const float* __restrict__ X, int64_t N, const int* __restrict__ rows,
                                                   const float* __restrict__ w, double* __restrict__ out) {
  const int j = blockIdx.y;
  const float* x = X + (int64_t)rows[j] * N;
  double a = 0.0, b = 0.0, c = 0.0;
  auto add = [&](float v, int64_t i) {
    if (v == v) {
      const double ww = w ? (double)w[i] : 1.0;
      a += ww; b += ww * v; c += ww * (double)v * v;
    }
  };
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((N & 3) == 0) {     // 16-byte loads, 4 in flight per lane: 4 consecutive rows each
    int64_t i = 4 * i0;
    for (; i + 12 * stride < N; i += 16 * stride) {
      float4 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = *reinterpret_cast<const float4*>(x + i + 4 * u * stride);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t b = i + 4 * u * stride;
        add(q[u].x, b); add(q[u].y, b + 1); add(q[u].z, b + 2); add(q[u].w, b + 3);
      }
    }
    for (; i < N; i += 4 * stride) {
      const float4 q = *reinterpret_cast<const float4*>(x + i);
      add(q.x, i); add(q.y, i + 1); add(q.z, i + 2); add(q.w, i + 3);
    }
  } else {
    for (int64_t i = i0; i < N; i += stride) add(x[i], i);
  }
  __shared__ double red[3][8];
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_down(a, o, 64); b += __shfl_down(b, o, 64); c += __shfl_down(c, o, 64);
  }
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][wv] = a; red[1][wv] = b; red[2][wv] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s0 = 0, s1 = 0, s2 = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { s0 += red[0][k]; s1 += red[1][k]; s2 += red[2][k]; }
    atomicAdd(out + 3 * j, s0); atomicAdd(out + 3 * j + 1, s1); atomicAdd(out + 3 * j + 2, s2);
  }
}

// The same moments over the FLATTENED [nf][N] span (N % 4 == 0): block b reads the 64 KiB at b * NS_SPAN of the
// listed rows laid end to end (at most two features per block), so the resident blocks stream one contiguous
// window of X instead of 64 slices of every feature at once. MEASURED before: 9.9 ms for 10M x 784 (3.1 TB/s).
#define NS_SPAN 16384
__global__ __launch_bounds__(256) void k_num_stats_flat(const float* __restrict__ X, int64_t N,
                                                        const int* __restrict__ rows, int nf,
                                                        const float* __restrict__ w, double* __restrict__ out) {
  const int64_t total = (int64_t)nf * N;
  const int64_t e0 = (int64_t)blockIdx.x * NS_SPAN;
  if (e0 >= total) return;
  const int64_t e1 = e0 + NS_SPAN < total ? e0 + NS_SPAN : total;
  __shared__ double red[3][4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t s = e0; s < e1;) {                // one or two features
    const int j = (int)(s / N);
    const int64_t fend = ((int64_t)j + 1) * N < e1 ? ((int64_t)j + 1) * N : e1;
    const float* x = X + (int64_t)rows[j] * N;
    const int64_t i0 = s - (int64_t)j * N, i1 = fend - (int64_t)j * N;
    double a = 0.0, b = 0.0, c = 0.0;
#pragma unroll 4
    for (int64_t i = i0 + 4 * (int64_t)threadIdx.x; i < i1; i += 4 * 256) {
      const float4 q = *reinterpret_cast<const float4*>(x + i);
      const float4 wq = w ? *reinterpret_cast<const float4*>(w + i) : make_float4(1.f, 1.f, 1.f, 1.f);
      const float v[4] = {q.x, q.y, q.z, q.w}, wv4[4] = {wq.x, wq.y, wq.z, wq.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (v[k] == v[k]) {
          const double ww = (double)wv4[k];
          a += ww; b += ww * v[k]; c += ww * (double)v[k] * v[k];
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_down(a, o, 64); b += __shfl_down(b, o, 64); c += __shfl_down(c, o, 64);
    }
    if (lane == 0) { red[0][wv] = a; red[1][wv] = b; red[2][wv] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
      const double s0 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
      const double s1 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
      const double s2 = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
      atomicAdd(out + 3 * j, s0); atomicAdd(out + 3 * j + 1, s1); atomicAdd(out + 3 * j + 2, s2);
    }
    __syncthreads();
    s = fend;
  }
}

// Z[r, col0 + j] = (isnan(x) ? fill_j : x - sub_j) * mul_j for the numeric rows listed in `rows`. A block owns
// NT_ROWS rows and walks the features in chunks of NT_FC through an [NT_FC][NT_ROWS + 1] LDS tile: every read is
// one feature's NT_ROWS rows (contiguous, 16-byte loads), every write a row's NT_FC-feature run (16-byte stores)
// — whole cache lines both ways.
// MEASURED before: one element per lane (5.9 ms for 2M x 784, 1.6 TB/s); 128-row x 32-feature tiles with 16-byte
// accesses, whose 64-byte row pieces left every written line partial (15.7 ms for 10M x 784, 3 TB/s).
template <typename T> struct NT_VEC;
template <> struct NT_VEC<__hip_bfloat16> { static constexpr int n = 8; };
template <> struct NT_VEC<float> { static constexpr int n = 4; };
__device__ __forceinline__ uint4 pack_row(const float* v, __hip_bfloat16*) {
  union { __hip_bfloat16 h[8]; uint4 u; } pk;
#pragma unroll
  for (int j = 0; j < 8; ++j) pk.h[j] = __float2bfloat16(v[j]);
  return pk.u;
}
__device__ __forceinline__ uint4 pack_row(const float* v, float*) {
  return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
}
// MEASURED r4 (10M x 784 bf16): 32 rows x 256 features 13.19 ms, 128 rows x 64 features 12.46 ms
// MEASURED r5: issuing the next (rows, feature chunk) item's loads before the current tile's stores (register
// pipeline) 14.0 ms — slower; not kept (scripts/experiments/num_transform_pipeline.diff).
#ifndef NT_ROWS
#define NT_ROWS 128
#endif
#ifndef NT_FC
#define NT_FC 64
#endif
template <typename T>
__global__ __launch_bounds__(256) void k_num_transform(const float* __restrict__ X, int64_t N, const int* __restrict__ rows,
                                                       int nf, const float* __restrict__ fill, const float* __restrict__ sub,
                                                       const float* __restrict__ mul, T* __restrict__ Z, int ldz, int col0,
                                                       float extra, int has_extra) {
  __shared__ float tile[NT_FC][NT_ROWS + 1];
  const int t = threadIdx.x;
  const bool vin = (N % 4) == 0;
  const bool lin = col0 == 0 && nf <= NT_FC && ldz == nf + has_extra;
  constexpr int VN = NT_VEC<T>::n, CPR = NT_FC / VN;          // 16-byte chunks per row and feature chunk
  for (int64_t r0 = (int64_t)blockIdx.x * NT_ROWS; r0 < N; r0 += (int64_t)gridDim.x * NT_ROWS) {
    for (int fc = 0; fc < nf; fc += NT_FC) {
      // read: thread t takes rows r0 + 4 (t % CPF) .. + 3 of features fc + t / CPF + FPP i
      constexpr int CPF = NT_ROWS / 4, FPP = 256 / CPF;
#pragma unroll
      for (int i = 0; i < NT_FC / FPP; ++i) {
        const int k = t / CPF + FPP * i, c = t % CPF;
        const int f = fc + k;
        const int64_t r = r0 + 4 * c;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (f < nf) {
          const float* x = X + (int64_t)rows[f] * N;
          if (vin && r + 3 < N) {
            const float4 q = *reinterpret_cast<const float4*>(x + r);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = r + j < N ? x[r + j] : 0.f;
          }
          const float fl = fill[f], sb = sub[f], ml = mul[f];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = ((v[j] != v[j]) ? fl : v[j]) - sb, v[j] *= ml;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[k][4 * c + j] = v[j];
      }
      __syncthreads();
      if (lin) {
        // whole rows (col0 == 0, ldz == nf + has_extra, one feature chunk): the block's output is ONE contiguous
        // span of NT_ROWS * ldz elements, written by consecutive lanes (the extra constant column included) —
        // MEASURED r6 (GLM 10M x 50, ldz 51): the 16-byte-row-chunk stores below cannot vectorise at an odd
        // ldz and ran 1.5 ms plus a 0.67 ms strided torch fill of the intercept column
        const int64_t nrow = min((int64_t)NT_ROWS, N - r0);
        const int span = (int)nrow * ldz;
        T* dst = Z + r0 * ldz;
        for (int o = t; o < span; o += 256) {
          const int rr = o / ldz, col = o - rr * ldz;
          st(dst, o, col < nf ? tile[col][rr] : extra);
        }
        __syncthreads();
        continue;
      }
      // write: VN consecutive features of one row per 16-byte store
      const bool vout = (ldz % VN) == 0 && ((col0 + fc) % VN) == 0;
      for (int idx = t; idx < NT_ROWS * CPR; idx += 256) {
        const int rr = idx / CPR, q = idx % CPR;
        const int64_t r = r0 + rr;
        const int fq = fc + q * VN;
        if (r >= N || fq >= nf) continue;
        float v[VN];
#pragma unroll
        for (int j = 0; j < VN; ++j) v[j] = tile[q * VN + j][rr];
        T* dst = Z + r * ldz + col0 + fq;
        if (vout && fq + VN <= nf) {
          *reinterpret_cast<uint4*>(dst) = pack_row(v, (T*)nullptr);
        } else {
#pragma unroll
          for (int j = 0; j < VN; ++j) if (fq + j < nf) st(dst, j, v[j]);
        }
      }
      __syncthreads();        // the tile is refilled for the next feature chunk / row range
    }
  }
}

}  // namespace

extern "C" {

int h2o_num_stats(const float* X, long long N, const int* rows, int nf, const float* w, double* out, hipStream_t s) {
  if (N <= 0 || nf <= 0) return 0;
  if ((N & 3) == 0) {
    const long long nb = ((long long)nf * N + NS_SPAN - 1) / NS_SPAN;
    hipLaunchKernelGGL(k_num_stats_flat, dim3((unsigned)nb), dim3(256), 0, s, X, (int64_t)N, rows, nf, w, out);
    return (int)hipGetLastError();
  }
  long long g = (N + 255) / 256;
  if (g > 64) g = 64;
  hipLaunchKernelGGL(k_num_stats, dim3((unsigned)g, (unsigned)nf), dim3(256), 0, s, X, (int64_t)N, rows, w, out);
  return (int)hipGetLastError();
}

// has_extra: also fill column nf of the whole-row layout (col0 == 0, ldz == nf + 1, nf <= NT_FC) with `extra`
// (the GLM intercept column); refused for any other layout (the caller fills it itself then)
int h2o_num_transform(const float* X, long long N, const int* rows, int nf, const float* fill, const float* sub,
                      const float* mul, void* Z, int ldz, int col0, int bf16, float extra, int has_extra,
                      hipStream_t s) {
  if (has_extra && (col0 != 0 || nf > NT_FC || ldz != nf + 1)) return (int)hipErrorInvalidValue;
  if (N <= 0 || nf <= 0) return 0;
  // 32-row blocks strided over a bounded grid
  long long gx = (N + NT_ROWS - 1) / NT_ROWS;
  if (gx > 16384) gx = 16384;
  dim3 grid((unsigned)gx);
  if (bf16)
    hipLaunchKernelGGL(k_num_transform<__hip_bfloat16>, grid, dim3(256), 0, s, X, (int64_t)N, rows, nf, fill, sub, mul,
                       (__hip_bfloat16*)Z, ldz, col0, extra, has_extra);
  else
    hipLaunchKernelGGL(k_num_transform<float>, grid, dim3(256), 0, s, X, (int64_t)N, rows, nf, fill, sub, mul, (float*)Z,
                       ldz, col0, extra, has_extra);
  return (int)hipGetLastError();
}

// wt (nullable): transposed copy to write along (tm_off/tm_in/tm_out: L layers' offsets and shapes)
int h2o_adadelta(float* p, const float* g, float* eg2, float* edx2, long long n, long long n_decay, float rho, float eps,
                 float l1, float l2, void* shadow, void* wt, int wt_f32, int L, const long long* tm_off,
                 const int* tm_in, const int* tm_out, const float* wpart, int S, long long inv_off,
                 const int* tile_start, const int* tiles_j, hipStream_t stream) {
  long long grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  WTMap tm{};
  if (wt) {
    if (L < 1 || L > 6) return (int)hipErrorInvalidValue;
    tm.wt = wt; tm.f32 = wt_f32; tm.L = L;
    for (int l = 0; l < L; ++l) { tm.w_off[l] = tm_off[l]; tm.n_in[l] = tm_in[l]; tm.n_out[l] = tm_out[l]; }
    if (wpart) {
      tm.wpart = wpart; tm.S = S; tm.inv_off = inv_off;
      for (int l = 0; l <= L; ++l) tm.tile_start[l] = tile_start[l];
      for (int l = 0; l < L; ++l) tm.tiles_j[l] = tiles_j[l];
    }
    // tiled update (H2O_ADADELTA_FLAT=1 keeps the per-element kernel): the 64 x 64 tile map of the weights, which
    // must be the one the split partials were written with, and weights laid out back to back from offset 0
    static int flat = -1;
    if (flat < 0) { const char* e = getenv("H2O_ADADELTA_FLAT"); flat = (e && e[0] == '1') ? 1 : 0; }
    bool ok = !flat;
    long long ts = 0, off = 0;
    int tsv[7], tjv[6];
    for (int l = 0; l < L && ok; ++l) {
      tjv[l] = (tm.n_in[l] + 63) / 64;
      tsv[l] = (int)ts;
      ts += (long long)((tm.n_out[l] + 63) / 64) * tjv[l];
      ok = tm.w_off[l] == off;
      off += (long long)tm.n_in[l] * tm.n_out[l];
      if (wpart) ok = ok && tsv[l] == tm.tile_start[l] && tjv[l] == tm.tiles_j[l];
    }
    tsv[L] = (int)ts;
    ok = ok && off == n_decay && ts < (1LL << 30) && (!wpart || tm.tile_start[L] == tsv[L]);
    if (ok) {
      for (int l = 0; l <= L; ++l) tm.tile_start[l] = tsv[l];
      for (int l = 0; l < L; ++l) tm.tiles_j[l] = tjv[l];
      // H2O_ADADELTA_STRIP=8 (default) | 16 | 64 rows per workgroup
      static int strip = 0;
      if (!strip) { const char* e = getenv("H2O_ADADELTA_STRIP"); strip = e ? atoi(e) : 8;
                    if (strip != 16 && strip != 64) strip = 8; }
      const long long grid2 = ts * (64 / strip) + (n - n_decay + 255) / 256;
      auto kern = strip == 8 ? k_adadelta_tiles<8> : strip == 64 ? k_adadelta_tiles<64> : k_adadelta_tiles<16>;
      hipLaunchKernelGGL(kern, dim3((unsigned)grid2), dim3(256), 0, stream, p, g, eg2, edx2, (int64_t)n,
                         (int64_t)n_decay, rho, eps, l1, l2, (__hip_bfloat16*)shadow, tm);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL(k_adadelta, dim3((unsigned)grid), dim3(256), 0, stream, p, g, eg2, edx2, (int64_t)n,
                     (int64_t)n_decay, rho, eps, l1, l2, (__hip_bfloat16*)shadow, tm);
  return (int)hipGetLastError();
}

int h2o_out_grad(const void* logits, const long long* ycls, const float* yreg, const float* w, const float* inv,
                 long long rows, int K, void* dO, float* db, int bf16, hipStream_t stream) {
  if (rows <= 0) return 0;
  const unsigned grid = (unsigned)((rows + 255) / 256);
  if (bf16)
    hipLaunchKernelGGL(k_out_grad<__hip_bfloat16>, dim3(grid), dim3(256), 0, stream, (const __hip_bfloat16*)logits,
                       ycls, yreg, w, inv, (int64_t)rows, K, (__hip_bfloat16*)dO, db);
  else
    hipLaunchKernelGGL(k_out_grad<float>, dim3(grid), dim3(256), 0, stream, (const float*)logits, ycls, yreg, w, inv,
                       (int64_t)rows, K, (float*)dO, db);
  return (int)hipGetLastError();
}


int h2o_bias_act_fwd(const void* x, const float* b, void* y, long long rows, int cols, int act, float drop,
                     unsigned long long seed, const unsigned long long* seed_dev, int bf16, hipStream_t stream) {
  const long long n = rows * (long long)cols;
  int grid = (int)((n + 255) / 256);
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  if (bf16)
    hipLaunchKernelGGL(k_bias_act_fwd<__hip_bfloat16>, dim3(grid), dim3(256), 0, stream, (const __hip_bfloat16*)x, b,
                       (__hip_bfloat16*)y, (int64_t)rows, cols, act, drop, seed, (const uint64_t*)seed_dev);
  else
    hipLaunchKernelGGL(k_bias_act_fwd<float>, dim3(grid), dim3(256), 0, stream, (const float*)x, b, (float*)y,
                       (int64_t)rows, cols, act, drop, seed, (const uint64_t*)seed_dev);
  return (int)hipGetLastError();
}

int h2o_bias_act_bwd(const void* gy, const void* y, void* gx, float* db, long long rows, int cols, int act,
                     float drop, unsigned long long seed, const unsigned long long* seed_dev, int bf16,
                     hipStream_t stream) {
  // enough row stripes to fill the chip: a [4096 x 200] mini-batch was 64 blocks (22.8 us); stripes of
  // 32 rows give 512 blocks (the per-stripe bias partial is one atomic per column)
  const int rpb = rows >= (1 << 16) ? 256 : 32;
  dim3 grid((cols + 63) / 64, (unsigned)((rows + rpb - 1) / rpb));
  if (bf16)
    hipLaunchKernelGGL(k_bias_act_bwd<__hip_bfloat16>, grid, dim3(256), 0, stream, (const __hip_bfloat16*)gy,
                       (const __hip_bfloat16*)y, (__hip_bfloat16*)gx, db, (int64_t)rows, cols, act, drop, seed, rpb,
                       (const uint64_t*)seed_dev);
  else
    hipLaunchKernelGGL(k_bias_act_bwd<float>, grid, dim3(256), 0, stream, (const float*)gy, (const float*)y,
                       (float*)gx, db, (int64_t)rows, cols, act, drop, seed, rpb, (const uint64_t*)seed_dev);
  return (int)hipGetLastError();
}

}  // extern "C"
