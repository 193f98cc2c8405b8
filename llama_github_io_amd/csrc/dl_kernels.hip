// DeepLearning training step on the matrix cores (reference: h2o-algos/src/main/java/hex/deeplearning/
// Neurons.java fprop / bprop, DeepLearningTask.map; the mini-batch replaces the reference's per-row Hogwild).
//
// One optimizer step of an MLP (bias + Rectifier/Tanh hidden layers with dropout, softmax-CE or squared-error
// output) is three launches instead of ~20 library GEMMs and elementwise kernels:
//
//  k_dl_rows   one workgroup per 16-row tile of the mini-batch. The tile's input rows are gathered from the
//              resident design matrix by row index, then the WHOLE network runs on that tile with the
//              activations in LDS: every layer is v_mfma_f32_16x16x32_bf16 over (activation tile in LDS) x
//              (bf16 weight rows streamed from L2), with bias / activation / dropout fused in the epilogue;
//              the output gradient (softmax - onehot) * w, and the backward pass dh = dA W, dA = dh * mask *
//              act'(h) run the same way on transposed weight copies. The tile writes its activations and
//              gradients TRANSPOSED ([units][rows]) for the weight-gradient GEMM and its per-column bias
//              gradient partial sums (fixed-order reduce later, no atomics).
//  k_dl_wgrad  dW_l = dA_lᵀ h_{l-1} for every layer in one launch: 64 x 64 output tiles, the mini-batch rows
//              (GEMM K) split over workgroups and, inside one, over 4 waves; partials summed in a fixed order
//              and written straight into the flat gradient buffer scaled by 1 / sum(w) of the batch (single
//              process) or raw plus the batch weight (data parallel). Trailing workgroups reduce the per-tile
//              bias partials of k_dl_rows (one wave per bias, fixed order).
//  MEASURED (r4, DL_TIMING phase clocks): staging the weights of layers 2+ in LDS per launch cost ~5 us of
//  loads at kernel start and gained < 0.4 us per later phase (their time is not the weight reads): dropped.
//  Prefetching layer 1's first round of weight fragments into registers before the gathers spilled (128 VGPRs).
//  MEASURED (r5): writing the layer-1 input transpose (hT0) from the 3 waves without a layer-1 tile while the other
//  13 run the layer-1 MFMAs: 31.1 -> 31.6 us per step (not on the critical path; scripts/experiments/dl_hT0_overlap.diff).
//  MEASURED (10M x 784 [200,200], 4096-row steps, rocprofv3): the first version (16-row tiles on 4 waves,
//  64 x 64 x 4-split weight tiles with fp32 slabs and a separate reduce) took 52 + 32 + 64 us per step:
//  latency-bound dependent L2 round trips and a serial 256-deep bias loop, not MFMA or HBM.
// The fused ADADELTA kernel (dense_kernels.hip) then updates the fp32 master weights and the bf16 weight
// shadow; k_dl_transpose refreshes the transposed shadow the backward pass reads.
//
// MFMA 16x16x32 bf16 operand maps (gfx950): lane l holds A[row l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][col
// l&15] (j = 0..7) and D[row 4(l>>4)+r][col l&15] (r = 0..3).
// fp32 (compute_dtype="float32", the H2O default): the same kernels on v_mfma_f32_16x16x4_f32 with fp32
// activations in LDS, the fp32 master weights read in place and fp32 transposed buffers. A lane loads 4
// consecutive k (one float4) of its A row and B column and issues 4 MFMAs, MFMA j taking element j: every
// MFMA pairs A[i][4q + j] with B[4q + j][n] for lane quarter q, so the 4 cover 16 k.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

#define DL_MAXL 6        // GEMM layers (hidden + output)
#define DL_ROWS 16       // rows per k_dl_rows tile
#define DL_THREADS 1024  // k_dl_rows workgroup: 16 waves (one 16-column output tile each per round)
#define DL_NW (DL_THREADS / 64)

struct DLArgs {
  const void* Z; long long ldz; const long long* ridx; int B; int Bpad;
  const float* w; const long long* ycls; const float* yreg;
  const float* P; const void* W; void* WT; const unsigned long long* step_dev;
  void* hT; void* dT; float* bpart; float* g; float* gsum;
  int L, K, act, regression;
  int n[DL_MAXL + 1];           // n[0] inputs, n[l] units of layer l, n[L] = outputs
  int kp[DL_MAXL + 1];          // n padded to 32 (GEMM K extent when the activation is an operand)
  int ld[DL_MAXL + 1];          // LDS row stride of activation tiles (kp + 8: spreads rows over banks)
  long long w_off[DL_MAXL], b_off[DL_MAXL];   // layer l+1's weights / biases in the flat parameter buffer
  long long h_off[DL_MAXL + 1], d_off[DL_MAXL + 1];
  int bias_off[DL_MAXL + 1], bias_total;
  float drop[DL_MAXL]; unsigned long long seed_base[DL_MAXL];
  int lds_off[DL_MAXL + 1];     // activation tiles l = 0..L-1, then the output-gradient tile
  int lds_g[2], lds_w;          // two gradient tiles, row weights
  int tiles_i[DL_MAXL], tiles_j[DL_MAXL], tile_start[DL_MAXL + 1];   // k_dl_wgrad block decode
  long long n_decay, n_total;
  int f32, pad_;                // 1: fp32 operands (Z, W, WT, hT, dT, LDS tiles), 0: bf16
  float in_drop; int lds_lg;    // input dropout ratio; K > 16: byte offset of the fp32 [16][K] logit tile
  unsigned long long in_seed;   // input dropout seed base
  int wsplit, maxout;           // k_dl_wgrad: batch-row (GEMM K) splits per 64 x 64 tile; 1: Maxout hidden layers
  int ng[DL_MAXL + 1];          // GEMM output width of layer l (2 n[l] for Maxout hidden layers: two channels)
  int kpg[DL_MAXL + 1], ldg[DL_MAXL + 1];   // ng padded to 32, LDS row stride of gradient tiles of width ng
  int lds_mx[DL_MAXL];          // Maxout: byte offset of layer l's [16][n[l]] winning-channel bytes
  int ae, no_wsum;               // 1: autoencoder (outputs reconstruct the undropped inputs, quadratic loss / K);
                                // no_wsum: the optimizer reads the split partials itself (no k_dl_wsum launch)
  float* wpart;                 // [tiles][wsplit][64 * 64] fp32 partial tiles, then the batch's 1 / sum(w)
};

#ifdef DL_TIMING
// per-workgroup phase clocks of the last k_dl_rows launch (diagnostic build only: scripts/build_alt.sh dlt
// -DDL_TIMING, read back with h2o_dl_timing)
__device__ unsigned long long g_dl_t[4096 * 16];
#define DLT(i) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_dl_t[blockIdx.x * 16 + (i)] = wall_clock64(); } while (0)
#else
#define DLT(i) do { } while (0)
#endif

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return (uint32_t)x;
}
// the dropout mask of dense_kernels.hip k_bias_act_fwd / k_bias_act_bwd (element index within the batch)
__device__ __forceinline__ bool dropped(uint64_t seed, int64_t i, uint32_t thr) {
  return hash32(seed ^ (uint64_t)i * 0x9E3779B97F4A7C15ULL) < thr;
}
__device__ __forceinline__ float act_f(int a, float v) {
  return a == 1 ? (v > 0.f ? v : 0.f) : (a == 2 ? tanhf(v) : (a == 3 ? (v > 0.f ? v : expm1f(v)) : v));
}
__device__ __forceinline__ float dact_from_y(int a, float y) {
  return a == 1 ? (y > 0.f ? 1.f : 0.f) : (a == 2 ? 1.f - y * y : (a == 3 ? (y > 0.f ? 1.f : y + 1.f) : 1.f));
}

// 8 bf16 of a global row [k, k+8) with a zero tail past `kvalid`; vector load when aligned
__device__ __forceinline__ bf16x8 load8(const bf16* row, int k, int kvalid, bool vec) {
  if (vec && k + 8 <= kvalid) return *reinterpret_cast<const bf16x8*>(row + k);
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float f = (k + j < kvalid) ? __bfloat162float(row[k + j]) : 0.f;
    v[j] = (__bf16)f;
  }
  return v;
}

// D(16 x 16 cols n0..n0+15) = A(LDS tile, 16 x K) * Bᵀ where B row n (global, contiguous along k) holds the
// operand column n: B[k][n] = Brow(n)[k]. K is a multiple of 32; A is zero past the valid extent.
// The B fragments come from L2 (every tile of the batch reads the same weights): KU k-steps of loads are
// issued before their MFMAs so KU round trips overlap instead of serialising one per MFMA.
#define KU 16
__device__ __forceinline__ f32x4 tile_mm(const bf16* A, int lda, const bf16* Bg, long long ldb, int n0, int nvalid,
                                         int K, int kvalid, bool vec) {
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int n = n0 + c;
  const bool nok = n < nvalid;
  const bf16* brow = Bg + (long long)(nok ? n : 0) * ldb;
  const bf16x8 z8 = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
  for (int kb = 0; kb < K; kb += 32 * KU) {
    bf16x8 b[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int k = kb + 32 * u + 8 * q;
      b[u] = (nok && kb + 32 * u < K) ? load8(brow, k, kvalid, vec) : z8;
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (kb + 32 * u < K) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + c * lda + kb + 32 * u + 8 * q);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[u], acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

// fp32 operands: 4 consecutive k of one row (zero tail past kvalid)
__device__ __forceinline__ float4 load4(const float* row, int k, int kvalid, bool vec) {
  if (vec && k + 4 <= kvalid) return *reinterpret_cast<const float4*>(row + k);
  float4 v;
  v.x = k < kvalid ? row[k] : 0.f;
  v.y = k + 1 < kvalid ? row[k + 1] : 0.f;
  v.z = k + 2 < kvalid ? row[k + 2] : 0.f;
  v.w = k + 3 < kvalid ? row[k + 3] : 0.f;
  return v;
}

#define KU4 8
__device__ __forceinline__ f32x4 tile_mm(const float* A, int lda, const float* Bg, long long ldb, int n0, int nvalid,
                                         int K, int kvalid, bool vec) {
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int n = n0 + c;
  const bool nok = n < nvalid;
  const float* brow = Bg + (long long)(nok ? n : 0) * ldb;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int kb = 0; kb < K; kb += 16 * KU4) {
    float4 b[KU4];
#pragma unroll
    for (int u = 0; u < KU4; ++u) {
      const int k = kb + 16 * u + 4 * q;
      b[u] = (nok && kb + 16 * u < K) ? load4(brow, k, kvalid, vec) : z4;
    }
#pragma unroll
    for (int u = 0; u < KU4; ++u) {
      if (kb + 16 * u < K) {
        const float4 a = *reinterpret_cast<const float4*>(A + c * lda + kb + 16 * u + 4 * q);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[u].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[u].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[u].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[u].w, acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

__device__ __forceinline__ float to_f(bf16 v) { return __bfloat162float(v); }
__device__ __forceinline__ float to_f(float v) { return v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ bf16 from_f<bf16>(float v) { return __float2bfloat16(v); }
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }

// column sums of the 16 x 16 D tile (rows 4q + r): in-lane over r, then across the 4 lane quarters
__device__ __forceinline__ float col_sum(f32x4 v) {
  float s = (v[0] + v[1]) + (v[2] + v[3]);
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  return s;
}

__device__ __forceinline__ void store4T(bf16* dst, f32x4 v) {   // 4 consecutive rows of one unit, 8 bytes
  union { bf16 h[4]; uint2 u; } pk;
  pk.h[0] = __float2bfloat16(v[0]); pk.h[1] = __float2bfloat16(v[1]);
  pk.h[2] = __float2bfloat16(v[2]); pk.h[3] = __float2bfloat16(v[3]);
  *reinterpret_cast<uint2*>(dst) = pk.u;
}
__device__ __forceinline__ void store4T(float* dst, f32x4 v) {  // fp32: 16 bytes
  *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
}

template <typename T>
__global__ __launch_bounds__(DL_THREADS) void k_dl_rows(DLArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* S = reinterpret_cast<T*>(smem);
  const T* Zg = reinterpret_cast<const T*>(a.Z);
  const T* Wg = reinterpret_cast<const T*>(a.W);
  const T* WTg = reinterpret_cast<const T*>(a.WT);
  T* hTg = reinterpret_cast<T*>(a.hT);
  T* dTg = reinterpret_cast<T*>(a.dT);
  constexpr int VE = 16 / sizeof(T);     // elements per 16-byte vector
  float* ws = reinterpret_cast<float*>(smem + a.lds_w);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, c = lane & 15;
  const int r0 = blockIdx.x * DL_ROWS;
  const int L = a.L;
  const uint64_t step = a.step_dev ? *a.step_dev : 0ull;
  DLT(0);
  __shared__ long long srow[DL_ROWS];
  __shared__ float sy[DL_ROWS];
  __shared__ long long scls[DL_ROWS];
  if (tid < DL_ROWS) {
    const int r = r0 + tid;
    const long long g = r < a.B ? a.ridx[r] : -1;
    srow[tid] = g;
    ws[tid] = g >= 0 ? a.w[g] : 0.f;
    if (a.ae) scls[tid] = -1;
    else if (a.regression) sy[tid] = g >= 0 ? a.yreg[g] : 0.f;
    else scls[tid] = g >= 0 ? a.ycls[g] : -1;
  }
  // zero every activation / gradient tile (K padding must read as zeros) except the input rows' data columns,
  // which the gather below writes in full — so the gather needs no barrier after the zeroing
  T* A0 = S + a.lds_off[0];
  const int n0 = a.n[0], ld0 = a.ld[0];
  {
    const int total = a.lds_w / 4;
    const int a0s = a.lds_off[0] * (int)sizeof(T) / 4, a0e = (a.lds_off[0] + DL_ROWS * ld0) * (int)sizeof(T) / 4;
    for (int i = tid; i < total; i += DL_THREADS)
      if (i < a0s || i >= a0e) reinterpret_cast<float*>(smem)[i] = 0.f;
    const int pw = ld0 - n0;
    for (int i = tid; i < DL_ROWS * pw; i += DL_THREADS) A0[(i / pw) * ld0 + n0 + i % pw] = from_f<T>(0.f);
  }
  DLT(1);
  // ---- gather the 16 input rows into activation tile 0: each thread reads its row's index itself (one
  // dependent round trip, index -> row, instead of index -> barrier -> row); padding rows are zero
  {
    const bool vec = (n0 % VE == 0) && (a.ldz % VE == 0);
    const int chunks = (n0 + VE - 1) / VE;
    for (int i = tid; i < DL_ROWS * chunks; i += DL_THREADS) {
      const int rr = i / chunks, k = (i - rr * chunks) * VE;
      const int r = r0 + rr;
      const long long g = r < a.B ? a.ridx[r] : -1;
      T* dst = A0 + rr * ld0 + k;
      if (g < 0) {
        if (vec) *reinterpret_cast<uint4*>(dst) = make_uint4(0u, 0u, 0u, 0u);
        else for (int j = 0; j < VE && k + j < n0; ++j) dst[j] = from_f<T>(0.f);
        continue;
      }
      const T* src = Zg + g * a.ldz;
      if (vec) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src + k);
      else for (int j = 0; j < VE && k + j < n0; ++j) dst[j] = src[k + j];
    }
  }
  __syncthreads();
  DLT(2);
  // input dropout (input_dropout_ratio): hash mask over (batch row, input), survivors scaled by 1 / keep
  if (a.in_drop > 0.f) {
    T* A0 = S + a.lds_off[0];
    const int n0 = a.n[0], ld0 = a.ld[0];
    const float keep = 1.f - a.in_drop;
    const uint32_t thr = (uint32_t)(a.in_drop * 4294967296.0);
    const uint64_t seed = a.in_seed ^ (step * 0x9E3779B97F4A7C15ULL);
    for (int i = tid; i < DL_ROWS * n0; i += DL_THREADS) {
      const int rr = i / n0, k = i - rr * n0;
      T* e = A0 + rr * ld0 + k;
      *e = dropped(seed, (int64_t)(r0 + rr) * n0 + k, thr) ? from_f<T>(0.f) : from_f<T>(to_f(*e) / keep);
    }
    __syncthreads();
  }
  // x transposed for the first weight gradient: hT_0[k][r0 + 4 g .. + 3]
  {
    const T* A0 = S + a.lds_off[0];
    T* dst = hTg + a.h_off[0];
    for (int i = tid; i < a.n[0] * 4; i += DL_THREADS) {
      const int k = i >> 2, g4 = (i & 3) * 4;
      f32x4 v = {to_f(A0[(g4 + 0) * a.ld[0] + k]), to_f(A0[(g4 + 1) * a.ld[0] + k]),
                 to_f(A0[(g4 + 2) * a.ld[0] + k]), to_f(A0[(g4 + 3) * a.ld[0] + k])};
      store4T(dst + (long long)k * a.Bpad + r0 + g4, v);
    }
  }
  // ---- forward: hidden layers
  for (int l = 1; l < L; ++l) {
    const T* Ain = S + a.lds_off[l - 1];
    T* Aout = S + a.lds_off[l];
    const int nin = a.n[l - 1], nout = a.n[l];
    const T* Wl = Wg + a.w_off[l - 1];
    const bool vec = (nin % VE == 0) && (a.w_off[l - 1] % VE == 0);
    const float drop = a.drop[l - 1], keep = 1.f - drop;
    const uint32_t thr = (uint32_t)(drop * 4294967296.0);
    const uint64_t seed = a.seed_base[l - 1] ^ (step * 0x9E3779B97F4A7C15ULL);
    const int NT = (nout + 15) / 16;
    unsigned char* win = a.maxout ? smem + a.lds_mx[l] : nullptr;
    for (int t = wv; t < NT; t += DL_NW) {
      const f32x4 acc = tile_mm(Ain, a.ld[l - 1], Wl, nin, t * 16, nout, a.kp[l - 1], nin, vec);
      // Maxout (Neurons.Maxout, 2 channels): channel 1 = weight / bias rows [nout, 2 nout)
      f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
      if (a.maxout)
        acc1 = tile_mm(Ain, a.ld[l - 1], Wl + (long long)nout * nin, nin, t * 16, nout, a.kp[l - 1], nin, vec);
      const int col = t * 16 + c;
      f32x4 o;
      if (col < nout) {
        const float b = a.P[a.b_off[l - 1] + col];
        const float b1 = a.maxout ? a.P[a.b_off[l - 1] + nout + col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v;
          if (a.maxout) {
            const float z0 = acc[r] + b, z1 = acc1[r] + b1;
            v = z1 > z0 ? z1 : z0;
            win[(4 * q + r) * nout + col] = z1 > z0 ? 1 : 0;
          } else {
            v = act_f(a.act, acc[r] + b);
          }
          if (drop > 0.f) v = dropped(seed, (int64_t)(r0 + 4 * q + r) * nout + col, thr) ? 0.f : v / keep;
          o[r] = v;
          Aout[(4 * q + r) * a.ld[l] + col] = from_f<T>(v);
        }
        store4T(hTg + a.h_off[l] + (long long)col * a.Bpad + r0 + 4 * q, o);
      }
    }
    __syncthreads();
    DLT(2 + l);
  }
  // ---- output layer + loss gradient (wave 0 when K <= 16; K > 16: logit tiles over the waves, then one wave
  // per row for the softmax, then one thread per class for the bias partials and the transposed gradient)
  T* GO = S + a.lds_off[L];
  if (a.K > 16) {
    float* LG = reinterpret_cast<float*>(smem + a.lds_lg);
    const int nin = a.n[L - 1], K = a.K;
    const T* Wo = Wg + a.w_off[L - 1];
    const bool vec = (nin % VE == 0) && (a.w_off[L - 1] % VE == 0);
    for (int t = wv; t < (K + 15) / 16; t += DL_NW) {
      const f32x4 acc = tile_mm(S + a.lds_off[L - 1], a.ld[L - 1], Wo, nin, t * 16, K, a.kp[L - 1], nin, vec);
      const int col = t * 16 + c;
      if (col < K) {
        const float b = a.P[a.b_off[L - 1] + col];
#pragma unroll
        for (int r = 0; r < 4; ++r) LG[(4 * q + r) * K + col] = acc[r] + b;
      }
    }
    __syncthreads();
    if (wv < DL_ROWS && a.ae) {
      // autoencoder: d/do of sum_k (o_k - x_k)^2 / K times the row weight (x: the input row before dropout)
      const int row = wv;
      float* lg = LG + row * K;
      const float wr = ws[row];
      const long long gr = srow[row];
      const T* xr = Zg + (gr < 0 ? 0 : gr) * a.ldz;
      for (int k = lane; k < K; k += 64) {
        const float gk = gr < 0 ? 0.f : 2.f * (lg[k] - to_f(xr[k])) * wr / (float)K;
        lg[k] = gk;
        GO[row * a.ld[L] + k] = from_f<T>(gk);
      }
    } else if (wv < DL_ROWS) {
      const int row = wv;
      float* lg = LG + row * K;
      float mx = -INFINITY;
      for (int k = lane; k < K; k += 64) mx = fmaxf(mx, lg[k]);
      for (int m = 32; m > 0; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
      float z = 0.f;
      for (int k = lane; k < K; k += 64) z += __expf(lg[k] - mx);
      for (int m = 32; m > 0; m >>= 1) z += __shfl_xor(z, m, 64);
      const float wr = ws[row];
      const long long cls = scls[row];
      for (int k = lane; k < K; k += 64) {
        const float gk = (__expf(lg[k] - mx) / z - (cls == k ? 1.f : 0.f)) * wr;
        lg[k] = gk;
        GO[row * a.ld[L] + k] = from_f<T>(gk);
      }
    }
    __syncthreads();
    for (int k = tid; k < K; k += DL_THREADS) {
      float cs = 0.f;
      for (int g4 = 0; g4 < DL_ROWS; g4 += 4) {
        const f32x4 v = {LG[(g4 + 0) * K + k], LG[(g4 + 1) * K + k], LG[(g4 + 2) * K + k], LG[(g4 + 3) * K + k]};
        cs += (v[0] + v[1]) + (v[2] + v[3]);
        store4T(dTg + a.d_off[L] + (long long)k * a.Bpad + r0 + g4, v);
      }
      a.bpart[(long long)blockIdx.x * (a.bias_total + 1) + a.bias_off[L] + k] = cs;
    }
  } else if (wv == 0) {
    const int nin = a.n[L - 1], K = a.K;
    const T* Wo = Wg + a.w_off[L - 1];
    const bool vec = (nin % VE == 0) && (a.w_off[L - 1] % VE == 0);
    const f32x4 acc = tile_mm(S + a.lds_off[L - 1], a.ld[L - 1], Wo, nin, 0, K, a.kp[L - 1], nin, vec);
    const bool cok = c < K;
    const float b = cok ? a.P[a.b_off[L - 1] + c] : 0.f;
    f32x4 g;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * q + r;
      const float o = cok ? acc[r] + b : -INFINITY;
      const float wr = ws[row];
      if (a.ae) {
        const long long gr = srow[row];
        g[r] = (cok && gr >= 0) ? 2.f * (o - to_f(Zg[gr * a.ldz + c])) * wr / (float)K : 0.f;
      } else if (a.regression) {
        g[r] = (c == 0) ? (o - sy[row]) * wr : 0.f;
      } else {
        float mx = o;
        for (int m = 1; m < 16; m <<= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
        const float e = cok ? __expf(o - mx) : 0.f;
        float z = e;
        for (int m = 1; m < 16; m <<= 1) z += __shfl_xor(z, m, 64);
        g[r] = cok ? (e / z - (scls[row] == c ? 1.f : 0.f)) * wr : 0.f;
      }
      GO[row * a.ld[L] + c] = from_f<T>(g[r]);
    }
    const float cs = col_sum(g);
    if (q == 0 && cok) a.bpart[(long long)blockIdx.x * (a.bias_total + 1) + a.bias_off[L] + c] = cs;
    if (cok) store4T(dTg + a.d_off[L] + (long long)c * a.Bpad + r0 + 4 * q, g);
  }
  __syncthreads();
  DLT(8);
  // ---- backward through the hidden layers
  const T* Gin = GO;
  int ldg_in = a.ld[L];
  for (int l = L - 1; l >= 1; --l) {
    T* Gout = S + a.lds_g[l & 1];
    const int nout = a.n[l], nnext = a.ng[l + 1];     // layer l+1's GEMM width (its WT rows)
    const int ldo = a.ldg[l];
    const unsigned char* win = a.maxout ? smem + a.lds_mx[l] : nullptr;
    const T* WTl = WTg + a.w_off[l];
    const bool vec = (nnext % VE == 0) && (a.w_off[l] % VE == 0);
    const float drop = a.drop[l - 1], keep = 1.f - drop;
    const uint32_t thr = (uint32_t)(drop * 4294967296.0);
    const uint64_t seed = a.seed_base[l - 1] ^ (step * 0x9E3779B97F4A7C15ULL);
    const T* H = S + a.lds_off[l];
    const int NT = (nout + 15) / 16;
    for (int t = wv; t < NT; t += DL_NW) {
      // dh = G_{l+1} W_{l+1}: B[k = unit of l+1][n = unit of l] = WT_{l+1}[n][k]
      const f32x4 acc = tile_mm(Gin, ldg_in, WTl, nnext, t * 16, nout, a.kpg[l + 1], nnext, vec);
      const int col = t * 16 + c;
      f32x4 gd = {0.f, 0.f, 0.f, 0.f};
      if (col < nout) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * q + r;
          float y = to_f(H[row * a.ld[l] + col]);
          float gg = acc[r];
          if (drop > 0.f) {
            const bool d = dropped(seed, (int64_t)(r0 + row) * nout + col, thr);
            gg = d ? 0.f : gg / keep;
            y = d ? 0.f : y * keep;
          }
          gd[r] = a.maxout ? gg : gg * dact_from_y(a.act, y);
        }
      }
      if (!a.maxout) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Gout[(4 * q + r) * ldo + col] = from_f<T>(gd[r]);
        const float cs = col_sum(gd);
        if (col < nout) {
          if (q == 0) a.bpart[(long long)blockIdx.x * (a.bias_total + 1) + a.bias_off[l] + col] = cs;
          store4T(dTg + a.d_off[l] + (long long)col * a.Bpad + r0 + 4 * q, gd);
        }
      } else {
        // the gradient flows to the winning channel only: GEMM columns col (channel 0) and nout + col (channel 1)
        f32x4 g0, g1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool w1 = col < nout && win[(4 * q + r) * nout + col] != 0;
          g0[r] = w1 ? 0.f : gd[r];
          g1[r] = w1 ? gd[r] : 0.f;
        }
        const float cs0 = col_sum(g0), cs1 = col_sum(g1);
        if (col < nout) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            Gout[(4 * q + r) * ldo + col] = from_f<T>(g0[r]);
            Gout[(4 * q + r) * ldo + nout + col] = from_f<T>(g1[r]);
          }
          if (q == 0) {
            a.bpart[(long long)blockIdx.x * (a.bias_total + 1) + a.bias_off[l] + col] = cs0;
            a.bpart[(long long)blockIdx.x * (a.bias_total + 1) + a.bias_off[l] + nout + col] = cs1;
          }
          store4T(dTg + a.d_off[l] + (long long)col * a.Bpad + r0 + 4 * q, g0);
          store4T(dTg + a.d_off[l] + (long long)(nout + col) * a.Bpad + r0 + 4 * q, g1);
        }
      }
    }
    __syncthreads();
    // zero the K padding of the gradient tile the next layer reads (columns past the written ones)
    {
      const int w0 = a.maxout ? 2 * nout : NT * 16;
      const int wz = a.kpg[l] - w0;
      for (int i = tid; i < DL_ROWS * wz; i += DL_THREADS) {
        const int rr = i / wz, cc = w0 + i % wz;
        Gout[rr * ldo + cc] = from_f<T>(0.f);
      }
    }
    __syncthreads();
    DLT(8 + l);
    Gin = Gout;
    ldg_in = ldo;
  }
  if (tid == 0) {
    float s = 0.f;
    for (int i = 0; i < DL_ROWS; ++i) s += ws[i];
    a.bpart[(long long)blockIdx.x * (a.bias_total + 1) + a.bias_total] = s;
  }
  DLT(15);
}

// dW_l[i][j] = sum_rows dA_l[row][i] h_{l-1}[row][j]: A[i][k = row] = dT_l[i][row], B[k = row][j] = hT_{l-1}[j][row].
// Workgroup = one 32 x 32 tile of one layer (2 x 2 MFMA tiles per wave); wave w accumulates row chunks
// w, w + 8, w + 16, ... (32 rows each); partial tiles meet in LDS and wave 0 sums them in wave order.
// Workgroups past the weight tiles reduce bias gradients from the k_dl_rows partials (wave = bias).
// dW_l[i][j] = sum_rows dA_l[row][i] h_{l-1}[row][j]: A[i][k = row] = dT_l[i][row], B[k = row][j] = hT_{l-1}[j][row]
// (both operands contiguous along the batch rows = GEMM K). One 64 x 64 output tile per (tile, split) workgroup of
// 4 waves: the batch rows are cut into `wsplit` ranges (enough workgroups to fill the chip) and each wave takes
// every 4th chunk of its workgroup's range with all 16 MFMA tiles of the 64 x 64 block in registers (per chunk 4 A
// and 4 B fragments feed 16 MFMAs). The 4 waves meet in LDS in wave order, the split partials in a global buffer,
// and k_dl_wsum sums them in split order (deterministic) into the gradient.
// MEASURED (r4): 32 x 32 tiles re-read every operand row 7-25 times from L2 (225 MB per fp32 step, 92 us).
// bf16: 32-row chunks, 8 rows per lane quarter (v_mfma_f32_16x16x32_bf16); fp32: 16-row chunks, 4 rows per lane
// quarter and 4 v_mfma_f32_16x16x4_f32 each.
#define WG4 4
// operand fragments of one chunk: 4 A rows-blocks and 4 B column-blocks per lane
struct FragB { bf16x8 a[4], b[4]; };
struct FragF { float4 a[4], b[4]; };
__device__ __forceinline__ void wg_load(FragB& f, const bf16* const (&ar)[4], const bf16* const (&br)[4],
                                        const bool (&aok)[4], const bool (&bok)[4], int ch) {
  const bf16x8 z8 = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f.a[u] = aok[u] ? *reinterpret_cast<const bf16x8*>(ar[u] + ch * 32) : z8;
    f.b[u] = bok[u] ? *reinterpret_cast<const bf16x8*>(br[u] + ch * 32) : z8;
  }
}
__device__ __forceinline__ void wg_load(FragF& f, const float* const (&ar)[4], const float* const (&br)[4],
                                        const bool (&aok)[4], const bool (&bok)[4], int ch) {
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f.a[u] = aok[u] ? *reinterpret_cast<const float4*>(ar[u] + ch * 16) : z4;
    f.b[u] = bok[u] ? *reinterpret_cast<const float4*>(br[u] + ch * 16) : z4;
  }
}
__device__ __forceinline__ void wg_mma(const FragB& f, f32x4 (&acc)[4][4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[u], f.b[v], acc[u][v], 0, 0, 0);
}
__device__ __forceinline__ void wg_mma(const FragF& f, f32x4 (&acc)[4][4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[u].x, f.b[v].x, acc[u][v], 0, 0, 0);
      acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[u].y, f.b[v].y, acc[u][v], 0, 0, 0);
      acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[u].z, f.b[v].z, acc[u][v], 0, 0, 0);
      acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[u].w, f.b[v].w, acc[u][v], 0, 0, 0);
    }
}
template <typename T> struct FragOf;
template <> struct FragOf<bf16> { typedef FragB type; };
template <> struct FragOf<float> { typedef FragF type; };

template <typename T>
__global__ __launch_bounds__(WG4 * 64) void k_dl_wgrad(DLArgs a, int G1, int scale_by_w) {
  __shared__ float red[WG4 - 1][16 * 4][64];
  __shared__ float s_sw;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int bst = a.bias_total + 1;
  const int S = a.wsplit;
  const int tiles = a.tile_start[a.L];
  if ((int)blockIdx.x >= tiles * S) {
    // trailing workgroups: sum(w) of the batch (fixed order) and the bias gradients
    if (wv == 0) {
      float sacc = 0.f;
      for (int g = lane; g < G1; g += 64) sacc += a.bpart[(long long)g * bst + a.bias_total];
      for (int o = 32; o > 0; o >>= 1) sacc += __shfl_xor(sacc, o, 64);
      if (lane == 0) s_sw = sacc;
    }
    __syncthreads();
    const float sw = s_sw;
    const float inv = scale_by_w ? 1.f / fmaxf(sw, 1e-12f) : 1.f;
    const int e = ((int)blockIdx.x - tiles * S) * WG4 + wv;
    if (e == 0 && lane == 0) {
      a.wpart[(long long)tiles * S * 4096] = inv;          // for k_dl_wsum
      if (!scale_by_w && a.gsum) *a.gsum = sw;
    }
    if (e >= a.bias_total) return;
    float sacc = 0.f;
    for (int g = lane; g < G1; g += 64) sacc += a.bpart[(long long)g * bst + e];
    for (int o = 32; o > 0; o >>= 1) sacc += __shfl_xor(sacc, o, 64);
    if (lane == 0) {
      int l = 1;
      while (l < a.L && e >= a.bias_off[l + 1]) ++l;
      a.g[a.b_off[l - 1] + (e - a.bias_off[l])] = sacc * inv;
    }
    return;
  }
  const int b = (int)blockIdx.x / S, sp = (int)blockIdx.x - b * S;
  int l = 0;
  while (l + 1 < a.L && b >= a.tile_start[l + 1]) ++l;          // GEMM layer l + 1 (0-based l)
  const int bt = b - a.tile_start[l];
  const int ti = bt / a.tiles_j[l], tj = bt - ti * a.tiles_j[l];
  const int ni = a.ng[l + 1], nj = a.n[l];
  const int i0 = ti * 64, j0 = tj * 64;
  const T* Ab = reinterpret_cast<const T*>(a.dT) + a.d_off[l + 1];
  const T* Bb = reinterpret_cast<const T*>(a.hT) + a.h_off[l];
  constexpr int CH = sizeof(T) == 2 ? 32 : 16;      // batch rows per chunk
  constexpr int LPQ = CH / 4;                       // rows per lane quarter
  f32x4 acc[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[u][v] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const T* ar[4];
  const T* br[4];
  bool aok[4], bok[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + u * 16 + c, j = j0 + u * 16 + c;
    aok[u] = i < ni; bok[u] = j < nj;
    ar[u] = Ab + (long long)(aok[u] ? i : 0) * a.Bpad + LPQ * q;
    br[u] = Bb + (long long)(bok[u] ? j : 0) * a.Bpad + LPQ * q;
  }
  const int nch = a.Bpad / CH;
  const int c0 = (int)((long long)nch * sp / S), c1 = (int)((long long)nch * (sp + 1) / S);
  // two-stage pipeline: the next chunk's fragments load while this chunk's MFMAs issue
  typename FragOf<T>::type f0, f1;
  int ch = c0 + wv;
  if (ch < c1) wg_load(f0, ar, br, aok, bok, ch);
  while (ch < c1) {
    const int n1 = ch + WG4;
    if (n1 < c1) wg_load(f1, ar, br, aok, bok, n1);
    wg_mma(f0, acc);
    if (n1 >= c1) break;
    const int n2 = n1 + WG4;
    if (n2 < c1) wg_load(f0, ar, br, aok, bok, n2);
    wg_mma(f1, acc);
    ch = n2;
  }
  // the 4 waves' tiles meet in LDS (wave order)
  if (wv > 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wv - 1][(u * 4 + v) * 4 + r][lane] = acc[u][v][r];
  }
  __syncthreads();
  const long long tile_off = (long long)b * S * 4096;
  float* mine = a.wpart + tile_off + (long long)sp * 4096;
  if (wv == 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = acc[u][v][r];
          for (int w = 0; w < WG4 - 1; ++w) t += red[w][(u * 4 + v) * 4 + r][lane];
          // partial tile element (row 16u + 4q + r, col 16v + c)
          mine[(u * 16 + 4 * q + r) * 64 + v * 16 + c] = t;
        }
  }
}

// dW = (sum over the split partials in split order) * inv, one thread per tile element (the next launch on the
// stream sees every partial: no cross-workgroup fences — an agent-scope release per workgroup wrote back L2)
__global__ __launch_bounds__(256) void k_dl_wsum(DLArgs a) {
  const int S = a.wsplit;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = (int)(e >> 12), el = (int)(e & 4095);
  if (b >= a.tile_start[a.L]) return;
  const float inv = a.wpart[(long long)a.tile_start[a.L] * S * 4096];   // 1 / sum(w) or 1 (k_dl_wgrad)
  int l = 0;
  while (l + 1 < a.L && b >= a.tile_start[l + 1]) ++l;
  const int bt = b - a.tile_start[l];
  const int ti = bt / a.tiles_j[l], tj = bt - ti * a.tiles_j[l];
  const int i = ti * 64 + (el >> 6), j = tj * 64 + (el & 63);
  const int ni = a.ng[l + 1], nj = a.n[l];
  if (i >= ni || j >= nj) return;
  const float* ps = a.wpart + (long long)b * S * 4096 + el;
  float t = 0.f;
  for (int s2 = 0; s2 < S; ++s2) t += ps[(long long)s2 * 4096];
  a.g[a.w_off[l] + (long long)i * nj + j] = t * inv;
}


// WT_l[j][i] = W_l[i][j] for every layer (the bf16 shadow the backward pass reads)
template <typename T>
__global__ __launch_bounds__(256) void k_dl_transpose(DLArgs a) {
  const T* W = reinterpret_cast<const T*>(a.W);
  T* WT = reinterpret_cast<T*>(a.WT);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < a.n_decay; e += (long long)gridDim.x * blockDim.x) {
    int l = 0;
    while (l + 1 < a.L && e >= a.w_off[l + 1]) ++l;
    const long long o = e - a.w_off[l];
    const int nin = a.n[l], i = (int)(o / nin), j = (int)(o - (long long)i * nin);
    WT[a.w_off[l] + (long long)j * a.ng[l + 1] + i] = W[e];
  }
}

}  // namespace

extern "C" {

int h2o_dl_args_size() { return (int)sizeof(DLArgs); }

// lds: bytes of dynamic LDS for k_dl_rows (activation + gradient tiles + row weights)
int h2o_dl_step(const DLArgs* a, int lds, int scale_by_w, hipStream_t s) {
  if (a->L < 1 || a->L > DL_MAXL || (a->K > 16 && ((a->regression && !a->ae) || a->lds_lg <= 0)) || a->Bpad % 128 != 0 ||
      lds > 160 * 1024)
    return (int)hipErrorInvalidValue;
  const int G1 = a->Bpad / DL_ROWS;
  if (a->wsplit < 1 || !a->wpart) return (int)hipErrorInvalidValue;
  const unsigned gsum_blocks = (unsigned)(((long long)a->tile_start[a->L] * 4096 + 255) / 256);
  const int bias_blocks = (a->bias_total + WG4 - 1) / WG4;
  const dim3 gw(a->tile_start[a->L] * a->wsplit + bias_blocks);
  if (a->f32) {
    hipLaunchKernelGGL(k_dl_rows<float>, dim3(G1), dim3(DL_THREADS), lds, s, *a);
    hipLaunchKernelGGL(k_dl_wgrad<float>, gw, dim3(WG4 * 64), 0, s, *a, G1, scale_by_w);
    if (!a->no_wsum) hipLaunchKernelGGL(k_dl_wsum, dim3(gsum_blocks), dim3(256), 0, s, *a);
  } else {
    hipLaunchKernelGGL(k_dl_rows<bf16>, dim3(G1), dim3(DL_THREADS), lds, s, *a);
    hipLaunchKernelGGL(k_dl_wgrad<bf16>, gw, dim3(WG4 * 64), 0, s, *a, G1, scale_by_w);
    if (!a->no_wsum) hipLaunchKernelGGL(k_dl_wsum, dim3(gsum_blocks), dim3(256), 0, s, *a);
  }
  return (int)hipGetLastError();
}

int h2o_dl_transpose(const DLArgs* a, hipStream_t s) {
  long long grid = (a->n_decay + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (a->f32) hipLaunchKernelGGL(k_dl_transpose<float>, dim3((unsigned)grid), dim3(256), 0, s, *a);
  else hipLaunchKernelGGL(k_dl_transpose<bf16>, dim3((unsigned)grid), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

}  // extern "C"

#ifdef DL_TIMING
extern "C" int h2o_dl_timing(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dl_t), sizeof(unsigned long long) * (size_t)n, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
