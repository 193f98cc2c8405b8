// Fused GBM row kernel (reference: hex/tree/gbm/GBM.java AddTreeContributions + ComputePredAndRes,
// hex/DistributionFactory.java negHalfGradient / gammaNum / gammaDenom).
//
// One pass over the rows per boosting iteration does what used to be ~30 small torch kernels:
//   f[i] += leaf_value[leaf_of_row[i]]        (previous tree's contribution; optional)
//   w_eff = w[i] * Bernoulli(sample_rate)     (row sampling, counter-based hash: no RNG state)
//   z = negHalfGradient(y, f); num/den = gammaNum/gammaDenom
//   aux[c][i] = (w_eff, w_eff*z, num, den) as four SoA planes (the histogram passes read only what they need)
//   block maxima of the four |planes| -> fixed-point scales of the histograms and of the leaf sums
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AMAX_SHARDS 64  // must match tree_kernels.hip

enum Dist { D_GAUSSIAN = 0, D_BERNOULLI = 1, D_QUASIBINOMIAL = 2, D_POISSON = 3, D_GAMMA = 4, D_TWEEDIE = 5,
            D_LAPLACE = 6, D_QUANTILE = 7, D_HUBER = 8, D_MODIFIED_HUBER = 9,
            // XGBoost binary:logistic (hex/tree/xgboost ObjFunction): Newton planes w = h, wY = -g
            D_XGB_LOGISTIC = 10 };

__device__ __forceinline__ unsigned long long smix(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float expc(float x) { return __expf(fminf(x, 80.f)); }

__global__ __launch_bounds__(256) void k_gbm_step(
    long long N, long long row0, int dist, const float* __restrict__ y, const float* __restrict__ w, float* __restrict__ f,
    const float* __restrict__ vals, const int* __restrict__ leaf, float sample_rate, unsigned long long seed,
    float p1 /*tweedie power | quantile alpha | huber delta*/, float* __restrict__ aux /*[4][N]*/,
    unsigned* __restrict__ amax_bits /*[AMAX_SHARDS][4], |.| as uint bits, pre-zeroed*/, int skip) {
  float ma = 0.f, mb = 0.f, mc = 0.f, md = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long long)gridDim.x * blockDim.x) {
    float fi = f[i];
    if (vals) { fi += vals[leaf[i]]; f[i] = fi; }
    float wi = w ? w[i] : 1.f;
    if (sample_rate < 1.f) {
      // keyed by the GLOBAL row index (row0 = this rank's first row): a row-sharded run samples exactly
      // the rows of the single-GPU run
      const float u = (float)(smix(seed ^ (unsigned long long)(row0 + i)) >> 40) * (1.0f / 16777216.0f);
      if (u >= sample_rate) wi = 0.f;
    }
    const float yi = y[i];
    float z, num, den;
    float p0 = wi;                     // plane 0: the histogram weight (w; XGBoost: the hessian)
    switch (dist) {
      case D_XGB_LOGISTIC: {
        const float p = 1.f / (1.f + expc(-fi));
        const float h = fmaxf(p * (1.f - p), 1e-16f);
        z = yi - p; num = wi * z; den = wi * h; p0 = den; break;
      }
      case D_BERNOULLI: {
        const float p = 1.f / (1.f + expc(-fi));
        z = yi - p; num = wi * z; den = wi * p * (1.f - p); break;
      }
      case D_QUASIBINOMIAL: {
        const float p = 1.f / (1.f + expc(-fi));
        z = (p == yi) ? 0.f : (p > 1.f ? yi / p : (p < 0.f ? (1.f - yi) / (p - 1.f) : yi - p));
        const float ff = yi - z;
        num = wi * z; den = wi * ff * (1.f - ff); break;
      }
      case D_POISSON: {
        const float mu = expc(fi);
        z = yi - mu; num = wi * yi; den = wi * mu; break;
      }
      case D_GAMMA: {
        z = yi * expc(-fi) - 1.f; num = wi * (z + 1.f); den = wi; break;
      }
      case D_TWEEDIE: {
        const float a = expc(fi * (1.f - p1)), b = expc(fi * (2.f - p1));
        z = yi * a - b; num = wi * yi * a; den = wi * b; break;
      }
      case D_LAPLACE: { z = fi > yi ? -0.5f : 0.5f; num = wi * z; den = wi; break; }
      case D_QUANTILE: { z = yi > fi ? 0.5f * p1 : 0.5f * (p1 - 1.f); num = wi * z; den = wi; break; }
      case D_HUBER: {
        const float r = yi - fi;
        z = fabsf(r) <= p1 ? r : (fi >= yi ? -p1 : p1); num = wi * z; den = wi; break;
      }
      case D_MODIFIED_HUBER: {
        const float s = 2.f * yi - 1.f, yf = s * fi;
        if (yf < -1.f) { z = 2.f * s; num = wi * 4.f * s; den = -wi * 4.f * yf; }
        else if (yf > 1.f) { z = 0.f; num = 0.f; den = 0.f; }
        else { z = -fi * s * s; num = wi * 2.f * s * (1.f - yf); den = wi * (1.f - yf) * (1.f - yf); }
        break;
      }
      default: { z = yi - fi; num = wi * z; den = wi; }
    }
    const float wz = wi * z;
    // skip bit 0: plane 0 is never read (unit weights: the histograms drop w); bit 2: num == wz for this
    // distribution and the leaf sums read plane 1 instead (88 of the pass's 352 MB at 11M rows)
    if (!(skip & 1)) aux[i] = p0;
    aux[N + i] = wz;
    if (!(skip & 4)) aux[2 * N + i] = num;
    aux[3 * N + i] = den;
    ma = fmaxf(ma, fabsf(p0));
    mb = fmaxf(mb, fabsf(wz));
    mc = fmaxf(mc, fabsf(num));
    md = fmaxf(md, fabsf(den));
  }
  // block max -> ONE atomic per component per block into one of AMAX_SHARDS shards (k_qscale folds the
  // shards): a single hot word would serialize every wave's atomic (~12 ns each at the memory side)
  for (int off = 32; off > 0; off >>= 1) {
    ma = fmaxf(ma, __shfl_xor(ma, off, 64));
    mb = fmaxf(mb, __shfl_xor(mb, off, 64));
    mc = fmaxf(mc, __shfl_xor(mc, off, 64));
    md = fmaxf(md, __shfl_xor(md, off, 64));
  }
  __shared__ float sm[4][4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[0][wv] = ma; sm[1][wv] = mb; sm[2][wv] = mc; sm[3][wv] = md; }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int c = threadIdx.x;
    float v = sm[c][0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) v = fmaxf(v, sm[c][k]);
    // non-negative floats order like their bit patterns
    atomicMax(amax_bits + 4 * (blockIdx.x & (AMAX_SHARDS - 1)) + c, __float_as_uint(v));
  }
}

// f[i] += vals[leaf[i]] only (final tree / multinomial classes)
__global__ void k_add_leaf(long long N, float* __restrict__ f, int fstride, const float* __restrict__ vals,
                           const int* __restrict__ leaf) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long long)gridDim.x * blockDim.x)
    f[i * fstride] += vals[leaf[i]];
}

extern "C" {
int h2o_gbm_step(long long N, long long row0, int dist, const void* y, const void* w, void* f, const void* vals, const void* leaf,
                 float sample_rate, unsigned long long seed, float p1, void* aux, void* amax_bits, int skip,
                 hipStream_t s) {
  const int blk = 256;
  long long grid = (N + blk - 1) / blk;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_gbm_step, dim3((unsigned)grid), dim3(blk), 0, s, N, row0, dist, (const float*)y, (const float*)w,
                     (float*)f, (const float*)vals, (const int*)leaf, sample_rate, seed, p1, (float*)aux,
                     (unsigned*)amax_bits, skip);
  return (int)hipGetLastError();
}

int h2o_add_leaf(long long N, void* f, int fstride, const void* vals, const void* leaf, hipStream_t s) {
  const int blk = 256;
  long long grid = (N + blk - 1) / blk;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_add_leaf, dim3((unsigned)grid), dim3(blk), 0, s, N, (float*)f, fstride, (const float*)vals,
                     (const int*)leaf);
  return (int)hipGetLastError();
}
}
