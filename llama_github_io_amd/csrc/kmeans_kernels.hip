// K-Means Lloyd step: fused squared-distance + argmin over all centers (reference:
// h2o-algos/src/main/java/hex/kmeans/KMeans.java, LloydsIterationTask.map / closest()).
//
// One workgroup = 256 rows. The center matrix (K x P) and the 256-row tile (padded to P+1 floats
// per row so the per-thread row reads hit distinct banks) are staged in LDS; every lane then owns
// one row and sweeps the centers with LDS-broadcast center reads (all lanes read the same word:
// no bank conflict). Output: closest center id and its squared distance per row; the per-center
// sums/counts are one device index_add on the host stream.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

namespace {

__global__ __launch_bounds__(256) void k_kmeans_assign(const float* __restrict__ X, int64_t N, int P,
                                                       const float* __restrict__ C, int K,
                                                       int* __restrict__ assign, float* __restrict__ mind) {
  extern __shared__ float sm[];
  float* Cs = sm;
  float* Xs = sm + (size_t)K * P;
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  for (int i = tid; i < K * P; i += 256) Cs[i] = C[i];
  const int rows = (int)((N - r0) < 256 ? (N - r0) : 256);
  for (int i = tid; i < rows * P; i += 256) {
    const int rr = i / P, cc = i - rr * P;
    Xs[rr * (P + 1) + cc] = X[(r0 + rr) * (int64_t)P + cc];
  }
  __syncthreads();
  if (tid >= rows) return;
  const float* xr = Xs + tid * (P + 1);
  float best = FLT_MAX;
  int bk = 0;
  for (int k = 0; k < K; ++k) {
    const float* c = Cs + k * P;
    float d = 0.f;
    int p = 0;
    for (; p + 4 <= P; p += 4) {
      const float t0 = xr[p] - c[p], t1 = xr[p + 1] - c[p + 1], t2 = xr[p + 2] - c[p + 2], t3 = xr[p + 3] - c[p + 3];
      d = fmaf(t0, t0, d); d = fmaf(t1, t1, d); d = fmaf(t2, t2, d); d = fmaf(t3, t3, d);
    }
    for (; p < P; ++p) { const float t = xr[p] - c[p]; d = fmaf(t, t, d); }
    if (d < best) { best = d; bk = k; }
  }
  assign[r0 + tid] = bk;
  mind[r0 + tid] = best;
}

// Lloyd step: assignment + per-block centroid partial sums. Rows are already in LDS, so each
// thread owns (center, dim) pairs and sweeps the block's rows: no atomics at all (a device-wide
// index_add into K*P addresses serializes ~N/K adds per address). Partials: slab[block][K][P+1]
// (last = weighted count), summed in fp64 by the caller.
__global__ __launch_bounds__(256) void k_kmeans_step(const float* __restrict__ X, int64_t N, int P,
                                                     const float* __restrict__ C, int K, const float* __restrict__ w,
                                                     int* __restrict__ assign, float* __restrict__ mind,
                                                     float* __restrict__ slab) {
  extern __shared__ float sm[];
  float* Cs = sm;
  float* Xs = sm + (size_t)K * P;
  int* sa = (int*)(Xs + 256 * (P + 1));
  float* sw = (float*)(sa + 256);
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  for (int i = tid; i < K * P; i += 256) Cs[i] = C[i];
  const int rows = (int)((N - r0) < 256 ? (N - r0) : 256);
  for (int i = tid; i < rows * P; i += 256) {
    const int rr = i / P, cc = i - rr * P;
    Xs[rr * (P + 1) + cc] = X[(r0 + rr) * (int64_t)P + cc];
  }
  __syncthreads();
  int bk = -1;
  if (tid < rows) {
    const float* xr = Xs + tid * (P + 1);
    float best = FLT_MAX;
    bk = 0;
    for (int k = 0; k < K; ++k) {
      const float* c = Cs + k * P;
      float d = 0.f;
      for (int p = 0; p < P; ++p) { const float t = xr[p] - c[p]; d = fmaf(t, t, d); }
      if (d < best) { best = d; bk = k; }
    }
    assign[r0 + tid] = bk;
    mind[r0 + tid] = best;
  }
  sa[tid] = bk;
  sw[tid] = (tid < rows) ? (w ? w[r0 + tid] : 1.f) : 0.f;
  __syncthreads();
  float* out = slab + (size_t)blockIdx.x * K * (P + 1);
  for (int pair = tid; pair < K * (P + 1); pair += 256) {
    const int k = pair / (P + 1), p = pair - k * (P + 1);
    float acc = 0.f;
    if (p < P) {
      for (int r = 0; r < rows; ++r) acc += (sa[r] == k) ? sw[r] * Xs[r * (P + 1) + p] : 0.f;
    } else {
      for (int r = 0; r < rows; ++r) acc += (sa[r] == k) ? sw[r] : 0.f;
    }
    out[pair] = acc;
  }
}

}  // namespace

extern "C" {

int h2o_kmeans_lds_bytes(int K, int P) { return (K * P + 256 * (P + 1)) * 4; }

int h2o_kmeans_assign(const float* X, long long N, int P, const float* C, int K, int* assign, float* mind,
                      hipStream_t stream) {
  const size_t lds = (size_t)(K * P + 256 * (P + 1)) * 4;
  if (lds > 160 * 1024 || N <= 0) return (int)hipErrorInvalidValue;
  const int grid = (int)((N + 255) / 256);
  hipLaunchKernelGGL(k_kmeans_assign, dim3(grid), dim3(256), lds, stream, X, (int64_t)N, P, C, K, assign, mind);
  return (int)hipGetLastError();
}

int h2o_kmeans_step(const float* X, long long N, int P, const float* C, int K, const float* w, int* assign, float* mind,
                    float* slab, hipStream_t stream) {
  const size_t lds = (size_t)(K * P + 256 * (P + 1) + 512) * 4;
  if (lds > 160 * 1024 || N <= 0) return (int)hipErrorInvalidValue;
  const int grid = (int)((N + 255) / 256);
  hipLaunchKernelGGL(k_kmeans_step, dim3(grid), dim3(256), lds, stream, X, (int64_t)N, P, C, K, w, assign, mind, slab);
  return (int)hipGetLastError();
}

}  // extern "C"
