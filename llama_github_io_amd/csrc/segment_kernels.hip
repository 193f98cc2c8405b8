// Grouped sums into few segments (ops/segment.py): out[s] = sum_{i : idx[i] == s} v[i].
//
// Reference role: the per-class / per-cluster / per-group reductions of the metric builders and
// MRTask reduces (e.g. hex/ModelMetricsClustering.java, hex/ModelMetricsMultinomial.java confusion
// matrix). torch.bincount(weights=fp64) lowers to global fp64 atomics on n addresses: with n = 10
// every atomic serialises at the memory side (MEASURED r3: 13.8 ms per 1M rows, 91 % of a KMeans job).
// Here every block privatises the n segment sums in LDS (ds_add_f64), writes its partial row, and a
// second launch sums the partials of each segment in block order. Only that cross-block order is fixed: the
// LDS atomics inside a block land in scheduling order, so the fp64 sums are not bit-reproducible run to run.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

template <typename I, typename T>
__global__ __launch_bounds__(256) void k_segsum_partial(const I* __restrict__ idx, const T* __restrict__ v, int64_t N,
                                                        int n, int64_t per, double* __restrict__ partial) {
  extern __shared__ double h[];
  for (int s = threadIdx.x; s < n; s += blockDim.x) h[s] = 0.0;
  __syncthreads();
  const int64_t a = (int64_t)blockIdx.x * per, b = a + per < N ? a + per : N;
  for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
    const int64_t s = (int64_t)idx[i];
    if (s >= 0 && s < n) atomicAdd(h + s, (double)v[i]);
  }
  __syncthreads();
  for (int s = threadIdx.x; s < n; s += blockDim.x) partial[(int64_t)blockIdx.x * n + s] = h[s];
}

__global__ void k_segsum_reduce(const double* __restrict__ partial, int G, int n, double* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  double acc = 0.0;
  for (int g = 0; g < G; ++g) acc += partial[(int64_t)g * n + s];
  out[s] = acc;
}

}  // namespace

extern "C" {

// idx_bytes: 4 (int32) or 8 (int64); val_bytes: 4 (float) or 8 (double). partial: [G][n] doubles.
int h2o_segsum(const void* idx, int idx_bytes, const void* v, int val_bytes, long long N, int n, int G, void* partial,
               void* out, hipStream_t s) {
  if (n <= 0 || n > 16384 || G <= 0 || N < 0) return (int)hipErrorInvalidValue;
  const int64_t per = (N + G - 1) / G;
  const size_t lds = (size_t)n * sizeof(double);
#define SEG(I, T) hipLaunchKernelGGL((k_segsum_partial<I, T>), dim3(G), dim3(256), lds, s, (const I*)idx, (const T*)v, \
                                     (int64_t)N, n, per, (double*)partial)
  if (idx_bytes == 8 && val_bytes == 8) SEG(int64_t, double);
  else if (idx_bytes == 8 && val_bytes == 4) SEG(int64_t, float);
  else if (idx_bytes == 4 && val_bytes == 8) SEG(int32_t, double);
  else if (idx_bytes == 4 && val_bytes == 4) SEG(int32_t, float);
  else return (int)hipErrorInvalidValue;
#undef SEG
  hipLaunchKernelGGL(k_segsum_reduce, dim3((n + 255) / 256), dim3(256), 0, s, (const double*)partial, G, n,
                     (double*)out);
  return (int)hipGetLastError();
}

}  // extern "C"
