// Device-resident input stream for gfx950: the batches of
// data_utils.py:176-196's tf.data pipeline
//   from_tensor_slices / CsvDataset -> shuffle(n, seed,
//   reshuffle_each_iteration=True) -> repeat() -> batch(B)
// produced on the device from the resident triple array, one launch per
// batch and no host work: output row b is stream position p = start + b,
// i.e. row pi_e(p mod n) of epoch e = p div n (batches straddle epochs as
// repeat().batch() does). pi_e is a stateless per-epoch permutation -- a
// 4-round Feistel network keyed by Philox4x32-10 and cycle-walked onto
// [0, n) (include/kge_hip.h kge_stream_desc) -- so no permutation array is
// needed; callers that stream many batches per epoch materialise pi_e once
// (kge_stream_permutation) and gather. Integer work only: one thread per row.
#include <algorithm>

#include "kge_step.h"

namespace kge {

// one Feistel pass over w = 2h bits
__device__ __forceinline__ uint64_t feistel_pass(uint64_t x, int h, PhiloxKey key, uint64_t epoch) {
  const uint64_t mask = (h >= 32) ? 0xFFFFFFFFull : ((1ull << h) - 1ull);
  uint64_t L = x >> h, R = x & mask;
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    const uint4 w = philox4x32_10(make_uint4((uint32_t)R, r, (uint32_t)epoch, (uint32_t)(epoch >> 32)), key);
    const uint64_t nl = R;
    R = (L ^ (uint64_t)w.x) & mask;
    L = nl;
  }
  return (L << h) | R;
}

// pi_epoch(k) on [0, n): cycle-walk the w-bit permutation (terminates: k's
// cycle returns to k < n)
__device__ __forceinline__ uint64_t stream_perm(uint64_t k, uint64_t n, int h, PhiloxKey key, uint64_t epoch) {
  uint64_t y = feistel_pass(k, h, key, epoch);
  while (y >= n) y = feistel_pass(y, h, key, epoch);
  return y;
}

template <typename T>
__global__ __launch_bounds__(256) void stream_batch_kernel(const T* __restrict__ tri, int64_t n, int64_t start,
                                                           int64_t batch, int h, PhiloxKey key, int shuffle,
                                                           T* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const uint64_t p = (uint64_t)(start + b);
  const uint64_t e = p / (uint64_t)n, k = p % (uint64_t)n;
  const uint64_t row = shuffle ? stream_perm(k, (uint64_t)n, h, key, e) : k;
  const T* src = tri + row * 3;
  T* dst = out + b * 3;
  dst[0] = src[0];
  dst[1] = src[1];
  dst[2] = src[2];
}

// Materialised permutations (kge_stream_permutation / kge_stream_batch_perm):
// the cycle walk is a dependent chain of Philox rounds -- at FB15k-237 size
// (n = 272,115 on a 2^20 domain, 26 % of values in range) the slowest of a
// batch's 1,024 rows walks ~20 times, ~23 us per batch launch. Computed once
// per epoch for all n positions in parallel, a batch becomes a gather.
__global__ __launch_bounds__(256) void stream_perm_kernel(int64_t n, int h, PhiloxKey key, uint64_t epoch,
                                                          int32_t* __restrict__ perm) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  perm[k] = (int32_t)stream_perm((uint64_t)k, (uint64_t)n, h, key, epoch);
}

template <typename T>
__global__ __launch_bounds__(256) void stream_gather_kernel(const T* __restrict__ tri, int64_t n, int64_t start,
                                                            int64_t batch, const int32_t* __restrict__ plo,
                                                            const int32_t* __restrict__ phi, int64_t e0,
                                                            T* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const int64_t p = start + b;
  const int64_t e = p / n, k = p - e * n;
  const int64_t row = (e == e0 ? plo : phi)[k];
  const T* src = tri + row * 3;
  T* dst = out + b * 3;
  dst[0] = src[0];
  dst[1] = src[1];
  dst[2] = src[2];
}

static int stream_half_bits(int64_t n) {
  int w = 2;
  while (w < 64 && (1ull << w) < (uint64_t)n) w += 2;
  return w / 2;
}

void launch_stream_perm(int64_t n, uint64_t seed, int64_t epoch, int32_t* perm, hipStream_t st) {
  const PhiloxKey key{(uint32_t)seed, (uint32_t)(seed >> 32)};
  hipLaunchKernelGGL(stream_perm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n,
                     stream_half_bits(n), key, (uint64_t)epoch, perm);
}

void launch_stream_gather(const void* tri, bool i64, int64_t n, int64_t start, int64_t batch, const int32_t* plo,
                          const int32_t* phi, int64_t e0, void* out, hipStream_t st) {
  const unsigned blocks = (unsigned)((batch + 255) / 256);
  if (i64)
    hipLaunchKernelGGL(stream_gather_kernel<int64_t>, dim3(blocks), dim3(256), 0, st, (const int64_t*)tri, n, start,
                       batch, plo, phi, e0, (int64_t*)out);
  else
    hipLaunchKernelGGL(stream_gather_kernel<int32_t>, dim3(blocks), dim3(256), 0, st, (const int32_t*)tri, n, start,
                       batch, plo, phi, e0, (int32_t*)out);
}

// ---- weight histograms (kge_histogram): per-workgroup LDS bins, one
// global 64-bit add per non-empty bin and workgroup
__global__ __launch_bounds__(256) void histogram_kernel(const float* __restrict__ x, int64_t n,
                                                        const double* __restrict__ lw, int bc,
                                                        unsigned long long* __restrict__ counts) {
  __shared__ unsigned int s_bin[256];
  for (int k = threadIdx.x; k < bc; k += 256) s_bin[k] = 0u;
  __syncthreads();
  const double lo = lw[0], width = lw[1];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double y = floor(((double)x[i] - lo) / width);
    const int k = !(y >= 0.0) ? 0 : (y >= (double)(bc - 1) ? bc - 1 : (int)y);
    atomicAdd(&s_bin[k], 1u);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < bc; k += 256)
    if (s_bin[k]) atomicAdd(&counts[k], (unsigned long long)s_bin[k]);
}

void launch_histogram(const float* x, int64_t n, const double* lw, int bc, unsigned long long* counts,
                      hipStream_t st) {
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 1024);
  hipLaunchKernelGGL(histogram_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, lw, bc, counts);
}

// ---- kge_copy16: the streaming copy bench.py measures the HBM peak with.
// One pass, no grid-stride loop: workgroup b copies the contiguous 16 KiB
// [b * 1024, (b + 1) * 1024) float4s, each lane four of them 4 KiB apart,
// every load issued before any store, non-temporal both ways (the fastest of
// the variants tools/copy_peak.hip measures: 6.2 TB/s vs 4.5-5.4 for
// grid-stride loops and 4.9 for hipMemcpy, profiles/r05c/copy_peak.txt)
typedef float kge_v4f __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy16_kernel(const kge_v4f* __restrict__ src, kge_v4f* __restrict__ dst,
                                                     int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  kge_v4f v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * 256 < n) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * 256 < n) __builtin_nontemporal_store(v[u], dst + base + u * 256);
}

void launch_copy16(const void* src, void* dst, int64_t n16, hipStream_t st) {
  const int64_t blocks = (n16 + 1023) / 1024;   // (kge_copy16 caps n16 at 2^40)
  hipLaunchKernelGGL(copy16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const kge_v4f*)src, (kge_v4f*)dst,
                     n16);
}

void launch_stream(const void* tri, bool i64, int64_t n, int64_t start, int64_t batch, uint64_t seed, int shuffle,
                   void* out, hipStream_t st) {
  const int w = 2 * stream_half_bits(n);
  const PhiloxKey key{(uint32_t)seed, (uint32_t)(seed >> 32)};
  const unsigned blocks = (unsigned)((batch + 255) / 256);
  if (i64)
    hipLaunchKernelGGL(stream_batch_kernel<int64_t>, dim3(blocks), dim3(256), 0, st, (const int64_t*)tri, n, start,
                       batch, w / 2, key, shuffle, (int64_t*)out);
  else
    hipLaunchKernelGGL(stream_batch_kernel<int32_t>, dim3(blocks), dim3(256), 0, st, (const int32_t*)tri, n, start,
                       batch, w / 2, key, shuffle, (int32_t*)out);
}

}  // namespace kge
