// HBM copy-rate microbenchmark (variants of a v4f streaming copy), to pick
// the kernel kge_copy16 uses for bench.py's measured peak.
// build: hipcc --offload-arch=gfx950 -O3 tools/copy_peak.hip -o tools/copy_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stride1(const v4f* __restrict__ s, v4f* __restrict__ d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = s[i];
}
__global__ __launch_bounds__(256) void k_unroll4(const v4f* __restrict__ s, v4f* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += 4 * stride) {
    v4f v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) v[u] = s[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) d[i + u * stride] = v[u];
  }
}
__global__ __launch_bounds__(256) void k_nt4(const v4f* __restrict__ s, v4f* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += 4 * stride) {
    v4f v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) v[u] = __builtin_nontemporal_load(s + i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) __builtin_nontemporal_store(v[u], d + i + u * stride);
  }
}
// one shot: block b copies the contiguous chunk [b * 256 * U, (b + 1) * 256 * U)
template <int U>
__global__ __launch_bounds__(256) void k_chunk(const v4f* __restrict__ s, v4f* __restrict__ d, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  v4f v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) v[u] = __builtin_nontemporal_load(s + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) __builtin_nontemporal_store(v[u], d + base + u * 256);
}
template <int U>
__global__ __launch_bounds__(256) void k_chunk_plain(const v4f* __restrict__ s, v4f* __restrict__ d, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  v4f v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) v[u] = s[base + u * 256];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) d[base + u * 256] = v[u];
}

int main() {
  const int64_t bytes = (int64_t)2 << 30, n = bytes / 16;
  v4f *s, *d;
  if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
  (void)hipMemset(s, 1, bytes);
  (void)hipMemset(d, 0, bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    for (int r = 0; r < 3; ++r) launch();
    (void)hipEventRecord(a);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    printf("%-28s %8.4f ms  %7.1f GB/s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
  };
  for (int g : {2048, 8192, 32768}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stride1 grid %d", g);
    run(nm, [&] { hipLaunchKernelGGL(k_stride1, dim3(g), dim3(256), 0, 0, s, d, n); });
    snprintf(nm, sizeof nm, "unroll4 grid %d", g);
    run(nm, [&] { hipLaunchKernelGGL(k_unroll4, dim3(g), dim3(256), 0, 0, s, d, n); });
    snprintf(nm, sizeof nm, "nt4 grid %d", g);
    run(nm, [&] { hipLaunchKernelGGL(k_nt4, dim3(g), dim3(256), 0, 0, s, d, n); });
  }
  run("chunk nt U=4", [&] { hipLaunchKernelGGL(k_chunk<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, 0, s, d, n); });
  run("chunk nt U=8", [&] { hipLaunchKernelGGL(k_chunk<8>, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, 0, s, d, n); });
  run("chunk plain U=4", [&] { hipLaunchKernelGGL(k_chunk_plain<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, 0, s, d, n); });
  run("chunk plain U=8", [&] { hipLaunchKernelGGL(k_chunk_plain<8>, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, 0, s, d, n); });
  run("hipMemcpyDtoD", [&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); });
  return 0;
}
