// Bandwidth of 8-byte global loads at a misaligned base (stride 8 per lane)
// vs aligned, vs two aligned loads + funnel shift (tools/, not the product).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_unal(const uint8_t* p, int64_t n, int off, uint64_t* out) {
  uint64_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    acc ^= *reinterpret_cast<const uint64_t*>(p + off + 8 * i);
  if (acc == 42) out[0] = acc;
}
__global__ void k_funnel(const uint8_t* p, int64_t n, int off, uint64_t* out) {
  uint64_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uintptr_t a = (uintptr_t)(p + off + 8 * i), al = a & ~(uintptr_t)7;
    const uint64_t w0 = *reinterpret_cast<const uint64_t*>(al);
    const uint64_t w1 = *reinterpret_cast<const uint64_t*>(al + 8);
    const int sh = (int)(a - al) * 8;
    acc ^= sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  }
  if (acc == 42) out[0] = acc;
}
__global__ void k_u16(const uint8_t* p, int64_t n, int off, uint64_t* out) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    acc ^= *reinterpret_cast<const uint16_t*>(p + off + 2 * i);
  if (acc == 42) out[0] = acc;
}

int main() {
  const int64_t bytes = (int64_t)4 << 30;
  uint8_t* p; uint64_t* o;
  hipMalloc(&p, bytes + 64); hipMalloc(&o, 64);
  hipMemset(p, 1, bytes + 64);
  const int64_t n = bytes / 8;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep)
    for (int off : {0, 3}) {
      float ms;
      hipEventRecord(a);
      hipLaunchKernelGGL(k_unal, dim3(8192), dim3(256), 0, 0, p, n, off, o);
      hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
      if (rep) printf("direct  off=%d: %.1f GB/s\n", off, bytes / ms / 1e6);
      hipEventRecord(a);
      hipLaunchKernelGGL(k_funnel, dim3(8192), dim3(256), 0, 0, p, n, off, o);
      hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
      if (rep) printf("funnel  off=%d: %.1f GB/s\n", off, bytes / ms / 1e6);
      hipEventRecord(a);
      hipLaunchKernelGGL(k_u16, dim3(8192), dim3(256), 0, 0, p, bytes / 2 - 8, off, o);
      hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
      if (rep) printf("u16     off=%d: %.1f GB/s\n", off, bytes / ms / 1e6);
    }
  return 0;
}
