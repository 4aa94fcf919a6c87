// Probe: do global loads at byte-misaligned addresses return the bytes at
// that address on this GPU (ROCm's unaligned mode for global memory)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void k(const uint8_t* src, uint64_t* out, uint32_t* out32) {
  const int i = threadIdx.x;  // byte offset
  out[i] = *reinterpret_cast<const uint64_t*>(src + i);
  out32[i] = *reinterpret_cast<const uint32_t*>(src + i);
}

int main() {
  uint8_t h[256];
  for (int i = 0; i < 256; ++i) h[i] = (uint8_t)(i * 37 + 11);
  uint8_t* d; uint64_t* o; uint32_t* o32;
  hipMalloc(&d, 256); hipMalloc(&o, 64 * 8); hipMalloc(&o32, 64 * 4);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, o32);
  uint64_t r[64]; uint32_t r32[64];
  hipMemcpy(r, o, 64 * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r32, o32, 64 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) {
    uint64_t e; uint32_t e32;
    memcpy(&e, h + i, 8); memcpy(&e32, h + i, 4);
    if (e != r[i] || e32 != r32[i]) ++bad;
  }
  printf("unaligned probe: %d mismatches of 64\n", bad);
  return bad != 0;
}
