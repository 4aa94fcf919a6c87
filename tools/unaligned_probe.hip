// Probe: do global loads at byte-misaligned addresses return the bytes at
// that address on this GPU (ROCm's unaligned mode for global memory)?
// dword, dwordx2 and dwordx4 loads at every byte offset 0..63.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void k(const uint8_t* src, uint64_t* out, uint32_t* out32,
                  uint4* out128) {
  const int i = threadIdx.x;  // byte offset
  out[i] = *reinterpret_cast<const uint64_t*>(src + i);
  out32[i] = *reinterpret_cast<const uint32_t*>(src + i);
  out128[i] = *reinterpret_cast<const uint4*>(src + i);
}

int main() {
  uint8_t h[256];
  for (int i = 0; i < 256; ++i) h[i] = (uint8_t)(i * 37 + 11);
  uint8_t* d; uint64_t* o; uint32_t* o32; uint4* o128;
  hipMalloc(&d, 256); hipMalloc(&o, 64 * 8); hipMalloc(&o32, 64 * 4);
  hipMalloc(&o128, 64 * 16);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, o32, o128);
  uint64_t r[64]; uint32_t r32[64]; uint8_t r128[64 * 16];
  hipMemcpy(r, o, 64 * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r32, o32, 64 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(r128, o128, 64 * 16, hipMemcpyDeviceToHost);
  int bad = 0, bad128 = 0;
  for (int i = 0; i < 64; ++i) {
    uint64_t e; uint32_t e32;
    memcpy(&e, h + i, 8); memcpy(&e32, h + i, 4);
    if (e != r[i] || e32 != r32[i]) ++bad;
    if (memcmp(r128 + 16 * i, h + i, 16)) {
      if (bad128 < 4) {
        printf("x4 off %d:", i);
        for (int b = 0; b < 16; ++b) printf(" %02x/%02x", r128[16 * i + b], h[i + b]);
        printf("\n");
      }
      ++bad128;
    }
  }
  printf("unaligned probe: %d dword/dwordx2 mismatches, %d dwordx4 mismatches of 64\n",
         bad, bad128);
  return (bad || bad128) != 0;
}
