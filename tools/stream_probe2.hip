// stream_probe2.hip — read-bandwidth ceilings of per-series wave streams
// (one wavefront streams one series' ts+val columns) by access shape and
// load policy: K consecutive points per lane (what k_fold does, each
// wave-instruction touching 16 B of every 64 B) vs lane-contiguous
// instructions (1 KB per wave-instruction), default vs non-temporal loads.
// Prints ms and GB/s.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef long long ll2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ ll2 ld(const ll2* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

template <bool NT>
__global__ void grid_stride(const ll2* a, const ll2* b, size_t n2, long long* out) {
  long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2;
       i += (size_t)gridDim.x * blockDim.x) {
    ll2 x = ld<NT>(a + i), y = ld<NT>(b + i);
    acc += x.x ^ y.y;
  }
  if (acc == 42) out[0] = acc;
}

// K consecutive points per lane (k_fold's shape)
template <int K, bool NT>
__global__ __launch_bounds__(256) void per_series(const long long* ts, const long long* val,
                           long long seg, long long nseg, long long* out) {
  const int lane = threadIdx.x & 63;
  const long long s = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;
  const long long lo = s * seg, hi = lo + seg;
  long long acc = 0;
  for (long long base = lo; base < hi; base += 64 * K) {
    const long long i0 = base + K * lane;
    if (i0 + K <= hi) {
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        ll2 x = ld<NT>((const ll2*)(ts + i0 + j)), y = ld<NT>((const ll2*)(val + i0 + j));
        acc += x.x ^ y.y;
      }
    }
  }
  if (acc == 42) out[0] = acc;
}

// lane-contiguous: instruction j reads points base + 128 j + 2 lane (+1)
template <int K, bool NT>
__global__ __launch_bounds__(256) void per_series_c(const long long* ts, const long long* val,
                           long long seg, long long nseg, long long* out) {
  const int lane = threadIdx.x & 63;
  const long long s = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;
  const long long lo = s * seg, hi = lo + seg;
  long long acc = 0;
  for (long long base = lo; base < hi; base += 64 * K) {
    if (base + 64 * K <= hi) {
#pragma unroll
      for (int j = 0; j < K / 2; ++j) {
        const long long i = base + 128 * j + 2 * lane;
        ll2 x = ld<NT>((const ll2*)(ts + i)), y = ld<NT>((const ll2*)(val + i));
        acc += x.x ^ y.y;
      }
    }
  }
  if (acc == 42) out[0] = acc;
}

// byte stream (the cells fold's value loads): lane reads NL x 16 B at
// stride STR bytes per lane from a running cursor, unaligned by +1 per step
template <int NL, int STR, bool NT>
__global__ __launch_bounds__(256) void bytes_lane(const unsigned char* p, long long seg,
                           long long nseg, long long* out) {
  const int lane = threadIdx.x & 63;
  const long long s = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;
  const unsigned char* b = p + s * seg;
  long long acc = 0;
  unsigned cur = 0;
  const unsigned lim = (unsigned)(seg - 64 * STR - 64);
  for (int it = 0; cur < lim; ++it) {
    const unsigned a = cur + STR * lane + (it & 1);
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const u4 w = NT ? __builtin_nontemporal_load((const u4*)(b + a + 16 * i))
                      : *(const u4*)(b + a + 16 * i);
      acc += w.x ^ w.w;
    }
    cur += 64 * STR;
  }
  if (acc == 42) out[0] = acc;
}

int main(int argc, char** argv) {
  const long long seg = 57344, nseg = argc > 1 ? atoll(argv[1]) : 100000;
  const size_t n = (size_t)seg * nseg;
  long long *ts, *val, *out;
  hipMalloc(&ts, n * 8); hipMalloc(&val, n * 8); hipMalloc(&out, 64);
  hipMemset(ts, 1, n * 8); hipMemset(val, 2, n * 8);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    hipEventRecord(a);
    const int R = 5;
    for (int r = 0; r < R; ++r) launch();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms / R, bytes / (ms / R) / 1e6);
  };
  const double B16 = 16.0 * n;
  run("grid_stride 8192x256", B16, [&] { grid_stride<false><<<8192, 256>>>((const ll2*)ts, (const ll2*)val, n / 2, out); });
  run("grid_stride 8192x256 nt", B16, [&] { grid_stride<true><<<8192, 256>>>((const ll2*)ts, (const ll2*)val, n / 2, out); });
  unsigned blocks = (unsigned)((nseg + 3) / 4);
  run("per_series K=8", B16, [&] { per_series<8, false><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  run("per_series K=8 nt", B16, [&] { per_series<8, true><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  run("per_series K=16 nt", B16, [&] { per_series<16, true><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  run("per_series_c K=8", B16, [&] { per_series_c<8, false><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  run("per_series_c K=8 nt", B16, [&] { per_series_c<8, true><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  run("per_series_c K=16 nt", B16, [&] { per_series_c<16, true><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  // cells-like byte stream over the same bytes: 10 B / point, 8 points/lane
  const long long bseg = seg * 10, bn = (long long)(8.0 * n / bseg);
  const unsigned char* bp = (const unsigned char*)ts;
  unsigned bblocks = (unsigned)((bn + 3) / 4);
  run("bytes 5x16B stride80", (double)bseg * bn, [&] { bytes_lane<5, 80, false><<<bblocks, 256>>>(bp, bseg, bn, out); });
  run("bytes 5x16B stride80 nt", (double)bseg * bn, [&] { bytes_lane<5, 80, true><<<bblocks, 256>>>(bp, bseg, bn, out); });
  run("bytes 10x16B stride160 nt", (double)bseg * bn, [&] { bytes_lane<10, 160, true><<<bblocks, 256>>>(bp, bseg, bn, out); });
  return 0;
}
