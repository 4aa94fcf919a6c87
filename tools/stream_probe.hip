// stream_probe.hip — read-bandwidth ceiling of the access pattern k_bucketize
// uses (one wavefront streams one series' ts+val columns, K consecutive
// points per lane), vs a plain grid-stride read, on the same 2 x N int64
// buffers.  Prints GB/s.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef long long ll2 __attribute__((ext_vector_type(2)));

__global__ void grid_stride(const ll2* a, const ll2* b, size_t n2, long long* out) {
  long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2;
       i += (size_t)gridDim.x * blockDim.x) {
    ll2 x = a[i], y = b[i];
    acc += x.x ^ y.y;
  }
  if (acc == 42) out[0] = acc;
}

template <int K>
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
        ll2 x = *(const ll2*)(ts + i0 + j), y = *(const ll2*)(val + i0 + j);
        acc += x.x ^ y.y;
      }
    }
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
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    hipEventRecord(a);
    const int R = 5;
    for (int r = 0; r < R; ++r) launch();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-22s %8.3f ms  %7.1f GB/s\n", name, ms / R, 16.0 * n / (ms / R) / 1e6);
  };
  run("grid_stride 2048x256", [&] { grid_stride<<<2048, 256>>>((const ll2*)ts, (const ll2*)val, n / 2, out); });
  run("grid_stride 8192x256", [&] { grid_stride<<<8192, 256>>>((const ll2*)ts, (const ll2*)val, n / 2, out); });
  unsigned blocks = (unsigned)((nseg + 3) / 4);
  run("per_series K=2", [&] { per_series<2><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  run("per_series K=8", [&] { per_series<8><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  run("per_series K=16", [&] { per_series<16><<<blocks, 256>>>(ts, val, seg, nseg, out); });
  return 0;
}
