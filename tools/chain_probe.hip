// chain_probe — how long one sequential Welford chain per bucket takes on
// gfx950 (StdDev.runDouble, Aggregators.java:547-568), the floor of a
// bit-exact cross-series `dev` over a 500k-member group (C4: 1,440 buckets).
//   A: the chain alone (values from a hash, no memory), IEEE division
//   B: the same with the division by n as a reciprocal product corrected to
//      the IEEE quotient (checked, falls back to the division)
//   C: B reading each member's value / state from a [S][NB] row matrix,
//      U members' loads in flight per lane
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/chain_probe.hip -o tools/chain_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ double hashv(uint32_t m, uint32_t b) {
  uint32_t h = m * 2654435761u ^ (b * 40503u + 0x9e3779b9u);
  h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12;
  return 3.0e9 + (double)(h & 0xFFFF);
}

// RN(d / n) from yh = RN(1/n), yl ~ 1/n - yh; exact unless d/n lies within
// 2u^2 of a midpoint, which the remainder test catches (then the division)
__device__ __forceinline__ double div_n(double d, double n, double yh, double yl) {
  const double q = __builtin_fma(d, yh, d * yl);
  const double r = __builtin_fma(-q, n, d);
  const uint64_t qb = (uint64_t)__double_as_longlong(q);
  const uint64_t e = qb & 0x7FF0000000000000ULL;
  const double half_ulp_n = __longlong_as_double((long long)(e - (53ULL << 52))) * n;
  const bool ok = (r == 0.0) | ((__builtin_fabs(r) < half_ulp_n) &
                                ((qb & 0x000FFFFFFFFFFFFFULL) != 0) &
                                (e > (100ULL << 52)) & (e < (2000ULL << 52)));
  return ok ? q : d / n;
}

template <int FAST>
__global__ __launch_bounds__(64) void k_chain_a(int64_t L, int NB, double* out) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  double mean = hashv(0, b), m2 = 0.0;
  double n = 1.0;
  for (int64_t m = 1; m < L; ++m) {
    const double x = hashv((uint32_t)m, b);
    n += 1.0;
    double q;
    if (FAST) {
      const double yh = 1.0 / n;  // off the chain
      const double yl = __builtin_fma(-n, yh, 1.0) / n;
      q = div_n(x - mean, n, yh, yl);
    } else {
      q = (x - mean) / n;
    }
    const double nm = mean + q;
    m2 += (x - mean) * (x - nm);
    mean = nm;
  }
  if (b < NB) out[b] = __builtin_sqrt(m2 / n) + mean * 0.0;
}

template <int FAST, int U>
__global__ __launch_bounds__(64) void k_chain_c(int64_t S, int64_t NB,
                                                const double* __restrict__ val,
                                                const uint8_t* __restrict__ st,
                                                double* out) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t bb = b < NB ? b : NB - 1;
  double mean = 0.0, m2 = 0.0, n = 0.0;
  int emit = 0;
  double xv[U];
  uint8_t sv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    xv[u] = val[(int64_t)u * NB + bb];
    sv[u] = st[(int64_t)u * NB + bb];
  }
  for (int64_t m0 = 0; m0 < S; m0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double x = xv[u];
      const uint8_t s = sv[u];
      const int64_t mn = m0 + U + u < S ? m0 + U + u : S - 1;
      xv[u] = val[mn * NB + bb];
      sv[u] = st[mn * NB + bb];
      if (s && x == x) {
        emit |= s == 2;
        if (n == 0.0) {
          mean = x;
          n = 1.0;
        } else {
          n += 1.0;
          double q;
          if (FAST) {
            const double yh = 1.0 / n;
            const double yl = __builtin_fma(-n, yh, 1.0) / n;
            q = div_n(x - mean, n, yh, yl);
          } else {
            q = (x - mean) / n;
          }
          const double nm = mean + q;
          m2 += (x - mean) * (x - nm);
          mean = nm;
        }
      }
    }
  }
  if (b < NB) out[b] = emit ? __builtin_sqrt(m2 / n) : -1.0;
}

__global__ void k_fill(int64_t n, double* v, uint8_t* s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    v[i] = hashv((uint32_t)(i / 1440), (uint32_t)(i % 1440));
    s[i] = (i % 97) ? 2 : 0;
  }
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t S = argc > 1 ? atoll(argv[1]) : 500000;
  const int64_t NB = 1440;
  double* out;
  CK(hipMalloc(&out, NB * 8));
  const unsigned nblk = (unsigned)((NB + 63) / 64);
  printf("chain_probe: S=%lld members, NB=%lld buckets (%u waves)\n",
         (long long)S, (long long)NB, nblk);
  float t;
  t = timeit([&] { hipLaunchKernelGGL(k_chain_a<0>, dim3(nblk), dim3(64), 0, 0, S, (int)NB, out); }, 2);
  printf("A  ieee div, no memory : %8.3f ms  %6.1f ns/step\n", t, t * 1e6 / S);
  t = timeit([&] { hipLaunchKernelGGL(k_chain_a<1>, dim3(nblk), dim3(64), 0, 0, S, (int)NB, out); }, 2);
  printf("B  fast div, no memory : %8.3f ms  %6.1f ns/step\n", t, t * 1e6 / S);
  double* val;
  uint8_t* st;
  CK(hipMalloc(&val, S * NB * 8));
  CK(hipMalloc(&st, S * NB));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, S * NB, val, st);
  CK(hipDeviceSynchronize());
#define RUNC(F, U)                                                                 \
  t = timeit([&] { hipLaunchKernelGGL((k_chain_c<F, U>), dim3(nblk), dim3(64), 0, 0, \
                                      S, NB, val, st, out); }, 2);                  \
  printf("C  %s div, U=%2d        : %8.3f ms  %6.1f ns/step  %6.1f GB/s\n",       \
         F ? "fast" : "ieee", U, t, t * 1e6 / S, S * NB * 9.0 / t / 1e6);
  RUNC(0, 8) RUNC(1, 8) RUNC(1, 16) RUNC(1, 24) RUNC(0, 24)
  // the same chain over 16 members per lane (the splitting k_group does)
  return 0;
}
