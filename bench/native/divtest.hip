#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <vector>
#include <random>
#include <cstring>
#include <algorithm>
__device__ double div0(double n, double d) {
#pragma clang fp contract(off)
  double r = __builtin_amdgcn_rcp(d);
  double q = n * r;
  return fma(fma(-d, q, n), r, q);
}
__device__ double div1(double n, double d) {
#pragma clang fp contract(off)
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  double q = n * r;
  return fma(fma(-d, q, n), r, q);
}
__global__ void k(const double* n, const double* d, double* o0, double* o1, double* oe, int N) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N) { o0[i] = div0(n[i], d[i]); o1[i] = div1(n[i], d[i]); oe[i] = n[i] / d[i]; }
}
int main() {
  const int N = 1 << 22;
  std::vector<double> n(N), d(N);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(0, 1), e(-60, 60);
  for (int i = 0; i < N; ++i) { n[i] = (u(g) - 0.3) * std::pow(10.0, e(g) / 4); d[i] = (0.5 + u(g)) * std::pow(10.0, e(g)); }
  double *dn, *dd, *o0, *o1, *oe;
  hipMalloc(&dn, N * 8); hipMalloc(&dd, N * 8); hipMalloc(&o0, N * 8); hipMalloc(&o1, N * 8); hipMalloc(&oe, N * 8);
  hipMemcpy(dn, n.data(), N * 8, hipMemcpyHostToDevice); hipMemcpy(dd, d.data(), N * 8, hipMemcpyHostToDevice);
  k<<<N / 256, 256>>>(dn, dd, o0, o1, oe, N);
  std::vector<double> r0(N), r1(N), re(N);
  hipMemcpy(r0.data(), o0, N * 8, hipMemcpyDeviceToHost); hipMemcpy(r1.data(), o1, N * 8, hipMemcpyDeviceToHost); hipMemcpy(re.data(), oe, N * 8, hipMemcpyDeviceToHost);
  auto ulp = [](double a, double b) { int64_t x, y; memcpy(&x, &a, 8); memcpy(&y, &b, 8); return std::llabs(x - y); };
  long long m0 = 0, m1 = 0, c0 = 0, c1 = 0, me = 0;
  for (int i = 0; i < N; ++i) {
    double ex = n[i] / d[i];
    long long a = ulp(r0[i], ex), b = ulp(r1[i], ex), c = ulp(re[i], ex);
    m0 = std::max(m0, a); m1 = std::max(m1, b); me = std::max(me, c); c0 += a != 0; c1 += b != 0;
  }
  printf("max ulp: div0 %lld (inexact %lld of %d), div1 %lld (inexact %lld), hip '/' %lld\n", m0, c0, N, m1, c1, me);
  return 0;
}
