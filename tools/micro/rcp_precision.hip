// Accuracy of v_rcp_f64 and of one / two Newton-Raphson refinements against
// IEEE 1/x on random doubles (how many refinements rcp_nr needs).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

__global__ void k(const double *x, double *r0, double *r1, double *r2, double *q, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = x[i];
  double r = __builtin_amdgcn_rcp(v);
  r0[i] = r;
  double e = fma(-v, r, 1.0);
  double ra = fma(r, e, r);
  r1[i] = ra;
  e = fma(-v, ra, 1.0);
  r2[i] = fma(ra, e, ra);
  q[i] = 1.0 / v;
}

int main() {
  const int n = 1 << 22;
  std::vector<double> h(n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-30.0, 30.0);
  for (int i = 0; i < n; ++i) h[i] = std::ldexp(1.0 + (g() >> 12) * 0x1p-52, (int)u(g)) * ((g() & 1) ? 1 : -1);
  double *d[5];
  for (auto &p : d) hipMalloc(&p, n * sizeof(double));
  hipMemcpy(d[0], h.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d[0], d[1], d[2], d[3], d[4], n);
  std::vector<double> a(n), b(n), c(n), q(n);
  hipMemcpy(a.data(), d[1], n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), d[2], n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), d[3], n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(q.data(), d[4], n * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0, m2 = 0;
  long long ne0 = 0, ne1 = 0, ne2 = 0;
  for (int i = 0; i < n; ++i) {
    const double ref = 1.0 / h[i];
    m0 = std::fmax(m0, std::fabs(a[i] - ref) / std::fabs(ref));
    m1 = std::fmax(m1, std::fabs(b[i] - ref) / std::fabs(ref));
    m2 = std::fmax(m2, std::fabs(c[i] - ref) / std::fabs(ref));
    ne0 += a[i] != ref;
    ne1 += b[i] != ref;
    ne2 += c[i] != ref;
  }
  printf("rcp: max rel %.3g (%lld/%d not IEEE)  +1 NR: %.3g (%lld)  +2 NR: %.3g (%lld)\n", m0, ne0, n,
         m1, ne1, m2, ne2);
  return 0;
}
