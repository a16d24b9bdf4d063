// Micro-benchmark: achievable HBM rate of algo 3's final-pass access pattern
// (tools/micro/stream_pattern.hip covers algo 2's).  Lanes = (16-step chunk,
// trajectory); per step each lane reads E x 2 float32 member planes (40 B)
// and writes one (x, y) float64 pair (16 B) into a time-major (T, B, 2)
// output.  Variants: loads only, + 16-B stores, + nt stores, 2 x 8-B stores.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int E = 5, N = 2, L = 16;

template <int MODE>  // 0 loads only, 1 double2 stores, 2 nt double2 stores, 3 two 8-B stores
__global__ __launch_bounds__(256) void k_final(const float *obs, long long B, long long T,
                                               double *out, double *sink) {
  const long long nc = (T + L - 1) / L;
  const long long bpc = (B + 255) / 256;
  const long long c = blockIdx.x / bpc;
  const long long b = (blockIdx.x % bpc) * 256 + threadIdx.x;
  if (c >= nc || b >= B) return;
  double acc = 0.0;
  const long long s = c * L, e = min(T, s + L);
  for (long long t = s; t < e; ++t) {
    float v[E][N];
#pragma unroll
    for (int u = 0; u < E; ++u)
#pragma unroll
      for (int j = 0; j < N; ++j) v[u][j] = obs[((t * E + u) * N + j) * B + b];
    double m0 = 0, m1 = 0;
#pragma unroll
    for (int u = 0; u < E; ++u) {
      m0 += v[u][0];
      m1 += v[u][1];
    }
    acc += m0 * 1e-9 + m1;
    double *o = out + (t * B + b) * 2;
    if (MODE == 1) *(double2 *)o = make_double2(m0, m1);
    if (MODE == 2) {
      __builtin_nontemporal_store(m0, o);
      __builtin_nontemporal_store(m1, o + 1);
    }
    if (MODE == 3) {
      o[0] = m0;
      o[1] = m1;
    }
  }
  if (acc == 1234.5) sink[b] = acc;
}

int main() {
  const long long B = 17408, T = 10000;
  const size_t nobs = (size_t)T * E * N * B;
  float *obs;
  double *out, *sink;
  hipMalloc(&obs, nobs * 4);
  hipMalloc(&out, (size_t)T * B * 16);
  hipMalloc(&sink, 1 << 24);
  hipMemset(obs, 0, nobs * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const long long nc = (T + L - 1) / L, bpc = (B + 255) / 256;
  dim3 grid((unsigned)(nc * bpc));
  auto time = [&](const char *name, auto launch, double bytes) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-28s %.3f ms  %.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const double rd = (double)nobs * 4, wr = (double)T * B * 16;
  time("loads only", [&] { hipLaunchKernelGGL(k_final<0>, grid, dim3(256), 0, 0, obs, B, T, out, sink); }, rd);
  time("loads + double2 stores", [&] { hipLaunchKernelGGL(k_final<1>, grid, dim3(256), 0, 0, obs, B, T, out, sink); }, rd + wr);
  time("loads + nt stores", [&] { hipLaunchKernelGGL(k_final<2>, grid, dim3(256), 0, 0, obs, B, T, out, sink); }, rd + wr);
  time("loads + 2x8B stores", [&] { hipLaunchKernelGGL(k_final<3>, grid, dim3(256), 0, 0, obs, B, T, out, sink); }, rd + wr);
  return 0;
}
