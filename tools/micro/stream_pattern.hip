// Micro-benchmark: achievable HBM rate of the smoother's access patterns.
//  A: time-major planes, one dword load per (t, e, j) per lane (K1 today)
//  B: same, plus 24 B/kp-ts of plane stores (y f32 + ev f64), like K1
//  C: blocked layout [t/4][e][j][b][4]: one 16-byte load per (4 t, e, j)
//  D: C plus the stores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int E = 5, N = 2;

template <bool STORE, bool NT = false, bool NTL = false>
__global__ __launch_bounds__(256) void k_planes(const float *obs, long long B, long long T,
                                                long long L, float *y, double *ev, double *sink) {
  const long long lane = blockIdx.x * 256ll + threadIdx.x;
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
      for (int j = 0; j < N; ++j) {
        const float *q = obs + ((t * E + u) * N + j) * B + b;
        v[u][j] = NTL ? __builtin_nontemporal_load(q) : *q;
      }
    double m0 = 0, m1 = 0;
#pragma unroll
    for (int u = 0; u < E; ++u) {
      m0 += v[u][0];
      m1 += v[u][1];
    }
    acc += m0 * 1e-9 + m1;
    if (STORE) {
      if (NT) {
        __builtin_nontemporal_store(v[2][0], y + (t * N + 0) * B + b);
        __builtin_nontemporal_store(v[2][1], y + (t * N + 1) * B + b);
        __builtin_nontemporal_store(m0, ev + (t * N + 0) * B + b);
        __builtin_nontemporal_store(m1, ev + (t * N + 1) * B + b);
      } else {
        y[(t * N + 0) * B + b] = v[2][0];
        y[(t * N + 1) * B + b] = v[2][1];
        ev[(t * N + 0) * B + b] = m0;
        ev[(t * N + 1) * B + b] = m1;
      }
    }
  }
  if (acc == 1234.5) sink[lane] = acc;
}

template <bool STORE>
__global__ __launch_bounds__(256) void k_blocked(const float4 *obs, long long B, long long T,
                                                 long long L, float4 *y, double *ev,
                                                 double *sink) {
  const long long nc = (T + L - 1) / L;
  const long long bpc = (B + 255) / 256;
  const long long c = blockIdx.x / bpc;
  const long long b = (blockIdx.x % bpc) * 256 + threadIdx.x;
  if (c >= nc || b >= B) return;
  double acc = 0.0;
  const long long s = c * L / 4, e = min(T, (c + 1) * L) / 4;
  for (long long t4 = s; t4 < e; ++t4) {
    float4 v[E][N];
#pragma unroll
    for (int u = 0; u < E; ++u)
#pragma unroll
      for (int j = 0; j < N; ++j) v[u][j] = obs[((t4 * E + u) * N + j) * B + b];
    double m0 = 0, m1 = 0;
#pragma unroll
    for (int u = 0; u < E; ++u) {
      m0 += v[u][0].x + v[u][0].y + v[u][0].z + v[u][0].w;
      m1 += v[u][1].x + v[u][1].y + v[u][1].z + v[u][1].w;
    }
    acc += m0 * 1e-9 + m1;
    if (STORE) {
      y[(t4 * N + 0) * B + b] = v[2][0];
      y[(t4 * N + 1) * B + b] = v[2][1];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ev[((t4 * 4 + k) * N + 0) * B + b] = m0 + k;
        ev[((t4 * 4 + k) * N + 1) * B + b] = m1 + k;
      }
    }
  }
  if (acc == 1234.5) sink[b] = acc;
}

int main() {
  const long long B = 17408, T = 10000, L = 625;
  const size_t nobs = (size_t)T * E * N * B;
  float *obs, *y;
  double *ev, *sink;
  hipMalloc(&obs, nobs * 4);
  hipMalloc(&y, (size_t)T * N * B * 4);
  hipMalloc(&ev, (size_t)T * N * B * 8);
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
  const double rd = (double)nobs * 4, wr = (double)T * N * B * 12;
  time("planes dword loads", [&] { hipLaunchKernelGGL(k_planes<false>, grid, dim3(256), 0, 0, obs, B, T, L, y, ev, sink); }, rd);
  time("planes dword + stores", [&] { hipLaunchKernelGGL(k_planes<true>, grid, dim3(256), 0, 0, obs, B, T, L, y, ev, sink); }, rd + wr);
  time("planes + nt stores", [&] { hipLaunchKernelGGL((k_planes<true, true>), grid, dim3(256), 0, 0, obs, B, T, L, y, ev, sink); }, rd + wr);
  time("planes nt loads + nt stores", [&] { hipLaunchKernelGGL((k_planes<true, true, true>), grid, dim3(256), 0, 0, obs, B, T, L, y, ev, sink); }, rd + wr);
  time("planes nt loads", [&] { hipLaunchKernelGGL((k_planes<false, false, true>), grid, dim3(256), 0, 0, obs, B, T, L, y, ev, sink); }, rd);
  time("blocked 16B loads", [&] { hipLaunchKernelGGL(k_blocked<false>, grid, dim3(256), 0, 0, (const float4 *)obs, B, T, L, (float4 *)y, ev, sink); }, rd);
  time("blocked 16B + stores", [&] { hipLaunchKernelGGL(k_blocked<true>, grid, dim3(256), 0, 0, (const float4 *)obs, B, T, L, (float4 *)y, ev, sink); }, rd + wr);
  return 0;
}
