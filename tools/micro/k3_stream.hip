// Micro-benchmark: the HBM rate of algo 3's member stream alone (k3_fwd's
// unit geometry: 64 trajectories x 4 waves x 32 steps, E = 5 float32 members
// x 2 coordinates per step, a D-step register ring, non-temporal loads,
// time-chunk-major unit order, 1024 x 17 x 10 000 trajectory-steps = 6.96 GB)
// under three member layouts:
//   0  [t][e][j][b]          (today: 10 loads of 256 B per wave-step, rows B*4 B apart)
//   1  [t][g][e][j][64]      (64-trajectory groups blocked: one 2.5 KB block per wave-step)
//   2  [g][t][e][j][64]      (group-major: each wave streams contiguous memory over time)
// and with F dependent FP64 FMAs per step and lane added (4 chains) -- the
// FP64 work of the real passes (~110-130 per step) -- to see what the work
// costs beside the stream (power: the shader clock, from s_memtime over the
// launch, is printed too).
// Prints TB/s per (layout, ring depth, grid, F) over 20 launches.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int E = 5, N = 2, KW = 4, SPW = 32;  // waves per unit, steps per wave

template <int LAYOUT>
__device__ __forceinline__ long long idx(long long t, int e, int j, long long b, long long B, long long T) {
  const long long g = b >> 6, l = b & 63;
  if (LAYOUT == 0) return ((t * E + e) * N + j) * B + b;
  if (LAYOUT == 1) return (((t * (B >> 6) + g) * E + e) * N + j) * 64 + l;
  return (((g * T + t) * E + e) * N + j) * 64 + l;
}

template <int LAYOUT, int D, int F = 0, bool W = false>
__global__ __launch_bounds__(256) void k_stream(const float *__restrict__ obs, long long B, long long T,
                                                long long units, unsigned *ctr, double *sink,
                                                unsigned long long *clk, float *ypl, double *evpl) {
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = __builtin_amdgcn_s_memtime();
  __shared__ unsigned tk;
  const long long ng = B / 64;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double acc = 0.0;
  while (true) {
    if (threadIdx.x == 0) tk = atomicAdd(ctr, 1u);
    __syncthreads();
    const long long u = __builtin_amdgcn_readfirstlane(tk);
    __syncthreads();
    if (u >= units) break;
    const long long c = u / ng, g = u % ng;
    const long long b = g * 64 + l;
    const long long s = (c * KW + w) * SPW;
    if (s >= T) continue;
    float v[D][E][N];
    auto fetch = [&](int q, long long t) {
#pragma unroll
      for (int e = 0; e < E; ++e)
#pragma unroll
        for (int j = 0; j < N; ++j) v[q][e][j] = __builtin_nontemporal_load(obs + idx<LAYOUT>(t, e, j, b, B, T));
    };
#pragma unroll
    for (int q = 0; q < D; ++q) fetch(q, s + q);
#pragma unroll 1
    for (int i0 = 0; i0 < SPW; i0 += D) {
#pragma unroll
      for (int q = 0; q < D; ++q) {
        double m = 0.0;
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int j = 0; j < N; ++j) m += (double)v[q][e][j];
        acc = fma(acc, 0.999, m);
        if constexpr (W) {  // the y (f32) / ev (f64) planes k3_bwd would read: 24 B per step
          const long long t = s + i0 + q;
          float2 yv = make_float2(v[q][0][0], v[q][0][1]);
          __builtin_nontemporal_store(yv.x, ypl + (t * B + b) * 2);
          __builtin_nontemporal_store(yv.y, ypl + (t * B + b) * 2 + 1);
          __builtin_nontemporal_store(m, evpl + (t * B + b) * 2);
          __builtin_nontemporal_store(m * 0.5, evpl + (t * B + b) * 2 + 1);
        }
        if constexpr (F > 0) {
          double c0 = m, c1 = m + 1.0, c2 = m + 2.0, c3 = m + 3.0;
#pragma unroll
          for (int k = 0; k < F / 4; ++k) {
            c0 = fma(c0, 0.9999, 1e-3);
            c1 = fma(c1, 0.9999, 1e-3);
            c2 = fma(c2, 0.9999, 1e-3);
            c3 = fma(c3, 0.9999, 1e-3);
          }
          acc += (c0 + c1) + (c2 + c3);
        }
        fetch(q, min(s + i0 + q + D, s + SPW - 1));
      }
    }
  }
  if (acc == 1234.5) sink[blockIdx.x] = acc;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[1] = __builtin_amdgcn_s_memtime();
}

static float *g_ypl = nullptr;
static double *g_evpl = nullptr;
template <int LAYOUT, int D, int F = 0, bool W = false>
void run(const float *obs, long long B, long long T, unsigned *ctr, double *sink, int grid) {
  static unsigned long long *clk = nullptr;
  if (!clk) (void)hipMalloc(&clk, 16);
  const long long units = (T / (KW * SPW)) * (B / 64);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9, tot = 0;
  const int reps = 20;
  for (int r = 0; r < reps + 2; ++r) {
    hipMemsetAsync(ctr, 0, 4);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_stream<LAYOUT, D, F, W>), dim3(grid), dim3(256), 0, 0, obs, B, T, units, ctr, sink, clk,
                       g_ypl, g_evpl);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (r >= 2) {
      tot += ms;
      if (ms < best) best = ms;
    }
  }
  const double bytes = (double)(units * KW * SPW) * 64 * E * N * 4;
  unsigned long long c[2];
  (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
  float last;
  hipEventElapsedTime(&last, a, b);
  printf("%s layout %d D %d F %3d grid %5d: mean %.3f ms (%.2f TB/s)  best %.3f ms (%.2f TB/s)  block-0 clock %.2f GHz\n",
         W ? "+planes" : "reads  ", LAYOUT, D, F, grid, tot / reps, bytes / (tot / reps * 1e-3) / 1e12, best,
         bytes / (best * 1e-3) / 1e12, (double)(c[1] - c[0]) / (last * 1e-3) / 1e9);
}

// pixel-like member values (hash of the index): random bits as the real
// workload has (zero-filled inputs switch less and run at a higher clock,
// MI355X_MICROARCH.md, DVFS give-back)
__global__ void k_fill(float *obs, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned h = (unsigned)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    obs[i] = 100.0f + (float)(h & 0xFFFFFF) * (500.0f / 16777216.0f);
  }
}

int main(int argc, char **argv) {
  const bool zero = argc > 1 && argv[1][0] == 'z';
  const long long B = 17408, T = 10240;  // T a multiple of the 128-step unit
  const size_t n = (size_t)T * E * N * B;
  float *obs;
  unsigned *ctr;
  double *sink;
  hipMalloc(&obs, n * 4);
  hipMalloc(&ctr, 4);
  hipMalloc(&sink, 1 << 20);
  if (zero) (void)hipMemset(obs, 0, n * 4);
  else hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, obs, n);
  printf("members: %s\n", zero ? "zero-filled" : "pixel-like random");
  (void)hipMalloc(&g_ypl, (size_t)T * B * 2 * 4);
  (void)hipMalloc(&g_evpl, (size_t)T * B * 2 * 8);
  for (int grid : {512}) {
    run<0, 2>(obs, B, T, ctr, sink, grid);
    run<0, 2, 0, true>(obs, B, T, ctr, sink, grid);
    run<0, 2, 64>(obs, B, T, ctr, sink, grid);
    run<0, 2, 64, true>(obs, B, T, ctr, sink, grid);
    run<0, 2, 128>(obs, B, T, ctr, sink, grid);
    run<0, 2, 128, true>(obs, B, T, ctr, sink, grid);
  }
  return 0;
}
