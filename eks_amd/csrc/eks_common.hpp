// Shared helpers of the EKS HIP translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>

#include "small_linalg.hpp"

namespace eks {

constexpr double kLog2Pi = 1.8378770664093453;  // log(2 pi)
constexpr double kLn2 = 0.6931471805599453;

constexpr int kMaxLatent = 6;   // r
constexpr int kMaxObs = 8;      // n (compiled kernels, eks_forward / eks_backward / eks_fit)
constexpr int kMaxObsRt = 64;   // n of eks_smooth's runtime-n kernel (eks_shape_rt.hip)
constexpr int kMaxMembers = 64; // E

int set_err(int code, const char *fmt, ...);
int check_launch(const char *what);
void clear_err();

// Optional per-kernel timing (eks_profile_begin/end): records a hipEvent on
// the launch stream before each kernel of an eks_smooth call and after the
// last one.  No-op unless profiling was switched on by the caller.
void prof_mark(hipStream_t s, const char *next_kernel);
void prof_call_begin();
void prof_call_end(hipStream_t s);
void prof_suspend(bool on);

template <int R>
EKS_DEV void load_vec(const double *p, double (&v)[R]) {
#pragma unroll
  for (int i = 0; i < R; ++i) v[i] = p[i];
}
template <int R>
EKS_DEV void store_vec(double *p, const double (&v)[R]) {
#pragma unroll
  for (int i = 0; i < R; ++i) p[i] = v[i];
}
template <int R, int C>
EKS_DEV void load_mat(const double *p, double (&M)[R][C]) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) M[i][j] = p[i * C + j];
}
template <int R, int C>
EKS_DEV void store_mat(double *p, const double (&M)[R][C]) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) p[i * C + j] = M[i][j];
}

// Packed per-trajectory model: [m0 | S0 | A | Q | C | offset]
template <int R, int N>
struct ParamLayout {
  static constexpr int m0 = 0;
  static constexpr int S0 = R;
  static constexpr int A = R + R * R;
  static constexpr int Q = R + 2 * R * R;
  static constexpr int C = R + 3 * R * R;
  static constexpr int off = R + 3 * R * R + N * R;
  static constexpr int len = R + 3 * R * R + N * R + N;
};

inline long long param_len(int n, int r) { return (long long)r + 3LL * r * r + (long long)n * r + n; }

// byte offset of the ev planes in a y / ev hand-off buffer (eks_yev_bytes)
__host__ __device__ inline size_t yev_ev_offset(long long B, long long T, int n, size_t ysize) {
  return ((size_t)T * n * B * ysize + 255) / 256 * 256;
}

inline unsigned grid_for(long long work, int block) {
  long long g = (work + block - 1) / block;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace eks

#include <type_traits>

namespace eks {

template <int V>
using ic = std::integral_constant<int, V>;

// r in [1, kMaxLatent]
template <typename F>
int dispatch_r(int r, F &&f) {
  switch (r) {
    case 1: return f(ic<1>{});
    case 2: return f(ic<2>{});
    case 3: return f(ic<3>{});
    case 4: return f(ic<4>{});
    case 5: return f(ic<5>{});
    case 6: return f(ic<6>{});
    default: return set_err(2 /*EKS_ERR_UNSUPPORTED*/, "latent dimension r=%d not supported (1..%d)", r, kMaxLatent);
  }
}

// n in [1, kMaxObs]
template <typename F>
int dispatch_n(int n, F &&f) {
  switch (n) {
    case 1: return f(ic<1>{});
    case 2: return f(ic<2>{});
    case 3: return f(ic<3>{});
    case 4: return f(ic<4>{});
    case 5: return f(ic<5>{});
    case 6: return f(ic<6>{});
    case 7: return f(ic<7>{});
    case 8: return f(ic<8>{});
    default: return set_err(2 /*EKS_ERR_UNSUPPORTED*/, "observation dimension n=%d not supported (1..%d)", n, kMaxObs);
  }
}

}  // namespace eks
