// Fused EKS hot path (eks_smooth in include/eks_hip.h):
//   ensemble (eks/ensemble_kalman.py:4-57)  ->  centring
//   -> forward filter (:59-107)  ->  RTS backward (:120-164)
//   -> projection C ms + offset (eks/multiview_pca_smoother.py:745, :756-765)
//
// algo 1, k_smooth_seq: one lane per trajectory, sequential in time.
//   Forward: the measurement update is done one scalar observation at a time
//   (R_t is diagonal), which is algebraically identical to the reference's
//   n x n solve, needs no matrix inverse and tolerates R_t[i,i] = 0 (frames
//   where all members agree).  The filtered mean and the packed upper
//   triangle of the filtered covariance are spilled to a TIME-MAJOR
//   workspace ws[t][k][b] so that the 64 lanes of a wave write (and later
//   read) 64 consecutive doubles per store.  The innovation NLL is
//   accumulated on the way (no extra memory traffic).
//   Backward: S[t] = A Vf[t] A^T + Q is recomputed from the spilled Vf[t]
//   (the reference stores it), J_t = (S[t]^-1 A Vf[t])^T, and only the mean
//   recursion is run (the wrappers discard Vs: :746), then the projection is
//   written straight to `out`.
// Member loads for step t+1 (and workspace loads for step t-1 in the backward
// sweep) are issued before step t's arithmetic, so their HBM latency hides
// under the recursion's dependency chain.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/eks_hip.h"
#include "eks_common.hpp"
#include "ensemble.hpp"
#include "small_linalg.hpp"

namespace eks {

template <int R>
struct Sym {
  static constexpr int len = R * (R + 1) / 2;
  static constexpr int idx(int i, int j) {
    return i <= j ? i * R - i * (i - 1) / 2 + (j - i) : j * R - j * (j - 1) / 2 + (i - j);
  }
};

// Load the E x N member values of one step into registers.
template <int E, int N, typename T>
EKS_DEV void load_members(const T *p, long long se, long long sj, T (&v)[E][N]) {
#pragma unroll
  for (int e = 0; e < E; ++e)
#pragma unroll
    for (int j = 0; j < N; ++j) v[e][j] = p[e * se + j * sj];
}

// ensemble + centring of one step: y = reduce(members) - offset, rv = var
template <int E, int N, typename T>
EKS_DEV void step_observation(const T (&v)[(E > 0 ? E : 1)][N], const T *p, long long se, long long sj, int Ert,
                              bool median, const double (&off)[N], double (&y)[N],
                              double (&rv)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double avg, var;
    if constexpr (E > 0) {
      T col[E];
#pragma unroll
      for (int e = 0; e < E; ++e) col[e] = v[e][j];
      ensemble_reduce<E, T>(col, median, avg, var);
    } else {
      ensemble_reduce_rt<T>(p + j * sj, se, Ert, median, avg, var);
    }
    y[j] = avg - off[j];
    rv[j] = var;
  }
}

// Kalman measurement update with diagonal R, one scalar observation at a time.
// m, P: prior in, posterior out.  Accumulates the innovation NLL terms.
template <int R, int N>
EKS_DEV void update_sequential(double (&m)[R], double (&P)[R][R], const double (&C)[N][R],
                               const double (&y)[N], const double (&rv)[N], double &quad,
                               double &det_m, int &det_e, bool &ok) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double v[R];
#pragma unroll
    for (int a = 0; a < R; ++a) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(P[a][k], C[i][k], s);
      v[a] = s;
    }
    double s = rv[i], hm = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      s = fma(C[i][k], v[k], s);
      hm = fma(C[i][k], m[k], hm);
    }
    ok = ok && !(s <= 0.0);  // NaN propagates as in numpy, not an error
    const double inv = 1.0 / s;
    const double e = y[i] - hm;
    quad = fma(e * e, inv, quad);
    int ex;
    det_m = frexp(det_m * s, &ex);
    det_e += ex;
    const double ei = e * inv;
#pragma unroll
    for (int a = 0; a < R; ++a) m[a] = fma(v[a], ei, m[a]);
#pragma unroll
    for (int a = 0; a < R; ++a) {
      const double ka = v[a] * inv;
#pragma unroll
      for (int c = a; c < R; ++c) {
        P[a][c] = fma(-ka, v[c], P[a][c]);
        if (c != a) P[c][a] = P[a][c];
      }
    }
  }
}

// prior of step t from the posterior of t-1:  m <- A m,  P <- A (P A^T) + Q
template <int R>
EKS_DEV void predict(double (&m)[R], double (&P)[R][R], const double (&A)[R][R],
                     const double (&Q)[R][R]) {
  double PAt[R][R], mp[R];
  matmul_nt<R, R, R>(P, A, PAt);
  matmul<R, R, R>(A, PAt, P);
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) P[i][j] += Q[i][j];
  matvec<R, R>(A, m, mp);
#pragma unroll
  for (int i = 0; i < R; ++i) m[i] = mp[i];
}

// One RTS mean step: given filtered (mf, Vf) at t and smoothed ms at t+1,
// ms <- mf + J (ms - A mf) with J = (S^-1 A Vf)^T, S = A Vf A^T + Q.
template <int R>
EKS_DEV void rts_mean_step(const double (&mf)[R], const double (&Vf)[R][R],
                           const double (&A)[R][R], const double (&Q)[R][R], double (&ms)[R],
                           bool &ok) {
  double VAt[R][R], S[R][R], X[R][R];
  matmul_nt<R, R, R>(Vf, A, VAt);
  matmul<R, R, R>(A, VAt, S);
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) S[i][j] += Q[i][j];
  matmul<R, R, R>(A, Vf, X);
  ok = gauss_solve<R, R>(S, X) && ok;
  double Amf[R], d[R];
  matvec<R, R>(A, mf, Amf);
#pragma unroll
  for (int i = 0; i < R; ++i) d[i] = ms[i] - Amf[i];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) s = fma(X[k][i], d[k], s);
    ms[i] = mf[i] + s;
  }
}

template <int R, int N>
EKS_DEV void write_projection(double *out, long long oj, const double (&C)[N][R],
                              const double (&ms)[R], const double (&off)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double s = off[j];
    // (C ms)_j + offset_j, summed as the reference's dot then add
    double cm = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) cm = fma(C[j][k], ms[k], cm);
    out[j * oj] = cm + s;
  }
}

template <int R, int N, int E, typename T>
__global__ __launch_bounds__(64) void k_smooth_seq(
    const T *__restrict__ obs, long long B, long long TT, int Ert, long long sb, long long st,
    long long se, long long sj, int median_i, const double *__restrict__ params,
    double *__restrict__ out, long long ob, long long ot, long long oj, double *__restrict__ ms_out,
    double *__restrict__ nll, double *__restrict__ ws, int32_t *__restrict__ status) {
  using L = ParamLayout<R, N>;
  constexpr int NS = Sym<R>::len;
  constexpr int K = R + NS;  // doubles spilled per step
  constexpr int EE = E > 0 ? E : 1;
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const bool median = median_i != 0;
  const double *pp = params + b * L::len;
  double m[R], P[R][R], A[R][R], Q[R][R], C[N][R], off[N];
  load_vec<R>(pp + L::m0, m);
  load_mat<R, R>(pp + L::S0, P);
  load_mat<R, R>(pp + L::A, A);
  load_mat<R, R>(pp + L::Q, Q);
  load_mat<N, R>(pp + L::C, C);
  load_vec<N>(pp + L::off, off);

  const T *ob_ = obs + b * sb;
  double *outb = out + b * ob;
  bool ok = true;
  double quad = 0.0, det_m = 1.0;
  int det_e = 0;

  // ---------------- forward sweep ----------------
  T cur[EE][N], nxt[EE][N];
  if constexpr (E > 0) load_members<E, N, T>(ob_, se, sj, cur);
  for (long long t = 0; t < TT; ++t) {
    const T *pt = ob_ + t * st;
    if constexpr (E > 0) {
      if (t + 1 < TT) load_members<E, N, T>(pt + st, se, sj, nxt);
    }
    double y[N], rv[N];
    step_observation<E, N, T>(cur, pt, se, sj, Ert, median, off, y, rv);
    if (t > 0) predict<R>(m, P, A, Q);
    update_sequential<R, N>(m, P, C, y, rv, quad, det_m, det_e, ok);
    double *w = ws + t * K * B + b;
#pragma unroll
    for (int i = 0; i < R; ++i) w[i * B] = m[i];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) w[(R + Sym<R>::idx(i, j)) * B] = P[i][j];
    if constexpr (E > 0) {
#pragma unroll
      for (int e = 0; e < E; ++e)
#pragma unroll
        for (int j = 0; j < N; ++j) cur[e][j] = nxt[e][j];
    }
  }
  if (nll) nll[b] = 0.5 * ((double)TT * N * kLog2Pi + log(det_m) + det_e * kLn2 + quad);

  // ---------------- backward sweep ----------------
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = m[i];
  write_projection<R, N>(outb + (TT - 1) * ot, oj, C, ms, off);
  if (ms_out) store_vec<R>(ms_out + (b * TT + TT - 1) * R, ms);
  double wcur[K], wnxt[K];
  if (TT >= 2) {
    const double *w = ws + (TT - 2) * K * B + b;
#pragma unroll
    for (int k = 0; k < K; ++k) wcur[k] = w[k * B];
  }
  for (long long t = TT - 2; t >= 0; --t) {
    if (t >= 1) {
      const double *w = ws + (t - 1) * K * B + b;
#pragma unroll
      for (int k = 0; k < K; ++k) wnxt[k] = w[k * B];
    }
    double mft[R], Vft[R][R];
#pragma unroll
    for (int i = 0; i < R; ++i) mft[i] = wcur[i];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) Vft[i][j] = wcur[R + Sym<R>::idx(i, j)];
    rts_mean_step<R>(mft, Vft, A, Q, ms, ok);
    write_projection<R, N>(outb + t * ot, oj, C, ms, off);
    if (ms_out) store_vec<R>(ms_out + (b * TT + t) * R, ms);
#pragma unroll
    for (int k = 0; k < K; ++k) wcur[k] = wnxt[k];
  }
  if (status) status[b] = ok ? 0 : EKS_SINGULAR;
}

}  // namespace eks

using namespace eks;

namespace {

// (r, n) shapes compiled into the fused path
template <typename F>
int dispatch_shape(int r, int n, F &&f) {
  if (r == 2 && n == 2) return f(ic<2>{}, ic<2>{});
  if (r == 3 && n == 4) return f(ic<3>{}, ic<4>{});
  if (r == 3 && n == 6) return f(ic<3>{}, ic<6>{});
  if (r == 3 && n == 8) return f(ic<3>{}, ic<8>{});
  return set_err(EKS_ERR_UNSUPPORTED,
                 "eks_smooth: (r=%d, n=%d) not compiled in (have (2,2) (3,4) (3,6) (3,8))", r, n);
}

template <typename F>
int dispatch_members(int E, F &&f) {
  switch (E) {
    case 2: return f(ic<2>{});
    case 3: return f(ic<3>{});
    case 4: return f(ic<4>{});
    case 5: return f(ic<5>{});
    case 6: return f(ic<6>{});
    case 8: return f(ic<8>{});
    default: return f(ic<0>{});  // runtime-E path
  }
}

size_t seq_workspace(int64_t B, int64_t T, int r) {
  const int K = r + r * (r + 1) / 2;
  return (size_t)B * (size_t)T * (size_t)K * sizeof(double);
}

}  // namespace

extern "C" {

size_t eks_smooth_workspace_bytes(int64_t B, int64_t T, int n, int r, int algo) {
  (void)n;
  (void)algo;
  return seq_workspace(B, T, r);
}

int eks_smooth(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
               int64_t sb, int64_t st, int64_t se, int64_t sj, int mode, const double *params,
               double *out, int64_t ob, int64_t ot, int64_t oj, double *ms, double *nll,
               void *workspace, size_t workspace_bytes, int algo, int32_t *status,
               void *stream) {
  if (!obs || !params || !out) return set_err(EKS_ERR_ARG, "eks_smooth: NULL pointer");
  if (B < 0 || T < 1 || E < 1) return set_err(EKS_ERR_ARG, "eks_smooth: need B>=0, T>=1, E>=1");
  if (E > kMaxMembers) return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth: E=%d > %d", E, kMaxMembers);
  if (mode != EKS_MEDIAN && mode != EKS_MEAN)
    return set_err(EKS_ERR_ARG, "%d averaging not supported", mode);
  if (obs_dtype != EKS_F32 && obs_dtype != EKS_F64) return set_err(EKS_ERR_ARG, "bad dtype");
  if (algo < 0 || algo > 1) return set_err(EKS_ERR_ARG, "eks_smooth: algo %d unknown", algo);
  if (B == 0) return EKS_OK;
  const size_t need = eks_smooth_workspace_bytes(B, T, n, r, algo);
  if (!workspace || workspace_bytes < need)
    return set_err(EKS_ERR_ARG, "eks_smooth: workspace of %zu bytes needed", need);
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto tag) -> int {
    using Tp = decltype(tag);
    return dispatch_shape(r, n, [&](auto Rc, auto Nc) {
      return dispatch_members(E, [&](auto Ec) {
        constexpr int RR = decltype(Rc)::value, NN = decltype(Nc)::value,
                      EE = decltype(Ec)::value;
        hipLaunchKernelGGL((k_smooth_seq<RR, NN, EE, Tp>), dim3(grid_for(B, 64)), dim3(64), 0, s,
                           (const Tp *)obs, B, T, E, sb, st, se, sj, mode == EKS_MEDIAN ? 1 : 0,
                           params, out, ob, ot, oj, ms, nll, (double *)workspace, status);
        return check_launch("k_smooth_seq");
      });
    });
  };
  return obs_dtype == EKS_F32 ? go(float{}) : go(double{});
}

}  // extern "C"
