// F3: the Newton ("opti") forward filter of eks/newton_eks.py:115-148.
//
//   k_newton   one lane per trajectory, information form exactly as the
//              reference evaluates it:
//                P    = inv(S0)                       (:123, used as a covariance)
//                P    = inv(inv(E + A P A^T) + B^T D^-1 B)          (:129, :141)
//                q[t] = A q[t-1] - P B^T D^-1 (B A q[t-1] - y[t])   (:130, :142)
//              with D = diag(ensemble_vars[t]), q[0] = mu0 and no update at
//              t = 0 (:121), P carried over between iterations, q updated in
//              place (the reference's `qnew = q` alias), and the trailing step
//              of :138-142 reading q[T-2] (= q[0] when T == 1).
//
// Per step the lane inverts two r x r matrices (partial-pivot Gauss-Jordan in
// VGPRs, r <= 6) and streams 16 n bytes of y / ensemble variances in and 8 r
// bytes of q out.  Latency-bound FP64 per lane; the arithmetic order follows
// the numpy expression order of the reference ((A @ P) @ A.T, (B @ A) @ q,
// ((P @ B.T) @ invD) @ res) so results agree to a few ulps of the state.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/eks_hip.h"
#include "eks_common.hpp"

namespace eks {

// out = inv(a) by Gaussian elimination with partial pivoting on [a | I];
// returns false on a zero pivot (numpy.linalg.inv raises LinAlgError).
template <int R>
EKS_DEV bool inverse(const double (&a)[R][R], double (&out)[R][R]) {
  double w[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      w[i][j] = a[i][j];
      out[i][j] = (i == j) ? 1.0 : 0.0;
    }
  return gauss_solve<R, R>(w, out);
}

template <int R, int N>
__global__ __launch_bounds__(64) void k_newton(
    long long B, long long TT, const double *__restrict__ y, const double *__restrict__ ev,
    const double *__restrict__ mu0g, const double *__restrict__ S0g,
    const double *__restrict__ Ag, const double *__restrict__ Bg, const double *__restrict__ Eg,
    int shared, int max_iter, double *__restrict__ q, int32_t *__restrict__ status) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long long pb = shared ? 0 : b;
  double A[R][R], Em[R][R], Bm[N][R], S0[R][R], P[R][R], BA[N][R];
  load_mat<R, R>(Ag + pb * R * R, A);
  load_mat<R, R>(Eg + pb * R * R, Em);
  load_mat<N, R>(Bg + pb * N * R, Bm);
  load_mat<R, R>(S0g + pb * R * R, S0);
  matmul<N, R, R>(Bm, A, BA);
  bool ok = inverse<R>(S0, P);  // :123

  const double *yb = y + b * TT * N;
  const double *eb = ev + b * TT * N;
  double *qb = q + b * TT * R;
  double q0[R];
  load_vec<R>(mu0g + pb * R, q0);
  store_vec<R>(qb, q0);  // :121

  for (int it = 0; it < max_iter; ++it) {
    double qp[R];
#pragma unroll
    for (int i = 0; i < R; ++i) qp[i] = q0[i];
    // t = 1 .. T-1; for T == 1 the trailing step runs once on t = 0 from q[0]
    const long long t_begin = TT > 1 ? 1 : 0;
    for (long long t = t_begin; t < TT; ++t) {
      double invd[N], yt[N];
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const double v = eb[t * N + k];
        ok = ok && (v != 0.0);
        invd[k] = 1.0 / v;
        yt[k] = yb[t * N + k];
      }
      // Ppred = E + (A P) A^T ; info = inv(Ppred) + (B^T invD) B ; P = inv(info)
      double AP[R][R], Pp[R][R], Pi[R][R];
      matmul<R, R, R>(A, P, AP);
      matmul_nt<R, R, R>(AP, A, Pp);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) Pp[i][j] = Em[i][j] + Pp[i][j];
      ok = inverse<R>(Pp, Pi) && ok;
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) {
          double s = 0.0;
#pragma unroll
          for (int k = 0; k < N; ++k) s = fma(Bm[k][i] * invd[k], Bm[k][j], s);
          Pp[i][j] = Pi[i][j] + s;
        }
      ok = inverse<R>(Pp, P) && ok;
      // res = (B A) q - y ; q = A q - ((P B^T) invD) res
      double res[N], Aq[R];
#pragma unroll
      for (int k = 0; k < N; ++k) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < R; ++j) s = fma(BA[k][j], qp[j], s);
        res[k] = s - yt[k];
      }
      matvec<R, R>(A, qp, Aq);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          double pbt = 0.0;
#pragma unroll
          for (int j = 0; j < R; ++j) pbt = fma(P[i][j], Bm[k][j], pbt);
          s = fma(pbt * invd[k], res[k], s);
        }
        qp[i] = Aq[i] - s;
      }
      store_vec<R>(qb + t * R, qp);
    }
    if (TT == 1) {
#pragma unroll
      for (int i = 0; i < R; ++i) q0[i] = qp[i];  // q[0] itself was updated in place
    }
  }
  if (status) status[b] = ok ? 0 : EKS_STATUS_SINGULAR;
}

// The same for any n <= kMaxObsRt (5+ cameras): n is a runtime loop bound,
// the observation matrix rows (B and B A) are read from global memory (a few
// KB per model, L1/L2 resident) and the per-step y / 1/ev from the input rows;
// every sum keeps the order of k_newton, so results equal the compiled kernel.
template <int R>
__global__ __launch_bounds__(64) void k_newton_rt(
    long long B, long long TT, int n, const double *__restrict__ y, const double *__restrict__ ev,
    const double *__restrict__ mu0g, const double *__restrict__ S0g,
    const double *__restrict__ Ag, const double *__restrict__ Bg, const double *__restrict__ Eg,
    int shared, int max_iter, double *__restrict__ q, int32_t *__restrict__ status) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long long pb = shared ? 0 : b;
  double A[R][R], Em[R][R], S0[R][R], P[R][R];
  load_mat<R, R>(Ag + pb * R * R, A);
  load_mat<R, R>(Eg + pb * R * R, Em);
  load_mat<R, R>(S0g + pb * R * R, S0);
  const double *Bm = Bg + pb * (long long)n * R;  // (n, R) row-major
  bool ok = inverse<R>(S0, P);  // :123
  const double *yb = y + b * TT * n;
  const double *eb = ev + b * TT * n;
  double *qb = q + b * TT * R;
  double q0[R];
  load_vec<R>(mu0g + pb * R, q0);
  store_vec<R>(qb, q0);  // :121
  for (int it = 0; it < max_iter; ++it) {
    double qp[R];
#pragma unroll
    for (int i = 0; i < R; ++i) qp[i] = q0[i];
    const long long t_begin = TT > 1 ? 1 : 0;
    for (long long t = t_begin; t < TT; ++t) {
      const double *et = eb + t * n, *yt = yb + t * n;
      double AP[R][R], Pp[R][R], Pi[R][R];
      matmul<R, R, R>(A, P, AP);
      matmul_nt<R, R, R>(AP, A, Pp);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) Pp[i][j] = Em[i][j] + Pp[i][j];
      ok = inverse<R>(Pp, Pi) && ok;
      double S[R][R];
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) S[i][j] = 0.0;
      for (int k = 0; k < n; ++k) {
        const double v = et[k];
        ok = ok && (v != 0.0);
        const double invd = 1.0 / v;
        double bk[R];
        load_vec<R>(Bm + k * R, bk);
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int j = 0; j < R; ++j) S[i][j] = fma(bk[i] * invd, bk[j], S[i][j]);
      }
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) Pp[i][j] = Pi[i][j] + S[i][j];
      ok = inverse<R>(Pp, P) && ok;
      // q = A q - ((P B^T) invD) ((B A) q - y), summed over k in order
      double Aq[R], acc[R];
      matvec<R, R>(A, qp, Aq);
#pragma unroll
      for (int i = 0; i < R; ++i) acc[i] = 0.0;
      for (int k = 0; k < n; ++k) {
        double bk[R], ba[R];
        load_vec<R>(Bm + k * R, bk);
#pragma unroll
        for (int j = 0; j < R; ++j) {  // (B A)[k][j]
          double s = 0.0;
#pragma unroll
          for (int u = 0; u < R; ++u) s = fma(bk[u], A[u][j], s);
          ba[j] = s;
        }
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < R; ++j) s = fma(ba[j], qp[j], s);
        const double res = s - yt[k];
        const double invd = 1.0 / et[k];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double pbt = 0.0;
#pragma unroll
          for (int j = 0; j < R; ++j) pbt = fma(P[i][j], bk[j], pbt);
          acc[i] = fma(pbt * invd, res, acc[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < R; ++i) qp[i] = Aq[i] - acc[i];
      store_vec<R>(qb + t * R, qp);
    }
    if (TT == 1) {
#pragma unroll
      for (int i = 0; i < R; ++i) q0[i] = qp[i];
    }
  }
  if (status) status[b] = ok ? 0 : EKS_STATUS_SINGULAR;
}

}  // namespace eks

using namespace eks;

extern "C" int eks_newton_filter(int64_t B, int64_t T, int n, int r, const double *y,
                                 const double *ev, const double *mu0, const double *S0,
                                 const double *A, const double *Bm, const double *E,
                                 int params_shared, int max_iter, double *q, int32_t *status,
                                 void *stream) {
  clear_err();
  if (!y || !ev || !mu0 || !S0 || !A || !Bm || !E || !q)
    return set_err(EKS_ERR_ARG, "eks_newton_filter: NULL pointer");
  if (B < 0 || T < 1) return set_err(EKS_ERR_ARG, "eks_newton_filter: need B >= 0, T >= 1");
  if (max_iter < 1) return set_err(EKS_ERR_ARG, "eks_newton_filter: max_iter must be >= 1");
  if (B == 0) return EKS_OK;
  hipStream_t s = (hipStream_t)stream;
  if (n > kMaxObs) {  // 5+ cameras: the runtime-n kernel
    if (n > kMaxObsRt)
      return set_err(EKS_ERR_UNSUPPORTED, "eks_newton_filter: n=%d > %d", n, kMaxObsRt);
    return dispatch_r(r, [&](auto Rc) {
      constexpr int RR = decltype(Rc)::value;
      hipLaunchKernelGGL((k_newton_rt<RR>), dim3(grid_for(B, 64)), dim3(64), 0, s, B, T, n, y, ev,
                         mu0, S0, A, Bm, E, params_shared, max_iter, q, status);
      return check_launch("k_newton_rt");
    });
  }
  return dispatch_r(r, [&](auto Rc) {
    return dispatch_n(n, [&](auto Nc) {
      constexpr int RR = decltype(Rc)::value, NN = decltype(Nc)::value;
      hipLaunchKernelGGL((k_newton<RR, NN>), dim3(grid_for(B, 64)), dim3(64), 0, s, B, T, y, ev,
                         mu0, S0, A, Bm, E, params_shared, max_iter, q, status);
      return check_launch("k_newton");
    });
  });
}
