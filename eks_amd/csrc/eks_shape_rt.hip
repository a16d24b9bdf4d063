// Fused smoother for (r, n) shapes without compiled kernels: any number of
// observed coordinates n (e.g. the multi-camera model with V > 4 cameras,
// n = 2V: the reference accepts any camera count,
// eks/multiview_pca_smoother.py:641-666) and runtime E.
//
// One lane per trajectory, sequential in time (algo 1's structure): the
// observation vector is never held whole -- each step streams its n columns
// one at a time (ensemble of column j -> scalar update with row j of C, read
// from the packed model), so registers do not grow with n.  Same arithmetic
// and update order as the compiled general-C kernels (kf_update with CI =
// kCGen): equal to them to ~1 ulp where both exist (tests/test_gpu_rt.py).
#include "smooth_impl.hpp"

namespace eks {

// one scalar observation y ~ N(c x, rv): kf_update's general-C body
template <int R>
EKS_DEV void kf_update_row_rt(double (&m)[R], double (&P)[R][R], const double *c, double y,
                              double rv, NllAcc &acc, bool &ok) {
  double cr[R], v[R];
#pragma unroll
  for (int k = 0; k < R; ++k) cr[k] = c[k];
#pragma unroll
  for (int a = 0; a < R; ++a) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) t = fma(P[a][k], cr[k], t);
    v[a] = t;
  }
  double s = rv, hm = 0.0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    s = fma(cr[k], v[k], s);
    hm = fma(cr[k], m[k], hm);
  }
  ok = ok && !(s <= 0.0);
  const double inv = rcp_nr(s);
  const double e = y - hm;
  acc.add(e, s, inv);
  const double ei = e * inv;
#pragma unroll
  for (int a = 0; a < R; ++a) m[a] = fma(v[a], ei, m[a]);
#pragma unroll
  for (int a = 0; a < R; ++a) {
    const double ka = v[a] * inv;
#pragma unroll
    for (int cc = a; cc < R; ++cc) {
      P[a][cc] = fma(-ka, v[cc], P[a][cc]);
      if (cc != a) P[cc][a] = P[a][cc];
    }
  }
}

template <int R>
EKS_DEV void project_rt(double *out, long long oj, const double *C, const double *off, int n,
                        const double (&ms)[R]) {
  for (int j = 0; j < n; ++j) {
    double cm = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) cm = fma(C[j * R + k], ms[k], cm);
    out[j * oj] = cm + off[j];
  }
}

template <int R, typename T>
__global__ __launch_bounds__(64) void k_smooth_seq_rt(SmoothArgs a) {
  constexpr int K = R + Sym<R>::len;
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long B = a.B, TT = a.T;
  const int n = a.n;
  if (b >= B) return;
  const bool median = a.median != 0;
  const double *pp = a.params + b * (long long)(R + 3 * R * R + n * R + n);  // eks_param_len
  double m[R], P[R][R], A[R][R], Q[R][R];
  load_vec<R>(pp, m);
  load_mat<R, R>(pp + R, P);
  load_mat<R, R>(pp + R + R * R, A);
  load_mat<R, R>(pp + R + 2 * R * R, Q);
  const double *C = pp + R + 3 * R * R;  // n x R, row-major
  const double *off = C + (long long)n * R;
  double *ws = (double *)a.ws;
  const T *ob = (const T *)a.obs + b * a.sb;
  bool ok = true;
  NllAcc acc;
  for (long long t = 0; t < TT; ++t) {
    if (t > 0) kf_predict<R, kAGen>(m, P, A, Q);
    const T *pt = ob + t * a.st;
    for (int j = 0; j < n; ++j) {
      double avg, var;
      ensemble_reduce_rt<T>(pt + j * a.sj, a.se, a.E, median, avg, var);
      kf_update_row_rt<R>(m, P, C + j * R, avg - off[j], var, acc, ok);
    }
    acc.renorm();
    store_state<R>(ws + t * K * B + b, B, m, P);
  }
  if (a.nll) a.nll[b] = acc.value((double)TT * n);
  if (!a.out) {
    if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
    return;
  }
  double *outb = a.out + b * a.ob;
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = m[i];
  project_rt<R>(outb + (TT - 1) * a.ot, a.oj, C, off, n, ms);
  if (a.ms) store_vec<R>(a.ms + (b * TT + TT - 1) * R, ms);
  for (long long t = TT - 2; t >= 0; --t) {
    double mc[R], Pc[R][R], J[R][R], d[R], nx[R];
    load_state<R>(ws + t * K * B + b, B, mc, Pc);
    ok = rts_gain<R, kAGen>(mc, Pc, A, Q, J, d) && ok;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = d[i];
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(J[i][k], ms[k], s);
      nx[i] = s;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = nx[i];
    project_rt<R>(outb + t * a.ot, a.oj, C, off, n, ms);
    if (a.ms) store_vec<R>(a.ms + (b * TT + t) * R, ms);
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
}

int launch_rt(const SmoothArgs &a) {
  if (a.dtype != EKS_F32 && a.dtype != EKS_F64)
    return set_err(EKS_ERR_UNSUPPORTED,
                   "eks_smooth: (r=%d, n=%d) runs the runtime-n kernel, which reads member "
                   "predictions (f32 / f64), not y / ev planes", a.r, a.n);
  auto go = [&](auto rtag, auto ttag) -> int {
    constexpr int R = decltype(rtag)::value;
    using T = decltype(ttag);
    prof_call_begin();
    prof_mark(a.stream, "k_smooth_seq_rt");
    hipLaunchKernelGGL((k_smooth_seq_rt<R, T>), dim3(grid_for(a.B, 64)), dim3(64), 0, a.stream,
                       a);
    prof_call_end(a.stream);
    return check_launch("k_smooth_seq_rt");
  };
  const bool f32 = a.dtype == EKS_F32;
  switch (a.r) {
    case 2: return f32 ? go(ic<2>{}, float{}) : go(ic<2>{}, double{});
    case 3: return f32 ? go(ic<3>{}, float{}) : go(ic<3>{}, double{});
    default:
      return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth: latent r=%d not compiled in (2, 3)", a.r);
  }
}

}  // namespace eks
