// Per-timestep building blocks of the EKS recursions, shared by the
// sequential (eks_smooth.hip) and time-parallel (eks_chunked.hip) kernels.
//
// Conventions: R = latent dimension r, N = observation dimension n.
// AI / CI are compile-time model-structure kinds (EKS_MODEL_* promises):
//   AI: kAGen, kAId (A = I: the single-view model, SURVEY.md §8 A6, and the
//       multi-camera model, eks/multiview_pca_smoother.py:724) or kADiag (A
//       and Q diagonal: the pupil model, eks/pupil_smoother.py:140-147);
//   CI: kCGen, kCId (C = I, R == N: single view) or kCPupil (C = the pupil
//       measurement matrix of eks/pupil_smoother.py:150-153, R = 3, N = 8).
// The host promises the structure and the kernels verify it per trajectory
// (status bit EKS_STATUS_BAD_MODEL on violation).
#pragma once
#include <type_traits>
#include "eks_common.hpp"
#include "ensemble.hpp"
#include "small_linalg.hpp"

namespace eks {

constexpr int kAGen = 0, kAId = 1, kADiag = 2;
constexpr int kCGen = 0, kCId = 1, kCPupil = 2;

template <int R>
struct Sym {
  static constexpr int len = R * (R + 1) / 2;
  static constexpr int idx(int i, int j) {
    return i <= j ? i * R - i * (i - 1) / 2 + (j - i) : j * R - j * (j - 1) / 2 + (i - j);
  }
};

// 1/x to ~1 ulp: hardware reciprocal + two Newton-Raphson steps (5 VALU ops
// instead of the ~10 of an IEEE division).
EKS_DEV double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// x / d correctly rounded (== IEEE division, as numpy's true_divide) for a
// small integer d, by one fma correction of x * RN(1/d) (Markstein); checked
// exhaustively against true division on random doubles for d in 3..10.
EKS_DEV double div_small_int(double x, double d, double inv_d) {
  const double q = x * inv_d;
  const double r = fma(-q, d, x);
  return fma(r, inv_d, q);
}

template <int R>
EKS_DEV bool is_identity(const double (&M)[R][R]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) ok = ok && (M[i][j] == (i == j ? 1.0 : 0.0));
  return ok;
}

template <int N, int R>
EKS_DEV bool is_identity_rect(const double (&M)[N][R]) {
  bool ok = (N == R);
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) ok = ok && (M[i][j] == (i == j ? 1.0 : 0.0));
  return ok;
}

template <int R>
EKS_DEV bool is_diagonal(const double (&M)[R][R]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) ok = ok && (i == j || M[i][j] == 0.0);
  return ok;
}

// C equals the pupil measurement matrix (eks/pupil_smoother.py:150-153)
template <int N, int R>
EKS_DEV bool is_pupil_c(const double (&M)[N][R]) {
  constexpr double P[8][3] = {{0, 1, 0}, {-.5, 0, 1}, {0, 1, 0}, {.5, 0, 1},
                              {.5, 1, 0}, {0, 0, 1},  {-.5, 1, 0}, {0, 0, 1}};
  bool ok = (N == 8 && R == 3);
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) ok = ok && (i < 8 && j < 3 && M[i][j] == P[i < 8 ? i : 0][j < 3 ? j : 0]);
  return ok;
}

// one ensemble column (E members in registers): the shared reduction of
// ensemble.hpp
template <int E, typename T>
EKS_DEV void ensemble_col(const T (&raw)[E], bool median, double &avg, double &var) {
  ensemble_reduce<E, T>(raw, median, avg, var);
}

// ---------------------------------------------------------------------------
// Kalman filter pieces
// ---------------------------------------------------------------------------
// prior of step t from the posterior of t-1:  m <- A m,  P <- A (P A^T) + Q
template <int R, int AI>
EKS_DEV void kf_predict(double (&m)[R], double (&P)[R][R], const double (&A)[R][R],
                        const double (&Q)[R][R]) {
  if constexpr (AI == kAId) {
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) {
        P[i][j] += Q[i][j];
        if (j != i) P[j][i] = P[i][j];
      }
  } else if constexpr (AI == kADiag) {  // A, Q diagonal
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int j = i; j < R; ++j) {
        const double t = (A[i][i] * P[i][j]) * A[j][j];
        P[i][j] = (i == j) ? t + Q[i][i] : t;
        if (j != i) P[j][i] = P[i][j];
      }
      m[i] *= A[i][i];
    }
  } else {
    double PAt[R][R], mp[R];
    matmul_nt<R, R, R>(P, A, PAt);
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) s = fma(A[i][k], PAt[k][j], s);
        P[i][j] = s + Q[i][j];
      }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < i; ++j) P[i][j] = P[j][i];
    matvec<R, R>(A, m, mp);
#pragma unroll
    for (int i = 0; i < R; ++i) m[i] = mp[i];
  }
}

// NLL accumulator: quad = sum e^2/s, log det = log(mant) + ex ln 2
struct NllAcc {
  double quad = 0.0, mant = 1.0;
  int ex = 0;
  EKS_DEV void add(double e, double s, double inv) {
    quad = fma(e * e, inv, quad);
    mant *= s;
  }
  EKS_DEV void renorm() {
    int k;
    mant = frexp(mant, &k);
    ex += k;
  }
  EKS_DEV double value(double n_terms) const {
    return 0.5 * (n_terms * kLog2Pi + log(mant) + ex * kLn2 + quad);
  }
};

// the same interface, accumulating nothing (smoothing calls without an NLL
// output: no per-step likelihood arithmetic)
struct NoAcc {
  EKS_DEV void add(double, double, double) {}
  EKS_DEV void renorm() {}
  EKS_DEV double value(double) const { return 0.0; }
};

// ---------------------------------------------------------------------------
// Pupil measurement rows (eks/pupil_smoother.py:150-153, PUPIL_KEYS order:
// top x, y, bottom x, y, right x, y, left x, y; state (diameter, com_x,
// com_y)), coefficients in half units.  Rows 0 / 2 ([0 1 0]) and 5 / 7
// ([0 0 1]) are equal: each pair is folded into ONE scalar observation
// (merge_obs), so a step is 6 sparse scalar updates instead of 8 dense ones.
// ---------------------------------------------------------------------------
// c . x for c = (H0, H1, H2) / 2, zero coefficients skipped: exact products
// by 1 and 1/2, the same value as the dense fma chain over the row
template <int H0, int H1, int H2>
EKS_DEV double cdot3(double x0, double x1, double x2) {
  constexpr double c0 = 0.5 * H0, c1 = 0.5 * H1, c2 = 0.5 * H2;
  double s = 0.0;
  if constexpr (H0 != 0) s = c0 * x0;
  if constexpr (H1 != 0) {
    if constexpr (H0 != 0) s = fma(c1, x1, s);
    else s = c1 * x1;
  }
  if constexpr (H2 != 0) {
    if constexpr (H0 != 0 || H1 != 0) s = fma(c2, x2, s);
    else s = c2 * x2;
  }
  return s;
}

// Two scalar observations (y1, r1), (y2, r2) of the same row c: their joint
// density is N(y; c x, r) N(y1 - y2; 0, r1 + r2) with
//   y = (r2 y1 + r1 y2) / (r1 + r2),  r = r1 r2 / (r1 + r2),
// i.e. one scalar observation plus a state-free NLL term (added to `acc`).
// r1 + r2 = 0 (both exact) is the reference's singular S.
template <typename Acc>
EKS_DEV void merge_obs(double y1, double r1, double y2, double r2, double &y, double &r,
                       Acc *acc, bool &ok) {
  const double sr = r1 + r2;
  ok = ok && !(sr <= 0.0);
  const double inv = rcp_nr(sr);
  y = fma(r2, y1, r1 * y2) * inv;
  r = (r1 * r2) * inv;
  if (acc) acc->add(y1 - y2, sr, inv);
}

// one scalar update of the filter state with pupil row H (kf_update's body)
template <int H0, int H1, int H2, typename Acc = NllAcc>
EKS_DEV void kf_update_row(double (&m)[3], double (&P)[3][3], double y, double rv, Acc &acc,
                           bool &ok) {
  double v[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) v[a] = cdot3<H0, H1, H2>(P[a][0], P[a][1], P[a][2]);
  const double s = rv + cdot3<H0, H1, H2>(v[0], v[1], v[2]);
  const double hm = cdot3<H0, H1, H2>(m[0], m[1], m[2]);
  ok = ok && !(s <= 0.0);
  const double inv = rcp_nr(s);
  const double e = y - hm;
  acc.add(e, s, inv);
  const double ei = e * inv;
#pragma unroll
  for (int a = 0; a < 3; ++a) m[a] = fma(v[a], ei, m[a]);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double ka = v[a] * inv;
#pragma unroll
    for (int c = a; c < 3; ++c) {
      P[a][c] = fma(-ka, v[c], P[a][c]);
      if (c != a) P[c][a] = P[a][c];
    }
  }
}

// Measurement update with diagonal R, one scalar observation at a time
// (algebraically the reference's kalman_dot with the n x n solve).
template <int R, int N, int CI, typename Acc = NllAcc>
EKS_DEV void kf_update(double (&m)[R], double (&P)[R][R], const double (&C)[N][R],
                       const double (&y)[N], const double (&rv)[N], Acc &acc, bool &ok) {
  if constexpr (CI == kCPupil) {
    static_assert(R == 3 && N == 8, "the pupil model is r = 3, n = 8");
    double ya, ra, yb, rb;
    merge_obs(y[0], rv[0], y[2], rv[2], ya, ra, &acc, ok);
    merge_obs(y[5], rv[5], y[7], rv[7], yb, rb, &acc, ok);
    kf_update_row<0, 2, 0, Acc>(m, P, ya, ra, acc, ok);
    kf_update_row<-1, 0, 2, Acc>(m, P, y[1], rv[1], acc, ok);
    kf_update_row<1, 0, 2, Acc>(m, P, y[3], rv[3], acc, ok);
    kf_update_row<1, 2, 0, Acc>(m, P, y[4], rv[4], acc, ok);
    kf_update_row<0, 0, 2, Acc>(m, P, yb, rb, acc, ok);
    kf_update_row<-1, 2, 0, Acc>(m, P, y[6], rv[6], acc, ok);
    acc.renorm();
    return;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double v[R], s, hm;
    if constexpr (CI == kCId) {
#pragma unroll
      for (int a = 0; a < R; ++a) v[a] = P[a][i];
      s = v[i] + rv[i];
      hm = m[i];
    } else {
#pragma unroll
      for (int a = 0; a < R; ++a) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) t = fma(P[a][k], C[i][k], t);
        v[a] = t;
      }
      s = rv[i];
      hm = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        s = fma(C[i][k], v[k], s);
        hm = fma(C[i][k], m[k], hm);
      }
    }
    ok = ok && !(s <= 0.0);  // NaN propagates as in numpy, not an error
    const double inv = rcp_nr(s);
    const double e = y[i] - hm;
    acc.add(e, s, inv);
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
  acc.renorm();
}

// Inverse of a small R x R matrix: adjugate / determinant (one reciprocal,
// short dependency chain) for R <= 3, Gauss-Jordan with partial pivoting
// above.  Used on well-conditioned matrices (S = A P A^T + Q, I + P J with
// P, J positive semi-definite).  false if singular.
template <int R>
EKS_DEV bool small_inverse(const double (&S)[R][R], double (&Si)[R][R]) {
  if constexpr (R == 1) {
    Si[0][0] = rcp_nr(S[0][0]);
    return S[0][0] != 0.0;
  } else if constexpr (R == 2) {
    const double det = fma(S[0][0], S[1][1], -S[0][1] * S[1][0]);
    const double id = rcp_nr(det);
    Si[0][0] = S[1][1] * id;
    Si[1][1] = S[0][0] * id;
    Si[0][1] = -S[0][1] * id;
    Si[1][0] = -S[1][0] * id;
    return det != 0.0;
  } else if constexpr (R == 3) {
    const double c00 = fma(S[1][1], S[2][2], -S[1][2] * S[2][1]);
    const double c01 = fma(S[1][2], S[2][0], -S[1][0] * S[2][2]);
    const double c02 = fma(S[1][0], S[2][1], -S[1][1] * S[2][0]);
    const double det = fma(S[0][0], c00, fma(S[0][1], c01, S[0][2] * c02));
    const double id = rcp_nr(det);
    Si[0][0] = c00 * id;
    Si[1][0] = c01 * id;
    Si[2][0] = c02 * id;
    Si[0][1] = fma(S[0][2], S[2][1], -S[0][1] * S[2][2]) * id;
    Si[1][1] = fma(S[0][0], S[2][2], -S[0][2] * S[2][0]) * id;
    Si[2][1] = fma(S[0][1], S[2][0], -S[0][0] * S[2][1]) * id;
    Si[0][2] = fma(S[0][1], S[1][2], -S[0][2] * S[1][1]) * id;
    Si[1][2] = fma(S[0][2], S[1][0], -S[0][0] * S[1][2]) * id;
    Si[2][2] = fma(S[0][0], S[1][1], -S[0][1] * S[1][0]) * id;
    return det != 0.0;
  } else {
    double a[R][R];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) {
        a[i][j] = S[i][j];
        Si[i][j] = (i == j) ? 1.0 : 0.0;
      }
    return gauss_solve<R, R>(a, Si);
  }
}

// RTS gain and offset at step t from the filtered (m, P):
//   S = A P A^T + Q,  J = P A^T S^-1,  d = m - J A m
// so that ms[t] = J ms[t+1] + d  (eks/ensemble_kalman.py:158, :161).
template <int R, int AI>
EKS_DEV bool rts_gain(const double (&m)[R], const double (&P)[R][R], const double (&A)[R][R],
                      const double (&Q)[R][R], double (&J)[R][R], double (&d)[R]) {
  double S[R][R], PAt[R][R], Si[R][R];
  if constexpr (AI == kAId) {
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) {
        S[i][j] = P[i][j] + Q[i][j];
        PAt[i][j] = P[i][j];
      }
  } else if constexpr (AI == kADiag) {
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) {
        PAt[i][j] = P[i][j] * A[j][j];
        S[i][j] = A[i][i] * PAt[i][j] + (i == j ? Q[i][i] : 0.0);
      }
  } else {
    matmul_nt<R, R, R>(P, A, PAt);
    matmul<R, R, R>(A, PAt, S);
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) S[i][j] += Q[i][j];
  }
  const bool ok = small_inverse<R>(S, Si);
  matmul<R, R, R>(PAt, Si, J);
  double Am[R];
  if constexpr (AI == kAId) {
#pragma unroll
    for (int i = 0; i < R; ++i) Am[i] = m[i];
  } else if constexpr (AI == kADiag) {
#pragma unroll
    for (int i = 0; i < R; ++i) Am[i] = A[i][i] * m[i];
  } else {
    matvec<R, R>(A, m, Am);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double s = m[i];
#pragma unroll
    for (int k = 0; k < R; ++k) s = fma(-J[i][k], Am[k], s);
    d[i] = s;
  }
  return ok;
}

template <int R, int N, int CI>
EKS_DEV void project_store(double *out, long long oj, const double (&C)[N][R],
                           const double (&ms)[R], const double (&off)[N]) {
  if constexpr (CI == kCPupil) {
    static_assert(R == 3 && N == 8, "the pupil model is r = 3, n = 8");
    const double o[8] = {cdot3<0, 2, 0>(ms[0], ms[1], ms[2]), cdot3<-1, 0, 2>(ms[0], ms[1], ms[2]),
                         cdot3<0, 2, 0>(ms[0], ms[1], ms[2]), cdot3<1, 0, 2>(ms[0], ms[1], ms[2]),
                         cdot3<1, 2, 0>(ms[0], ms[1], ms[2]), cdot3<0, 0, 2>(ms[0], ms[1], ms[2]),
                         cdot3<-1, 2, 0>(ms[0], ms[1], ms[2]), cdot3<0, 0, 2>(ms[0], ms[1], ms[2])};
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j * oj] = o[j] + off[j];
    return;
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double cm;
    if constexpr (CI == kCId) {
      cm = ms[j];
    } else {
      cm = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) cm = fma(C[j][k], ms[k], cm);
    }
    out[j * oj] = cm + off[j];
  }
}

}  // namespace eks

namespace eks {

// ---------------------------------------------------------------------------
// Time-parallel (associative) filtering elements, Sarkka & Garcia-Fernandez,
// "Temporal parallelization of Bayesian smoothers" (IEEE TAC 2021).  An
// element summarises a chunk of steps [s, e) as a function of the unknown
// state x_{s-1}:
//     p(x_{e-1} | x_{s-1}, y_{s..e-1}) = N(Ab x_{s-1} + bb, Cb)
//     p(y_{s..e-1} | x_{s-1})          ~ exp(-1/2 x^T Jb x + eta^T x)
// It is built here one step and one scalar observation at a time (R_t is
// diagonal), so no matrix inverse is needed inside a chunk.
// ---------------------------------------------------------------------------
template <int R>
struct Elem {
  double Ab[R][R], bb[R], Cb[R][R], eta[R], Jb[R][R];
  static constexpr int len = R * R + R + Sym<R>::len + R + Sym<R>::len;

  EKS_DEV void set_identity() {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      bb[i] = 0.0;
      eta[i] = 0.0;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        Ab[i][j] = (i == j) ? 1.0 : 0.0;
        Cb[i][j] = 0.0;
        Jb[i][j] = 0.0;
      }
    }
  }
  // strided store / load: component k at p[k * stride]
  EKS_DEV void store(double *p, long long stride) const {
    int k = 0;
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) p[(k++) * stride] = Ab[i][j];
#pragma unroll
    for (int i = 0; i < R; ++i) p[(k++) * stride] = bb[i];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) p[(k++) * stride] = Cb[i][j];
#pragma unroll
    for (int i = 0; i < R; ++i) p[(k++) * stride] = eta[i];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) p[(k++) * stride] = Jb[i][j];
  }
  EKS_DEV void load(const double *p, long long stride) {
    int k = 0;
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) Ab[i][j] = p[(k++) * stride];
#pragma unroll
    for (int i = 0; i < R; ++i) bb[i] = p[(k++) * stride];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) Cb[i][j] = Cb[j][i] = p[(k++) * stride];
#pragma unroll
    for (int i = 0; i < R; ++i) eta[i] = p[(k++) * stride];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) Jb[i][j] = Jb[j][i] = p[(k++) * stride];
  }
};

// One scalar observation y ~ N(c x_t, r) absorbed into the element, given
// v = Cb c, g = Ab^T c, s = c Cb c + r, hb = c bb.
template <int R>
EKS_DEV void absorb_scalar(Elem<R> &E, const double (&v)[R], const double (&g)[R], double s,
                           double hb, double y, bool &ok, NllAcc *acc) {
  ok = ok && !(s <= 0.0);
  const double inv = rcp_nr(s);
  const double e0 = y - hb;
  const double ei = e0 * inv;
  if (acc) acc->add(e0, s, inv);
#pragma unroll
  for (int a = 0; a < R; ++a) {
    const double ga = g[a] * inv;
    E.eta[a] = fma(g[a], ei, E.eta[a]);
#pragma unroll
    for (int c = a; c < R; ++c) {
      E.Jb[a][c] = fma(ga, g[c], E.Jb[a][c]);
      if (c != a) E.Jb[c][a] = E.Jb[a][c];
    }
  }
#pragma unroll
  for (int a = 0; a < R; ++a) {
    const double ka = v[a] * inv;
    E.bb[a] = fma(ka, e0, E.bb[a]);
#pragma unroll
    for (int c = 0; c < R; ++c) E.Ab[a][c] = fma(-ka, g[c], E.Ab[a][c]);
#pragma unroll
    for (int c = a; c < R; ++c) {
      E.Cb[a][c] = fma(-ka, v[c], E.Cb[a][c]);
      if (c != a) E.Cb[c][a] = E.Cb[a][c];
    }
  }
}

// the same for pupil row H (sparse c)
template <int H0, int H1, int H2>
EKS_DEV void absorb_row(Elem<3> &E, double y, double r, bool &ok, NllAcc *acc) {
  double v[3], g[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    v[a] = cdot3<H0, H1, H2>(E.Cb[a][0], E.Cb[a][1], E.Cb[a][2]);
    g[a] = cdot3<H0, H1, H2>(E.Ab[0][a], E.Ab[1][a], E.Ab[2][a]);
  }
  const double s = r + cdot3<H0, H1, H2>(v[0], v[1], v[2]);
  const double hb = cdot3<H0, H1, H2>(E.bb[0], E.bb[1], E.bb[2]);
  absorb_scalar<3>(E, v, g, s, hb, y, ok, acc);
}

// Absorb one time step (predict with A, Q; update with the N scalar
// observations of y, rv) into the running element.
// With `acc`, the step's terms of the element's likelihood constant are
// accumulated too: conditioned on x_{s-1} each scalar observation is
// y_i ~ N(hb_i + g_i x_{s-1}, s_i), so
//   -log p(y_{s..e-1} | x) = K + 1/2 x^T Jb x - eta^T x,
//   K = 1/2 sum_i (log 2 pi + log s_i + e0_i^2 / s_i)   (acc.value)
// which elem_nll_share turns into the chunk's NLL share.
// the predict half: E <- (A Ab, A bb, A Cb A^T + Q)
template <int R, int AI>
EKS_DEV void elem_predict(Elem<R> &E, const double (&A)[R][R], const double (&Q)[R][R]) {
  if constexpr (AI == kAId) {
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) {
        E.Cb[i][j] += Q[i][j];
        if (j != i) E.Cb[j][i] = E.Cb[i][j];
      }
  } else if constexpr (AI == kADiag) {  // A, Q diagonal
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int j = 0; j < R; ++j) E.Ab[i][j] *= A[i][i];
      E.bb[i] *= A[i][i];
#pragma unroll
      for (int j = i; j < R; ++j) {
        const double t = (A[i][i] * E.Cb[i][j]) * A[j][j];
        E.Cb[i][j] = (i == j) ? t + Q[i][i] : t;
        if (j != i) E.Cb[j][i] = E.Cb[i][j];
      }
    }
  } else {
    double T1[R][R], T2[R][R], b2[R];
    matmul<R, R, R>(A, E.Ab, T1);
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) E.Ab[i][j] = T1[i][j];
    matvec<R, R>(A, E.bb, b2);
#pragma unroll
    for (int i = 0; i < R; ++i) E.bb[i] = b2[i];
    matmul_nt<R, R, R>(E.Cb, A, T2);
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) {
        double s = Q[i][j];
#pragma unroll
        for (int k = 0; k < R; ++k) s = fma(A[i][k], T2[k][j], s);
        E.Cb[i][j] = s;
      }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < i; ++j) E.Cb[i][j] = E.Cb[j][i];
  }
}

// one scalar observation y ~ N(c x, rv) with a general row c
template <int R>
EKS_DEV void absorb_gen_row(Elem<R> &E, const double (&c)[R], double y, double rv, bool &ok,
                            NllAcc *acc) {
  double v[R], g[R];
#pragma unroll
  for (int a = 0; a < R; ++a) {
    double tv = 0.0, tg = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      tv = fma(E.Cb[a][k], c[k], tv);
      tg = fma(E.Ab[k][a], c[k], tg);
    }
    v[a] = tv;
    g[a] = tg;
  }
  double s = rv, hb = 0.0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    s = fma(c[k], v[k], s);
    hb = fma(c[k], E.bb[k], hb);
  }
  absorb_scalar<R>(E, v, g, s, hb, y, ok, acc);
}

template <int R, int N, int AI, int CI>
EKS_DEV void elem_absorb(Elem<R> &E, const double (&A)[R][R], const double (&Q)[R][R],
                         const double (&C)[N][R], const double (&y)[N], const double (&rv)[N],
                         bool &ok, NllAcc *acc = nullptr) {
  elem_predict<R, AI>(E, A, Q);
  if constexpr (CI == kCPupil) {
    static_assert(R == 3 && N == 8, "the pupil model is r = 3, n = 8");
    double ya, ra, yb, rb;
    merge_obs(y[0], rv[0], y[2], rv[2], ya, ra, acc, ok);
    merge_obs(y[5], rv[5], y[7], rv[7], yb, rb, acc, ok);
    absorb_row<0, 2, 0>(E, ya, ra, ok, acc);
    absorb_row<-1, 0, 2>(E, y[1], rv[1], ok, acc);
    absorb_row<1, 0, 2>(E, y[3], rv[3], ok, acc);
    absorb_row<1, 2, 0>(E, y[4], rv[4], ok, acc);
    absorb_row<0, 0, 2>(E, yb, rb, ok, acc);
    absorb_row<-1, 2, 0>(E, y[6], rv[6], ok, acc);
    if (acc) acc->renorm();
    return;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if constexpr (CI == kCId) {
      double v[R], g[R];
#pragma unroll
      for (int a = 0; a < R; ++a) {
        v[a] = E.Cb[a][i];
        g[a] = E.Ab[i][a];
      }
      absorb_scalar<R>(E, v, g, v[i] + rv[i], E.bb[i], y[i], ok, acc);
    } else {
      absorb_gen_row<R>(E, C[i], y[i], rv[i], ok, acc);
    }
  }
  if (acc) acc->renorm();
}

// determinant of a small matrix (adjugate for R <= 3, pivoted elimination above)
template <int R>
EKS_DEV double small_det(const double (&S)[R][R]) {
  if constexpr (R == 1) {
    return S[0][0];
  } else if constexpr (R == 2) {
    return fma(S[0][0], S[1][1], -S[0][1] * S[1][0]);
  } else if constexpr (R == 3) {
    const double c00 = fma(S[1][1], S[2][2], -S[1][2] * S[2][1]);
    const double c01 = fma(S[1][2], S[2][0], -S[1][0] * S[2][2]);
    const double c02 = fma(S[1][0], S[2][1], -S[1][1] * S[2][0]);
    return fma(S[0][0], c00, fma(S[0][1], c01, S[0][2] * c02));
  } else {
    double a[R][R];
    double det = 1.0;
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) a[i][j] = S[i][j];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      int p = k;
#pragma unroll
      for (int i = k + 1; i < R; ++i)
        if (fabs(a[i][k]) > fabs(a[p][k])) p = i;
      if (p != k) {
        det = -det;
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const double t = a[k][j];
          a[k][j] = a[p][j];
          a[p][j] = t;
        }
      }
      det *= a[k][k];
      if (a[k][k] == 0.0) return 0.0;
      const double inv = 1.0 / a[k][k];
#pragma unroll
      for (int i = k + 1; i < R; ++i) {
        const double f = a[i][k] * inv;
#pragma unroll
        for (int j = k + 1; j < R; ++j) a[i][j] = fma(-f, a[k][j], a[i][j]);
      }
    }
    return det;
  }
}

// Filtered state (m, P) at step s-1 combined with the element of [s, e):
//   P' = Ab (I + P Jb)^-1 P Ab^T + Cb,   m' = Ab (I + P Jb)^-1 (m + P eta) + bb
template <int R>
EKS_DEV bool compose_state(double (&m)[R], double (&P)[R][R], const Elem<R> &E) {
  double W[R][R], Mi[R][R], v[R], PAt[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double pe = m[i];
#pragma unroll
    for (int k = 0; k < R; ++k) pe = fma(P[i][k], E.eta[k], pe);
    v[i] = pe;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double t = (i == j) ? 1.0 : 0.0, u = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        t = fma(P[i][k], E.Jb[k][j], t);
        u = fma(P[i][k], E.Ab[j][k], u);
      }
      W[i][j] = t;
      PAt[i][j] = u;
    }
  }
  const bool ok = small_inverse<R>(W, Mi);  // (I + P Jb)^-1
  double x0[R], XP[R][R];
  matvec<R, R>(Mi, v, x0);
  matmul<R, R, R>(Mi, PAt, XP);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double s = E.bb[i];
#pragma unroll
    for (int k = 0; k < R; ++k) s = fma(E.Ab[i][k], x0[k], s);
    m[i] = s;
  }
  double Pn[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double s = E.Cb[i][j];
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(E.Ab[i][k], XP[k][j], s);
      Pn[i][j] = s;
    }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) P[i][j] = 0.5 * (Pn[i][j] + Pn[j][i]);
  return ok;
}

// NLL share of the chunk [s, e) summarised by element E, given the filtered
// x_{s-1} ~ N(m, P) (eks/ensemble_kalman.py:94-105's innovations, summed over
// the chunk):
//   -log E_x[exp(-K - 1/2 x^T Jb x + eta^T x)]
//     = K - eta^T m + 1/2 m^T Jb m - 1/2 h^T (I + P Jb)^-1 P h + 1/2 log det(I + P Jb),
//   h = eta - Jb m,
// K = `kconst` (elem_absorb's accumulator).  Equal to the sum of the per-step
// innovation terms of the sequential filter over the chunk (the algebra of
// the Gaussian integral), without re-running that filter.
template <int R>
EKS_DEV double elem_nll_share(const double (&m)[R], const double (&P)[R][R], const Elem<R> &E,
                              double kconst, bool &ok) {
  double W[R][R], Mi[R][R], h[R], Ph[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double t = E.eta[i];
#pragma unroll
    for (int k = 0; k < R; ++k) t = fma(-E.Jb[i][k], m[k], t);
    h[i] = t;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) t = fma(P[i][k], h[k], t);
    Ph[i] = t;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double w = (i == j) ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) w = fma(P[i][k], E.Jb[k][j], w);
      W[i][j] = w;
    }
  }
  const double det = small_det<R>(W);
  ok = small_inverse<R>(W, Mi) && ok && det > 0.0;
  double quad = 0.0, lin = 0.0, jm = 0.0;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double u = 0.0, jmi = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      u = fma(Mi[i][k], Ph[k], u);
      jmi = fma(E.Jb[i][k], m[k], jmi);
    }
    quad = fma(h[i], u, quad);
    lin = fma(E.eta[i], m[i], lin);
    jm = fma(m[i], jmi, jm);
  }
  return kconst - lin + 0.5 * jm - 0.5 * quad + 0.5 * log(det);
}

// compose_state plus the chunk-level RTS map across the chunk.  With the
// filtered (m, P) at the boundary x_b = x_{s-1} and the element of [s, e):
//   p(x_b | y_{..e-1}) = N(mt, Pt),  Pt = (I + P Jb)^-1 P,  mt = (I + P Jb)^-1 (m + P eta)
//   p(x_e | x_b, y_{s..e-1}) = N(Ab x_b + bb, Cb)   (x_e = x_{e-1})
// so (x_b, x_e) is jointly Gaussian given y_{..e-1}, x_e's marginal is the
// filtered state at e-1 (= compose_state), and since x_b is independent of
// the later observations given x_e, the smoothed means obey
//   ms_b = mt + G (ms_e - m'),   G = Pt Ab^T P'^-1
// i.e. the affine map ms_b = G ms_e + g with g = mt - G m'.  This replaces
// the per-step RTS recursion (eks/ensemble_kalman.py:158-161) composed over
// the chunk; it needs P' (a filtered covariance) invertible, which fails
// only for an exactly observed state (R_ii = 0) at the chunk's last step.
// (m, P) are replaced by the filtered state at e-1.  false if singular.
template <int R>
EKS_DEV bool compose_state_rts(double (&m)[R], double (&P)[R][R], const Elem<R> &E,
                               double (&G)[R][R], double (&g)[R]) {
  double W[R][R], Mi[R][R], v[R], PAt[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double pe = m[i];
#pragma unroll
    for (int k = 0; k < R; ++k) pe = fma(P[i][k], E.eta[k], pe);
    v[i] = pe;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double t = (i == j) ? 1.0 : 0.0, u = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        t = fma(P[i][k], E.Jb[k][j], t);
        u = fma(P[i][k], E.Ab[j][k], u);
      }
      W[i][j] = t;
      PAt[i][j] = u;
    }
  }
  bool ok = small_inverse<R>(W, Mi);  // (I + P Jb)^-1
  double mt[R], XP[R][R];              // XP = Pt Ab^T
  matvec<R, R>(Mi, v, mt);
  matmul<R, R, R>(Mi, PAt, XP);
  double mn[R], Pn[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double s = E.bb[i];
#pragma unroll
    for (int k = 0; k < R; ++k) s = fma(E.Ab[i][k], mt[k], s);
    mn[i] = s;
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double s = E.Cb[i][j];
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(E.Ab[i][k], XP[k][j], s);
      Pn[i][j] = s;
    }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) P[i][j] = 0.5 * (Pn[i][j] + Pn[j][i]);
  double Pi[R][R];
  ok = small_inverse<R>(P, Pi) && ok;
  // an exactly observed coordinate leaves P' singular up to rounding: then
  // det P' / prod diag P' (1 for a diagonal P', 0 for a singular one) is at
  // rounding level and G would be noise -> report it (caller falls back)
  {
    double dg = 1.0, tr = 0.0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      dg *= P[i][i];
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(P[i][k], Pi[k][i], s);
      tr += s;  // trace(P' P'^-1) = R when the inverse is accurate
    }
    ok = ok && dg > 0.0 && fabs(tr - (double)R) < 1e-6;
  }
  matmul<R, R, R>(XP, Pi, G);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double s = mt[i];
#pragma unroll
    for (int k = 0; k < R; ++k) s = fma(-G[i][k], mn[k], s);
    g[i] = s;
    m[i] = mn[i];
  }
  return ok;
}

}  // namespace eks

namespace eks {

// Full associative composition of two filtering elements, i earlier than j
// (Sarkka & Garcia-Fernandez 2021, Lemma 8):
//   M = (I + Ci Jj)^-1
//   A = Aj M Ai                      b = Aj M (bi + Ci eta_j) + bj
//   C = Aj M Ci Aj^T + Cj            eta = Ai^T M^T (eta_j - Jj bi) + eta_i
//   J = Ai^T M^T Jj Ai + Ji
template <int R>
EKS_DEV bool compose_elem(const Elem<R> &Ei, const Elem<R> &Ej, Elem<R> &out) {
  double W[R][R], M[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double t = (i == j) ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) t = fma(Ei.Cb[i][k], Ej.Jb[k][j], t);
      W[i][j] = t;
      M[i][j] = (i == j) ? 1.0 : 0.0;
    }
  const bool ok = small_inverse<R>(W, M);  // M = W^-1
  double AjM[R][R], MAi[R][R];  // Aj M, and M Ai (whose transpose is Ai^T M^T)
  matmul<R, R, R>(Ej.Ab, M, AjM);
  matmul<R, R, R>(M, Ei.Ab, MAi);
  // A = (Aj M) Ai
  matmul<R, R, R>(AjM, Ei.Ab, out.Ab);
  // b = (Aj M)(bi + Ci eta_j) + bj
  double v[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double t = Ei.bb[i];
#pragma unroll
    for (int k = 0; k < R; ++k) t = fma(Ei.Cb[i][k], Ej.eta[k], t);
    v[i] = t;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double t = Ej.bb[i];
#pragma unroll
    for (int k = 0; k < R; ++k) t = fma(AjM[i][k], v[k], t);
    out.bb[i] = t;
  }
  // C = (Aj M) Ci Aj^T + Cj
  double T1[R][R];
  matmul<R, R, R>(AjM, Ei.Cb, T1);
  double Cn[R][R];
  matmul_nt<R, R, R>(T1, Ej.Ab, Cn);
  // eta = (M Ai)^T (eta_j - Jj bi) + eta_i
  double w[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double t = Ej.eta[i];
#pragma unroll
    for (int k = 0; k < R; ++k) t = fma(-Ej.Jb[i][k], Ei.bb[k], t);
    w[i] = t;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double t = Ei.eta[i];
#pragma unroll
    for (int k = 0; k < R; ++k) t = fma(MAi[k][i], w[k], t);
    out.eta[i] = t;
  }
  // J = (M Ai)^T Jj Ai + Ji
  double T2[R][R], Jn[R][R];
  matmul<R, R, R>(Ej.Jb, Ei.Ab, T2);
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double t = Ei.Jb[i][j];
#pragma unroll
      for (int k = 0; k < R; ++k) t = fma(MAi[k][i], T2[k][j], t);
      Jn[i][j] = t;
    }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      out.Cb[i][j] = 0.5 * ((Cn[i][j] + Ej.Cb[i][j]) + (Cn[j][i] + Ej.Cb[j][i]));
      out.Jb[i][j] = 0.5 * (Jn[i][j] + Jn[j][i]);
    }
  return ok;
}

// Move a whole element between lanes of a wave (__shfl_up / __shfl_down).
template <int R, bool UP>
EKS_DEV Elem<R> shfl_elem(const Elem<R> &E, int delta) {
  Elem<R> o;
  auto mv = [&](double x) { return UP ? __shfl_up(x, delta, 64) : __shfl_down(x, delta, 64); };
#pragma unroll
  for (int i = 0; i < R; ++i) {
    o.bb[i] = mv(E.bb[i]);
    o.eta[i] = mv(E.eta[i]);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      o.Ab[i][j] = mv(E.Ab[i][j]);
      o.Cb[i][j] = mv(E.Cb[i][j]);
      o.Jb[i][j] = mv(E.Jb[i][j]);
    }
  }
  return o;
}

}  // namespace eks
