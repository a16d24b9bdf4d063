// Register-resident small dense linear algebra for the EKS kernels (gfx950).
//
// Every matrix here is at most 8x8 and every loop bound is a template
// constant, so after full unrolling all indices are static and the arrays
// live in VGPRs (no scratch).  Row pivoting is done with data-dependent
// selects instead of dynamic row indices for the same reason.
#pragma once
#include <hip/hip_runtime.h>

#define EKS_DEV __device__ __forceinline__

namespace eks {

// y = M x            (M: R x C)
template <int R, int C>
EKS_DEV void matvec(const double (&M)[R][C], const double (&x)[C], double (&y)[R]) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < C; ++k) s = fma(M[i][k], x[k], s);
    y[i] = s;
  }
}

// Z = X Y            (X: R x K, Y: K x C)
template <int R, int K, int C>
EKS_DEV void matmul(const double (&X)[R][K], const double (&Y)[K][C], double (&Z)[R][C]) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k) s = fma(X[i][k], Y[k][j], s);
      Z[i][j] = s;
    }
}

// Z = X Y^T          (X: R x K, Y: C x K)
template <int R, int K, int C>
EKS_DEV void matmul_nt(const double (&X)[R][K], const double (&Y)[C][K], double (&Z)[R][C]) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k) s = fma(X[i][k], Y[j][k], s);
      Z[i][j] = s;
    }
}

// Gaussian elimination with partial pivoting, the algorithm of LAPACK gesv
// (np.linalg.solve): solves a X = b in place (b <- X).  `a` is destroyed.
// Returns false on an exactly-zero pivot (numpy raises LinAlgError there).
// det_mant * 2^det_exp accumulates |det a| without overflow.
template <int N, int M>
EKS_DEV bool gauss_solve(double (&a)[N][N], double (&b)[N][M], double &det_mant, int &det_exp) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    // bring the largest |a[i][k]|, i >= k, to row k (first maximum wins)
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const bool sw = fabs(a[i][k]) > fabs(a[k][k]);
#pragma unroll
      for (int j = k; j < N; ++j) {
        const double t = a[k][j];
        a[k][j] = sw ? a[i][j] : t;
        a[i][j] = sw ? t : a[i][j];
      }
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const double t = b[k][j];
        b[k][j] = sw ? b[i][j] : t;
        b[i][j] = sw ? t : b[i][j];
      }
    }
    const double piv = a[k][k];
    ok = ok && (piv != 0.0);
    int e;
    det_mant = frexp(det_mant * fabs(piv), &e);
    det_exp += e;
    const double inv = 1.0 / piv;
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const double f = a[i][k] * inv;
#pragma unroll
      for (int j = k + 1; j < N; ++j) a[i][j] = fma(-f, a[k][j], a[i][j]);
#pragma unroll
      for (int j = 0; j < M; ++j) b[i][j] = fma(-f, b[k][j], b[i][j]);
    }
  }
#pragma unroll
  for (int k = N - 1; k >= 0; --k) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double s = b[k][j];
#pragma unroll
      for (int i = k + 1; i < N; ++i) s = fma(-a[k][i], b[i][j], s);
      b[k][j] = s / a[k][k];
    }
  }
  return ok;
}

template <int N, int M>
EKS_DEV bool gauss_solve(double (&a)[N][N], double (&b)[N][M]) {
  double dm = 1.0;
  int de = 0;
  return gauss_solve<N, M>(a, b, dm, de);
}

}  // namespace eks
