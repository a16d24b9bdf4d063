// HIP kernels and C ABI of libeks_hip.so (see include/eks_hip.h).
//
// Target: gfx950 (MI355X, CDNA4), wave64.  Everything on the recursion path
// is float64 in VGPRs; per-step matrices are at most 8x8, so there is no
// MFMA here (DESIGN.md explains the roofline: the fused path is bound by HBM
// bandwidth and FP64 issue, not by matrix throughput).
//
// Kernels
//   k_ensemble        eks/ensemble_kalman.py:4-57     one thread per (b, t, j)
//   k_forward_dense   eks/ensemble_kalman.py:59-117   one lane per trajectory,
//                     LU solve of the n x n innovation covariance exactly as
//                     the reference's kalman_dot (drop-in API, full R)
//   k_backward        eks/ensemble_kalman.py:120-164  one lane per trajectory
//   k_kalman_dot      eks/ensemble_kalman.py:110-117
//   k_smooth_seq      fused hot path, one lane per trajectory: ensemble ->
//                     forward (sequential scalar updates, R diagonal) ->
//                     RTS backward -> projection; time-major workspace
// The time-parallel chunked-scan kernels live in eks_chunked.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include "../../include/eks_hip.h"
#include "ensemble.hpp"
#include "eks_common.hpp"
#include "small_linalg.hpp"

namespace eks {

// ------------------------------------------------------------------------
// error reporting
// ------------------------------------------------------------------------
static thread_local std::string g_err;

int set_err(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

void clear_err() { g_err.clear(); }

// ------------------------------------------------------------------------
// per-kernel timing of eks_smooth calls (profiling aid)
// ------------------------------------------------------------------------
struct Prof {
  bool on = false;
  int max_calls = 0, call = -1, mark = 0;
  static constexpr int kMarks = 16;  // a split-selection fit call has 10-12 marks
  std::vector<hipEvent_t> ev;
  std::vector<int> nmarks;
  std::vector<std::string> names;  // [call * kMarks + mark]: kernel launched after the mark
};
static thread_local Prof g_prof;
// > 0 while a launcher times a multi-stream call as one interval (its inner
// launchers' marks would interleave across streams)
static thread_local int g_prof_suspend = 0;

void prof_suspend(bool on) { g_prof_suspend += on ? 1 : -1; }

void prof_call_begin() {
  if (!g_prof.on || g_prof_suspend) return;
  if (g_prof.call + 1 >= g_prof.max_calls) return;
  ++g_prof.call;
  g_prof.mark = 0;
}

void prof_mark(hipStream_t s, const char *next_kernel) {
  if (!g_prof.on || g_prof_suspend || g_prof.call < 0 || g_prof.call >= g_prof.max_calls) return;
  if (g_prof.mark >= Prof::kMarks) return;
  hipEventRecord(g_prof.ev[g_prof.call * Prof::kMarks + g_prof.mark], s);
  g_prof.names[g_prof.call * Prof::kMarks + g_prof.mark] = next_kernel ? next_kernel : "";
  ++g_prof.mark;
  g_prof.nmarks[g_prof.call] = g_prof.mark;
}

void prof_call_end(hipStream_t s) { prof_mark(s, nullptr); }

int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(EKS_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return EKS_OK;
}

// ------------------------------------------------------------------------
// A1: ensemble reduction, one thread per (b, t, j)
// ------------------------------------------------------------------------
template <int E, typename T>
__global__ __launch_bounds__(256) void k_ensemble(const T *__restrict__ obs, long long B,
                                                  long long TT, int Ert, int n, long long sb,
                                                  long long st, long long se, long long sj,
                                                  int median, double *__restrict__ preds,
                                                  double *__restrict__ vars) {
  const long long total = B * TT * n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long j = i % n;
    const long long bt = i / n;
    const long long t = bt % TT;
    const long long b = bt / TT;
    const T *p = obs + b * sb + t * st + j * sj;
    double avg, var;
    if constexpr (E > 0) {
      T raw[E];
#pragma unroll
      for (int e = 0; e < E; ++e) raw[e] = p[e * se];
      ensemble_reduce<E, T>(raw, median != 0, avg, var);
    } else {
      ensemble_reduce_rt<T>(p, se, Ert, median != 0, avg, var);
    }
    preds[i] = avg;
    vars[i] = var;
  }
}

// ------------------------------------------------------------------------
// A2/A3: drop-in forward filter with the dense n x n solve of kalman_dot
// ------------------------------------------------------------------------
template <int R, int N>
__global__ __launch_bounds__(64) void k_forward_dense(
    long long B, long long TT, const double *__restrict__ y, const double *__restrict__ ev,
    const double *__restrict__ m0g, const double *__restrict__ S0g, const double *__restrict__ Ag,
    const double *__restrict__ Qg, const double *__restrict__ Cg, const double *__restrict__ Rg,
    int shared, double *__restrict__ mf, double *__restrict__ Vf, double *__restrict__ S,
    double *__restrict__ nll, int32_t *__restrict__ status) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long long pb = shared ? 0 : b;
  double A[R][R], Q[R][R], C[N][R], Roff[N][N], m[R], P[R][R];
  load_mat<R, R>(Ag + pb * R * R, A);
  load_mat<R, R>(Qg + pb * R * R, Q);
  load_mat<N, R>(Cg + pb * N * R, C);
  if (Rg) {
    load_mat<N, N>(Rg + pb * N * N, Roff);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = 0; j < N; ++j) Roff[i][j] = 0.0;
  }
  load_vec<R>(m0g + pb * R, m);
  load_mat<R, R>(S0g + pb * R * R, P);

  const double *yb = y + b * TT * N;
  const double *eb = ev + b * TT * N;
  double *mfb = mf ? mf + b * TT * R : nullptr;
  double *Vfb = Vf ? Vf + b * TT * R * R : nullptr;
  double *Sb = S ? S + b * TT * R * R : nullptr;
  bool ok = true;
  double quad = 0.0, det_m = 1.0;
  int det_e = 0;
  double mprev[R], Vprev[R][R];
  for (long long t = 0; t < TT; ++t) {
    if (t > 0) {
      // S[t-1] = A Vf[t-1] A^T + Q  (:101); prior mean A mf[t-1]  (:102)
      double VAt[R][R];
      matmul_nt<R, R, R>(Vprev, A, VAt);
      matmul<R, R, R>(A, VAt, P);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) P[i][j] += Q[i][j];
      matvec<R, R>(A, mprev, m);
      if (Sb) store_mat<R, R>(Sb + (t - 1) * R * R, P);
    } else if (Sb) {
      store_mat<R, R>(Sb, P);  // S[0] = S0 (:96); overwritten at t = 1
    }
    // innovation covariance R_t + C (P C^T)   (:112)
    double PCt[R][N], sig[N][N];
    matmul_nt<R, R, N>(P, C, PCt);
    matmul<N, R, N>(C, PCt, sig);
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = 0; j < N; ++j) sig[i][j] += (i == j) ? eb[t * N + i] : Roff[i][j];
    // right-hand sides [ y - C m | C P ]  (:94-95, :102-105)
    double rhs[N][1 + R], e0[N];
    double Cm[N];
    matvec<N, R>(C, m, Cm);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      e0[i] = yb[t * N + i] - Cm[i];
      rhs[i][0] = e0[i];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) s = fma(C[i][k], P[k][j], s);
        rhs[i][1 + j] = s;
      }
    }
    ok = gauss_solve<N, 1 + R>(sig, rhs, det_m, det_e) && ok;
#pragma unroll
    for (int i = 0; i < N; ++i) quad = fma(e0[i], rhs[i][0], quad);
    // mf = m + P (C^T x0);  Vf = P - P (C^T X)
    double ctx[R][1 + R];
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int c = 0; c < 1 + R; ++c) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) s = fma(C[i][k], rhs[i][c], s);
        ctx[k][c] = s;
      }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(P[i][k], ctx[k][0], s);
      mprev[i] = m[i] + s;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        double u = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) u = fma(P[i][k], ctx[k][1 + j], u);
        Vprev[i][j] = P[i][j] - u;
      }
    }
    if (mfb) store_vec<R>(mfb + t * R, mprev);
    if (Vfb) store_mat<R, R>(Vfb + t * R * R, Vprev);
  }
  if (Sb && TT >= 2) {
    double z[R][R] = {};
    store_mat<R, R>(Sb + (TT - 1) * R * R, z);  // never written by the reference
  }
  if (nll) nll[b] = 0.5 * ((double)TT * N * kLog2Pi + log(det_m) + det_e * kLn2 + quad);
  if (status) status[b] = ok ? 0 : EKS_STATUS_SINGULAR;
}

// ------------------------------------------------------------------------
// A4: drop-in RTS backward pass
// ------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(64) void k_backward(long long B, long long TT,
                                                 const double *__restrict__ mf,
                                                 const double *__restrict__ Vf,
                                                 const double *__restrict__ S,
                                                 const double *__restrict__ Ag, int shared,
                                                 double *__restrict__ ms, double *__restrict__ Vs,
                                                 double *__restrict__ CV,
                                                 int32_t *__restrict__ status) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (b >= B) return;
  double A[R][R];
  load_mat<R, R>(Ag + (shared ? 0 : b) * R * R, A);
  const double *mfb = mf + b * TT * R;
  const double *Vfb = Vf + b * TT * R * R;
  const double *Sb = S + b * TT * R * R;
  double msn[R], Vsn[R][R];
  load_vec<R>(mfb + (TT - 1) * R, msn);
  load_mat<R, R>(Vfb + (TT - 1) * R * R, Vsn);
  if (ms) store_vec<R>(ms + b * TT * R + (TT - 1) * R, msn);
  if (Vs) store_mat<R, R>(Vs + b * TT * R * R + (TT - 1) * R * R, Vsn);
  bool ok = true;
  for (long long t = TT - 2; t >= 0; --t) {
    double mft[R], Vft[R][R], St[R][R], X[R][R];
    load_vec<R>(mfb + t * R, mft);
    load_mat<R, R>(Vfb + t * R * R, Vft);
    load_mat<R, R>(Sb + t * R * R, St);
    double Sc[R][R];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) Sc[i][j] = St[i][j];
    matmul<R, R, R>(A, Vft, X);            // rhs = A Vf[t]
    ok = gauss_solve<R, R>(Sc, X) && ok;   // X = S^-1 A Vf ; J = X^T  (:158)
    // ms = mf + J (ms[t+1] - A mf)  (:161)
    double Amf[R], d[R];
    matvec<R, R>(A, mft, Amf);
#pragma unroll
    for (int i = 0; i < R; ++i) d[i] = msn[i] - Amf[i];
    double msc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(X[k][i], d[k], s);
      msc[i] = mft[i] + s;
    }
    if (Vs || CV) {
      // W = (Vs[t+1] - S) J^T ; Vs[t] = Vf + J W  (:160) ; CV[t] = Vs[t+1] J^T (:162)
      double D[R][R], W[R][R], CVt[R][R], Vsc[R][R];
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) D[i][j] = Vsn[i][j] - St[i][j];
      // J^T = X, so (D J^T) = D X
      matmul<R, R, R>(D, X, W);
      matmul<R, R, R>(Vsn, X, CVt);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) {
          double s = 0.0;
#pragma unroll
          for (int k = 0; k < R; ++k) s = fma(X[k][i], W[k][j], s);
          Vsc[i][j] = Vft[i][j] + s;
        }
      if (CV) store_mat<R, R>(CV + b * (TT - 1) * R * R + t * R * R, CVt);
      if (Vs) store_mat<R, R>(Vs + b * TT * R * R + t * R * R, Vsc);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) Vsn[i][j] = Vsc[i][j];
    }
    if (ms) store_vec<R>(ms + b * TT * R + t * R, msc);
#pragma unroll
    for (int i = 0; i < R; ++i) msn[i] = msc[i];
  }
  if (status) status[b] = ok ? 0 : EKS_STATUS_SINGULAR;
}

// ------------------------------------------------------------------------
// A3: kalman_dot, one problem, one thread (the reference calls it per step)
// ------------------------------------------------------------------------
template <int R, int N>
__global__ void k_kalman_dot(int k, const double *x, const double *Vg, const double *Cg,
                             const double *Rg, double *out, int32_t *status) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double V[R][R], C[N][R], Rm[N][N];
  load_mat<R, R>(Vg, V);
  load_mat<N, R>(Cg, C);
  load_mat<N, N>(Rg, Rm);
  double VCt[R][N], sig[N][N];
  matmul_nt<R, R, N>(V, C, VCt);  // V C^T
  matmul<N, R, N>(C, VCt, sig);   // C (V C^T)
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) sig[i][j] += Rm[i][j];
  bool ok = true;
  for (int c = 0; c < k; ++c) {
    double a[N][N], rhs[N][1];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      rhs[i][0] = x[i * k + c];
#pragma unroll
      for (int j = 0; j < N; ++j) a[i][j] = sig[i][j];
    }
    ok = gauss_solve<N, 1>(a, rhs) && ok;
    double ct[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < N; ++i) s = fma(C[i][q], rhs[i][0], s);
      ct[q] = s;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < R; ++q) s = fma(V[i][q], ct[q], s);
      out[i * k + c] = s;
    }
  }
  if (status) status[0] = ok ? 0 : EKS_STATUS_SINGULAR;
}

// ------------------------------------------------------------------------
// A2/A3 for any n <= kMaxObsRt (5+ cameras): one wave per trajectory, the
// n x n system of kalman_dot in LDS with lane i owning row i, solved by the
// elimination of gauss_solve (partial pivoting, first maximum); every sum in
// the order of k_forward_dense, so n <= 8 inputs give the compiled kernel's
// numbers.  Latency bound (O(n) dependent elimination rounds per step): the
// reference's own per-step solve, for the drop-in API -- eks_smooth's fused
// kernels are the throughput path.
// ------------------------------------------------------------------------
struct RtLds {  // LDS layout of the runtime-n solve (doubles)
  int n, nc, ld;
  size_t a, rhs, pct, e0, cs, ctx, total;
  __host__ __device__ RtLds(int n_, int r) : n(n_), nc(1 + r), ld(n_ + 1) {
    a = 0;
    rhs = a + (size_t)n * ld;
    pct = rhs + (size_t)n * nc;
    e0 = pct + (size_t)r * n;
    cs = e0 + n;
    ctx = cs + (size_t)n * r;
    total = ctx + (size_t)r * nc;
  }
};

// Solve a X = rhs in LDS (a: n x n, stride ld; rhs: n x nc), one wave.
// Returns the pivots' |det| accumulation like gauss_solve; ok false on a
// zero pivot.  Lane i < n owns row i.
EKS_DEV bool lds_gauss_solve(double *a, double *rhs, int n, int ld, int nc, double &det_m,
                             int &det_e) {
  const int l = threadIdx.x;
  bool ok = true;
  for (int k = 0; k < n; ++k) {
    // the first maximum of |a[i][k]|, i >= k (NaNs never win, as in the
    // compiled bubble: a NaN pivot candidate keeps its row)
    const double akk = a[k * ld + k];
    int p = k;
    if (akk == akk) {
      double v = (l > k && l < n) ? fabs(a[l * ld + k]) : -1.0;
      if (!(v == v)) v = -1.0;
      int idx = l;
      double best = fabs(akk);
      // lanes with v > |a[k][k]| compete; ties -> smallest index
      double cv = v > best ? v : -1.0;
      int ci = v > best ? idx : n;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const double ov = __shfl_xor(cv, off, 64);
        const int oi = __shfl_xor(ci, off, 64);
        if (ov > cv || (ov == cv && oi < ci)) {
          cv = ov;
          ci = oi;
        }
      }
      if (ci < n) p = ci;
    }
    if (p != k) {
      for (int j = l; j < n; j += 64)
        if (j >= k) {
          const double t = a[k * ld + j];
          a[k * ld + j] = a[p * ld + j];
          a[p * ld + j] = t;
        }
      if (l < nc) {
        const double t = rhs[k * nc + l];
        rhs[k * nc + l] = rhs[p * nc + l];
        rhs[p * nc + l] = t;
      }
    }
    __syncthreads();
    const double piv = a[k * ld + k];
    ok = ok && (piv != 0.0);
    int e;
    det_m = frexp(det_m * fabs(piv), &e);
    det_e += e;
    const double inv = 1.0 / piv;
    if (l > k && l < n) {
      const double f = a[l * ld + k] * inv;
      for (int j = k + 1; j < n; ++j) a[l * ld + j] = fma(-f, a[k * ld + j], a[l * ld + j]);
      for (int c = 0; c < nc; ++c) rhs[l * nc + c] = fma(-f, rhs[k * nc + c], rhs[l * nc + c]);
    }
    __syncthreads();
  }
  if (l < nc) {  // back substitution, one rhs column per lane
    for (int k = n - 1; k >= 0; --k) {
      double sum = rhs[k * nc + l];
      for (int i = k + 1; i < n; ++i) sum = fma(-a[k * ld + i], rhs[i * nc + l], sum);
      rhs[k * nc + l] = sum / a[k * ld + k];
    }
  }
  __syncthreads();
  return ok;
}

template <int R>
__global__ __launch_bounds__(64) void k_forward_dense_rt(
    long long B, long long TT, int n, const double *__restrict__ y, const double *__restrict__ ev,
    const double *__restrict__ m0g, const double *__restrict__ S0g, const double *__restrict__ Ag,
    const double *__restrict__ Qg, const double *__restrict__ Cg, const double *__restrict__ Rg,
    int shared, double *__restrict__ mf, double *__restrict__ Vf, double *__restrict__ S,
    double *__restrict__ nll, int32_t *__restrict__ status) {
  extern __shared__ double sh[];
  const long long b = blockIdx.x;
  const int l = threadIdx.x;
  if (b >= B) return;
  const RtLds L(n, R);
  double *a = sh + L.a, *rhs = sh + L.rhs, *pct = sh + L.pct, *e0s = sh + L.e0, *Cs = sh + L.cs,
         *ctx = sh + L.ctx;
  const int nc = L.nc, ld = L.ld;
  const long long pb = shared ? 0 : b;
  double A[R][R], Q[R][R], m[R], P[R][R];
  load_mat<R, R>(Ag + pb * R * R, A);
  load_mat<R, R>(Qg + pb * R * R, Q);
  load_vec<R>(m0g + pb * R, m);
  load_mat<R, R>(S0g + pb * R * R, P);
  const double *Cb = Cg + pb * (long long)n * R;
  const double *Rb = Rg ? Rg + pb * (long long)n * n : nullptr;
  for (int i = l; i < n * R; i += 64) Cs[i] = Cb[i];
  __syncthreads();
  const double *yb = y + b * TT * n;
  const double *eb = ev + b * TT * n;
  double *mfb = mf ? mf + b * TT * R : nullptr;
  double *Vfb = Vf ? Vf + b * TT * R * R : nullptr;
  double *Sb = S ? S + b * TT * R * R : nullptr;
  bool ok = true;
  double quad = 0.0, det_m = 1.0;
  int det_e = 0;
  double mprev[R], Vprev[R][R];
  for (long long t = 0; t < TT; ++t) {
    if (t > 0) {
      double VAt[R][R];
      matmul_nt<R, R, R>(Vprev, A, VAt);
      matmul<R, R, R>(A, VAt, P);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) P[i][j] += Q[i][j];
      matvec<R, R>(A, mprev, m);
      if (Sb && l == 0) store_mat<R, R>(Sb + (t - 1) * R * R, P);
    } else if (Sb && l == 0) {
      store_mat<R, R>(Sb, P);
    }
    // P C^T (R x n): lane j computes column j
    if (l < n) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        double sum = 0.0;
#pragma unroll
        for (int q = 0; q < R; ++q) sum = fma(P[k][q], Cs[l * R + q], sum);
        pct[k * n + l] = sum;
      }
    }
    __syncthreads();
    if (l < n) {  // row l of R_t + C (P C^T) and of [ y - C m | C P ]
      double Cl[R];
#pragma unroll
      for (int k = 0; k < R; ++k) Cl[k] = Cs[l * R + k];
      for (int j = 0; j < n; ++j) {
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) sum = fma(Cl[k], pct[k * n + j], sum);
        sum += (l == j) ? eb[t * n + l] : (Rb ? Rb[(long long)l * n + j] : 0.0);
        a[l * ld + j] = sum;
      }
      double cm = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) cm = fma(Cl[k], m[k], cm);
      const double e = yb[t * n + l] - cm;
      e0s[l] = e;
      rhs[l * nc] = e;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) sum = fma(Cl[k], P[k][j], sum);
        rhs[l * nc + 1 + j] = sum;
      }
    }
    __syncthreads();
    ok = lds_gauss_solve(a, rhs, n, ld, nc, det_m, det_e) && ok;
    // quad += e0 . x0 (in row order); C^T [x0 | X] (R x nc), one lane per entry
    if (l == 0)
      for (int i = 0; i < n; ++i) quad = fma(e0s[i], rhs[i * nc], quad);
    if (l < R * nc) {
      const int k = l / nc, c = l % nc;
      double sum = 0.0;
      for (int i = 0; i < n; ++i) sum = fma(Cs[i * R + k], rhs[i * nc + c], sum);
      ctx[k * nc + c] = sum;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double sum = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) sum = fma(P[i][k], ctx[k * nc], sum);
      mprev[i] = m[i] + sum;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        double u = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) u = fma(P[i][k], ctx[k * nc + 1 + j], u);
        Vprev[i][j] = P[i][j] - u;
      }
    }
    if (l == 0) {
      if (mfb) store_vec<R>(mfb + t * R, mprev);
      if (Vfb) store_mat<R, R>(Vfb + t * R * R, Vprev);
    }
    __syncthreads();  // LDS reused by the next step
  }
  if (l == 0) {
    if (Sb && TT >= 2) {
      double z[R][R] = {};
      store_mat<R, R>(Sb + (TT - 1) * R * R, z);
    }
    if (nll) nll[b] = 0.5 * ((double)TT * n * kLog2Pi + log(det_m) + det_e * kLn2 + quad);
    if (status) status[b] = ok ? 0 : EKS_STATUS_SINGULAR;
  }
}

// kalman_dot for any n <= kMaxObsRt: one wave, the same LDS solve
template <int R>
__global__ __launch_bounds__(64) void k_kalman_dot_rt(int n, int k, const double *x, const double *Vg,
                                                      const double *Cg, const double *Rg,
                                                      double *out, int32_t *status) {
  extern __shared__ double sh[];
  const int l = threadIdx.x;
  const RtLds L(n, 0);  // rhs: one column at a time (nc = 1)
  double *a = sh + L.a, *rhs = sh + L.rhs;
  double *vct = sh + L.total;  // V C^T (R x n)
  double V[R][R];
  load_mat<R, R>(Vg, V);
  if (l < n) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double sum = 0.0;
#pragma unroll
      for (int q = 0; q < R; ++q) sum = fma(V[i][q], Cg[l * R + q], sum);
      vct[i * n + l] = sum;
    }
  }
  __syncthreads();
  bool ok = true;
  for (int c = 0; c < k; ++c) {
    if (l < n) {
      for (int j = 0; j < n; ++j) {
        double sum = 0.0;
#pragma unroll
        for (int q = 0; q < R; ++q) sum = fma(Cg[l * R + q], vct[q * n + j], sum);
        a[l * L.ld + j] = sum + Rg[(long long)l * n + j];
      }
      rhs[l] = x[l * k + c];
    }
    __syncthreads();
    double dm = 1.0;
    int de = 0;
    ok = lds_gauss_solve(a, rhs, n, L.ld, 1, dm, de) && ok;
    if (l < R) {
      double ct[R];
#pragma unroll
      for (int q = 0; q < R; ++q) {
        double sum = 0.0;
        for (int i = 0; i < n; ++i) sum = fma(Cg[i * R + q], rhs[i], sum);
        ct[q] = sum;
      }
      double sum = 0.0;
#pragma unroll
      for (int q = 0; q < R; ++q) sum = fma(V[l][q], ct[q], sum);
      out[l * k + c] = sum;
    }
    __syncthreads();
  }
  if (l == 0 && status) status[0] = ok ? 0 : EKS_STATUS_SINGULAR;
}

}  // namespace eks

// ==========================================================================
// C ABI
// ==========================================================================
using namespace eks;

extern "C" {

const char *eks_last_error(void) { return g_err.c_str(); }
int eks_version(void) { return 100; }
int eks_max_latent(void) { return kMaxLatent; }
int eks_max_obs(void) { return kMaxObs; }
int eks_max_members(void) { return kMaxMembers; }
int64_t eks_param_len(int n, int r) { return param_len(n, r); }

int eks_profile_begin(int max_calls) {
  g_err.clear();
  for (hipEvent_t e : g_prof.ev) hipEventDestroy(e);
  g_prof = Prof();
  if (max_calls <= 0) return EKS_OK;
  g_prof.ev.resize((size_t)max_calls * Prof::kMarks);
  for (auto &e : g_prof.ev)
    if (hipEventCreate(&e) != hipSuccess) return set_err(EKS_ERR_HIP, "hipEventCreate failed");
  g_prof.nmarks.assign(max_calls, 0);
  g_prof.names.assign((size_t)max_calls * Prof::kMarks, std::string());
  g_prof.max_calls = max_calls;
  g_prof.on = true;
  return EKS_OK;
}

int eks_profile_end(double *kernel_ms, char *names, int max_kernels, int name_len) {
  g_err.clear();
  if (!g_prof.on) return set_err(EKS_ERR_ARG, "eks_profile_end: profiling not started");
  const int calls = g_prof.call + 1;
  // total milliseconds per kernel name over all recorded calls, in order of
  // first appearance
  std::vector<std::string> order;
  std::vector<double> total;
  for (int c = 0; c < calls; ++c) {
    const int m = g_prof.nmarks[c];
    if (m < 2) continue;
    hipEvent_t *ev = &g_prof.ev[c * Prof::kMarks];
    if (hipEventSynchronize(ev[m - 1]) != hipSuccess)
      return set_err(EKS_ERR_HIP, "hipEventSynchronize failed");
    for (int k = 0; k + 1 < m; ++k) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
      const std::string &nm = g_prof.names[c * Prof::kMarks + k];
      size_t i = 0;
      while (i < order.size() && order[i] != nm) ++i;
      if (i == order.size()) {
        order.push_back(nm);
        total.push_back(0.0);
      }
      total[i] += ms;
    }
  }
  const int nk = std::min((int)order.size(), max_kernels);
  for (int k = 0; k < max_kernels; ++k) kernel_ms[k] = k < nk ? total[k] : 0.0;
  if (names && name_len > 0)
    for (int k = 0; k < nk; ++k)
      std::snprintf(names + (size_t)k * name_len, name_len, "%s", order[k].c_str());
  for (hipEvent_t e : g_prof.ev) hipEventDestroy(e);
  g_prof = Prof();
  return nk;
}

int eks_ensemble(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int64_t sb,
                 int64_t st, int64_t se, int64_t sj, int mode, double *preds, double *vars,
                 void *stream) {
  g_err.clear();
  if (!obs || !preds || !vars) return set_err(EKS_ERR_ARG, "eks_ensemble: NULL pointer");
  if (B < 0 || T < 0 || n < 1 || E < 1) return set_err(EKS_ERR_ARG, "eks_ensemble: bad sizes");
  if (E > kMaxMembers) return set_err(EKS_ERR_UNSUPPORTED, "eks_ensemble: E=%d > %d", E, kMaxMembers);
  if (mode != EKS_MEDIAN && mode != EKS_MEAN)
    return set_err(EKS_ERR_ARG, "%d averaging not supported", mode);
  if (obs_dtype != EKS_F32 && obs_dtype != EKS_F64) return set_err(EKS_ERR_ARG, "bad dtype");
  const long long total = (long long)B * T * n;
  if (total == 0) return EKS_OK;
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = (unsigned)std::min<long long>(grid_for(total, 256), 8192);
  auto launch = [&](auto Ec, auto tag) -> int {
    using Tp = decltype(tag);
    constexpr int EE = decltype(Ec)::value;
    hipLaunchKernelGGL((k_ensemble<EE, Tp>), dim3(grid), dim3(256), 0, s, (const Tp *)obs, B, T,
                       E, n, sb, st, se, sj, mode == EKS_MEDIAN ? 1 : 0, preds, vars);
    return check_launch("k_ensemble");
  };
  auto by_e = [&](auto tag) -> int {
    switch (E) {
      case 1: return launch(ic<1>{}, tag);
      case 2: return launch(ic<2>{}, tag);
      case 3: return launch(ic<3>{}, tag);
      case 4: return launch(ic<4>{}, tag);
      case 5: return launch(ic<5>{}, tag);
      case 6: return launch(ic<6>{}, tag);
      case 8: return launch(ic<8>{}, tag);
      default: return launch(ic<0>{}, tag);
    }
  };
  return obs_dtype == EKS_F32 ? by_e(float{}) : by_e(double{});
}

int eks_forward(int64_t B, int64_t T, int n, int r, const double *y, const double *ev,
                const double *m0, const double *S0, const double *A, const double *Q,
                const double *C, const double *R, int params_shared, double *mf, double *Vf,
                double *S, double *nll, int32_t *status, void *stream) {
  g_err.clear();
  if (!y || !ev || !m0 || !S0 || !A || !Q || !C)
    return set_err(EKS_ERR_ARG, "eks_forward: NULL input");
  if (B < 0 || T < 1) return set_err(EKS_ERR_ARG, "eks_forward: need B >= 0, T >= 1");
  if (B == 0) return EKS_OK;
  hipStream_t s = (hipStream_t)stream;
  if (n > kMaxObs) {  // 5+ cameras: one wave per trajectory, the solve in LDS
    if (n > kMaxObsRt) return set_err(EKS_ERR_UNSUPPORTED, "eks_forward: n=%d > %d", n, kMaxObsRt);
    return dispatch_r(r, [&](auto Rc) {
      constexpr int RR = decltype(Rc)::value;
      const size_t lds = RtLds(n, RR).total * sizeof(double);
      hipLaunchKernelGGL((k_forward_dense_rt<RR>), dim3((unsigned)B), dim3(64), lds, s, B, T, n,
                         y, ev, m0, S0, A, Q, C, R, params_shared, mf, Vf, S, nll, status);
      return check_launch("k_forward_dense_rt");
    });
  }
  return dispatch_r(r, [&](auto Rc) {
    return dispatch_n(n, [&](auto Nc) {
      constexpr int RR = decltype(Rc)::value, NN = decltype(Nc)::value;
      hipLaunchKernelGGL((k_forward_dense<RR, NN>), dim3(grid_for(B, 64)), dim3(64), 0, s, B, T,
                         y, ev, m0, S0, A, Q, C, R, params_shared, mf, Vf, S, nll, status);
      return check_launch("k_forward_dense");
    });
  });
}

int eks_backward(int64_t B, int64_t T, int r, const double *mf, const double *Vf, const double *S,
                 const double *A, int params_shared, double *ms, double *Vs, double *CV,
                 int32_t *status, void *stream) {
  g_err.clear();
  if (!mf || !Vf || !S || !A) return set_err(EKS_ERR_ARG, "eks_backward: NULL input");
  if (B < 0 || T < 1) return set_err(EKS_ERR_ARG, "eks_backward: need B >= 0, T >= 1");
  if (B == 0) return EKS_OK;
  hipStream_t s = (hipStream_t)stream;
  return dispatch_r(r, [&](auto Rc) {
    constexpr int RR = decltype(Rc)::value;
    hipLaunchKernelGGL((k_backward<RR>), dim3(grid_for(B, 64)), dim3(64), 0, s, B, T, mf, Vf, S,
                       A, params_shared, ms, Vs, CV, status);
    return check_launch("k_backward");
  });
}

int eks_kalman_dot(int n, int r, int k, const double *x, const double *V, const double *C,
                   const double *R, double *out, int32_t *status, void *stream) {
  g_err.clear();
  if (!x || !V || !C || !R || !out) return set_err(EKS_ERR_ARG, "eks_kalman_dot: NULL pointer");
  if (k < 1) return set_err(EKS_ERR_ARG, "eks_kalman_dot: k must be >= 1");
  hipStream_t s = (hipStream_t)stream;
  if (n > kMaxObs) {
    if (n > kMaxObsRt) return set_err(EKS_ERR_UNSUPPORTED, "eks_kalman_dot: n=%d > %d", n, kMaxObsRt);
    return dispatch_r(r, [&](auto Rc) {
      constexpr int RR = decltype(Rc)::value;
      const size_t lds = (RtLds(n, 0).total + (size_t)RR * n) * sizeof(double);
      hipLaunchKernelGGL((k_kalman_dot_rt<RR>), dim3(1), dim3(64), lds, s, n, k, x, V, C, R, out,
                         status);
      return check_launch("k_kalman_dot_rt");
    });
  }
  return dispatch_r(r, [&](auto Rc) {
    return dispatch_n(n, [&](auto Nc) {
      constexpr int RR = decltype(Rc)::value, NN = decltype(Nc)::value;
      hipLaunchKernelGGL((k_kalman_dot<RR, NN>), dim3(1), dim3(64), 0, s, k, x, V, C, R, out,
                         status);
      return check_launch("k_kalman_dot");
    });
  });
}

}  // extern "C"
