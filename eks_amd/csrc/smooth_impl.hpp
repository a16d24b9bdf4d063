// Fused smoother kernels (eks_smooth): the sequential lane-per-trajectory
// algorithm (algo 1) and the exact time-parallel chunked scan (algo 2).
//
// Included by one translation unit per (r, n) shape (eks_shape_*.hip) so
// the template instantiations compile in parallel.
//
// ---------------------------------------------------------------------------
// algo 2: each trajectory's T steps are cut into NC chunks of L steps; one
// lane owns one (chunk, trajectory) pair, lanes of a wave = 64 consecutive
// trajectories of the same chunk, so every load/store of the time-major
// intermediates below is one coalesced 256..512-byte access per wave.
//
//  K1 k_c1_elem    members -> ensemble (median, var/E) -> y (raw), ev stored
//                  time-major; builds the chunk's filtering element
//                  (kf_steps.hpp, Elem) or, for chunk 0, runs the plain filter
//  K2 k_c2_fscan   per trajectory, sequential over chunks: filtered state at
//                  every chunk start (state (x) element composition)
//  K3 k_c3_rerun   re-runs the Kalman filter over the chunk from its exact
//                  start state, writes a checkpoint every LS steps, and
//                  accumulates the chunk's RTS map ms[s] = G ms[e] + g in
//                  FORWARD order (G = J_s ... J_{e-1}) plus its NLL share
//  K4 k_c4_bscan   per trajectory, sequential over chunks in reverse:
//                  smoothed mean entering every chunk from the right, NLL sum
//  K5 k_c5_final   per LS-step sub-chunk, last to first: re-runs the filter
//                  from the checkpoint keeping (J_t, d_t) in registers, then
//                  the RTS mean recursion backwards, writes C ms + offset
//
// Exactness: K3/K5 run the same sequential recursion as algo 1 from start
// states that agree with the sequential filter to rounding; only K2/K4's
// chunk compositions are extra arithmetic.  The filter and RTS recursions
// are contractive, so those rounding differences do not grow.
// ---------------------------------------------------------------------------
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/eks_hip.h"
#include "eks_common.hpp"
#include "ensemble.hpp"
#include "kf_steps.hpp"
#include "small_linalg.hpp"

namespace eks {

struct SmoothArgs {
  const void *obs;
  int dtype;
  long long B, T;
  int E, n, r;
  long long sb, st, se, sj;
  int median;
  const double *params;
  double *out;
  long long ob, ot, oj;
  double *ms;
  double *nll;
  char *ws;
  size_t ws_bytes;
  int flags;
  int algo;
  int32_t *status;
  hipStream_t stream;
};

constexpr long long kTargetLanes = 256LL * 16 * 64;  // 4 waves per SIMD
constexpr long long kMinChunk = 64;

inline int sub_len(int r) { return r <= 2 ? 8 : 4; }
inline int elem_len(int r) { return r * r + r + r * (r + 1) / 2 + r + r * (r + 1) / 2; }
inline int state_len(int r) { return r + r * (r + 1) / 2; }

inline long long round_up(long long x, long long m) { return (x + m - 1) / m * m; }

inline long long chunk_len(long long B, long long T, int r) {
  const long long ls = sub_len(r);
  const long long nc = std::max(1LL, (kTargetLanes + B - 1) / B);
  long long L = std::max(kMinChunk, (T + nc - 1) / nc);
  L = round_up(L, ls);
  if (L >= T) L = round_up(T, ls);
  return L;
}

struct ChunkPlan {
  long long L = 0, NC = 0, NSUB = 0;
  int LS = 8;
  size_t y_off = 0, ev_off = 0, elem_off = 0, cstart_off = 0, bwd_off = 0, nllp_off = 0,
         msend_off = 0, ckpt_off = 0, total = 0;
};

inline size_t align256(size_t x) { return (x + 255) / 256 * 256; }

inline ChunkPlan make_plan(long long B, long long T, int r, int n, long long L) {
  ChunkPlan p;
  p.LS = sub_len(r);
  p.L = L;
  p.NC = (T + L - 1) / L;
  p.NSUB = L / p.LS;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align256(off + bytes);
    return o;
  };
  const size_t Bz = (size_t)B;
  p.y_off = take((size_t)T * n * Bz * 8);  // sized for f64 y
  p.ev_off = take((size_t)T * n * Bz * 8);
  p.elem_off = take((size_t)p.NC * elem_len(r) * Bz * 8);
  p.cstart_off = take((size_t)p.NC * state_len(r) * Bz * 8);
  p.bwd_off = take((size_t)p.NC * (r * r + r) * Bz * 8);
  p.nllp_off = take((size_t)p.NC * Bz * 8);
  p.msend_off = take((size_t)p.NC * r * Bz * 8);
  p.ckpt_off = take((size_t)p.NC * p.NSUB * state_len(r) * Bz * 8);
  p.total = off;
  return p;
}

inline size_t seq_workspace_bytes(long long B, long long T, int r) {
  return (size_t)B * (size_t)T * (size_t)state_len(r) * 8;
}

// model of one trajectory in registers
template <int R, int N>
struct Model {
  double m0[R], S0[R][R], A[R][R], Q[R][R], C[N][R], off[N];
  EKS_DEV void load(const double *pp, bool with_prior) {
    using L = ParamLayout<R, N>;
    if (with_prior) {
      load_vec<R>(pp + L::m0, m0);
      load_mat<R, R>(pp + L::S0, S0);
    }
    load_mat<R, R>(pp + L::A, A);
    load_mat<R, R>(pp + L::Q, Q);
    load_mat<N, R>(pp + L::C, C);
    load_vec<N>(pp + L::off, off);
  }
  template <bool AI, bool CI>
  EKS_DEV bool valid() const {
    bool ok = true;
    if constexpr (AI) ok = ok && is_identity<R>(A);
    if constexpr (CI) ok = ok && is_identity_rect<N, R>(C);
    return ok;
  }
};

template <int R>
EKS_DEV void store_state(double *p, long long stride, const double (&m)[R],
                         const double (&P)[R][R]) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) p[(k++) * stride] = m[i];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = i; j < R; ++j) p[(k++) * stride] = P[i][j];
}

template <int R>
EKS_DEV void load_state(const double *p, long long stride, double (&m)[R], double (&P)[R][R]) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) m[i] = p[(k++) * stride];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = i; j < R; ++j) P[i][j] = P[j][i] = p[(k++) * stride];
}

// E x N members of step t (compile-time E) into registers
template <int E, int N, typename T>
EKS_DEV void load_step(const T *p, long long se, long long sj, T (&v)[E][N]) {
#pragma unroll
  for (int e = 0; e < E; ++e)
#pragma unroll
    for (int j = 0; j < N; ++j) v[e][j] = p[e * se + j * sj];
}

// ensemble of one step: raw average and variance per coordinate
template <int E, int N, typename T>
EKS_DEV void reduce_step(const T (&v)[(E > 0 ? E : 1)][N], const T *p, long long se,
                         long long sj, int Ert, bool median, double (&avg)[N], double (&var)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if constexpr (E > 0) {
      T col[E];
#pragma unroll
      for (int e = 0; e < E; ++e) col[e] = v[e][j];
      ensemble_col<E, T>(col, median, avg[j], var[j]);
    } else {
      ensemble_reduce_rt<T>(p + j * sj, se, Ert, median, avg[j], var[j]);
    }
  }
}

EKS_DEV void flag(int32_t *status, long long b, int bits) {
  if (bits) atomicOr(status + b, bits);
}

// ===========================================================================
// algo 1: one lane per trajectory, sequential in time
// ===========================================================================
template <int R, int N, int E, typename T, bool AI, bool CI>
__global__ __launch_bounds__(64) void k_smooth_seq(SmoothArgs a) {
  constexpr int K = R + Sym<R>::len;
  constexpr int EE = E > 0 ? E : 1;
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long B = a.B, TT = a.T;
  if (b >= B) return;
  const bool median = a.median != 0;
  Model<R, N> md;
  md.load(a.params + b * ParamLayout<R, N>::len, true);
  if (!md.template valid<AI, CI>()) flag(a.status, b, EKS_STATUS_BAD_MODEL);
  double *ws = (double *)a.ws;
  const T *ob = (const T *)a.obs + b * a.sb;
  double *outb = a.out + b * a.ob;
  bool ok = true;
  NllAcc acc;
  double m[R], P[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    m[i] = md.m0[i];
#pragma unroll
    for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
  }
  T cur[EE][N], nxt[EE][N];
  if constexpr (E > 0) load_step<E, N, T>(ob, a.se, a.sj, cur);
  for (long long t = 0; t < TT; ++t) {
    const T *pt = ob + t * a.st;
    if constexpr (E > 0) {
      if (t + 1 < TT) load_step<E, N, T>(pt + a.st, a.se, a.sj, nxt);
    }
    double y[N], rv[N];
    reduce_step<E, N, T>(cur, pt, a.se, a.sj, a.E, median, y, rv);
#pragma unroll
    for (int j = 0; j < N; ++j) y[j] -= md.off[j];
    if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
    kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
    store_state<R>(ws + t * K * B + b, B, m, P);
    if constexpr (E > 0) {
#pragma unroll
      for (int e = 0; e < E; ++e)
#pragma unroll
        for (int j = 0; j < N; ++j) cur[e][j] = nxt[e][j];
    }
  }
  if (a.nll) a.nll[b] = acc.value((double)TT * N);
  // backward
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = m[i];
  project_store<R, N, CI>(outb + (TT - 1) * a.ot, a.oj, md.C, ms, md.off);
  if (a.ms) store_vec<R>(a.ms + (b * TT + TT - 1) * R, ms);
  double mc[R], Pc[R][R], mn[R], Pn[R][R];
  if (TT >= 2) load_state<R>(ws + (TT - 2) * K * B + b, B, mc, Pc);
  for (long long t = TT - 2; t >= 0; --t) {
    if (t >= 1) load_state<R>(ws + (t - 1) * K * B + b, B, mn, Pn);
    double J[R][R], d[R];
    ok = rts_gain<R, AI>(mc, Pc, md.A, md.Q, J, d) && ok;
    double msn[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = d[i];
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(J[i][k], ms[k], s);
      msn[i] = s;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = msn[i];
    project_store<R, N, CI>(outb + t * a.ot, a.oj, md.C, ms, md.off);
    if (a.ms) store_vec<R>(a.ms + (b * TT + t) * R, ms);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      mc[i] = mn[i];
#pragma unroll
      for (int j = 0; j < R; ++j) Pc[i][j] = Pn[i][j];
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
}

// ===========================================================================
// algo 2 kernels
// ===========================================================================
struct Lane {
  long long c, b;
  EKS_DEV bool init(long long B, long long NC) {
    const long long lane = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (lane >= NC * B) return false;
    c = lane / B;
    b = lane - c * B;
    return true;
  }
};

template <int R, int N, int E, typename T, typename YT, bool AI, bool CI>
__global__ __launch_bounds__(256) void k_c1_elem(SmoothArgs a, ChunkPlan p) {
  constexpr int EE = E > 0 ? E : 1;
  Lane ln;
  const long long B = a.B, TT = a.T;
  if (!ln.init(B, p.NC)) return;
  const long long c = ln.c, b = ln.b;
  const bool median = a.median != 0;
  Model<R, N> md;
  md.load(a.params + b * ParamLayout<R, N>::len, c == 0);
  if (c == 0 && !md.template valid<AI, CI>()) flag(a.status, b, EKS_STATUS_BAD_MODEL);
  YT *ybuf = (YT *)(a.ws + p.y_off);
  double *evbuf = (double *)(a.ws + p.ev_off);
  const long long s = c * p.L, e = min(TT, s + p.L);
  const T *ob = (const T *)a.obs + b * a.sb;
  bool ok = true;
  Elem<R> El;
  double m[R], P[R][R];
  NllAcc acc;
  if (c == 0) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = md.m0[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
    }
  } else {
    El.set_identity();
  }
  T cur[EE][N], nxt[EE][N];
  if constexpr (E > 0) load_step<E, N, T>(ob + s * a.st, a.se, a.sj, cur);
  for (long long t = s; t < e; ++t) {
    const T *pt = ob + t * a.st;
    if constexpr (E > 0) {
      if (t + 1 < e) load_step<E, N, T>(pt + a.st, a.se, a.sj, nxt);
    }
    double avg[N], rv[N], y[N];
    reduce_step<E, N, T>(cur, pt, a.se, a.sj, a.E, median, avg, rv);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      ybuf[(t * N + j) * B + b] = (YT)avg[j];
      evbuf[(t * N + j) * B + b] = rv[j];
      y[j] = avg[j] - md.off[j];
    }
    if (c == 0) {
      if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
      kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
    } else {
      elem_absorb<R, N, AI, CI>(El, md.A, md.Q, md.C, y, rv, ok);
    }
    if constexpr (E > 0) {
#pragma unroll
      for (int q = 0; q < E; ++q)
#pragma unroll
        for (int j = 0; j < N; ++j) cur[q][j] = nxt[q][j];
    }
  }
  if (c == 0) {
    // chunk 0 summarised as the known filtered state: Ab = 0, bb = m, Cb = P
    El.set_identity();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      El.bb[i] = m[i];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        El.Ab[i][j] = 0.0;
        El.Cb[i][j] = P[i][j];
      }
    }
  }
  El.store((double *)(a.ws + p.elem_off) + (c * Elem<R>::len) * B + b, B);
  if (!ok) flag(a.status, b, c == 0 ? EKS_STATUS_SINGULAR : EKS_STATUS_SCAN);
}

template <int R, int N>
__global__ __launch_bounds__(64) void k_c2_fscan(SmoothArgs a, ChunkPlan p) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long B = a.B;
  if (b >= B) return;
  constexpr int KS = R + Sym<R>::len;
  const double *elem = (const double *)(a.ws + p.elem_off);
  double *cst = (double *)(a.ws + p.cstart_off);
  double m[R], P[R][R];
  {
    using L = ParamLayout<R, N>;
    const double *pp = a.params + b * L::len;
    load_vec<R>(pp + L::m0, m);
    load_mat<R, R>(pp + L::S0, P);
    store_state<R>(cst + b, B, m, P);  // chunk 0 starts from the prior
  }
  Elem<R> El;
  El.load(elem + b, B);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    m[i] = El.bb[i];
#pragma unroll
    for (int j = 0; j < R; ++j) P[i][j] = El.Cb[i][j];
  }
  bool ok = true;
  for (long long c = 1; c < p.NC; ++c) {
    store_state<R>(cst + (c * KS) * B + b, B, m, P);
    if (c + 1 < p.NC) {
      El.load(elem + (c * Elem<R>::len) * B + b, B);
      ok = compose_state<R>(m, P, El) && ok;
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SCAN);
}

// y / ev of step t (time-major planes) with the centring offset applied
template <int N, typename YT>
EKS_DEV void read_yev(const YT *ybuf, const double *evbuf, long long t, long long B, long long b,
                      const double (&off)[N], double (&y)[N], double (&rv)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    y[j] = (double)ybuf[(t * N + j) * B + b] - off[j];
    rv[j] = evbuf[(t * N + j) * B + b];
  }
}

template <int R, int N, typename YT, bool AI, bool CI>
__global__ __launch_bounds__(256) void k_c3_rerun(SmoothArgs a, ChunkPlan p) {
  Lane ln;
  const long long B = a.B, TT = a.T;
  if (!ln.init(B, p.NC)) return;
  const long long c = ln.c, b = ln.b;
  constexpr int KS = R + Sym<R>::len;
  Model<R, N> md;
  md.load(a.params + b * ParamLayout<R, N>::len, false);
  const YT *ybuf = (const YT *)(a.ws + p.y_off);
  const double *evbuf = (const double *)(a.ws + p.ev_off);
  double *ckpt = (double *)(a.ws + p.ckpt_off) + (c * p.NSUB * KS) * B + b;
  double m[R], P[R][R];
  load_state<R>((const double *)(a.ws + p.cstart_off) + (c * KS) * B + b, B, m, P);
  const long long s = c * p.L, e = min(TT, s + p.L);
  double G[R][R], g[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    g[i] = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) G[i][j] = (i == j) ? 1.0 : 0.0;
  }
  bool ok = true;
  NllAcc acc;
  int sub = 0, k = 0;
  double y[N], rv[N], yn[N], rvn[N];
  read_yev<N, YT>(ybuf, evbuf, s, B, b, md.off, y, rv);
  for (long long t = s; t < e; ++t) {
    if (t + 1 < e) read_yev<N, YT>(ybuf, evbuf, t + 1, B, b, md.off, yn, rvn);
    if (sub == 0) store_state<R>(ckpt + (k * KS) * B, B, m, P);
    if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
    kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
    if (t + 1 < TT) {
      double J[R][R], d[R], GJ[R][R];
      ok = rts_gain<R, AI>(m, P, md.A, md.Q, J, d) && ok;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        double sg = g[i];
#pragma unroll
        for (int q = 0; q < R; ++q) sg = fma(G[i][q], d[q], sg);
        g[i] = sg;
      }
      matmul<R, R, R>(G, J, GJ);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) G[i][j] = GJ[i][j];
    } else {  // ms[T-1] = mf[T-1]: the map ends in a constant
#pragma unroll
      for (int i = 0; i < R; ++i) {
        double sg = g[i];
#pragma unroll
        for (int q = 0; q < R; ++q) sg = fma(G[i][q], m[q], sg);
        g[i] = sg;
      }
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) G[i][j] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
      y[j] = yn[j];
      rv[j] = rvn[j];
    }
    if (++sub == p.LS) {
      sub = 0;
      ++k;
    }
  }
  double *bw = (double *)(a.ws + p.bwd_off) + (c * (R * R + R)) * B + b;
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) bw[(i * R + j) * B] = G[i][j];
#pragma unroll
  for (int i = 0; i < R; ++i) bw[(R * R + i) * B] = g[i];
  ((double *)(a.ws + p.nllp_off))[c * B + b] = acc.value((double)(e - s) * N);
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
}

template <int R>
__global__ __launch_bounds__(64) void k_c4_bscan(SmoothArgs a, ChunkPlan p) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long B = a.B;
  if (b >= B) return;
  const double *bw = (const double *)(a.ws + p.bwd_off);
  double *msend = (double *)(a.ws + p.msend_off);
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = 0.0;
  for (long long c = p.NC - 1; c >= 0; --c) {
    const double *q = bw + (c * (R * R + R)) * B + b;
    double nx[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = q[(R * R + i) * B];
#pragma unroll
      for (int j = 0; j < R; ++j) s = fma(q[(i * R + j) * B], ms[j], s);
      nx[i] = s;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = nx[i];
    if (c >= 1) {
#pragma unroll
      for (int i = 0; i < R; ++i) msend[((c - 1) * R + i) * B + b] = ms[i];
    }
  }
  if (a.nll) {
    const double *np_ = (const double *)(a.ws + p.nllp_off);
    double s = 0.0;
    for (long long c = 0; c < p.NC; ++c) s += np_[c * B + b];
    a.nll[b] = s;
  }
}

template <int R, int N, typename YT, bool AI, bool CI, int LS>
__global__ __launch_bounds__(256) void k_c5_final(SmoothArgs a, ChunkPlan p) {
  Lane ln;
  const long long B = a.B, TT = a.T;
  if (!ln.init(B, p.NC)) return;
  const long long c = ln.c, b = ln.b;
  constexpr int KS = R + Sym<R>::len;
  Model<R, N> md;
  md.load(a.params + b * ParamLayout<R, N>::len, false);
  const YT *ybuf = (const YT *)(a.ws + p.y_off);
  const double *evbuf = (const double *)(a.ws + p.ev_off);
  const double *ckpt = (const double *)(a.ws + p.ckpt_off) + (c * p.NSUB * KS) * B + b;
  double ms[R];
  if (c + 1 < p.NC) {
    const double *me = (const double *)(a.ws + p.msend_off);
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = me[(c * R + i) * B + b];
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = 0.0;
  }
  const long long s = c * p.L, e = min(TT, s + p.L);
  const int nsub = (int)((e - s + LS - 1) / LS);
  bool ok = true;
  NllAcc dummy;
  double *outb = a.out + b * a.ob;
  for (int k = nsub - 1; k >= 0; --k) {
    const long long t0 = s + (long long)k * LS;
    const int cnt = (int)min((long long)LS, e - t0);
    double m[R], P[R][R];
    load_state<R>(ckpt + (k * KS) * B, B, m, P);
    double Jr[LS][R][R], dr[LS][R];
#pragma unroll
    for (int j = 0; j < LS; ++j) {
      if (j < cnt) {
        const long long t = t0 + j;
        double y[N], rv[N];
        read_yev<N, YT>(ybuf, evbuf, t, B, b, md.off, y, rv);
        if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
        kf_update<R, N, CI>(m, P, md.C, y, rv, dummy, ok);
        if (t + 1 < TT) {
          ok = rts_gain<R, AI>(m, P, md.A, md.Q, Jr[j], dr[j]) && ok;
        } else {
#pragma unroll
          for (int i = 0; i < R; ++i) {
            dr[j][i] = m[i];
#pragma unroll
            for (int q = 0; q < R; ++q) Jr[j][i][q] = 0.0;
          }
        }
      }
    }
#pragma unroll
    for (int j = LS - 1; j >= 0; --j) {
      if (j < cnt) {
        const long long t = t0 + j;
        double nx[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double sm = dr[j][i];
#pragma unroll
          for (int q = 0; q < R; ++q) sm = fma(Jr[j][i][q], ms[q], sm);
          nx[i] = sm;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) ms[i] = nx[i];
        project_store<R, N, CI>(outb + t * a.ot, a.oj, md.C, ms, md.off);
        if (a.ms) store_vec<R>(a.ms + (b * TT + t) * R, ms);
      }
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
}

// ===========================================================================
// host launcher for one (R, N, AI, CI)
// ===========================================================================
template <typename F>
int dispatch_members_c(int E, F &&f) {
  switch (E) {
    case 3: return f(ic<3>{});
    case 4: return f(ic<4>{});
    case 5: return f(ic<5>{});
    default: return f(ic<0>{});
  }
}

template <int R, int N, bool AI, bool CI>
int launch_shape(const SmoothArgs &a, int algo, long long L) {
  const bool f32 = a.dtype == EKS_F32;
  if (algo == 1) {
    auto go = [&](auto tag) -> int {
      using Tp = decltype(tag);
      return dispatch_members_c(a.E, [&](auto Ec) {
        constexpr int EE = decltype(Ec)::value;
        prof_call_begin();
        prof_mark(a.stream, "k_smooth_seq");
        hipLaunchKernelGGL((k_smooth_seq<R, N, EE, Tp, AI, CI>), dim3(grid_for(a.B, 64)),
                           dim3(64), 0, a.stream, a);
        prof_call_end(a.stream);
        return check_launch("k_smooth_seq");
      });
    };
    return f32 ? go(float{}) : go(double{});
  }
  const ChunkPlan p = make_plan(a.B, a.T, R, N, L);
  const unsigned g256 = grid_for(p.NC * a.B, 256);
  const unsigned g64 = grid_for(a.B, 64);
  // y is stored as float when it is exactly a member value (odd-E median of f32)
  const bool y32 = f32 && a.median && (a.E == 3 || a.E == 5);
  auto rest = [&](auto ytag) -> int {
    using YT = decltype(ytag);
    prof_mark(a.stream, "k_c2_fscan");
    hipLaunchKernelGGL((k_c2_fscan<R, N>), dim3(g64), dim3(64), 0, a.stream, a, p);
    if (int rc = check_launch("k_c2_fscan")) return rc;
    prof_mark(a.stream, "k_c3_rerun");
    hipLaunchKernelGGL((k_c3_rerun<R, N, YT, AI, CI>), dim3(g256), dim3(256), 0, a.stream, a, p);
    if (int rc = check_launch("k_c3_rerun")) return rc;
    prof_mark(a.stream, "k_c4_bscan");
    hipLaunchKernelGGL((k_c4_bscan<R>), dim3(g64), dim3(64), 0, a.stream, a, p);
    if (int rc = check_launch("k_c4_bscan")) return rc;
    constexpr int LS = R <= 2 ? 8 : 4;
    prof_mark(a.stream, "k_c5_final");
    hipLaunchKernelGGL((k_c5_final<R, N, YT, AI, CI, LS>), dim3(g256), dim3(256), 0, a.stream, a,
                       p);
    prof_call_end(a.stream);
    return check_launch("k_c5_final");
  };
  auto k1 = [&](auto tag, auto ytag) -> int {
    using Tp = decltype(tag);
    using YT = decltype(ytag);
    return dispatch_members_c(a.E, [&](auto Ec) {
      constexpr int EE = decltype(Ec)::value;
      prof_call_begin();
      prof_mark(a.stream, "k_c1_elem");
      hipLaunchKernelGGL((k_c1_elem<R, N, EE, Tp, YT, AI, CI>), dim3(g256), dim3(256), 0,
                         a.stream, a, p);
      return check_launch("k_c1_elem");
    });
  };
  int rc;
  if (y32) {
    rc = k1(float{}, float{});
    return rc ? rc : rest(float{});
  }
  rc = f32 ? k1(float{}, double{}) : k1(double{}, double{});
  return rc ? rc : rest(double{});
}

// per-shape entry points (defined in eks_shape_*.hip)
int launch_22(const SmoothArgs &a, int algo, long long L);
int launch_34(const SmoothArgs &a, int algo, long long L);
int launch_36(const SmoothArgs &a, int algo, long long L);
int launch_38(const SmoothArgs &a, int algo, long long L);

}  // namespace eks
