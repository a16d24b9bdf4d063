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

template <int R, typename T, int E>
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
  constexpr bool kYev = is_yev<T>::value;  // the caller's y / ev planes (EKS_YEV32 / 64)
  using YT = typename yev_y<T>::type;
  const YT *ob = (const YT *)a.obs + (kYev ? 0 : b * a.sb);
  const double *evp = kYev ? (const double *)((const char *)a.obs +
                                              yev_ev_offset(B, TT, n, sizeof(YT)))
                           : nullptr;
  bool ok = true;
  NllAcc acc;
  for (long long t = 0; t < TT; ++t) {
    if (t > 0) kf_predict<R, kAGen>(m, P, A, Q);
    for (int j = 0; j < n; ++j) {
      double avg, var;
      if constexpr (kYev) {
        avg = (double)ob[(t * n + j) * B + b];
        var = evp[(t * n + j) * B + b];
      } else {
        column_reduce<E, YT>(ob + t * a.st + j * a.sj, a.se, a.E, median, avg, var);
      }
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

// ---------------------------------------------------------------------------
// Time-parallel form (few long trajectories: the 5+ camera batch of
// eks/multiview_pca_smoother.py:641-666 is ~17 keypoints x 50 k frames, one
// lane per trajectory leaves the GPU idle).  Algo 2's pipeline with the
// observation model streamed row by row:
//   K1 k_rt_c1   (chunk, trajectory) lanes: ensemble of each step's n columns
//                (y / ev planes for K3), the chunk's filtering element built one
//                scalar row at a time (chunk 0: the filter from the prior)
//   K2           the chunk scan of algo 2 (k_c2_fscan / _g, R-only)
//   K3 k_rt_c3   filter re-run from the chunk's start state, every step's RTS
//                gain (J_t, d_t) into the (J, d) planes, the chunk's RTS map
//                and NLL share
//   K4           the backward chunk scan of algo 2 (k_c4_bscan / _g)
//   K5 k_rt_c5   ms_t = J_t ms_{t+1} + d_t over the chunk, projected with the
//                n rows of C
// Same arithmetic per step as k_smooth_seq_rt (kf_update_row_rt, rts_gain),
// the chunk algebra of algo 2 (tests/test_gpu_rt.py).
// ---------------------------------------------------------------------------
template <int R>
EKS_DEV void load_row(const double *c, double (&cr)[R]) {
#pragma unroll
  for (int k = 0; k < R; ++k) cr[k] = c[k];
}

// ring of the columns' model rows (c_j, offset_j)
template <int R>
struct RowRing {
  double c[kRtDP][R], o[kRtDP];
  EKS_DEV void fetch(int k, const double *C, const double *off, int j) {
#pragma unroll
    for (int u = 0; u < R; ++u) c[k][u] = C[j * R + u];
    o[k] = off[j];
  }
};

template <int R, typename T, int E>
__global__ __launch_bounds__(kBlock) void k_rt_c1(SmoothArgs a, ChunkPlan p) {
  zero_scan_sync(a, p);
  Lane<false> ln;
  if (!ln.init(a.B, p.NC)) return;
  const long long c = ln.c;
  const unsigned b = ln.b;
  const long long B = a.B, TT = a.T;
  const int n = a.n;
  const bool median = a.median != 0;
  const double *pp = a.params + (long long)b * param_stride<R, 0>(n);
  using L = ParamLayout<R, 0>;
  double A[R][R], Q[R][R];
  load_mat<R, R>(pp + L::A, A);
  load_mat<R, R>(pp + L::Q, Q);
  const double *C = pp + L::C, *off = C + (long long)n * R;
  constexpr bool kYev = is_yev<T>::value;  // the caller's y / ev planes (EKS_YEV32 / 64)
  using YT = typename yev_y<T>::type;
  double *ybuf = (double *)(a.ws + p.y_off), *evbuf = (double *)(a.ws + p.ev_off);
  const YT *ob = kYev ? nullptr : (const YT *)a.obs + (long long)b * a.sb;
  const long long s = c * p.L, e = min(TT, s + p.L);
  const bool first = c == 0;
  bool ok = true;
  Elem<R> El;
  El.set_identity();
  double m[R], P[R][R];
  if (first) {
    load_vec<R>(pp + L::m0, m);
    load_mat<R, R>(pp + L::S0, P);
  }
  NllAcc acc;
  auto begin = [&](long long t) {
    if (first) {
      if (t > 0) kf_predict<R, kAGen>(m, P, A, Q);
    } else {
      elem_predict<R, kAGen>(El, A, Q);
    }
  };
  auto end = [&](long long) { acc.renorm(); };
  auto absorb = [&](const double (&cr)[R], double y, double var) {
    if (first)
      kf_update_row_rt<R>(m, P, cr, y, var, acc, ok);
    else
      absorb_gen_row<R>(El, cr, y, var, ok, &acc);
  };
  RowRing<R> rr;
  if constexpr (kYev || E > 0) {
    constexpr int EE = E > 0 ? E : 1;
    YT mr[kRtDP][EE];        // members (member input)
    YT yr[kRtDP];            // plane values (y / ev input)
    double er[kRtDP];
    auto fetch = [&](int k, long long t, int j) {
      rr.fetch(k, C, off, j);
      if constexpr (kYev) {
        yr[k] = pl((const YT *)p.ysrc, t * n + j, B, b);
        er[k] = pl((const double *)p.evsrc, t * n + j, B, b);
      } else {
        const YT *pc = ob + t * a.st + j * a.sj;
#pragma unroll
        for (int u = 0; u < EE; ++u) mr[k][u] = pc[(long long)u * a.se];
      }
    };
    auto col = [&](int k, long long t, int j) {
      double avg, var;
      if constexpr (kYev) {
        avg = (double)yr[k];
        var = er[k];
      } else {
        ensemble_reduce<EE, YT>(mr[k], median, avg, var);
        pl(ybuf, t * n + j, B, b) = avg;
        pl(evbuf, t * n + j, B, b) = var;
      }
      absorb(rr.c[k], avg - rr.o[k], var);
    };
    rt_columns(s, e, n, fetch, col, begin, end);
  } else {  // runtime E: no member ring
    for (long long t = s; t < e; ++t) {
      begin(t);
      for (int j = 0; j < n; ++j) {
        double avg, var, cr[R];
        column_reduce<0, YT>(ob + t * a.st + j * a.sj, a.se, a.E, median, avg, var);
        pl(ybuf, t * n + j, B, b) = avg;
        pl(evbuf, t * n + j, B, b) = var;
        load_row<R>(C + j * R, cr);
        absorb(cr, avg - off[j], var);
      }
      end(t);
    }
  }
  if (first) {  // the filtered state (Ab = 0), as c1_chunk
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
  El.store((double *)(a.ws + p.elem_off) + ((long long)b * p.NC + c) * Elem<R>::len, 1);
  if (!ok) flag(a.status, b, first ? EKS_STATUS_SINGULAR : EKS_STATUS_SCAN);
}

template <int R, typename YT>
__global__ __launch_bounds__(kBlock) void k_rt_c3(SmoothArgs a, ChunkPlan p) {
  Lane<false> ln;
  if (!ln.init(a.B, p.NC)) return;
  const long long c = ln.c;
  const unsigned b = ln.b;
  const long long B = a.B, TT = a.T;
  const int n = a.n;
  constexpr int KS = R + Sym<R>::len, MR = R * R + R;
  const double *pp = a.params + (long long)b * param_stride<R, 0>(n);
  using L = ParamLayout<R, 0>;
  double A[R][R], Q[R][R];
  load_mat<R, R>(pp + L::A, A);
  load_mat<R, R>(pp + L::Q, Q);
  const double *C = pp + L::C, *off = C + (long long)n * R;
  const YT *ybuf = (const YT *)p.ysrc;
  const double *evbuf = (const double *)p.evsrc;
  double *jdp = (double *)(a.ws + p.jd_off);
  double m[R], P[R][R], G[R][R], g[R];
  load_state_pl<R>((const double *)(a.ws + p.cstart_off), c * KS, B, b, m, P);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    g[i] = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) G[i][j] = (i == j) ? 1.0 : 0.0;
  }
  const long long s = c * p.L, e = min(TT, s + p.L);
  bool ok = true;
  NllAcc acc;
  RowRing<R> rr;
  YT yr[kRtDP];
  double er[kRtDP];
  auto fetch = [&](int k, long long t, int j) {
    rr.fetch(k, C, off, j);
    yr[k] = pl(ybuf, t * n + j, B, b);
    er[k] = pl(evbuf, t * n + j, B, b);
  };
  auto col = [&](int k, long long, int) {
    kf_update_row_rt<R>(m, P, rr.c[k], (double)yr[k] - rr.o[k], er[k], acc, ok);
  };
  auto begin = [&](long long t) {
    if (t > 0) kf_predict<R, kAGen>(m, P, A, Q);
  };
  auto end = [&](long long t) {
    acc.renorm();
    if (!p.smooth) return;
    double J[R][R], d[R];
    if (t + 1 < TT) {
      ok = rts_gain<R, kAGen>(m, P, A, Q, J, d) && ok;
    } else {  // ms[T-1] = mf[T-1]: the map ends in a constant
#pragma unroll
      for (int i = 0; i < R; ++i) {
        d[i] = m[i];
#pragma unroll
        for (int k = 0; k < R; ++k) J[i][k] = 0.0;
      }
    }
    store_jd<R>(jdp, t, B, b, J, d);
    double GJ[R][R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double sg = g[i];
#pragma unroll
      for (int u = 0; u < R; ++u) sg = fma(G[i][u], d[u], sg);
      g[i] = sg;
    }
    matmul<R, R, R>(G, J, GJ);
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int k = 0; k < R; ++k) G[i][k] = GJ[i][k];
  };
  rt_columns(s, e, n, fetch, col, begin, end);
  pl((double *)(a.ws + p.nllp_off), c, B, b) = acc.value((double)(e - s) * n);
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
  if (!p.smooth) return;
  double *bw = (double *)(a.ws + p.bwd_off) + ((long long)b * p.NC + c) * MR;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    bw[R * R + i] = g[i];
#pragma unroll
    for (int k = 0; k < R; ++k) bw[i * R + k] = G[i][k];
  }
}

template <int R>
__global__ __launch_bounds__(kBlock) void k_rt_c5(SmoothArgs a, ChunkPlan p) {
  Lane<false> ln;
  if (!ln.init(a.B, p.NC)) return;
  const long long c = ln.c;
  const unsigned b = ln.b;
  const long long B = a.B, TT = a.T;
  const int n = a.n;
  constexpr int MR = R * R + R;
  const double *pp = a.params + (long long)b * param_stride<R, 0>(n);
  const double *C = pp + ParamLayout<R, 0>::C, *off = C + (long long)n * R;
  double ms[R];
  c5_ms_in<R, false>(a, p, c, b, ms);
  const double *jdp = (const double *)(a.ws + p.jd_off);
  const long long s = c * p.L, e = min(TT, s + p.L);
  double *outb = a.out + (long long)b * a.ob;
  for (long long t = e - 1; t >= s; --t) {
    double f[MR], nx[R];
#pragma unroll
    for (int k = 0; k < MR; ++k) f[k] = pl(jdp, t * MR + k, B, b);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double sm = f[R * R + i];
#pragma unroll
      for (int k = 0; k < R; ++k) sm = fma(f[i * R + k], ms[k], sm);
      nx[i] = sm;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = nx[i];
    project_rt<R>(outb + t * a.ot, a.oj, C, off, n, ms);
    if (a.ms) store_vec<R>(a.ms + ((long long)b * TT + t) * R, ms);
  }
}

// the time-parallel form runs when the trajectories alone do not fill the
// GPU (chunk_len < T) unless eks_debug_set(EKS_DBG_RT_FORM) forces one
bool rt_chunked(long long B, long long T, int r) {
  if (g_rt_form == 1) return false;
  if (g_rt_form == 2) return T >= 2;
  return chunk_len(B, T, r) < T;
}

long long rt_chunk_len(long long B, long long T, int r, bool smooth) {
  long long L = smooth ? chunk_len_smooth(B, T, r) : chunk_len(B, T, r);
  if (L >= T) L = std::max(1LL, (T + 1) / 2);  // forced on a short trajectory: two chunks
  return L;
}

size_t rt_workspace_bytes(long long B, long long T, int n, int r) {
  size_t w = seq_workspace_bytes(B, T, r);
  if (!rt_chunked(B, T, r)) return w;
  for (int sm = 0; sm < 2; ++sm)
    w = std::max(w, make_plan(B, T, r, n, rt_chunk_len(B, T, r, sm != 0), true).total);
  return w;
}

template <int R, typename T>
int launch_rt_chunked(const SmoothArgs &a) {
  ChunkPlan p = make_plan(a.B, a.T, R, a.n, rt_chunk_len(a.B, a.T, R, a.out != nullptr), true);
  p.smooth = a.out != nullptr;
  p.yB = a.B;
  p.jd = p.smooth ? 1 : 0;
  // K3 reads the caller's planes (their y type) or the f64 planes K1 wrote
  using YT = typename std::conditional<is_yev<T>::value, typename yev_y<T>::type, double>::type;
  if constexpr (is_yev<T>::value) {
    p.ysrc = (const char *)a.obs;
    p.evsrc = p.ysrc + yev_ev_offset(a.B, a.T, a.n, sizeof(YT));
  } else {
    p.ysrc = a.ws + p.y_off;
    p.evsrc = a.ws + p.ev_off;
  }
  const unsigned gch = grid_for(p.NC * a.B, kBlock), g64 = grid_for(a.B, 64);
  const bool wave_scan = p.NC > wave_scan_chunks();
  int rc;
  prof_call_begin();
  prof_mark(a.stream, "k_rt_c1");
  auto k1 = [&](auto Ec) {
    constexpr int EE = decltype(Ec)::value;
    hipLaunchKernelGGL((k_rt_c1<R, T, EE>), dim3(gch), dim3(kBlock), 0, a.stream, a, p);
    return check_launch("k_rt_c1");
  };
  if constexpr (is_yev<T>::value)
    rc = k1(ic<0>{});  // the members are not read: E does not matter
  else
    rc = dispatch_members_c(a.E, k1);
  if (rc) return rc;
  prof_mark(a.stream, "k_c2_fscan");
  if (!wave_scan)
    hipLaunchKernelGGL((k_c2_fscan<R, 0>), dim3(g64), dim3(64), 0, a.stream, a, p);
  else
    hipLaunchKernelGGL((k_c2_fscan_g<R, 0>), dim3((unsigned)(a.B * p.G)), dim3(256), 0, a.stream,
                       a, p);
  if ((rc = check_launch("k_c2_fscan"))) return rc;
  prof_mark(a.stream, "k_rt_c3");
  hipLaunchKernelGGL((k_rt_c3<R, YT>), dim3(gch), dim3(kBlock), 0, a.stream, a, p);
  if ((rc = check_launch("k_rt_c3"))) return rc;
  if (!p.smooth) {
    prof_mark(a.stream, "k_c4_nll");
    hipLaunchKernelGGL((k_c4_nll<R>), dim3((unsigned)a.B), dim3(64), 0, a.stream, a, p);
    prof_call_end(a.stream);
    return check_launch("k_c4_nll");
  }
  prof_mark(a.stream, "k_c4_bscan");
  if (!wave_scan)
    hipLaunchKernelGGL((k_c4_bscan<R>), dim3(g64), dim3(64), 0, a.stream, a, p);
  else
    hipLaunchKernelGGL((k_c4_bscan_g<R>), dim3((unsigned)(a.B * p.G)), dim3(256), 0, a.stream, a,
                       p);
  if ((rc = check_launch("k_c4_bscan"))) return rc;
  prof_mark(a.stream, "k_rt_c5");
  hipLaunchKernelGGL((k_rt_c5<R>), dim3(gch), dim3(kBlock), 0, a.stream, a, p);
  prof_call_end(a.stream);
  return check_launch("k_rt_c5");
}

int launch_rt(const SmoothArgs &a) {
  // algo 1 asks for the sequential form (batch.smooth's re-run after a
  // time-parallel breakdown)
  const bool chunked = a.algo != 1 && rt_chunked(a.B, a.T, a.r);
  auto go = [&](auto rtag, auto ttag) -> int {
    constexpr int R = decltype(rtag)::value;
    using T = decltype(ttag);
    if (chunked) return launch_rt_chunked<R, T>(a);
    prof_call_begin();
    prof_mark(a.stream, "k_smooth_seq_rt");
    auto k = [&](auto Ec) {
      constexpr int EE = decltype(Ec)::value;
      hipLaunchKernelGGL((k_smooth_seq_rt<R, T, EE>), dim3(grid_for(a.B, 64)), dim3(64), 0,
                         a.stream, a);
      return check_launch("k_smooth_seq_rt");
    };
    int rc;
    if constexpr (is_yev<T>::value)
      rc = k(ic<0>{});
    else
      rc = dispatch_members_c(a.E, k);
    prof_call_end(a.stream);
    return rc;
  };
  auto by_type = [&](auto rtag) -> int {
    switch (a.dtype) {
      case EKS_F32: return go(rtag, float{});
      case EKS_F64: return go(rtag, double{});
      case EKS_YEV32: return go(rtag, YevIn<float>{});
      default: return go(rtag, YevIn<double>{});
    }
  };
  switch (a.r) {
    case 2: return by_type(ic<2>{});
    case 3: return by_type(ic<3>{});
    default:
      return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth: latent r=%d not compiled in (2, 3)", a.r);
  }
}

}  // namespace eks
