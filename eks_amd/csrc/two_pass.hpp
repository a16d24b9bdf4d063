// algo 3 of eks_smooth: the exact smoother in TWO passes over the member
// predictions (included by smooth_impl.hpp, inside namespace eks).
//
// algo 2 spills the ensemble output (y, ev: 24 B per keypoint-timestep at
// n = 2) and re-runs the filter twice (K3, K5) to obtain the smoothed mean
// entering each chunk.  algo 3 gets those boundary means from the filtering
// elements alone -- compose_state_rts: the chunk-level RTS map
// ms_b = G ms_e + g follows from the boundary's filtered state and the
// chunk's element -- so the members are read once to build elements and
// once to smooth, and nothing per step is stored in between:
//
//  P1 k3_elem    fine chunk (L = 16 steps) per lane, members -> ensemble ->
//                filtering element (planes); the 4 waves of a block are 4
//                consecutive fine chunks of 64 trajectories, composed (LDS
//                tree) into one coarse (64-step) element
//  P2 k3_coarse  8 waves (x S sub-parts) per 64 (/ S) trajectories over the
//                coarse elements (parallel scan, shuffles + LDS): filtered
//                state entering each coarse chunk, coarse RTS maps, then the
//                smoothed mean at every coarse boundary
//  P3 k3_fine    one lane per (coarse chunk, trajectory): the same over its 4
//                fine elements -> filtered state entering / smoothed mean at
//                the last step of every fine chunk
//  P4 k3_final_s fine chunk per lane: members again -> ensemble -> filter
//                from the exact start state; the filtered states of the first
//                8-step sub-chunk are kept in LDS, the second's in registers;
//                RTS backwards from the chunk's known last-step mean (no
//                filter re-run); writes C ms + offset (and ms / the chunk's
//                NLL share).  k3_final is the earlier (y, ev)-stash variant.
//
// HBM bytes per keypoint-timestep (single view, E = 5): P1 40 + 7 (fine
// elements) + 1.75 (coarse), P2 ~2, P3 7 + 3.5, P4 40 + 3.5 + 16 ~= 121,
// against algo 2's ~139, and one fewer filter pass.
//
// Exactness: P4 runs the reference recursion (kf_update / rts_gain) from
// start states and last-step means that equal the sequential ones up to the
// rounding of the element compositions (contractive, as in algo 2).  A
// singular boundary covariance (exactly observed state at a chunk's last
// step) sets EKS_STATUS_SCAN; batch.smooth(check=True) then re-runs algo 1.

#ifndef EKS_K3_FPL
#define EKS_K3_FPL 1     // fine chunks per k3_elem lane (2: 128-step coarse chunks, halves k3_coarse but 256 VGPRs in k3_elem, measured slower)
#endif
#ifndef EKS_K3_WV
#define EKS_K3_WV 4      // waves per k3_elem block
#endif
constexpr int kFPL = EKS_K3_FPL, kWV = EKS_K3_WV;
constexpr int kNF = kFPL * kWV;  // fine chunks per coarse chunk
#ifndef EKS_K3_D
#define EKS_K3_D 2       // member prefetch distance (steps) of k3_elem
#endif
#ifndef EKS_K3_DF
#define EKS_K3_DF 2      // member prefetch distance (steps) of k3_final
#endif
constexpr int kNS = 2;   // sub-chunks per fine chunk in k3_final
// occupancy target of the streaming kernels: their LDS / state already limit
// them to 2 waves per SIMD, so the compiler may spend the whole register file
// on keeping member prefetches in flight instead of trimming it for waves
// that could never be resident
#ifndef EKS_K3_FULLPATH
#define EKS_K3_FULLPATH 0  // 1: guard-free unrolled step loop in k3_final_s (measured 35 % slower)
#endif
// Keep the member prefetches where they are issued: without a scheduling
// barrier the machine scheduler sinks them next to their use (to save
// registers), so every step waits for its own loads (vmcnt(0) each step).
#ifndef EKS_PIN
#define EKS_PIN 0  // measured neutral
#endif
#if EKS_PIN
#define EKS_PIN_LOADS() __builtin_amdgcn_sched_barrier(0)
#else
#define EKS_PIN_LOADS() ((void)0)
#endif
#ifndef EKS_K3_WPE
#define EKS_K3_WPE  // e.g. __attribute__((amdgpu_waves_per_eu(2, 2))): measured spills
#endif
#ifndef EKS_K3E_WPE
#define EKS_K3E_WPE
#endif
#ifndef EKS_K3_MERGED
#define EKS_K3_MERGED 0  // 1: the fine walk inside the final pass (measured slower: prologue latency)
#endif


constexpr int sub_len3(int r, int n) { return sub_len_c(r, n); }
constexpr int fine_len3(int r, int n) { return kNS * sub_len3(r, n); }

struct Plan3 {
  long long L = 16, NCf = 0, NCc = 0;
  size_t fel_off = 0, cel_off = 0, ccs_off = 0, cmap_off = 0, cms_off = 0, fcs_off = 0,
         fms_off = 0, nllp_off = 0, prm_off = 0, total = 0;
};

inline Plan3 make_plan3(long long B, long long T, int r, int n) {
  Plan3 p;
  p.L = fine_len3(r, n);
  p.NCf = (T + p.L - 1) / p.L;
  p.NCc = (p.NCf + kNF - 1) / kNF;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align256(off + bytes);
    return o;
  };
  const size_t Bz = (size_t)B;
  p.fel_off = take((size_t)p.NCf * elem_len(r) * Bz * 8);
  p.cel_off = take((size_t)p.NCc * elem_len(r) * Bz * 8);
  p.ccs_off = take((size_t)p.NCc * state_len(r) * Bz * 8);
  p.cmap_off = take((size_t)p.NCc * (r * r + r) * Bz * 8);
  p.cms_off = take((size_t)(p.NCc + 1) * r * Bz * 8);
  if (!EKS_K3_MERGED) {  // per-fine-chunk start states / last-step means (k3_fine)
    p.fcs_off = take((size_t)p.NCf * state_len(r) * Bz * 8);
    p.fms_off = take((size_t)p.NCf * r * Bz * 8);
  }
  p.nllp_off = take((size_t)p.NCf * Bz * 8);
  p.prm_off = take((size_t)param_len(n, r) * Bz * 8);  // k_model_planes
  p.total = off;
  return p;
}

// Step sources of the two member passes: a D-deep register ring of raw step
// data, reduced to (raw average, variance) on use.
template <int E, int N, typename T, int D>
struct MemberRing {
  T v[D][E][N];
  const T *ob;
  long long st, se, sj;
  bool median;
  EKS_DEV void init(const SmoothArgs &a, unsigned b) {
    ob = (const T *)a.obs + (long long)b * a.sb;
    st = a.st;
    se = a.se;
    sj = a.sj;
    median = a.median != 0;
  }
  EKS_DEV void fetch(int slot, long long t) {
#if EKS_NT_LOAD
    const T *p = ob + t * st;
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int j = 0; j < N; ++j) v[slot][e][j] = __builtin_nontemporal_load(p + e * se + j * sj);
#else
    load_step<E, N, T>(ob + t * st, se, sj, v[slot]);
#endif
  }
  EKS_DEV void get(int slot, double (&avg)[N], double (&rv)[N]) const {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      T col[E];
#pragma unroll
      for (int e = 0; e < E; ++e) col[e] = v[slot][e][j];
      ensemble_col<E, T>(col, median, avg[j], rv[j]);
    }
  }
};

// the ensemble handed over as y / ev planes (EKS_YEV32 / EKS_YEV64 inputs)
template <int N, typename YT, int D>
struct YevRing {
  YT y[D][N];
  double ev[D][N];
  const YT *yb;
  const double *eb;
  long long B;
  unsigned b;
  EKS_DEV void init(const SmoothArgs &a, unsigned bb) {
    yb = (const YT *)a.obs;
    eb = (const double *)((const char *)a.obs + yev_ev_offset(a.B, a.T, N, sizeof(YT)));
    B = a.B;
    b = bb;
  }
  EKS_DEV void fetch(int slot, long long t) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
#if EKS_NT_LOAD
      y[slot][j] = __builtin_nontemporal_load(&pl(yb, t * N + j, B, b));
      ev[slot][j] = __builtin_nontemporal_load(&pl(eb, t * N + j, B, b));
#else
      y[slot][j] = pl(yb, t * N + j, B, b);
      ev[slot][j] = pl(eb, t * N + j, B, b);
#endif
    }
  }
  EKS_DEV void get(int slot, double (&avg)[N], double (&rv)[N]) const {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      avg[j] = (double)y[slot][j];
      rv[j] = ev[slot][j];
    }
  }
};

template <int E, int N, typename T, int D>
struct SrcOf {
  using type = MemberRing<E, N, T, D>;
};
template <int E, int N, typename YT, int D>
struct SrcOf<E, N, YevIn<YT>, D> {
  using type = YevRing<N, YT, D>;
};

// element component k of fine / coarse chunk c lives in plane (c * EL + k)
template <int R>
EKS_DEV void store_elem_pl(double *base, long long c, long long B, unsigned b, const Elem<R> &El) {
  El.store(&pl(base, c * Elem<R>::len, B, b), B);
}
template <int R>
EKS_DEV void load_elem_pl(const double *base, long long c, long long B, unsigned b, Elem<R> &El) {
  El.load(&pl(base, c * Elem<R>::len, B, b), B);
}

// ---------------------------------------------------------------------------
// P1: fine elements + coarse aggregates
// ---------------------------------------------------------------------------
template <int R, int N, int E, typename T, int AI, int CI>
__global__ __launch_bounds__(64 * kWV) EKS_K3E_WPE void k3_elem(SmoothArgs a, Plan3 p) {
  constexpr int EL = Elem<R>::len;
  constexpr int D = EKS_K3_D;
  __shared__ double sh[kWV][EL][64];
  // the wave index is uniform: keep it (and every time index) in SGPRs
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const long long B = a.B, TT = a.T;
  const long long ng = (B + 63) / 64;
  const long long cc = blockIdx.x / ng;
  const unsigned b = (unsigned)((blockIdx.x - cc * ng) * 64 + l);
  bool ok = true, okf = true;  // element / composition, and the plain filter of chunk 0
  Elem<R> Acc;  // the lane's kFPL consecutive fine chunks, composed
  Acc.set_identity();
#pragma unroll 1
  for (int u = 0; u < kFPL; ++u) {
  const long long f = cc * kNF + w * kFPL + u;
  const bool live = (long long)b < B && f < p.NCf;
  Elem<R> El;
  El.set_identity();
  if (live) {
    Model<R, N> md;  // structure checked by k_model_planes
    load_model_pl<R, N, AI, CI>((const double *)(a.ws + p.prm_off), B, b, f == 0, md);
    const long long s = f * p.L, e = min(TT, s + p.L);
    typename SrcOf<E, N, T, D>::type src;
    src.init(a, b);
    // the step loop, specialised per chunk kind (hoisted branch: the filter
    // state and the element are never live together).  Full chunks (all but
    // a trajectory's last) run a compile-time loop whose prefetches are
    // unconditional: a load under a lane-divergent `if` is merged into its
    // ring slot by a copy that waits for it, i.e. no prefetch at all.
    auto stream = [&](auto &&absorb) {
      constexpr int LF = fine_len3(R, N);
      if (e - s == LF) {
        // full chunk: the same loads on every path (see k3_final_s); the
        // clamped tail re-reads the last step (a cache hit) instead of branching
#pragma unroll
        for (int q = 0; q < D; ++q) src.fetch(q, s + q);
#pragma unroll 1
        for (int i0 = 0; i0 < LF; i0 += D) {
#pragma unroll
          for (int q = 0; q < D; ++q) {
            const long long t = s + i0 + q;
            double avg[N], rv[N], y[N];
            src.get(q, avg, rv);
            src.fetch(q, min(t + D, s + LF - 1));
            EKS_PIN_LOADS();
#pragma unroll
            for (int j = 0; j < N; ++j) y[j] = avg[j] - md.off[j];
            absorb(t, y, rv);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < D; ++q)
          if (s + q < e) src.fetch(q, s + q);
        for (long long t0 = s; t0 < e; t0 += D) {
#pragma unroll
          for (int q = 0; q < D; ++q) {
            const long long t = t0 + q;
            if (t < e) {
              double avg[N], rv[N], y[N];
              src.get(q, avg, rv);
              if (t + D < e) src.fetch(q, t + D);
              EKS_PIN_LOADS();
#pragma unroll
              for (int j = 0; j < N; ++j) y[j] = avg[j] - md.off[j];
              absorb(t, y, rv);
            }
          }
        }
      }
    };
    if (f == 0) {  // the first chunk: the plain filter from the prior,
                   // summarised as the known filtered state (Ab = 0)
      double m[R], P[R][R];
      NllAcc acc;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        m[i] = md.m0[i];
#pragma unroll
        for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
      }
      stream([&](long long t, const double (&y)[N], const double (&rv)[N]) {
        if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
        kf_update<R, N, CI>(m, P, md.C, y, rv, acc, okf);
      });
#pragma unroll
      for (int i = 0; i < R; ++i) {
        El.bb[i] = m[i];
#pragma unroll
        for (int j = 0; j < R; ++j) {
          El.Ab[i][j] = 0.0;
          El.Cb[i][j] = P[i][j];
        }
      }
    } else {
      stream([&](long long, const double (&y)[N], const double (&rv)[N]) {
        elem_absorb<R, N, AI, CI>(El, md.A, md.Q, md.C, y, rv, ok);
      });
    }
    store_elem_pl<R>((double *)(a.ws + p.fel_off), f, B, b, El);
    if (u == 0) {
      Acc = El;
    } else {
      Elem<R> Et;
      ok = compose_elem<R>(Acc, El, Et) && ok;
      Acc = Et;
    }
  }
  }
  // coarse element = ordered tree over the block's waves (log2 kWV rounds;
  // dead waves hold the identity, which composes exactly)
  Acc.store(&sh[w][0][l], 64);
#pragma unroll
  for (int st2 = 1; st2 < kWV; st2 <<= 1) {
    __syncthreads();
    if ((w & (2 * st2 - 1)) == 0) {
      Elem<R> Ea, Eb, Et;
      Ea.load(&sh[w][0][l], 64);
      Eb.load(&sh[w + st2][0][l], 64);
      ok = compose_elem<R>(Ea, Eb, Et) && ok;
      Et.store(&sh[w][0][l], 64);
    }
  }
  if (w == 0 && (long long)b < B) {
    Elem<R> Ec;
    Ec.load(&sh[0][0][l], 64);
    store_elem_pl<R>((double *)(a.ws + p.cel_off), cc, B, b, Ec);
  }
  if ((long long)b < B)
    flag(a.status, b, (ok ? 0 : EKS_STATUS_SCAN) | (okf ? 0 : EKS_STATUS_SINGULAR));
}

// ---------------------------------------------------------------------------
// P2: coarse scan.  A block = kNP waves x 64 trajectories; wave w owns a
// contiguous run of coarse chunks (a "part") of the block's trajectories, so
// every element load is one 512-byte row segment:
//   (a) compose the part's elements, (b) exclusive prefix over the parts
//   through LDS (part 0's aggregate is a state; later parts' aggregates are
//   folded in with compose_state), (c) walk the part: filtered state
//   entering every coarse chunk + its RTS map, the part's maps composed in
//   forward order, (d) the smoothed mean entering the part from the right =
//   the later parts' maps applied to ms[T-1] = mf[T-1], (e) walk back:
//   smoothed mean at every coarse boundary.
// ---------------------------------------------------------------------------
#ifndef EKS_K3_NP
#define EKS_K3_NP 8
#endif
constexpr int kNP = EKS_K3_NP;

// Small batches (an 8-GPU shard) leave most CUs idle with one trajectory per
// lane, and the chains are latency bound: S > 1 splits every wave into S
// sub-parts of TW = 64 / S trajectories (TW * 8-byte row segments), i.e.
// kNP * S parts per trajectory, each S times shorter.  Inside a wave the
// part aggregates are scanned with shuffles; across waves through LDS as
// above.  The partition depends on S, so results for different S agree to
// rounding, not bit for bit.
template <int R>
EKS_DEV Elem<R> shfl_up_elem(const Elem<R> &e, int d) {
  double v[Elem<R>::len];
  e.store(v, 1);
#pragma unroll
  for (int k = 0; k < Elem<R>::len; ++k) v[k] = __shfl_up(v[k], d, 64);
  Elem<R> o;
  o.load(v, 1);
  return o;
}

// S from a sweep at T = 10 000 (tools/gpu_ssweep.sh), k3_coarse ms for
// S = 1 / 2 / 4 (/ 8):  B = 2 176 (one 8-GPU shard of config 4): 0.083 /
// 0.053 / 0.040 / 0.066;  B = 4 352: 0.086 / 0.059 / 0.076;  B = 6 528:
// 0.090 / 0.071 / 0.082;  B = 8 704: 0.106 / 0.125 / 0.119 / 0.180.
// EKS_K3_S overrides.
inline int coarse_subparts(long long B) {
  if (const char *s = getenv("EKS_K3_S")) {
    const int v = atoi(s);
    if (v == 1 || v == 2 || v == 4 || v == 8) return v;
  }
  return B <= 3072 ? 4 : B <= 7680 ? 2 : 1;
}

template <int R, int S>
__global__ __launch_bounds__(64 * kNP) void k3_coarse(SmoothArgs a, Plan3 p) {
  constexpr int KS = R + Sym<R>::len, MP = R * R + R, EL = Elem<R>::len;
  constexpr int TW = 64 / S, NPT = kNP * S;
  __shared__ double shE[kNP][EL][TW];
  __shared__ double shF[NPT][MP][TW];
  __shared__ double shM[R][TW];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int sub = l / TW, tl = l % TW;
  const int gp = w * S + sub;  // part index
  const long long B = a.B;
  const long long bl = blockIdx.x * (long long)TW + tl;
  const bool live = bl < B;
  const unsigned b = live ? (unsigned)bl : 0u;  // dead lanes shadow trajectory 0, store nothing
  const long long NC = p.NCc;
  const long long q = (NC + NPT - 1) / NPT;
  const long long c0 = min(NC, (long long)gp * q), c1 = min(NC, c0 + q);
  const double *cel = (const double *)(a.ws + p.cel_off);
  double *ccs = (double *)(a.ws + p.ccs_off);
  double *cmap = (double *)(a.ws + p.cmap_off);
  double *cms = (double *)(a.ws + p.cms_off);
  bool ok = true;
  // (a) the chain is latency bound: kPF elements are always in flight
  constexpr int kPF = 2;
  Elem<R> agg, ring[kPF];
  agg.set_identity();
#pragma unroll
  for (int u = 0; u < kPF; ++u)
    if (c0 + u < c1) load_elem_pl<R>(cel, c0 + u, B, b, ring[u]);
  for (long long c = c0; c < c1; c += kPF) {
#pragma unroll
    for (int u = 0; u < kPF; ++u) {
      if (c + u < c1) {
        const Elem<R> e = ring[u];
        if (c + u + kPF < c1) load_elem_pl<R>(cel, c + u + kPF, B, b, ring[u]);
        Elem<R> t;
        ok = compose_elem<R>(agg, e, t) && ok;
        agg = t;
      }
    }
  }
  // (b) filtered state entering c0.  Inside the wave: inclusive scan of the S
  // part aggregates, excl = the wave's parts before this one composed.
  Elem<R> excl;
  if constexpr (S > 1) {
#pragma unroll
    for (int k = 1; k < S; k <<= 1) {
      const Elem<R> o = shfl_up_elem<R>(agg, TW * k);
      if (sub >= k) {
        Elem<R> t;
        ok = compose_elem<R>(o, agg, t) && ok;
        agg = t;
      }
    }
    excl = shfl_up_elem<R>(agg, TW);
  }
  if (sub == S - 1) agg.store(&shE[w][0][tl], TW);  // the wave's aggregate
  __syncthreads();
  double m[R], P[R][R];
  auto set_state = [&](const Elem<R> &e) {  // an element starting at the prior is a state
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = e.bb[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = e.Cb[i][j];
    }
  };
  if (w > 0) {
    Elem<R> e0;
    e0.load(&shE[0][0][tl], TW);
    set_state(e0);
    for (int v = 1; v < w; ++v) {
      Elem<R> ev;
      ev.load(&shE[v][0][tl], TW);
      ok = compose_state<R>(m, P, ev) && ok;
    }
    if (sub > 0) ok = compose_state<R>(m, P, excl) && ok;
  } else if (sub > 0) {
    set_state(excl);
  }
  long long c = c0;
  if (gp == 0) {  // coarse chunk 0 is a state: its end state is the walk's start
    Elem<R> e0;
    load_elem_pl<R>(cel, 0, B, b, e0);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = e0.bb[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = e0.Cb[i][j];
    }
    c = 1;
  }
  // (c) walk
  Affine<R> F;  // this part's maps composed: ms(boundary c0) = F(ms(boundary c1))
  F.set_identity();
#pragma unroll
  for (int u = 0; u < kPF; ++u)
    if (c + u < c1) load_elem_pl<R>(cel, c + u, B, b, ring[u]);
  for (; c < c1; c += kPF) {
#pragma unroll
    for (int u = 0; u < kPF; ++u) {
      const long long cu = c + u;
      if (cu < c1) {
        const Elem<R> e = ring[u];
        if (cu + kPF < c1) load_elem_pl<R>(cel, cu + kPF, B, b, ring[u]);
        if (live) store_state_pl<R>(ccs, cu * KS, B, b, m, P);
        Affine<R> mp;
        ok = compose_state_rts<R>(m, P, e, mp.G, mp.g) && ok;
        if (live) {
          int k = 0;
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int j = 0; j < R; ++j) pl(cmap, cu * MP + (k++), B, b) = mp.G[i][j];
#pragma unroll
          for (int i = 0; i < R; ++i) pl(cmap, cu * MP + (k++), B, b) = mp.g[i];
        }
        F = F.after(mp);
      }
    }
  }
  // (d) ms[T-1] = mf[T-1]: the filtered mean after the last coarse chunk,
  // held by the part that contains it
  const int plast = (int)((NC - 1) / q);
  {
    int k = 0;
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) shF[gp][k++][tl] = F.G[i][j];
#pragma unroll
    for (int i = 0; i < R; ++i) shF[gp][k++][tl] = F.g[i];
  }
  if (gp == plast)
#pragma unroll
    for (int i = 0; i < R; ++i) {
      shM[i][tl] = m[i];
      if (live) pl(cms, NC * R + i, B, b) = m[i];
    }
  __syncthreads();
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = shM[i][tl];
  for (int v = plast; v > gp; --v) {  // parts after plast are empty (identity maps)
    double nx[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double sm = shF[v][R * R + i][tl];
#pragma unroll
      for (int k = 0; k < R; ++k) sm = fma(shF[v][i * R + k][tl], ms[k], sm);
      nx[i] = sm;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = nx[i];
  }
  // (e) walk back (maps prefetched kPM ahead)
  constexpr int kPM = 4;
  const long long cl = max(c0, 1LL);
  double Gr[kPM][R][R], gr[kPM][R];
  auto load_map = [&](long long cb, double (&G)[R][R], double (&g)[R]) {
    int k = 0;
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) G[i][j] = pl(cmap, cb * MP + (k++), B, b);
#pragma unroll
    for (int i = 0; i < R; ++i) g[i] = pl(cmap, cb * MP + (k++), B, b);
  };
#pragma unroll
  for (int u = 0; u < kPM; ++u)
    if (c1 - 1 - u >= cl) load_map(c1 - 1 - u, Gr[u], gr[u]);
  for (long long cb0 = c1 - 1; cb0 >= cl; cb0 -= kPM) {
#pragma unroll
    for (int u = 0; u < kPM; ++u) {
      const long long cb = cb0 - u;
      if (cb >= cl) {
        double nx[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double sm = gr[u][i];
#pragma unroll
          for (int j = 0; j < R; ++j) sm = fma(Gr[u][i][j], ms[j], sm);
          nx[i] = sm;
        }
        if (cb - kPM >= cl) load_map(cb - kPM, Gr[u], gr[u]);
#pragma unroll
        for (int i = 0; i < R; ++i) {
          ms[i] = nx[i];
          if (live) pl(cms, cb * R + i, B, b) = ms[i];  // smoothed mean at the last step of chunk cb-1
        }
      }
    }
  }
  if (live && !ok) flag(a.status, b, EKS_STATUS_SCAN);
}

// ---------------------------------------------------------------------------
// P3: fine walk, one lane per (coarse chunk, trajectory)
// ---------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(kBlock) void k3_fine(SmoothArgs a, Plan3 p) {
  constexpr int KS = R + Sym<R>::len;
  Lane<true> ln;
  const long long B = a.B;
  if (!ln.init(B, p.NCc)) return;
  const long long cc = ln.c;
  const unsigned b = ln.b;
  const double *fel = (const double *)(a.ws + p.fel_off);
  double *fcs = (double *)(a.ws + p.fcs_off);
  double *fms = (double *)(a.ws + p.fms_off);
  const long long f0 = cc * kNF, f1 = min(p.NCf, f0 + kNF);
  bool ok = true;
  double m[R], P[R][R];
  if (cc > 0) load_state_pl<R>((const double *)(a.ws + p.ccs_off), cc * KS, B, b, m, P);
  double G[kNF][R][R], g[kNF][R];
#pragma unroll
  for (int j = 0; j < kNF; ++j) {
    const long long f = f0 + j;
    if (f < f1) {
      Elem<R> El;
      load_elem_pl<R>(fel, f, B, b, El);
      if (f == 0) {  // the first fine chunk starts at the prior (read from the model by P4)
#pragma unroll
        for (int i = 0; i < R; ++i) {
          m[i] = El.bb[i];
#pragma unroll
          for (int k = 0; k < R; ++k) P[i][k] = El.Cb[i][k];
        }
      } else {
        store_state_pl<R>(fcs, f * KS, B, b, m, P);
        ok = compose_state_rts<R>(m, P, El, G[j], g[j]) && ok;
      }
    }
  }
  // smoothed mean at the last step of the coarse chunk, then right to left
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = pl((const double *)(a.ws + p.cms_off), (cc + 1) * R + i, B, b);
#pragma unroll
  for (int j = kNF - 1; j >= 0; --j) {
    const long long f = f0 + j;
    if (f < f1) {
#pragma unroll
      for (int i = 0; i < R; ++i) pl(fms, f * R + i, B, b) = ms[i];
      if (j > 0) {
        double nx[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double s = g[j][i];
#pragma unroll
          for (int k = 0; k < R; ++k) s = fma(G[j][i][k], ms[k], s);
          nx[i] = s;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) ms[i] = nx[i];
      }
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SCAN);
}

// ---------------------------------------------------------------------------
// P4: final smoothing pass
// ---------------------------------------------------------------------------
template <int R, int N, int E, typename T, typename YT, int AI, int CI, int LS>
__global__ __launch_bounds__(kBlock) void k3_final(SmoothArgs a, Plan3 p) {
  constexpr int KS = R + Sym<R>::len;
  constexpr int D = EKS_K3_DF;
  constexpr int NST = (kNS - 1) * LS;  // steps kept in LDS
  __shared__ YT ys[NST][N][kBlock];
  __shared__ double es[NST][N][kBlock];
  Lane<true> ln;
  const long long B = a.B, TT = a.T;
  if (!ln.init(B, p.NCf)) return;
  const long long c = ln.c;
  const unsigned b = ln.b;
  const int tid = threadIdx.x;
  Model<R, N> md;
  load_model_pl<R, N, AI, CI>((const double *)(a.ws + p.prm_off), B, b, c == 0, md);
  const long long s = c * p.L, e = min(TT, s + p.L);
  const bool last = e == TT;
  const int nsub = (int)((e - s + LS - 1) / LS);
  typename SrcOf<E, N, T, D>::type src;
  src.init(a, b);
#pragma unroll
  for (int q = 0; q < D; ++q)
    if (s + q < e) src.fetch(q, s + q);
  double m[R], P[R][R], m0c[R], P0c[R][R], msE[R];
  if (c == 0) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = md.m0[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
    }
  } else {
    load_state_pl<R>((const double *)(a.ws + p.fcs_off), c * KS, B, b, m, P);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    m0c[i] = m[i];
    msE[i] = last ? 0.0 : pl((const double *)(a.ws + p.fms_off), c * R + i, B, b);
#pragma unroll
    for (int j = 0; j < R; ++j) P0c[i][j] = P[i][j];
  }
  bool ok = true;
  NllAcc acc;
  double Jr[LS][R][R], dr[LS][R];
  // forward: filter every step; stash the early sub-chunks, keep the last
  // sub-chunk's RTS gains
#pragma unroll
  for (int i = 0; i < kNS * LS; ++i) {
    const long long t = s + i;
    const int k = i / LS, q = i % LS;
    if (t < e) {
      double avg[N], rv[N], y[N];
      src.get(i % D, avg, rv);
      if (t + D < e) src.fetch(i % D, t + D);
      if (k < kNS - 1 && k < nsub - 1) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          ys[i][j][tid] = (YT)avg[j];
          es[i][j][tid] = rv[j];
        }
      }
#pragma unroll
      for (int j = 0; j < N; ++j) y[j] = avg[j] - md.off[j];
      if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
      kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
      if (k == nsub - 1) {
        if (t == e - 1) {
#pragma unroll
          for (int u = 0; u < R; ++u) {
            dr[q][u] = last ? m[u] : msE[u];
#pragma unroll
            for (int v = 0; v < R; ++v) Jr[q][u][v] = 0.0;
          }
        } else {
          ok = rts_gain<R, AI>(m, P, md.A, md.Q, Jr[q], dr[q]) && ok;
        }
      }
    }
  }
  if (a.nll) pl((double *)(a.ws + p.nllp_off), c, B, b) = acc.value((double)(e - s) * N);
  double *outb = a.out + (long long)b * a.ob;
  // (x, y) pairs adjacent and 16-byte aligned (the time-major default
  // layout): one 16-byte store per step instead of two 8-byte ones
  const bool vec2 = N == 2 && a.oj == 1 && ((a.ob | a.ot) & 1) == 0 &&
                    (((uintptr_t)a.out) & 15) == 0;
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = 0.0;
  auto rts_back = [&](long long t0) {
#pragma unroll
    for (int q = LS - 1; q >= 0; --q) {
      const long long t = t0 + q;
      if (t < e) {
        double nx[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double sm = dr[q][i];
#pragma unroll
          for (int u = 0; u < R; ++u) sm = fma(Jr[q][i][u], ms[u], sm);
          nx[i] = sm;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) ms[i] = nx[i];
        if constexpr (N == 2) {
          if (vec2) {
            double cm[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              if constexpr (CI == kCId) {
                cm[j] = ms[j] + md.off[j];
              } else {
                double u = 0.0;
#pragma unroll
                for (int k = 0; k < R; ++k) u = fma(md.C[j][k], ms[k], u);
                cm[j] = u + md.off[j];
              }
            }
    #if EKS_NT_OUT  // streaming (non-temporal) output stores (smooth_impl.hpp)
        __builtin_nontemporal_store(cm[0], outb + t * a.ot);
        __builtin_nontemporal_store(cm[1], outb + t * a.ot + 1);
#else
        *(double2 *)(outb + t * a.ot) = make_double2(cm[0], cm[1]);
#endif
          } else {
            project_store<R, N, CI>(outb + t * a.ot, a.oj, md.C, ms, md.off);
          }
        } else {
          project_store<R, N, CI>(outb + t * a.ot, a.oj, md.C, ms, md.off);
        }
        if (a.ms) store_vec<R>(a.ms + ((long long)b * TT + t) * R, ms);
      }
    }
  };
  rts_back(s + (long long)(nsub - 1) * LS);
  // earlier sub-chunks (kNS = 2: at most one), re-run from the chunk start
  // with the stashed (y, ev)
  if (nsub >= 2) {
    static_assert(kNS == 2, "the re-run below assumes two sub-chunks");
    NllAcc dummy;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = m0c[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = P0c[i][j];
    }
#pragma unroll
    for (int q = 0; q < LS; ++q) {
      const long long t = s + q;
      double y[N], rv[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        y[j] = (double)ys[q][j][tid] - md.off[j];
        rv[j] = es[q][j][tid];
      }
      if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
      kf_update<R, N, CI>(m, P, md.C, y, rv, dummy, ok);
      ok = rts_gain<R, AI>(m, P, md.A, md.Q, Jr[q], dr[q]) && ok;
    }
    rts_back(s);
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
}

// P4, state-stash form: the forward sweep keeps the FILTERED STATE of every
// step (LDS for the early sub-chunks, registers for the last one) instead of
// (y, ev), so the backward sweep computes the RTS gains without re-running
// the filter (one filter pass per step instead of 1.5).
template <int R, int N, int E, typename T, typename YT, int AI, int CI, int LS, bool WALK>
__global__ __launch_bounds__(kBlock) EKS_K3_WPE void k3_final_s(SmoothArgs a, Plan3 p) {
  constexpr int KS = R + Sym<R>::len;
  constexpr int D = EKS_K3_DF;
  constexpr int NST = (kNS - 1) * LS;  // steps kept in LDS
  __shared__ double fs[NST][KS][kBlock];
  const long long B = a.B, TT = a.T;
  const int tid = threadIdx.x;
  long long c;
  unsigned b;
  if constexpr (WALK) {  // block = the kNF fine chunks of one coarse chunk x 64 trajectories
    static_assert(64 * kNF == kBlock, "one wave per fine chunk of a coarse chunk");
    const long long ng = (B + 63) / 64;
    const long long cc = blockIdx.x / ng;
    b = (unsigned)((blockIdx.x - cc * ng) * 64 + (tid & 63));
    c = cc * kNF + (tid >> 6);
    if ((long long)b >= B || c >= p.NCf) return;
  } else {
    Lane<true> ln;
    if (!ln.init(B, p.NCf)) return;
    c = ln.c;
    b = ln.b;
  }
  Model<R, N> md;
  load_model_pl<R, N, AI, CI>((const double *)(a.ws + p.prm_off), B, b, c == 0, md);
  const long long s = c * p.L, e = min(TT, s + p.L);
  const bool last = e == TT;
  const int nsub = (int)((e - s + LS - 1) / LS);
  typename SrcOf<E, N, T, D>::type src;
  src.init(a, b);
  constexpr int LF = kNS * LS;
  const bool full = EKS_K3_FULLPATH && e - s == LF;  // all chunks but a trajectory's last: no runtime guards
  if (full) {
#pragma unroll
    for (int q = 0; q < D; ++q) src.fetch(q, s + q);
  } else {
#pragma unroll
    for (int q = 0; q < D; ++q)
      if (s + q < e) src.fetch(q, s + q);
  }
  double m[R], P[R][R], msE[R];
  bool ok = true;
  if constexpr (WALK) {
    // the fine walk of P3, redundantly per wave (the block's 4 waves read the
    // same 4 elements: one HBM fetch, L1/L2 hits after): filtered state
    // entering this fine chunk, and the smoothed mean at its last step = the
    // later fine chunks' RTS maps applied to the coarse boundary mean
    const long long cc = c / kNF, f0 = cc * kNF, f1 = min(p.NCf, f0 + kNF);
    const int w = (int)(c - f0);
    Elem<R> El[kNF];
#pragma unroll
    for (int j = 0; j < kNF; ++j)
      if (f0 + j < f1) load_elem_pl<R>((const double *)(a.ws + p.fel_off), f0 + j, B, b, El[j]);
    double wm[R], wP[R][R], G[kNF][R][R], g[kNF][R];
    if (cc > 0) load_state_pl<R>((const double *)(a.ws + p.ccs_off), cc * KS, B, b, wm, wP);
#pragma unroll
    for (int j = 0; j < kNF; ++j) {
      const long long f = f0 + j;
      if (f < f1) {
        if (j == w) {
#pragma unroll
          for (int i = 0; i < R; ++i) {
            m[i] = wm[i];
#pragma unroll
            for (int k = 0; k < R; ++k) P[i][k] = wP[i][k];
          }
        }
        if (f == 0) {  // the first chunk's element is its end state
#pragma unroll
          for (int i = 0; i < R; ++i) {
            wm[i] = El[j].bb[i];
#pragma unroll
            for (int k = 0; k < R; ++k) wP[i][k] = El[j].Cb[i][k];
          }
        } else {
          bool okw = compose_state_rts<R>(wm, wP, El[j], G[j], g[j]);
          if (j > w) ok = ok && okw;  // maps this chunk does not use are checked elsewhere
        }
      }
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
      msE[i] = last ? 0.0 : pl((const double *)(a.ws + p.cms_off), (cc + 1) * R + i, B, b);
#pragma unroll
    for (int j = kNF - 1; j >= 0; --j) {
      if (j > w && f0 + j < f1) {
        double nx[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double sm = g[j][i];
#pragma unroll
          for (int k = 0; k < R; ++k) sm = fma(G[j][i][k], msE[k], sm);
          nx[i] = sm;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) msE[i] = nx[i];
      }
    }
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        m[i] = md.m0[i];
#pragma unroll
        for (int k = 0; k < R; ++k) P[i][k] = md.S0[i][k];
      }
    }
  } else {
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        m[i] = md.m0[i];
#pragma unroll
        for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
      }
    } else {
      load_state_pl<R>((const double *)(a.ws + p.fcs_off), c * KS, B, b, m, P);
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
      msE[i] = last ? 0.0 : pl((const double *)(a.ws + p.fms_off), c * R + i, B, b);
  }
  NllAcc acc;
  double Mr[LS][KS];  // filtered states of the last sub-chunk
  auto pack = [&](double (&dst)[KS]) {
    int k = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) dst[k++] = m[i];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) dst[k++] = P[i][j];
  };
  auto fwd = [&](auto fullc) {
    constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
    for (int i = 0; i < LF; ++i) {
      const long long t = s + i;
      const int k = i / LS, q = i % LS;
      if (FULL || t < e) {
        double avg[N], rv[N], y[N];
        src.get(i % D, avg, rv);
        if (FULL) {
          if (i + D < LF) src.fetch(i % D, t + D);
        } else if (t + D < e) {
          src.fetch(i % D, t + D);
        }
        EKS_PIN_LOADS();
#pragma unroll
        for (int j = 0; j < N; ++j) y[j] = avg[j] - md.off[j];
        if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
        kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
        if (FULL ? k == kNS - 1 : k == nsub - 1) {
          pack(Mr[q]);
        } else if (k < kNS - 1) {
          double st[KS];
          pack(st);
#pragma unroll
          for (int u = 0; u < KS; ++u) fs[i][u][tid] = st[u];
        }
      }
    }
  };
  if (full)
    fwd(std::true_type{});
  else
    fwd(std::false_type{});
  if (a.nll) pl((double *)(a.ws + p.nllp_off), c, B, b) = acc.value((double)(e - s) * N);
  double *outb = a.out + (long long)b * a.ob;
  const bool vec2 = N == 2 && a.oj == 1 && ((a.ob | a.ot) & 1) == 0 &&
                    (((uintptr_t)a.out) & 15) == 0;
  double ms[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = 0.0;
  auto emit = [&](long long t) {
    if constexpr (N == 2) {
      if (vec2) {
        double cm[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (CI == kCId) {
            cm[j] = ms[j] + md.off[j];
          } else {
            double u = 0.0;
#pragma unroll
            for (int k = 0; k < R; ++k) u = fma(md.C[j][k], ms[k], u);
            cm[j] = u + md.off[j];
          }
        }
#if EKS_NT_OUT  // streaming (non-temporal) output stores (smooth_impl.hpp)
        __builtin_nontemporal_store(cm[0], outb + t * a.ot);
        __builtin_nontemporal_store(cm[1], outb + t * a.ot + 1);
#else
        *(double2 *)(outb + t * a.ot) = make_double2(cm[0], cm[1]);
#endif
      } else {
        project_store<R, N, CI>(outb + t * a.ot, a.oj, md.C, ms, md.off);
      }
    } else {
      project_store<R, N, CI>(outb + t * a.ot, a.oj, md.C, ms, md.off);
    }
    if (a.ms) store_vec<R>(a.ms + ((long long)b * TT + t) * R, ms);
  };
  // one RTS step backwards from the filtered state st of step t
  auto rts_step = [&](const double (&st)[KS]) {
    double mf[R], Pf[R][R], J[R][R], d[R], nx[R];
    int k = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) mf[i] = st[k++];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) Pf[i][j] = Pf[j][i] = st[k++];
    ok = rts_gain<R, AI>(mf, Pf, md.A, md.Q, J, d) && ok;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double sm = d[i];
#pragma unroll
      for (int u = 0; u < R; ++u) sm = fma(J[i][u], ms[u], sm);
      nx[i] = sm;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = nx[i];
  };
  // the last sub-chunk, from registers; its last step's mean is known
#pragma unroll
  for (int q = LS - 1; q >= 0; --q) {
    const long long t = s + (long long)(nsub - 1) * LS + q;
    if (t < e) {
      if (t == e - 1) {
#pragma unroll
        for (int i = 0; i < R; ++i) ms[i] = last ? Mr[q][i] : msE[i];
      } else {
        rts_step(Mr[q]);
      }
      emit(t);
    }
  }
  // the earlier sub-chunks, from LDS
  for (int k = nsub - 2; k >= 0; --k) {
#pragma unroll
    for (int q = LS - 1; q >= 0; --q) {
      const int i = k * LS + q;
      double st[KS];
#pragma unroll
      for (int u = 0; u < KS; ++u) st[u] = fs[i][u][tid];
      rts_step(st);
      emit(s + i);
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
}

// NLL of each trajectory = sum of its fine chunks' shares (fixed order)
template <int R>
__global__ __launch_bounds__(64) void k3_nll(SmoothArgs a, Plan3 p) {
  const long long b = blockIdx.x;
  const int l = threadIdx.x;
  if (b >= a.B || !a.nll) return;
  const double *np_ = (const double *)(a.ws + p.nllp_off);
  double s = 0.0;
  for (long long c = l; c < p.NCf; c += 64) s += np_[c * a.B + b];
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) s += __shfl_xor(s, k, 64);
  if (l == 0) a.nll[b] = s;
}

// host: the four (five with NLL) launches of one algo-3 call
template <int R, int N, int AI, int CI>
int launch_algo3(const SmoothArgs &a, hipEvent_t after_elem = nullptr, hipStream_t cont = nullptr) {
  constexpr int LS = sub_len_c(R, N);
  const Plan3 p = make_plan3(a.B, a.T, R, N);
  const bool yev = a.dtype == EKS_YEV32 || a.dtype == EKS_YEV64;
  const bool f32 = a.dtype == EKS_F32;
  const bool y32 = yev ? a.dtype == EKS_YEV32 : (f32 && a.median && (a.E == 3 || a.E == 5));
  const unsigned ng = (unsigned)((a.B + 63) / 64);
  const unsigned g1 = (unsigned)(p.NCc * ng);
  const unsigned g3 = (unsigned)(p.NCc * blocks_per_chunk(a.B));
  const unsigned g4 = (unsigned)(p.NCf * blocks_per_chunk(a.B));
  auto run = [&](auto tag, auto ytag, auto Ec) -> int {
    using Tp = decltype(tag);
    using YT = decltype(ytag);
    constexpr int EE = decltype(Ec)::value;
    int rc;
    prof_call_begin();
    prof_mark(a.stream, "k_model_planes");
    hipLaunchKernelGGL((k_model_planes<R, N, AI, CI>), dim3(grid_for(a.B, 256)), dim3(256), 0, a.stream,
                       a.params, a.B, (double *)(a.ws + p.prm_off), a.status);
    if ((rc = check_launch("k_model_planes"))) return rc;
    prof_mark(a.stream, "k3_elem");
    hipLaunchKernelGGL((k3_elem<R, N, EE, Tp, AI, CI>), dim3(g1), dim3(64 * kWV), 0, a.stream, a, p);
    if ((rc = check_launch("k3_elem"))) return rc;
    if (after_elem && hipEventRecord(after_elem, a.stream) != hipSuccess)
      return set_err(EKS_ERR_HIP, "eks_smooth algo 3: hipEventRecord failed");
    // (split calls) the rest of this half's chain continues on `cont`
    const hipStream_t sc = cont ? cont : a.stream;
    if (cont && hipStreamWaitEvent(cont, after_elem, 0) != hipSuccess)
      return set_err(EKS_ERR_HIP, "eks_smooth algo 3: hipStreamWaitEvent failed");
    prof_mark(sc, "k3_coarse");
    switch (coarse_subparts(a.B)) {
      case 8: hipLaunchKernelGGL((k3_coarse<R, 8>), dim3(grid_for(a.B, 8)), dim3(64 * kNP), 0, sc, a, p); break;
      case 4: hipLaunchKernelGGL((k3_coarse<R, 4>), dim3(grid_for(a.B, 16)), dim3(64 * kNP), 0, sc, a, p); break;
      case 2: hipLaunchKernelGGL((k3_coarse<R, 2>), dim3(grid_for(a.B, 32)), dim3(64 * kNP), 0, sc, a, p); break;
      default: hipLaunchKernelGGL((k3_coarse<R, 1>), dim3(grid_for(a.B, 64)), dim3(64 * kNP), 0, sc, a, p);
    }
    if ((rc = check_launch("k3_coarse"))) return rc;
#if EKS_K3_MERGED
    prof_mark(sc, "k3_final");
    hipLaunchKernelGGL((k3_final_s<R, N, EE, Tp, YT, AI, CI, LS, true>), dim3(g1), dim3(kBlock), 0,
                       sc, a, p);
#else
    prof_mark(sc, "k3_fine");
    hipLaunchKernelGGL((k3_fine<R>), dim3(g3), dim3(kBlock), 0, sc, a, p);
    if ((rc = check_launch("k3_fine"))) return rc;
    prof_mark(sc, "k3_final");
    hipLaunchKernelGGL((k3_final_s<R, N, EE, Tp, YT, AI, CI, LS, false>), dim3(g4), dim3(kBlock), 0,
                       sc, a, p);
#endif
    if ((rc = check_launch("k3_final"))) return rc;
    if (a.nll) {
      prof_mark(sc, "k3_nll");
      hipLaunchKernelGGL((k3_nll<R>), dim3((unsigned)a.B), dim3(64), 0, sc, a, p);
      if ((rc = check_launch("k3_nll"))) return rc;
    }
    prof_call_end(sc);
    return 0;
  };
  if (yev) {
    if (y32) return run(YevIn<float>{}, float{}, ic<0>{});
    return run(YevIn<double>{}, double{}, ic<0>{});
  }
  auto by_e = [&](auto tag, auto ytag) -> int {
    switch (a.E) {
      case 3: return run(tag, ytag, ic<3>{});
      case 4: return run(tag, ytag, ic<4>{});
      case 5: return run(tag, ytag, ic<5>{});
      default: return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth algo 3: E=%d not compiled in", a.E);
    }
  };
  if (y32) return by_e(float{}, float{});
  return f32 ? by_e(float{}, double{}) : by_e(double{}, double{});
}

// ---------------------------------------------------------------------------
// Two half-batches on two streams (EKS_A3_SPLIT = 1 / 2; off by default:
// measured no faster).  k3_coarse holds a whole CU per block (242 VGPRs x 8
// waves, 83 KB LDS) for a latency-bound chain, and k3_fine is short; in one
// stream nothing else runs beside them (15 % of the config-4 step).  Split
// into halves A and B (A = whole 64-trajectory groups): mode 1 starts B's
// chain on a side stream when A's k3_elem is done; mode 2 continues A's
// scans + final pass on a high-priority side stream while B's k3_elem
// follows on the caller's stream.  Either way one half's member pass streams
// beside the other half's scans; the caller's stream then joins the side
// stream.  Each half is an ordinary algo-3 call on its own workspace range
// (planes pitched by the half's B), so results are bit-identical to two
// separate calls on the halves (and to the one-piece call whenever the
// half's coarse sub-part count S equals the whole's, e.g. config 4's
// 17 408 -> 2 x 8 704, S = 1).  Measured at config 4 (profiles/r02/split):
// the kernels do overlap (A's k3_coarse runs beside B's k3_elem) but the
// coarse scan is starved (0.94 instead of 0.25 ms) while k3_elem keeps its
// 0.80 ms: the step is bound by its total HBM traffic (22.2 GB at 5.3 TB/s),
// which overlap does not reduce (4.21 / 4.21 / 4.22 ms for one stream /
// mode 1 / mode 2).
// ---------------------------------------------------------------------------
constexpr long long kSplitMinB = 8192;

inline int a3_split_mode() {  // read per call (tests switch it)
  const char *e = getenv("EKS_A3_SPLIT");
  return e ? atoi(e) : 0;
}

struct SplitRes {  // per device: the side stream and the fork / join events
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

inline SplitRes *split_res() {
  static SplitRes res[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  SplitRes &r = res[dev];
  if (!r.side) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    if (hipStreamCreateWithPriority(&r.side, hipStreamNonBlocking, greatest) != hipSuccess ||
        hipEventCreateWithFlags(&r.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r.join, hipEventDisableTiming) != hipSuccess) {
      r.side = nullptr;
      return nullptr;
    }
  }
  return &r;
}

template <int R, int N, int AI, int CI>
int launch_algo3_split(const SmoothArgs &a) {
  const int mode = a3_split_mode();
  const bool members = a.dtype == EKS_F32 || a.dtype == EKS_F64;
  const long long b0 = (a.B / 2 + 63) / 64 * 64;  // half A: whole 64-trajectory groups
  bool go = members && a.phase == 0 && b0 < a.B && mode > 0 && a.B >= kSplitMinB;
  SmoothArgs A = a, Bh = a;
  if (go) {
    A.B = b0;
    A.ws_bytes = align256(make_plan3(b0, a.T, R, N).total);
    Bh.B = a.B - b0;
    Bh.ws = a.ws + A.ws_bytes;
    Bh.ws_bytes = make_plan3(Bh.B, a.T, R, N).total;
    go = A.ws_bytes + Bh.ws_bytes <= a.ws_bytes;
  }
  SplitRes *sr = go ? split_res() : nullptr;
  if (!sr) return launch_algo3<R, N, AI, CI>(a);
  const size_t esz = a.dtype == EKS_F32 ? 4 : 8;
  Bh.obs = (const char *)a.obs + (size_t)(b0 * a.sb) * esz;
  Bh.params = a.params + b0 * ParamLayout<R, N>::len;
  Bh.out = a.out + b0 * a.ob;
  Bh.ms = a.ms ? a.ms + b0 * a.T * R : nullptr;
  Bh.nll = a.nll ? a.nll + b0 : nullptr;
  Bh.status = a.status ? a.status + b0 : nullptr;
  prof_call_begin();
  prof_mark(a.stream, "k3_split");
  prof_suspend(true);
  int rc;
  if (mode == 1) {  // B's whole chain on the side stream after A's k3_elem
    Bh.stream = sr->side;
    rc = launch_algo3<R, N, AI, CI>(A, sr->fork);
    if (!rc && hipStreamWaitEvent(sr->side, sr->fork, 0) != hipSuccess)
      rc = set_err(EKS_ERR_HIP, "eks_smooth algo 3 split: hipStreamWaitEvent failed");
    if (!rc) rc = launch_algo3<R, N, AI, CI>(Bh);
  } else {  // A's scans + final pass on the (high-priority) side stream, B on the caller's
    Bh.stream = a.stream;
    rc = launch_algo3<R, N, AI, CI>(A, sr->fork, sr->side);
    if (!rc) rc = launch_algo3<R, N, AI, CI>(Bh);
  }
  // join even after a failed half so the side stream never outlives the call
  if (hipEventRecord(sr->join, sr->side) != hipSuccess ||
      hipStreamWaitEvent(a.stream, sr->join, 0) != hipSuccess)
    rc = rc ? rc : set_err(EKS_ERR_HIP, "eks_smooth algo 3 split: join failed");
  prof_suspend(false);
  prof_call_end(a.stream);
  return rc;
}
