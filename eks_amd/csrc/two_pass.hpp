// algo 3 of eks_smooth: the exact smoother in TWO passes over the member
// predictions, each pass carrying its time recursion across chunks itself
// (included by smooth_impl.hpp, inside namespace eks).
//
// Time is cut into fine chunks of L steps (L = 16 at r = n = 2).  A *unit*
// is one coarse chunk (4 consecutive fine chunks, one wave each) of 64
// trajectories: 256 threads.  Both passes are persistent kernels that take
// units from an atomic ticket counter, so the unit a unit waits for (the
// previous coarse chunk in the pass's direction, same trajectories) holds a
// smaller ticket, i.e. is already running or done: the waits always end,
// whatever the dispatch order.  Each pass is a chained scan over coarse
// chunks: a unit waits for the value its neighbour publishes, combines it
// with its own aggregate and publishes its own.  No scan kernels, no
// per-chunk element planes.
//
//  k3_fwd  members -> ensemble -> filtering element of each fine chunk
//          (kf_steps.hpp Elem; the plain filter from the prior for chunk 0);
//          the 4 elements composed in LDS (two rounds); wave 0 waits for the
//          filtered state entering the coarse chunk, publishes the state
//          leaving it (= the start state of the next coarse chunk), and
//          waves 1-3 write their fine chunk's start state
//          (compose_state of the entering state with the elements before).
//  k3_bwd  units in reverse time order.  Members again -> ensemble -> the
//          filter from the exact start state; the filtered state of every
//          step kept on chip (the first NL steps in LDS, the last NR in
//          registers) and the fine chunk's RTS map ms[s] = G ms[e] + g
//          accumulated in forward order (algo 2's K3 rule).  Wave 0 waits for
//          the smoothed mean at the first step of the next coarse chunk,
//          applies the 4 maps right to left (handing each wave the mean at
//          the first step after its chunk) and publishes the mean at the
//          coarse chunk's first step; then every wave runs the RTS recursion
//          backwards over its steps (eks/ensemble_kalman.py:156-162) and
//          writes C ms + offset (+ ms, + the chunk's NLL share).
//
// HBM bytes per keypoint-timestep (single view, E = 5): k3_fwd 40 (members)
// + 2.5 (fine start states: 5 doubles per 16 steps); k3_bwd 40 + 2.5 + 16
// (outputs); the chain payloads (5 + 2 doubles per 64 steps) < 1.  About
// 100 B, against the four-kernel version's 125.5 measured (fine and coarse
// element planes, coarse scan, fine walk).
//
// Exactness: k3_bwd runs the reference recursions (kf_update, rts_gain) from
// start states and boundary means that equal the sequential ones up to the
// rounding of the element compositions / map applications (contractive, as
// in algo 2).  Determinism: a unit only ever combines its own aggregate with
// its neighbour's published value, so the association order of every
// operation depends on T alone: results are bit-reproducible and a slice of
// the batch smooths to the same bits as the whole.
//
// Hand-offs inside a launch (MI355X_MICROARCH.md, inter-workgroup
// visibility): payloads are stored write-through (agent-scope relaxed
// atomic stores, `sc1`) by the one wave that publishes, which then drains
// (`s_waitcnt vmcnt(0)`) before one agent-scope flag store; the consumer
// polls the flag with agent-scope loads and reads the payload with
// agent-scope (`sc1`, L1-bypassing) loads.  Flags and tickets are zeroed by a
// memset at the start of every call (a memset node under graph capture).
// Every spin is bounded: a unit that gives up flags its trajectories
// EKS_STATUS_SCAN (batch.smooth(check=True) then re-runs algo 1) and still
// publishes, so nothing behind it hangs.

constexpr int kWV = 4;  // waves per unit = fine chunks per coarse chunk

// In-kernel phase stamps (profiling builds only: -DEKS_STAMPS=1, read back by
// eks_dbg_stamps / tools/stamps_run.py): s_memtime at the phase boundaries of
// every unit, per (pass, block, unit, wave); slot 0 = the unit's (group, chunk).
// Stored by lane 0 with a vector store.  Compiled out of the shipped library.
#ifndef EKS_STAMPS
#define EKS_STAMPS 0
#endif
constexpr int kStampBlocks = 512, kStampIts = 128;
#if EKS_STAMPS
static __device__ unsigned long long g_stamps[2 * kStampBlocks * kStampIts * 32];
#define EKS_STAMP(PASS, K)                                                                    \
  do {                                                                                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                               \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kStampBlocks && it < kStampIts)               \
      g_stamps[(((size_t)(PASS) * kStampBlocks + blockIdx.x) * kStampIts + it) * 32 +        \
               (threadIdx.x >> 6) * 8 + (K)] =                                               \
          (K) == 0 ? (((unsigned long long)wk.grp << 32) | (unsigned long long)wk.c) : t_;    \
  } while (0)
// wave 0's chain detail (after both waves' slot-0 words are written at the
// unit's start): the look-back's end time into wave 1's slot 0, the number
// of units folded into wave 2's
#define EKS_STAMP_AUX(PASS, WSLOT, VAL)                                                       \
  do {                                                                                        \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kStampBlocks && it < kStampIts)               \
      g_stamps[(((size_t)(PASS) * kStampBlocks + blockIdx.x) * kStampIts + it) * 32 +        \
               (WSLOT) * 8] = (unsigned long long)(VAL);                                     \
  } while (0)
#else
#define EKS_STAMP(PASS, K) \
  do {                     \
  } while (0)
#define EKS_STAMP_AUX(PASS, WSLOT, VAL) \
  do {                                  \
  } while (0)
#endif

// fine chunk geometry of k3_bwd: NR steps' filtered states in registers, NL
// in LDS; LDS per block <= 80 KB so two 256-thread blocks share a CU (the
// register file allows two waves per SIMD), after the 3 waves' RTS maps
constexpr int reg_steps3(int r, int n) { return (r <= 2 && n <= 2) ? 9 : sub_len_c(r, n); }
constexpr int lds_steps3(int r, int n) {
  return ((80 * 1024 - 3 * (r * r + r) * 64 * 8 - 256) / ((r + r * (r + 1) / 2) * 8 * 256)) < 1
             ? 1
             : (80 * 1024 - 3 * (r * r + r) * 64 * 8 - 256) / ((r + r * (r + 1) / 2) * 8 * 256);
}
constexpr int fine_len3(int r, int n) { return reg_steps3(r, n) + lds_steps3(r, n); }

struct Plan3 {
  // NCc / units: k3_bwd's 4-chunk units; NCu / units_f: k3_fwd's (4 x FPW)
  long long L = 16, NCf = 0, NCc = 0, NCu = 0, ng = 0, units = 0, units_f = 0;
  // sync block (zeroed every call): ticket counters (own 128-byte lines),
  // then one flag word per unit for each pass
  size_t sync_bytes = 0, flag1_off = 0, flag2_off = 0;
  size_t fst_off = 0, inc2_off = 0, nllp_off = 0, prm_off = 0, total = 0;
  // look-back aggregates: k3_fwd's unit elements, k3_bwd's unit maps
  size_t agg1_off = 0, agg2_off = 0;
};

inline Plan3 make_plan3(long long B, long long T, int r, int n) {
  Plan3 p;
  p.L = fine_len3(r, n);
  p.NCf = (T + p.L - 1) / p.L;
  p.NCc = (p.NCf + kWV - 1) / kWV;
  const int kpu = kWV * (r <= 2 ? 2 : 1);  // k3_fwd's fine chunks per unit (fwd_fpw)
  p.NCu = (p.NCf + kpu - 1) / kpu;
  p.ng = (B + 63) / 64;
  p.units = p.NCc * p.ng;
  p.units_f = p.NCu * p.ng;
  p.flag1_off = 256;
  p.flag2_off = p.flag1_off + (size_t)p.units_f * 4;
  p.sync_bytes = align256(p.flag2_off + (size_t)p.units * 4);
  size_t off = p.sync_bytes;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align256(off + bytes);
    return o;
  };
  const size_t Bz = (size_t)B;
  // start state of fine chunk f (f >= 1; entry KPU c is also the state
  // k3_fwd's chain hands from its unit c-1 to c)
  p.fst_off = take((size_t)(std::max(kWV * p.NCc, kpu * p.NCu) + 1) * state_len(r) * Bz * 8);
  // smoothed mean at the first step of coarse chunk c (k3_bwd's chain)
  p.inc2_off = take((size_t)p.NCc * r * Bz * 8);
  p.nllp_off = take((size_t)p.NCf * Bz * 8);
  p.prm_off = take((size_t)param_len(n, r) * Bz * 8);  // k_model_planes
  // a unit's aggregate, published for the look-back of later units when the
  // value it waits for is not there yet: k3_fwd's element of unit c (planes
  // c * EL ..), k3_bwd's RTS map of unit c (its 4 chunk maps composed; planes
  // c * MP ..)
  p.agg1_off = take((size_t)p.NCu * elem_len(r) * Bz * 8);
  p.agg2_off = take((size_t)p.NCc * (r * r + r) * Bz * 8);
  p.total = off;
  return p;
}

// Step sources of the two member passes: a D-deep register ring of raw step
// data, reduced to (raw average, variance) on use.
// Raw buffer loads of the members: the step's base address goes into the
// buffer descriptor (scalar, advanced per step), member e / coordinate j's
// offset into soffset (scalar) and the trajectory's into a 32-bit voffset:
// no vector address arithmetic per load.  launch_algo3 slices the batch so
// that voffset + soffset stays below 2^32 (the descriptor's range).
EKS_DEV __amdgpu_buffer_rsrc_t member_rsrc(const void *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, -1, 0x00020000);
}
template <typename T, bool NT>
EKS_DEV T member_load(__amdgpu_buffer_rsrc_t rs, unsigned voff, int soff) {
  constexpr int aux = NT ? 2 : 0;  // nt: streamed once
  if constexpr (sizeof(T) == 4)
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, aux));
  else
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, aux));
}

template <int E, int N, typename T, int D, bool NT = kNtLoad>
struct MemberRing {
  T v[D][E][N];
  const char *base;  // uniform
  unsigned loff;     // trajectory b's byte offset
  long long stb;     // bytes per step
  int seb, sjb;      // bytes per member / coordinate
  bool median;
  // the uniform fields once, outside any lane-dependent branch (a value
  // merged at a divergent join is divergent to the compiler: the buffer
  // descriptor would need a waterfall loop per load)
  EKS_DEV void init(const SmoothArgs &a) {
    base = (const char *)a.obs;
    stb = a.st * (long long)sizeof(T);
    seb = (int)(a.se * (long long)sizeof(T));
    sjb = (int)(a.sj * (long long)sizeof(T));
    median = a.median != 0;
    loff = 0;
  }
  EKS_DEV void lane(const SmoothArgs &a, unsigned b) {
    loff = (unsigned)((unsigned long long)b * (unsigned long long)a.sb * sizeof(T));
  }
  EKS_DEV void fetch(int slot, long long t) {
    const __amdgpu_buffer_rsrc_t rs = member_rsrc(base + t * stb);
    // the E x N member offsets from the two strides (the compiler may hoist
    // them; an empty asm that kept them per fetch -- against SGPR spills seen
    // before the k3_bwd waitcnt fix -- measured 1.3 % slower after it)
    const int seb_ = seb, sjb_ = sjb;
    int off_e = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      int off = off_e;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        v[slot][e][j] = member_load<T, NT>(rs, loff, off);
        off += sjb_;
      }
      off_e += seb_;
    }
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
template <int N, typename YT, int D, bool NT = kNtLoad>
struct YevRing {
  YT y[D][N];
  double ev[D][N];
  const YT *yb;
  const double *eb;
  long long B;
  unsigned b;
  EKS_DEV void init(const SmoothArgs &a) {
    yb = (const YT *)a.obs;
    eb = (const double *)((const char *)a.obs + yev_ev_offset(a.B, a.T, N, sizeof(YT)));
    B = a.B;
    b = 0;
  }
  EKS_DEV void lane(const SmoothArgs &, unsigned bb) { b = bb; }
  EKS_DEV void fetch(int slot, long long t) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if constexpr (NT) {
        y[slot][j] = __builtin_nontemporal_load(&pl(yb, t * N + j, B, b));
        ev[slot][j] = __builtin_nontemporal_load(&pl(eb, t * N + j, B, b));
      } else {
        y[slot][j] = pl(yb, t * N + j, B, b);
        ev[slot][j] = pl(eb, t * N + j, B, b);
      }
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

template <int E, int N, typename T, int D, bool NT = kNtLoad>
struct SrcOf {
  using type = MemberRing<E, N, T, D, NT>;
};
template <int E, int N, typename YT, int D, bool NT>
struct SrcOf<E, N, YevIn<YT>, D, NT> {
  using type = YevRing<N, YT, D, NT>;
};

// Look-back payloads in time-major planes, stored write-through / loaded
// L1-bypassing (handoff.hpp).
template <int R>
EKS_DEV void elem_store_pl_wt(const Elem<R> &E, double *base, long long plane0, long long B,
                              unsigned b) {
  double v[Elem<R>::len];
  E.store(v, 1);
#pragma unroll
  for (int k = 0; k < Elem<R>::len; ++k) st_wt(&pl(base, plane0 + k, B, b), v[k]);
}
template <int R>
EKS_DEV void elem_load_pl_wt(Elem<R> &E, const double *base, long long plane0, long long B,
                             unsigned b) {
  double v[Elem<R>::len];
#pragma unroll
  for (int k = 0; k < Elem<R>::len; ++k) v[k] = ld_wt(&pl(base, plane0 + k, B, b));
  E.load(v, 1);
}
template <int R>
EKS_DEV void state_load_pl_wt(const double *base, long long plane0, long long B, unsigned b,
                              double (&m)[R], double (&P)[R][R]) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) m[i] = ld_wt(&pl(base, plane0 + (k++), B, b));
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = i; j < R; ++j) P[i][j] = P[j][i] = ld_wt(&pl(base, plane0 + (k++), B, b));
}
template <int R>
EKS_DEV void state_store_pl_wt(double *base, long long plane0, long long B, unsigned b,
                               const double (&m)[R], const double (&P)[R][R]) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) st_wt(&pl(base, plane0 + (k++), B, b), m[i]);
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = i; j < R; ++j) st_wt(&pl(base, plane0 + (k++), B, b), P[i][j]);
}
// ms <- G ms + g (the one expression every application of a chunk map uses,
// so that a mean carried through any number of maps has the same bits
// whichever unit applies them)
template <int R>
EKS_DEV void apply_map(const double (&G)[R][R], const double (&g)[R], double (&ms)[R]) {
  double nx[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    double sm = g[u];
#pragma unroll
    for (int q = 0; q < R; ++q) sm = fma(G[u][q], ms[q], sm);
    nx[u] = sm;
  }
#pragma unroll
  for (int u = 0; u < R; ++u) ms[u] = nx[u];
}

// H <- F o H for affine maps (F applied after H): G = F.G H.G, g = F.G H.g + F.g
template <int R>
EKS_DEV void compose_map(const double (&FG)[R][R], const double (&Fg)[R], double (&HG)[R][R],
                         double (&Hg)[R]) {
  double G[R][R], g[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
#pragma unroll
    for (int v = 0; v < R; ++v) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < R; ++q) t = fma(FG[u][q], HG[q][v], t);
      G[u][v] = t;
    }
    double t = Fg[u];
#pragma unroll
    for (int q = 0; q < R; ++q) t = fma(FG[u][q], Hg[q], t);
    g[u] = t;
  }
#pragma unroll
  for (int u = 0; u < R; ++u) {
    Hg[u] = g[u];
#pragma unroll
    for (int v = 0; v < R; ++v) HG[u][v] = G[u][v];
  }
}

// The first D steps of a lane's chunk into the ring (issued ahead: for the
// next unit while the current one finishes its tail).
template <int D, typename Src>
EKS_DEV void prefetch_head(Src &src, long long s, long long e) {
#pragma unroll
  for (int q = 0; q < D; ++q) src.fetch(q, min(s + q, e - 1));
}

// Feed the steps [s, e) of one lane (e - s <= LF; the ring's head loaded by
// prefetch_head) to absorb(t, y - offset, rv).  Full chunks run a
// compile-time loop whose prefetches are unconditional (a load under a
// lane-divergent `if` is merged into its ring slot by a copy that waits for
// it, i.e. no prefetch at all); the clamped tail re-reads the last step (a
// cache hit) instead of branching.
template <int LF, int D, int N, typename Src, typename F>
EKS_DEV void stream_steps(Src &src, long long s, long long e, const double (&off)[N], F &&absorb) {
  if (e - s == LF) {
#pragma unroll 1
    for (int i0 = 0; i0 < LF; i0 += D) {
#pragma unroll
      for (int q = 0; q < D; ++q) {
        if (LF % D == 0 || i0 + q < LF) {
          const long long t = s + i0 + q;
          double avg[N], rv[N], y[N];
          src.get(q, avg, rv);
          src.fetch(q, min(t + D, s + LF - 1));
#pragma unroll
          for (int j = 0; j < N; ++j) y[j] = avg[j] - off[j];
          absorb(t, y, rv);
        }
      }
    }
  } else {
    for (long long t0 = s; t0 < e; t0 += D) {
#pragma unroll
      for (int q = 0; q < D; ++q) {
        const long long t = t0 + q;
        if (t < e) {
          double avg[N], rv[N], y[N];
          src.get(q, avg, rv);
          if (t + D < e) src.fetch(q, t + D);
#pragma unroll
          for (int j = 0; j < N; ++j) y[j] = avg[j] - off[j];
          absorb(t, y, rv);
        }
      }
    }
  }
}

// Persistent grid: as many 256-thread blocks as can be resident (the
// occupancy query, cached per kernel), at most one per unit.
template <auto Kernel>
unsigned persistent_grid(long long units) {
  static int resident = 0;  // one device type per process
  if (resident <= 0) {
    int nb = 0, dev = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, Kernel, 256, 0) != hipSuccess || nb < 1)
      nb = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu < 1)
      ncu = 256;
    resident = nb * ncu;
  }
  return (unsigned)std::max(1LL, std::min(units, (long long)resident));
}

// ---------------------------------------------------------------------------
// Ticket schedule of one pass (mode 0: k3_fwd, mode 1: k3_bwd): a ticket is a
// unit, time-chunk major (k3_bwd: time chunks counted from the end), so the
// unit a unit waits for holds a smaller ticket.  (Round 4's one-launch form
// of both passes, k3_fused, measured no better at any size and was removed.)
// ---------------------------------------------------------------------------
struct Sched3 {
  int mode = 0;  // 0 fwd, 1 bwd
  long long ng = 0, NCu = 0, NCc = 0;
};
struct Work3 {
  int phase;  // 0 a k3_fwd unit, 1 a k3_bwd unit, 2 none (the grid drains)
  long long c, grp;  // time chunk (k3_bwd: counted from the end), group
};
inline Sched3 make_sched3(const Plan3 &p, int mode) {
  Sched3 s;
  s.mode = mode;
  s.ng = p.ng;
  s.NCu = p.NCu;
  s.NCc = p.NCc;
  return s;
}
// 32-bit arithmetic only
template <int MODE>
EKS_DEV Work3 decode3(const Sched3 &s, unsigned t) {
  Work3 w{2, 0, 0};
  const unsigned nc = (unsigned)(MODE == 0 ? s.NCu : s.NCc), ng = (unsigned)s.ng;
  if (t < nc * ng) {
    const unsigned c = t / ng;
    w.phase = MODE;
    w.c = c;
    w.grp = t - c * ng;
  }
  return w;
}

// ---------------------------------------------------------------------------
// k3_fwd: filtering elements + the forward chain (filtered states).  A unit
// is KPU = 4 x FPW fine chunks: each wave streams FPW consecutive ones (two
// at r = 2: 128-step units, half the chain links and half the per-unit tail
// of a one-chunk wave; r = 3 elements are too large for that LDS).
// ---------------------------------------------------------------------------
template <int R>
constexpr int fwd_fpw() { return R <= 2 ? 2 : 1; }

// LDS of one k3_fwd unit (doubles): each wave's first element (FPW = 2), each
// wave's element then the prefix compositions, the state entering the unit
template <int R>
constexpr int fwd_lds_doubles() {
  return ((fwd_fpw<R>() > 1 ? kWV : 1) + kWV) * Elem<R>::len * 64 + (R + Sym<R>::len) * 64;
}

// The k3_fwd units of consecutive tickets from t on (the run ends when the
// tickets run out).  Member loads are non-temporal: nothing re-reads them
// soon (7 GB at config 4 pass through the caches before k3_bwd).
template <int R, int N, int E, typename T, int AI, int CI>
EKS_DEV unsigned k3_fwd_run(const SmoothArgs &a, const Plan3 &p, const Sched3 &sc, unsigned t,
                            double *lds, unsigned *tk, unsigned *ctr, int &it) {
  constexpr int EL = Elem<R>::len, KS = R + Sym<R>::len;
  constexpr int D = is_yev<T>::value ? kK3YevD : kK3D;
  constexpr int LF = fine_len3(R, N);
  constexpr int FPW = fwd_fpw<R>(), KPU = kWV * FPW;
  constexpr int NA = FPW > 1 ? kWV : 1;
  auto &shA = *reinterpret_cast<double (*)[NA][EL][64]>(lds);  // each wave's first element (FPW = 2)
  auto &shX = *reinterpret_cast<double (*)[kWV][EL][64]>(lds + NA * EL * 64);  // each wave's element, then prefixes
  auto &shS = *reinterpret_cast<double (*)[KS][64]>(lds + (NA + kWV) * EL * 64);  // state entering the unit
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const long long B = a.B, TT = a.T;
  unsigned *flags = (unsigned *)(a.ws + p.flag1_off);
  double *fst = (double *)(a.ws + p.fst_off);
  double *agg1 = (double *)(a.ws + p.agg1_off);
  const double *prm = (const double *)(a.ws + p.prm_off);
  // member ring, persists across the units of the run
  typename SrcOf<E, N, T, D>::type src;
  src.init(a);
  Model<R, N> md;
  // model + the first member steps of unit wk (structure checked by
  // k_model_planes).  Lanes past the last trajectory read trajectory 0 (their
  // results are never stored): every branch here is wave-uniform.
  auto head = [&](const Work3 &wk) {
    if (wk.phase != 0) return;
    const long long c = wk.c, g = wk.grp, ff = (c * kWV + w) * FPW;
    const unsigned bb = (unsigned)(g * 64 + l);
    const unsigned bl = (long long)bb < B ? bb : 0u;
    if (ff < p.NCf) {
      load_model_pl<R, N, AI, CI>(prm, B, bl, ff == 0, md);
      src.lane(a, bl);
      const long long s = ff * p.L;
      prefetch_head<D>(src, s, min(TT, s + p.L));
    }
  };
  auto load_state_sh = [&](double (&m)[R], double (&P)[R][R]) {
    int k = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) m[i] = shS[k++][l];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = i; j < R; ++j) P[i][j] = P[j][i] = shS[k++][l];
  };
  Work3 wk = decode3<0>(sc, t);  // uniform: every index below in SGPRs
  head(wk);
  while (wk.phase == 0) {
    EKS_STAMP(0, 0);
    EKS_STAMP(0, 1);
    unsigned tnext = 0;
    if (threadIdx.x == 0) tnext = atomicAdd(ctr, 1u);  // consumed after the streaming
    const long long cu = wk.c, grp = wk.grp;
    const long long f0 = (cu * kWV + w) * FPW;  // the wave's first fine chunk
    const unsigned b = (unsigned)(grp * 64 + l);
    const bool lane_ok = (long long)b < B;
    const bool live = lane_ok && f0 < p.NCf;
    bool ok = true, okf = true;  // element / composition, and the plain filter of chunk 0
    Elem<R> El;                  // the wave's last element (E_B), or its only one
    El.set_identity();
    if constexpr (FPW > 1) El.store(&shA[w][0][l], 64);  // E_A of a dead wave
    if (f0 < p.NCf) {  // (dead lanes: trajectory 0's data, replaced by the identity below)
      const long long s0 = f0 * p.L, e0 = min(TT, s0 + FPW * p.L);
      auto absorb_el = [&](long long, const double (&y)[N], const double (&rv)[N]) {
        elem_absorb<R, N, AI, CI>(El, md.A, md.Q, md.C, y, rv, ok);
      };
      if (f0 == 0) {  // the first chunk: the plain filter from the prior,
                      // summarised as the known filtered state (Ab = 0)
        const long long e = min(TT, s0 + p.L);
        double m[R], P[R][R];
        NllAcc acc;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          m[i] = md.m0[i];
#pragma unroll
          for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
        }
        stream_steps<LF, D, N>(src, s0, e, md.off,
                               [&](long long tt, const double (&y)[N], const double (&rv)[N]) {
                                 if (tt > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
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
        if constexpr (FPW > 1) {
          El.store(&shA[w][0][l], 64);
          El.set_identity();
          if (e0 > e) {
            prefetch_head<D>(src, e, e0);
            stream_steps<LF, D, N>(src, e, e0, md.off, absorb_el);
          }
        }
      } else if constexpr (FPW > 1) {
        // both chunks as one stream; the first element is parked in LDS at
        // the boundary (a wave-uniform branch once per 16 steps)
        const long long sb = s0 + p.L;
        stream_steps<FPW * LF, D, N>(src, s0, e0, md.off,
                                     [&](long long tt, const double (&y)[N], const double (&rv)[N]) {
                                       if (tt == sb) {
                                         El.store(&shA[w][0][l], 64);
                                         El.set_identity();
                                       }
                                       absorb_el(tt, y, rv);
                                     });
        if (e0 <= sb) {  // no second chunk (the trajectory ends in the first)
          El.store(&shA[w][0][l], 64);
          El.set_identity();
        }
      } else {
        stream_steps<LF, D, N>(src, s0, e0, md.off, absorb_el);
      }
    }
    // wave 0: the neighbour's flag polled now, read at the chain point (the
    // load flies during the element stores, the barrier and the compositions)
    unsigned early = 0u;
    if (kEarlyPoll && w == 0 && cu > 0) early = ld_flag(flags + grp * p.NCu + cu - 1);
    if (!lane_ok) {  // a dead lane's chain stays exact (identity elements)
      El.set_identity();
      if constexpr (FPW > 1) El.store(&shA[w][0][l], 64);
      ok = okf = true;
    }
    // X_w = the wave's elements composed (own LDS data: no barrier needed)
    if constexpr (FPW > 1) {
      Elem<R> Ea, Et;
      Ea.load(&shA[w][0][l], 64);
      ok = compose_elem<R>(Ea, El, Et) && ok;
      Et.store(&shX[w][0][l], 64);
    } else {
      El.store(&shX[w][0][l], 64);
    }
    EKS_STAMP(0, 2);
    if (threadIdx.x == 0) tk[(it + 1) & 1] = tnext;
    __syncthreads();
    EKS_STAMP(0, 3);
    const unsigned tn = __builtin_amdgcn_readfirstlane(tk[(it + 1) & 1]);
    const Work3 wn = decode3<0>(sc, tn);
    // the next unit's first member steps in flight during this unit's tail
    // (wave 0 after its chain wait: vmcnt counts in order, so a prefetch
    // issued before the poll would hold the poll back until it lands)
    if (w != 0) head(wn);
    // prefix over the waves (dead chunks / lanes hold the identity, which
    // composes exactly): round 1 X01 -> slot 1, X23 -> slot 3
    if (w == 1 || w == 3) {
      Elem<R> Ea, Eb, Et;
      Ea.load(&shX[w - 1][0][l], 64);
      Eb.load(&shX[w][0][l], 64);
      ok = compose_elem<R>(Ea, Eb, Et) && ok;
      Et.store(&shX[w][0][l], 64);
    }
    __syncthreads();
    // round 2: X012 -> slot 2 (wave 2); the unit's element X0123 (wave 0)
    Elem<R> Ec;
    if (w == 2) {
      Elem<R> Ea, Eb, Et;
      Ea.load(&shX[1][0][l], 64);
      Eb.load(&shX[2][0][l], 64);
      ok = compose_elem<R>(Ea, Eb, Et) && ok;
      Et.store(&shX[2][0][l], 64);
    } else if (w == 0) {
      Elem<R> Ea, Eb;
      Ea.load(&shX[1][0][l], 64);
      Eb.load(&shX[3][0][l], 64);
      ok = compose_elem<R>(Ea, Eb, Ec) && ok;
    }
    if (w == 0) {
      // the chain: filtered state entering unit cu = the state leaving unit
      // cu - 1 (for cu = 0 any state: chunk 0's element has Ab = 0).
      // Decoupled look-back: if unit cu - 1 has not published that state yet,
      // this unit publishes its own element for the units after it, then walks
      // back to the nearest unit j whose leaving state is published and folds
      // the elements of units j+1 .. cu-1 into it.  compose_state is a left
      // fold of state (x) element, so the state has the same bits whichever j
      // it starts from: results do not depend on timing.
      double m[R], P[R][R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        m[i] = 0.0;
#pragma unroll
        for (int j = 0; j < R; ++j) P[i][j] = 0.0;
      }
      if (cu > 0) {
        const unsigned *fl = flags + grp * p.NCu;  // group-major: a walk reads consecutive words
        long long j = cu - 1;
        const bool agg = cu + 1 < p.NCu;  // (the last unit has no successor)
        if (kEagerAgg) {
          // the aggregate's stores go out with the neighbour's poll (the poll's
          // wait covers them), then its flag: later units fold it instead of
          // waiting for this unit's own chain wait
          if (agg && lane_ok) elem_store_pl_wt<R>(Ec, agg1, cu * EL, B, b);
          const bool ready = inc_ready(fl + j, a.wait_ticks);
          if (agg) publish_flag(flags + grp * p.NCu + cu, l, kAggReady);
          if (!ready) j = look_back(fl, j, 1, -1, p.NCu, a.wait_ticks, ok);
        } else if (!(kEarlyPoll && inc_ready_early(early, a.wait_ticks)) &&
                   !inc_ready(fl + j, a.wait_ticks)) {
          if (agg) {
            if (lane_ok) elem_store_pl_wt<R>(Ec, agg1, cu * EL, B, b);
            publish_flag(flags + grp * p.NCu + cu, l, kAggReady);
          }
          j = look_back(fl, j, 1, -1, p.NCu, a.wait_ticks, ok);
        }
        EKS_STAMP_AUX(0, 1, __builtin_amdgcn_s_memtime());
        EKS_STAMP_AUX(0, 2, cu - 1 - j);
        if (lane_ok) {
          state_load_pl_wt<R>(fst, ((j + 1) * KPU) * KS, B, b, m, P);
          // fold the elements of units j+1 .. cu-1, the next one's loads in
          // flight while one is composed (a walk back over many units is then
          // ~one L2 / MALL latency per element, not a load round trip each)
          if (j + 1 < cu) {
            Elem<R> Ei;
            elem_load_pl_wt<R>(Ei, agg1, (j + 1) * EL, B, b);
            for (long long i = j + 1; i < cu; ++i) {
              Elem<R> En;
              if (i + 1 < cu) elem_load_pl_wt<R>(En, agg1, (i + 1) * EL, B, b);
              ok = compose_state<R>(m, P, Ei) && ok;
              Ei = En;
            }
          }
        }
      }
      {
        int k = 0;
#pragma unroll
        for (int i = 0; i < R; ++i) shS[k++][l] = m[i];
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int j = i; j < R; ++j) shS[k++][l] = P[i][j];
      }
      ok = compose_state<R>(m, P, Ec) && ok;  // the state leaving unit cu
      if (cu + 1 < p.NCu) {
        if (lane_ok) state_store_pl_wt<R>(fst, ((cu + 1) * KPU) * KS, B, b, m, P);
        publish_flag(flags + grp * p.NCu + cu, l, kIncReady);
      }
      head(wn);
    }
    EKS_STAMP(0, 4);
    __syncthreads();
    EKS_STAMP(0, 5);
    // fine start states: wave w's first chunk starts from the entering state
    // composed with the waves before it (slots 0 / 1 / 2 = X0 / X01 / X012;
    // wave 0's is the entering state itself, stored by the unit before), its
    // second from that composed with its first element
    if (live) {
      double m[R], P[R][R];
      load_state_sh(m, P);
      if (w >= 1) {
        Elem<R> Ep;
        Ep.load(&shX[w - 1][0][l], 64);
        ok = compose_state<R>(m, P, Ep) && ok;
        store_state_pl<R>(fst, f0 * KS, B, b, m, P);
      }
      if constexpr (FPW > 1) {
        if (f0 + 1 < p.NCf) {
          Elem<R> Ea;
          Ea.load(&shA[w][0][l], 64);
          ok = compose_state<R>(m, P, Ea) && ok;
          store_state_pl<R>(fst, (f0 + 1) * KS, B, b, m, P);
        }
      }
    }
    if (lane_ok)
      flag(a.status, b, (ok ? 0 : EKS_STATUS_SCAN) | (okf ? 0 : EKS_STATUS_SINGULAR));
    EKS_STAMP(0, 6);
    __syncthreads();  // LDS free for the next unit
    EKS_STAMP(0, 7);
    t = tn;
    wk = wn;
    ++it;
  }
  return t;
}

template <int R, int N, int E, typename T, int AI, int CI>
__global__ __launch_bounds__(64 * kWV) void k3_fwd(SmoothArgs a, Plan3 p, Sched3 sc) {
  __shared__ double lds[fwd_lds_doubles<R>()];
  __shared__ unsigned tk[2];
  unsigned *ctr = (unsigned *)a.ws;
  if (threadIdx.x == 0) tk[0] = atomicAdd(ctr, 1u);
  __syncthreads();
  int it = 0;
  k3_fwd_run<R, N, E, T, AI, CI>(a, p, sc, __builtin_amdgcn_readfirstlane(tk[0]), lds, tk, ctr,
                                 it);
}

// ---------------------------------------------------------------------------
// k3_bwd: the final smoothing pass + the backward chain (smoothed means)
// ---------------------------------------------------------------------------
// LDS of one k3_bwd unit (doubles): the filtered states of the first NL
// steps of every lane, the RTS maps of waves 1..3 (then their entering means)
template <int R, int N>
constexpr int bwd_lds_doubles() {
  return lds_steps3(R, N) * (R + Sym<R>::len) * 64 * kWV + (kWV - 1) * (R * R + R) * 64;
}

// an empty use of the model registers a later loop reads (see k3_bwd_run)
template <int R, int N, int AI, int CI>
EKS_DEV void touch_model(Model<R, N> &md) {
#pragma unroll
  for (int j = 0; j < N; ++j) asm volatile("" : "+v"(md.off[j]));
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int k = 0; k < R; ++k) {
      asm volatile("" : "+v"(md.Q[i][k]));
      if constexpr (AI != kAId) asm volatile("" : "+v"(md.A[i][k]));
    }
  if constexpr (CI != kCId)
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int k = 0; k < R; ++k) asm volatile("" : "+v"(md.C[j][k]));
}

// The k3_bwd units of consecutive tickets from t on (the run ends when the
// tickets run out).  LB: the backward chain's look-back (publish the unit's maps, walk, fold).
// It only pays where few groups share the chip (the 8-GPU shard's k3_bwd:
// 0.365 -> 0.348 ms) and adds SGPR pressure to the hot loop (21 -> 153
// v_readlane in the ISA; config 4 measured the same either way), so it is a
// separate instantiation, launched for small batches (a3_bwd_lookback).
template <int R, int N, int E, typename T, int AI, int CI, bool NLL, bool LB>
EKS_DEV unsigned k3_bwd_run(const SmoothArgs &a, const Plan3 &p, const Sched3 &sc, unsigned t,
                            double *lds, unsigned *tk, unsigned *ctr, int &it) {
  constexpr int KS = R + Sym<R>::len, MP = R * R + R;
  constexpr int D = is_yev<T>::value ? kK3YevD : kK3BD;
  constexpr int NR = reg_steps3(R, N), NL = lds_steps3(R, N), LF = NR + NL;
  auto &fs = *reinterpret_cast<double (*)[NL][KS][64 * kWV]>(lds);  // filtered states, first NL steps
  auto &shM = *reinterpret_cast<double (*)[kWV - 1][MP][64]>(lds + NL * KS * 64 * kWV);  // maps of waves 1..3
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const int tid = threadIdx.x;
  const long long B = a.B, TT = a.T;
  unsigned *flags = (unsigned *)(a.ws + p.flag2_off);
  const double *fst = (const double *)(a.ws + p.fst_off);
  double *inc = (double *)(a.ws + p.inc2_off);
  double *agg2 = (double *)(a.ws + p.agg2_off);
  const double *prm = (const double *)(a.ws + p.prm_off);
  const bool vec2 = N == 2 && a.oj == 1 && ((a.ob | a.ot) & 1) == 0 &&
                    (((uintptr_t)a.out) & 15) == 0;
  Work3 wk = decode3<1>(sc, t);  // uniform: every index below in SGPRs
  while (wk.phase == 1) {
    EKS_STAMP(1, 0);
    EKS_STAMP(1, 1);
    unsigned tnext = 0;
    if (tid == 0) tnext = atomicAdd(ctr, 1u);
    const long long cr = wk.c, grp = wk.grp;
    const long long cc = p.NCc - 1 - cr;  // units in reverse time order
    const long long f = cc * kWV + w;
    const unsigned b = (unsigned)(grp * 64 + l);
    const bool lane_ok = (long long)b < B;
    const bool live = lane_ok && f < p.NCf;
    bool ok = true, okc = true;  // recursions, and the chain wait
    Model<R, N> md;
    // the last NR steps keep their RTS gains (J_t, d_t) from the forward
    // sweep in registers; the first NL keep filtered states in LDS
    double Jr[NR][R][R], dr[NR][R];
    Affine<R> Mp;       // this chunk's RTS map: ms[s] = G ms[e] + g
    Mp.set_identity();
    const long long s = f * p.L, e = min(TT, s + p.L);
    // a whole fine chunk with a successor step after it (wave-uniform)
    // (the single-view shape only: elsewhere the guarded loop, half the code)
    const bool full = R == 2 && N == 2 && e - s == LF && e < TT;
    // wave-uniform branch: lanes past the last trajectory run on trajectory
    // 0's data and store nothing
    const unsigned bl = lane_ok ? b : 0u;
    if (f < p.NCf) {
      load_model_pl<R, N, AI, CI>(prm, B, bl, f == 0, md);
      double m[R], P[R][R];
      if (f == 0) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          m[i] = md.m0[i];
#pragma unroll
          for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
        }
      } else {
        load_state_pl<R>(fst, f * KS, B, bl, m, P);
      }
      typename SrcOf<E, N, T, D>::type src;
      src.init(a);
      src.lane(a, bl);
#pragma unroll
      for (int q = 0; q < D; ++q)
        if (s + q < e) src.fetch(q, s + q);
      typename std::conditional<NLL, NllAcc, NoAcc>::type acc;  // NLL shares only when asked for
      // one forward step i (time tt) of the re-run.  FULL: a whole chunk that
      // is not the trajectory's last (every step present, every step has a
      // successor): no run-time guards, so no value merges at each step
      auto fwd_step = [&](const int i, const long long tt, auto full) {
        constexpr bool FULL = decltype(full)::value;
        double avg[N], rv[N], y[N];
        src.get(i % D, avg, rv);
        if (FULL ? i + D < LF : tt + D < e) src.fetch(i % D, tt + D);
#pragma unroll
        for (int j = 0; j < N; ++j) y[j] = avg[j] - md.off[j];
        if (FULL ? (i > 0 || f > 0) : tt > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
        kf_update<R, N, CI, decltype(acc)>(m, P, md.C, y, rv, acc, ok);
        if (i < NL) {
          double st[KS];
          int k = 0;
#pragma unroll
          for (int u = 0; u < R; ++u) st[k++] = m[u];
#pragma unroll
          for (int u = 0; u < R; ++u)
#pragma unroll
            for (int v = u; v < R; ++v) st[k++] = P[u][v];
#pragma unroll
          for (int u = 0; u < KS; ++u) fs[i < NL ? i : 0][u][tid] = st[u];
        }
        const int ir = i >= NL ? i - NL : 0;
        // the chunk's map in forward order: G <- G J_t, g <- g + G d_t
        // (the trajectory's last step: ms[T-1] = mf[T-1], a constant)
        if (FULL || tt + 1 < TT) {
          double J[R][R], d[R];
          ok = rts_gain<R, AI>(m, P, md.A, md.Q, J, d) && ok;
          if (i >= NL) {
#pragma unroll
            for (int u = 0; u < R; ++u) {
              dr[ir][u] = d[u];
#pragma unroll
              for (int v = 0; v < R; ++v) Jr[ir][u][v] = J[u][v];
            }
          }
          Affine<R> step;
#pragma unroll
          for (int u = 0; u < R; ++u) {
            step.g[u] = d[u];
#pragma unroll
            for (int v = 0; v < R; ++v) step.G[u][v] = J[u][v];
          }
          Mp = Mp.after(step);
        } else {
          if (i >= NL) {
#pragma unroll
            for (int u = 0; u < R; ++u) dr[ir][u] = m[u];
          }
#pragma unroll
          for (int u = 0; u < R; ++u) {
            double sg = Mp.g[u];
#pragma unroll
            for (int v = 0; v < R; ++v) sg = fma(Mp.G[u][v], m[v], sg);
            Mp.g[u] = sg;
          }
#pragma unroll
          for (int u = 0; u < R; ++u)
#pragma unroll
            for (int v = 0; v < R; ++v) Mp.G[u][v] = 0.0;
        }
      };
      if (full) {
#pragma unroll
        for (int i = 0; i < LF; ++i) {
          fwd_step(i, s + i, std::true_type{});
          if constexpr (kK3BSched) __builtin_amdgcn_sched_barrier(0);  // one step's registers at a time
        }
      } else {
#pragma unroll
        for (int i = 0; i < LF; ++i)
          if (s + i < e) fwd_step(i, s + i, std::false_type{});
      }
      if (NLL && lane_ok) pl((double *)(a.ws + p.nllp_off), f, B, b) = acc.value((double)(e - s) * N);
      // the model registers the backward sweep reads (offsets; Q, A, C when
      // not the identity) marked complete here, on every path: otherwise the
      // waitcnt pass, merging the paths around each `if (tt < e)`, re-waits
      // for their loads at every emitted step -- vmcnt counts the output
      // stores too, so each step waited for the previous step's store
      touch_model<R, N, AI, CI>(md);
      if (!lane_ok) {
        ok = true;
        Mp.set_identity();
      }
    }
    EKS_STAMP(1, 2);
    // wave 0: the next unit's flag polled now, read at the chain point
    unsigned early = 0u;
    if (kEarlyPoll && w == 0 && cc + 1 < p.NCc) early = ld_flag(flags + grp * p.NCc + cc + 1);
    if (w >= 1) {
      int k = 0;
#pragma unroll
      for (int u = 0; u < R; ++u)
#pragma unroll
        for (int v = 0; v < R; ++v) shM[w - 1][k++][l] = Mp.G[u][v];
#pragma unroll
      for (int u = 0; u < R; ++u) shM[w - 1][k++][l] = Mp.g[u];
    }
    __syncthreads();
    EKS_STAMP(1, 3);
    double ms[R];  // smoothed mean at the first step after this chunk
    if (w == 0) {
      // the chain: the mean at the first step of coarse chunk cc+1, published
      // by its unit (for the last coarse chunk: unused, its last map is
      // constant).  The unit's map U = M0 o M1 o M2 o M3 (its 4 chunk maps,
      // composed right to left in a fixed order) carries that mean to the
      // mean at the unit's first step, which the unit publishes.  Decoupled
      // look-back as in k3_fwd: if unit cc+1 has not published its mean yet,
      // this unit publishes U for the units before it, walks forward to the
      // nearest unit j with a published mean and carries that mean back
      // through the maps U of units j-1 .. cc+1 with the expression every
      // unit uses (apply_map): the same bits whichever j it starts from.
      // The walk's loads go out KLB units at a time (one round trip per KLB
      // units instead of one per chunk map).
      constexpr int KLB = 4;
      double UG[R][R], Ug[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        Ug[u] = shM[kWV - 2][R * R + u][l];
#pragma unroll
        for (int v = 0; v < R; ++v) UG[u][v] = shM[kWV - 2][u * R + v][l];
      }
#pragma unroll
      for (int v = kWV - 2; v >= 1; --v) {
        double G[R][R], g[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
          g[u] = shM[v - 1][R * R + u][l];
#pragma unroll
          for (int q = 0; q < R; ++q) G[u][q] = shM[v - 1][u * R + q][l];
        }
        compose_map<R>(G, g, UG, Ug);
      }
      compose_map<R>(Mp.G, Mp.g, UG, Ug);
#pragma unroll
      for (int u = 0; u < R; ++u) ms[u] = 0.0;
      if (cc + 1 < p.NCc) {
        const unsigned *fl = flags + grp * p.NCc;  // group-major
        long long j = cc + 1;
        auto store_agg = [&]() {
          if (lane_ok) {
#pragma unroll
            for (int u = 0; u < R; ++u) {
#pragma unroll
              for (int q = 0; q < R; ++q) st_wt(&pl(agg2, cc * MP + u * R + q, B, b), UG[u][q]);
              st_wt(&pl(agg2, cc * MP + R * R + u, B, b), Ug[u]);
            }
          }
        };
        const bool early_ok = kEarlyPoll && inc_ready_early(early, a.wait_ticks);
        if (!LB) {
          if (!early_ok && !wait_flag(fl + j, a.wait_ticks, kIncReady)) okc = false;
        } else if (early_ok) {
        } else if (kEagerAgg) {  // (as k3_fwd: U published with the poll)
          if (cc > 0) store_agg();
          const bool ready = inc_ready(fl + j, a.wait_ticks);
          if (cc > 0) publish_flag(flags + grp * p.NCc + cc, l, kAggReady);
          if (!ready) j = look_back(fl, j, 1, +1, p.NCc, a.wait_ticks, okc);
        } else if (!inc_ready(fl + j, a.wait_ticks)) {
          if (cc > 0) {
            store_agg();
            publish_flag(flags + grp * p.NCc + cc, l, kAggReady);
          }
          j = look_back(fl, j, 1, +1, p.NCc, a.wait_ticks, okc);
        }
        EKS_STAMP_AUX(1, 1, __builtin_amdgcn_s_memtime());
        EKS_STAMP_AUX(1, 2, j - cc - 1);
        if (lane_ok) {
#pragma unroll
          for (int u = 0; u < R; ++u) ms[u] = ld_wt(&pl(inc, j * R + u, B, b));
          for (long long i0 = j - 1; i0 > cc; i0 -= KLB) {
            double G[KLB][R][R], g[KLB][R];
#pragma unroll
            for (int k = 0; k < KLB; ++k) {
              const long long i = i0 - k > cc ? i0 - k : i0;  // (past cc: a re-load, unused)
#pragma unroll
              for (int u = 0; u < R; ++u) {
#pragma unroll
                for (int q = 0; q < R; ++q) G[k][u][q] = ld_wt(&pl(agg2, i * MP + u * R + q, B, b));
                g[k][u] = ld_wt(&pl(agg2, i * MP + R * R + u, B, b));
              }
            }
#pragma unroll
            for (int k = 0; k < KLB; ++k)
              if (i0 - k > cc) apply_map<R>(G[k], g[k], ms);
          }
        }
      }
      // right to left through waves 3, 2, 1: hand each its entering mean
      double mnext[R];
#pragma unroll
      for (int u = 0; u < R; ++u) mnext[u] = ms[u];
#pragma unroll
      for (int v = kWV - 1; v >= 1; --v) {
        double G[R][R], g[R];
        int k = 0;
#pragma unroll
        for (int u = 0; u < R; ++u)
#pragma unroll
          for (int q = 0; q < R; ++q) G[u][q] = shM[v - 1][k++][l];
#pragma unroll
        for (int u = 0; u < R; ++u) g[u] = shM[v - 1][k++][l];
#pragma unroll
        for (int u = 0; u < R; ++u) shM[v - 1][u][l] = ms[u];
        apply_map<R>(G, g, ms);
      }
      if (cc > 0) {  // the mean at this coarse chunk's first step: U(mean entering the unit)
        apply_map<R>(UG, Ug, mnext);
        if (lane_ok)
#pragma unroll
          for (int u = 0; u < R; ++u) st_wt(&pl(inc, cc * R + u, B, b), mnext[u]);
        publish_flag(flags + grp * p.NCc + cc, l, kIncReady);
      }
    }
    EKS_STAMP(1, 4);
    __syncthreads();
    EKS_STAMP(1, 5);
    if (w >= 1)
#pragma unroll
      for (int u = 0; u < R; ++u) ms[u] = shM[w - 1][u][l];
    if (live) {
      double *outb = a.out + (long long)b * a.ob;
      auto emit = [&](long long tt) {
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
            if constexpr (kNtOut) {  // streaming (non-temporal) output stores
              __builtin_nontemporal_store(cm[0], outb + tt * a.ot);
              __builtin_nontemporal_store(cm[1], outb + tt * a.ot + 1);
            } else {
              *(double2 *)(outb + tt * a.ot) = make_double2(cm[0], cm[1]);
            }
          } else {
            project_store<R, N, CI>(outb + tt * a.ot, a.oj, md.C, ms, md.off);
          }
        } else {
          project_store<R, N, CI>(outb + tt * a.ot, a.oj, md.C, ms, md.off);
        }
        if (a.ms) store_vec<R>(a.ms + ((long long)b * TT + tt) * R, ms);
      };
      // one RTS step backwards from the filtered state st of step tt
      auto rts_step = [&](const double (&st)[KS], long long tt) {
        double mf[R], Pf[R][R];
        int k = 0;
#pragma unroll
        for (int i = 0; i < R; ++i) mf[i] = st[k++];
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int j = i; j < R; ++j) Pf[i][j] = Pf[j][i] = st[k++];
        if (tt + 1 == TT) {  // ms[T-1] = mf[T-1]
#pragma unroll
          for (int i = 0; i < R; ++i) ms[i] = mf[i];
          return;
        }
        double J[R][R], d[R], nx[R];
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
      // the last NR steps from registers, then the first NL from LDS
      auto bwd_reg = [&](const int i, const long long tt, auto fullc) {
        double nx[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
          double sm = dr[i - NL][u];
#pragma unroll
          for (int v = 0; v < R; ++v) sm = fma(Jr[i - NL][u][v], ms[v], sm);
          nx[u] = sm;
        }
        if constexpr (decltype(fullc)::value) {
#pragma unroll
          for (int u = 0; u < R; ++u) ms[u] = nx[u];
        } else {
          const bool last = tt + 1 == TT;  // ms[T-1] = mf[T-1] (J_t unset)
#pragma unroll
          for (int u = 0; u < R; ++u) ms[u] = last ? dr[i - NL][u] : nx[u];
        }
        emit(tt);
      };
      auto bwd_lds = [&](const int i, const long long tt) {
        double st[KS];
#pragma unroll
        for (int u = 0; u < KS; ++u) st[u] = fs[i][u][tid];
        rts_step(st, tt);
        emit(tt);
      };
      if (full) {
#pragma unroll
        for (int i = LF - 1; i >= NL; --i) bwd_reg(i, s + i, std::true_type{});
#pragma unroll
        for (int i = NL - 1; i >= 0; --i) bwd_lds(i, s + i);
      } else {
#pragma unroll
        for (int i = LF - 1; i >= NL; --i)
          if (s + i < e) bwd_reg(i, s + i, std::false_type{});
#pragma unroll
        for (int i = NL - 1; i >= 0; --i)
          if (s + i < e) bwd_lds(i, s + i);
      }
    }
    EKS_STAMP(1, 6);
    if (lane_ok)
      flag(a.status, b, (ok ? 0 : EKS_STATUS_SINGULAR) | (okc ? 0 : EKS_STATUS_SCAN));
    if (tid == 0) tk[(it + 1) & 1] = tnext;
    __syncthreads();  // LDS free for the next unit, its ticket visible
    EKS_STAMP(1, 7);
    t = __builtin_amdgcn_readfirstlane(tk[(it + 1) & 1]);
    wk = decode3<1>(sc, t);
    ++it;
  }
  return t;
}

template <int R, int N, int E, typename T, int AI, int CI, bool NLL, bool LB>
__global__ __launch_bounds__(64 * kWV, 2) void k3_bwd(SmoothArgs a, Plan3 p, Sched3 sc) {
  __shared__ double lds[bwd_lds_doubles<R, N>()];
  __shared__ unsigned tk[2];
  unsigned *ctr = (unsigned *)a.ws + 32;
  if (threadIdx.x == 0) tk[0] = atomicAdd(ctr, 1u);
  __syncthreads();
  int it = 0;
  k3_bwd_run<R, N, E, T, AI, CI, NLL, LB>(a, p, sc, __builtin_amdgcn_readfirstlane(tk[0]), lds, tk,
                                         ctr, it);
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

// k3_bwd's look-back instantiation (LB): for batches of at most kLbGroups
// 64-trajectory groups, where several time chunks of a group are resident at
// once (eks_debug_set(EKS_DBG_A3_LB): 1 never, 2 always, 0 this rule).
// Measured: 128 videos (34 groups) k3_bwd 0.336 -> 0.320 ms with it, 256
// videos (68 groups) 0.525 -> 0.544 ms
constexpr long long kLbGroups = 48;
inline bool a3_bwd_lookback(const Plan3 &p) {
  if (g_a3_lb == 1) return false;
  if (g_a3_lb == 2) return true;
  return kLbAll || p.ng <= kLbGroups;
}

// host: the launches of one algo-3 call
template <int R, int N, int AI, int CI>
int launch_algo3_one(const SmoothArgs &a) {
  const Plan3 p = make_plan3(a.B, a.T, R, N);
  const bool yev = a.dtype == EKS_YEV32 || a.dtype == EKS_YEV64;
  const bool f32 = a.dtype == EKS_F32;
  auto run = [&](auto tag, auto Ec) -> int {
    using Tp = decltype(tag);
    constexpr int EE = decltype(Ec)::value;
    int rc;
    prof_call_begin();
    prof_mark(a.stream, "k_model_planes");
    // tickets and chain flags start at zero every call: k_model_planes zeroes
    // them (sync_bytes is a multiple of 256), or a memset node when the
    // caller's workspace is not 16-byte aligned
    const bool zk = ((uintptr_t)a.ws & 15) == 0;
    if (!zk && hipMemsetAsync(a.ws, 0, p.sync_bytes, a.stream) != hipSuccess)
      return set_err(EKS_ERR_HIP, "eks_smooth algo 3: hipMemsetAsync failed");
    hipLaunchKernelGGL((k_model_planes<R, N, AI, CI>), dim3(grid_for(a.B, 256)), dim3(256), 0, a.stream,
                       a.params, a.B, (double *)(a.ws + p.prm_off), a.status, (uint4 *)a.ws,
                       zk ? (long long)(p.sync_bytes / sizeof(uint4)) : 0LL);
    if ((rc = check_launch("k_model_planes"))) return rc;
    // the single-view model: the throughput shape (config 4)
    constexpr bool kSingleView = R == 2 && N == 2 && AI == kAId && CI == kCId;
    {
      prof_mark(a.stream, "k3_fwd");
      hipLaunchKernelGGL((k3_fwd<R, N, EE, Tp, AI, CI>),
                         dim3(persistent_grid<k3_fwd<R, N, EE, Tp, AI, CI>>(p.units_f)),
                         dim3(64 * kWV), 0, a.stream, a, p, make_sched3(p, 0));
      if ((rc = check_launch("k3_fwd"))) return rc;
      prof_mark(a.stream, "k3_bwd");
      const Sched3 sb = make_sched3(p, 1);
      // the look-back instantiation only for small batches of the
      // single-view shape
      bool lb = false;
      if constexpr (kSingleView) lb = a3_bwd_lookback(p);
      // (the look-back instantiation exists for the single-view shape only)
      auto bwd = [&](auto nll, auto lbc) {
        constexpr bool NL_ = decltype(nll)::value, LB_ = decltype(lbc)::value;
        hipLaunchKernelGGL((k3_bwd<R, N, EE, Tp, AI, CI, NL_, LB_>),
                           dim3(persistent_grid<k3_bwd<R, N, EE, Tp, AI, CI, NL_, LB_>>(p.units)),
                           dim3(64 * kWV), 0, a.stream, a, p, sb);
      };
      auto bwd_nll = [&](auto nll) {
        if constexpr (kSingleView) {
          if (lb) bwd(nll, std::true_type{});
          else bwd(nll, std::false_type{});
        } else {
          bwd(nll, std::false_type{});
        }
      };
      if (a.nll) bwd_nll(std::true_type{});
      else bwd_nll(std::false_type{});
      if ((rc = check_launch("k3_bwd"))) return rc;
    }
    if (a.nll) {
      prof_mark(a.stream, "k3_nll");
      hipLaunchKernelGGL((k3_nll<R>), dim3((unsigned)a.B), dim3(64), 0, a.stream, a, p);
      if ((rc = check_launch("k3_nll"))) return rc;
    }
    prof_call_end(a.stream);
    return 0;
  };
  if (yev) {
    if (a.dtype == EKS_YEV32) return run(YevIn<float>{}, ic<0>{});
    return run(YevIn<double>{}, ic<0>{});
  }
  auto by_e = [&](auto tag) -> int {
    switch (a.E) {
      case 3: return run(tag, ic<3>{});
      case 4: return run(tag, ic<4>{});
      case 5: return run(tag, ic<5>{});
      default: return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth algo 3: E=%d not compiled in", a.E);
    }
  };
  return f32 ? by_e(float{}) : by_e(double{});
}

// The member loads address trajectory b as a 32-bit byte offset b * sb *
// sizeof(T) (plus the member / coordinate offset) from the step's base.  A
// batch whose offsets do not fit (members stored trajectory-major with > 4 GB
// between the first and last trajectory) runs as consecutive slices on the
// same stream and workspace: algo 3's results depend on T only, so the
// slices give the bits of the one-piece call.
template <int R, int N, int AI, int CI>
int launch_algo3(const SmoothArgs &a) {
  const bool yev = a.dtype == EKS_YEV32 || a.dtype == EKS_YEV64;
  const long long esz = a.dtype == EKS_F32 ? 4 : 8;
  const long long per = yev ? 0 : a.sb * esz;  // bytes between trajectories
  // the largest member / coordinate offset of a step (buffer soffset)
  const long long soff = yev ? 0 : ((a.E - 1) * a.se + (N - 1) * a.sj) * esz + esz;
  // (eks_debug_set(EKS_DBG_A3_SLICE_BYTES) lowers the 4 GB span: tests of the slicing)
  const long long span = g_a3_slice_bytes > 0 && g_a3_slice_bytes < (1LL << 32) ? g_a3_slice_bytes
                                                                               : (1LL << 32);
  const long long lim = span - soff;
  if (per <= 0 || (a.B - 1) * per < lim) return launch_algo3_one<R, N, AI, CI>(a);
  const long long cap = std::max(1LL, lim / per);  // trajectories per slice
  if (lim <= 0)
    return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth algo 3: member strides beyond 4 GB per step");
  for (long long b0 = 0; b0 < a.B; b0 += cap) {
    SmoothArgs s = a;
    s.B = std::min(cap, a.B - b0);
    s.obs = (const char *)a.obs + b0 * per;
    s.params = a.params + b0 * ParamLayout<R, N>::len;
    s.out = a.out + b0 * a.ob;
    s.ms = a.ms ? a.ms + b0 * a.T * R : nullptr;
    s.nll = a.nll ? a.nll + b0 : nullptr;
    s.status = a.status + b0;
    if (const int rc = launch_algo3_one<R, N, AI, CI>(s)) return rc;
  }
  return 0;
}

