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
//                  time-major; builds the chunk's filtering element (stored
//                  trajectory-major, one row per (b, c), for the scans)
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
#include <cmath>
#include <cstdlib>

#include "../../include/eks_hip.h"
#include "eks_common.hpp"
#include "ensemble.hpp"
#include "handoff.hpp"
#include "kf_steps.hpp"
#include "small_linalg.hpp"
#include "tuning.hpp"

namespace eks {


// debug / fault-injection settings (eks_debug_set; defined in eks_smooth_api.hip)
extern long long g_wait_ticks;      // chain wait bound (wall_clock64 ticks), < 0: forced timeouts
extern long long g_a3_slice_bytes;  // algo-3 member offset span per slice (0: 4 GB)
extern long long g_a3_mode;         // retired key EKS_DBG_A3_MODE (round 5: one launch form)
extern long long g_rt_form;         // runtime-n smoother form (eks_shape_rt.hip rt_chunked)
extern long long g_a3_lb;           // k3_bwd look-back instantiation (two_pass.hpp a3_bwd_lookback)

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
  // time-sharded smoothing (eks_smooth_seg): this call covers global frames
  // [t_base, t_base + T) of trajectories T_total long; phase 0 = whole
  // pipeline, 1 / 2 / 3 = the three per-segment phases
  long long t_base = 0, T_total = 0;
  int phase = 0;
  const double *seg_in = nullptr;
  double *seg_out = nullptr;
  // bound of every in-launch chain wait, in wall_clock64 ticks (handoff.hpp)
  long long wait_ticks = kDefaultWaitTicks;
};

// Target number of (chunk, trajectory) lanes: enough 256-thread blocks that
// the last partial round of resident blocks (the tail) is a small fraction of
// the kernel.  EKS_TARGET_LANES overrides it (tuning experiments).
constexpr long long kTargetLanesDefault = 256LL * 16 * 64;
constexpr long long kMinChunk = 16;

// above this many chunks per trajectory the chunk scans run one wave per
// trajectory (EKS_WAVE_SCAN_CHUNKS overrides it: tuning and tests)
inline long long wave_scan_chunks() {
  static long long v = [] {
    const char *e = getenv("EKS_WAVE_SCAN_CHUNKS");
    return e ? atoll(e) : 24LL;
  }();
  return v;
}

// waves per trajectory of the parallel chunk scans: enough that each thread
// composes at most ~4 chunks before the in-wave scan
inline int scan_waves(long long NC) {
  static const int forced = [] {  // EKS_SCAN_WAVES: tuning / tests
    const char *e = getenv("EKS_SCAN_WAVES");
    return e ? atoi(e) : 0;
  }();
  if (forced == 1 || forced == 4 || forced == 8) return forced;
  // 4 waves (one per SIMD) beat 8 at configs 2 / 3 / 5 (NC = 3 125 / 1 563 /
  // 17 858: 0.147 / 0.301 / 2.92 -> 0.142 / 0.295 / 2.88 ms per step,
  // tools/scan_waves_sweep.sh): the waves of one trajectory's block share the
  // FP64 pipes of one CU, and W = 4 halves the serial cross-wave LDS prefix
  return NC > 256 ? 4 : 1;
}

inline long long target_lanes() {
  static long long v = [] {
    const char *e = getenv("EKS_TARGET_LANES");
    long long x = e ? atoll(e) : 0;
    return x > 0 ? x : kTargetLanesDefault;
  }();
  return v;
}

// checkpoint interval LS of K3/K5 (steps): K5 keeps LS steps of (J_t, d_t)
// in registers, so it shrinks as the state / observation grow.
constexpr int sub_len_c(int r, int n) { return (r <= 2 && n <= 2) ? 8 : (n <= 4 ? 4 : 2); }
inline int sub_len(int r, int n) { return sub_len_c(r, n); }
inline int elem_len(int r) { return r * r + r + r * (r + 1) / 2 + r + r * (r + 1) / 2; }
inline int state_len(int r) { return r + r * (r + 1) / 2; }

inline long long round_up(long long x, long long m) { return (x + m - 1) / m * m; }

inline bool uniform_lanes(long long B);

// Chunk length L.
// Many trajectories (whole blocks per chunk): short enough that B * NC lanes
// fill the GPU (L_fill), long enough that the chunk scans stay short
// (L_scan = sqrt(2 T / 64)).
// Few trajectories (chunk-major lanes): the per-step FP64 work of K1 / K3 /
// K5 keeps a SIMD busy with one wave (a second wave per SIMD buys ~nothing:
// config 2 at L = 16 vs 32), so L is as long as still gives every SIMD a
// wave: L_fill = B T / (1024 SIMDs x 64 lanes), at least kMinChunk; and at
// most the length that balances the per-lane chunk work against the chunk
// scans' compositions, L_scan = sqrt(2 T rho / 512), rho = composition /
// step cost ratio (2.6 for r <= 2, 0.8 for r = 3).  Config 5's B = 1 smooth
// of 1M frames: L 56 -> 16, its K3 + K5 0.49 -> 0.20 ms.
inline long long chunk_len(long long B, long long T, int r) {
  const long long ls = 8;  // a multiple of every checkpoint interval
  static const long long forced = [] {  // EKS_CHUNK_LEN: tuning experiments only
    const char *e = getenv("EKS_CHUNK_LEN");
    return e ? atoll(e) : 0LL;
  }();
  if (forced > 0) return std::min(round_up(forced, ls), round_up(T, ls));
  long long L;
  if (uniform_lanes(B)) {
    const long long nc = std::max(1LL, (target_lanes() + B - 1) / B);
    const long long l_fill = (T + nc - 1) / nc;
    const long long l_scan = (long long)std::ceil(std::sqrt(2.0 * (double)T / 64.0));
    L = std::max(kMinChunk, std::max(l_fill, l_scan));
  } else {
    const double rho = r <= 2 ? 2.6 : 0.8;
    const long long l_scan = std::llround(std::sqrt(2.0 * (double)T * rho / 512.0));
    const long long l_fill = (B * T + 65535) / 65536;
    L = std::max(kMinChunk, std::min(l_fill, l_scan));
  }
  L = round_up(L, ls);
  if (L >= T) L = round_up(T, ls);
  return L;
}

// (J, d) mode shapes (see ChunkPlan::jd)
inline bool jd_shape(long long B, int r, int n) {
  static const int off = [] {  // EKS_NO_JD: tuning experiments only
    const char *e = getenv("EKS_NO_JD");
    return e ? atoi(e) : 0;
  }();
  // B >= 8: the (J, d) planes are time-major (B values per row); with fewer
  // trajectories a wave's loads scatter over 64 rows (config 5's B = 1
  // smooth: K3 + K5 0.20 -> 0.24 ms with them)
  return !off && !uniform_lanes(B) && B >= 8 && B <= 256 && r >= 3 && n >= 4;
}

// Chunk length of a smoothing call: with few trajectories (B <= 256,
// chunk-major lanes) the group-mode scans cost ~the same for any chunk
// count, so the chunks are as short as the checkpoint grid allows
// (kMinChunk): more waves per SIMD for K1 / K3 / K5 (config 2: L 32 -> 16,
// 0.114 -> 0.104 ms per step).  Filter-only calls keep chunk_len's choice.
inline long long chunk_len_smooth(long long B, long long T, int r) {
  const long long L = chunk_len(B, T, r);
  if (getenv("EKS_CHUNK_LEN") || uniform_lanes(B) || B > 256 || L >= T) return L;
  const long long Ls = std::min(L, kMinChunk);
  return (T + Ls - 1) / Ls > wave_scan_chunks() ? Ls : L;
}

struct ChunkPlan {
  long long L = 0, NC = 0, NSUB = 0;
  int LS = 8;
  int smooth = 1;  // 0: filter only (out == NULL): NLL, no backward pass
  // filter-only call of the whole pipeline: each chunk's NLL share is taken in
  // closed form from its element (K1 stores the element's likelihood
  // constant, K2 adds the start-state terms: elem_nll_share), so K3 does not
  // re-run the filter
  int nll_closed = 0;
  // ... and the wave-parallel K2 sums the shares itself (no K4 NLL launch)
  int nll_fused = 0;
  // members shared by all trajectories (batch stride 0, e.g. candidate models
  // of one trajectory): y / ev are stored once, as a single plane column
  long long yB = 0;
  EKS_DEV unsigned ylane(unsigned b) const { return yB == 1 ? 0u : b; }
  // single-column planes (yB = 1) read by waves whose lanes all lie in one
  // chunk (UNI, or B a multiple of 64): K1 loads them with scalar loads
  int ywave = 0;
  size_t y_off = 0, ev_off = 0, elem_off = 0, cstart_off = 0, bwd_off = 0, nllp_off = 0,
         msend_off = 0, ckpt_off = 0, total = 0;
  // chained chunk scans (k_c2_fscan_g / k_c4_bscan_g): G blocks per
  // trajectory, block g owning chunks [g CPB, (g+1) CPB); their sync words
  // (two tickets, then per-(trajectory, block) flags: K2 totals, K2 NLL
  // partials, K4 totals) are zeroed by K1 (or a memset) every call
  int G = 1;
  long long CPB = 0;
  size_t sync_off = 0, sync_bytes = 0, agg_off = 0, magg_off = 0, part_off = 0;
  EKS_DEV unsigned *sync(char *ws) const { return (unsigned *)(ws + sync_off); }
  int GF = 1;  // the flag arrays' stride (max of the chunk- and group-level G)
  EKS_DEV unsigned *flags(char *ws, int k, long long B) const {
    return sync(ws) + 64 + (size_t)k * (size_t)B * (size_t)GF;
  }
  // where K3 / K5 read y / ev: the workspace planes K1 wrote, or (EKS_YEV
  // input) the caller's planes
  const char *ysrc = nullptr, *evsrc = nullptr;
  // Group mode (few trajectories, chunk-major lanes, smoothing calls): a
  // *group* is the run of one trajectory's chunks inside one 256-lane block
  // of K1 / K3 / K5 (B <= 256: every block holds ~256 / B consecutive chunks
  // of every trajectory).  K1 scans its elements within the group (LDS) and
  // stores inclusive prefixes plus the group total; K2 scans only the NG
  // group totals per trajectory; K3 starts chunk c from its group's start
  // state composed with the prefix before c, scans its RTS maps within the
  // group right to left (suffixes, group totals, group NLL sums); K4 scans
  // the group totals; K5 applies its suffix to the mean entering the group
  // from the right.  The chained scans then see ~NC B / 256 groups instead
  // of NC chunks per trajectory.
  int grp = 0;
  long long NG = 0;   // K1 blocks = groups per trajectory (the last may lack some b)
  long long gnc = 0;  // in a K2 / K4 plan over groups: the chunk count (0 otherwise)
  int GG = 1;         // G of the group-level scans
  long long CPBG = 0;
  size_t gagg_off = 0, gst_off = 0, gmap_off = 0, gms_off = 0, gnll_off = 0;
  // (J, d) mode (few trajectories, heavy observation models: r = 3, n >= 4):
  // K3 stores every step's RTS gain (J_t, d_t) in time-major planes and K5
  // only runs the backward mean recursion from them, instead of re-running
  // the filter from checkpoints (config 3: n = 8 dense C)
  int jd = 0;
  size_t jd_off = 0;
  // groups of trajectory b in a plan over groups (the last block may not hold b)
  EKS_DEV long long count_of(long long b, long long B) const {
    return gnc ? ((gnc - 1) * B + b) / 256 + 1 : NC;
  }
};

inline size_t align256(size_t x) { return (x + 255) / 256 * 256; }

// force_jd: the (J, d) planes whatever jd_shape says (the runtime-n pipeline
// always runs K5 from them)
inline ChunkPlan make_plan(long long B, long long T, int r, int n, long long L,
                           bool force_jd = false) {
  ChunkPlan p;
  p.LS = sub_len(r, n);
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
  if (force_jd || jd_shape(B, r, n)) p.jd_off = take((size_t)T * (r * r + r) * Bz * 8);
  if (p.NC > wave_scan_chunks()) {
    // blocks per trajectory: few lanes in all -> ~1 chunk per thread (the
    // scan is latency bound); many -> q chunks per thread so the chip holds
    // ~2 blocks per CU (the Hillis-Steele trees cost ~6 compositions per
    // lane, the per-thread runs 1 per chunk: config 5's 64 x 17 858 chunks,
    // q = 2 / 4 / 8 / 16: K2 0.238 / 0.188 / 0.175 / 0.194 ms,
    // profiles/r05/ab9).  At most 64 blocks: their totals are combined by
    // one wave.
    static const long long qt_force = [] {  // EKS_SCAN_QT: tuning experiments only
      const char *e = getenv("EKS_SCAN_QT");
      return e ? atoll(e) : 0LL;
    }();
    auto blocks = [&](long long nc, int &G, long long &cpb) {
      const long long qt = qt_force > 0 ? qt_force
                                        : std::min<long long>(8, std::max<long long>(1, B * nc / (256LL * 256 * 2)));
      G = (int)std::min<long long>(64, std::max<long long>(1, (nc + 256 * qt - 1) / (256 * qt)));
      cpb = (nc + G - 1) / G;
    };
    blocks(p.NC, p.G, p.CPB);
    if (!uniform_lanes(B) && B <= 256) {  // group-mode planes (used by smoothing calls)
      p.NG = (p.NC * B + 255) / 256;
      blocks(p.NG, p.GG, p.CPBG);
      p.gagg_off = take(Bz * (size_t)p.NG * elem_len(r) * 8);
      p.gst_off = take((size_t)p.NG * state_len(r) * Bz * 8);
      p.gmap_off = take(Bz * (size_t)p.NG * (r * r + r) * 8);
      p.gms_off = take((size_t)p.NG * r * Bz * 8);
      p.gnll_off = take((size_t)p.NG * Bz * 8);
    }
    p.GF = std::max(p.G, p.GG);
    const size_t BG = Bz * (size_t)p.GF;
    p.sync_bytes = align256(256 + 3 * BG * 4);
    p.sync_off = take(p.sync_bytes);
    p.agg_off = take(BG * elem_len(r) * 8);
    p.magg_off = take(BG * (r * r + r) * 8);
    p.part_off = take(BG * 2 * 8);
  }
  p.total = off;
  return p;
}

inline size_t seq_workspace_bytes(long long B, long long T, int r) {
  return (size_t)B * (size_t)T * (size_t)state_len(r) * 8;
}

// parameter row stride; N = 0: the runtime-n kernels (eks_shape_rt.hip)
template <int R, int N>
EKS_DEV long long param_stride(int n) {
  return N > 0 ? (long long)ParamLayout<R, N>::len : (long long)R + 3LL * R * R + (long long)n * (R + 1);
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
  template <int AI, int CI>
  EKS_DEV bool valid() const {
    bool ok = true;
    if constexpr (AI == kAId) ok = ok && is_identity<R>(A);
    if constexpr (AI == kADiag) ok = ok && is_diagonal<R>(A) && is_diagonal<R>(Q);
    if constexpr (CI == kCId) ok = ok && is_identity_rect<N, R>(C);
    if constexpr (CI == kCPupil) ok = ok && is_pupil_c<N, R>(C);
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

// Input tag: instead of member predictions the caller hands over the
// ensemble output itself (y / ev planes written by eks_fit, EKS_YEV32/64),
// time-major [t*N + j][b]: y of type YT, then ev (f64) at yev_ev_offset.
template <typename YT>
struct YevIn {
  using y_type = YT;
};
template <typename T>
struct is_yev : std::false_type {};
template <typename YT>
struct is_yev<YevIn<YT>> : std::true_type {};
template <typename T>
struct yev_y {
  using type = T;
};
template <typename YT>
struct yev_y<YevIn<YT>> {
  using type = YT;
};


// ===========================================================================
// algo 1: one lane per trajectory, sequential in time
// ===========================================================================
template <int R, int N, int E, typename T, int AI, int CI>
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
  auto step = [&](long long t, double (&y)[N], const double (&rv)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) y[j] -= md.off[j];
    if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
    kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
    store_state<R>(ws + t * K * B + b, B, m, P);
  };
  if constexpr (is_yev<T>::value) {  // ensemble handed over as y / ev planes
    using YT = typename yev_y<T>::type;
    const YT *yb = (const YT *)a.obs;
    const double *eb =
        (const double *)((const char *)a.obs + yev_ev_offset(B, TT, N, sizeof(YT)));
    for (long long t = 0; t < TT; ++t) {
      double y[N], rv[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        y[j] = (double)yb[(t * N + j) * B + b];
        rv[j] = eb[(t * N + j) * B + b];
      }
      step(t, y, rv);
    }
  } else {
    const T *ob = (const T *)a.obs + b * a.sb;
    T cur[EE][N], nxt[EE][N];
    if constexpr (E > 0) load_step<E, N, T>(ob, a.se, a.sj, cur);
    for (long long t = 0; t < TT; ++t) {
      const T *pt = ob + t * a.st;
      if constexpr (E > 0) {
        if (t + 1 < TT) load_step<E, N, T>(pt + a.st, a.se, a.sj, nxt);
      }
      double y[N], rv[N];
      reduce_step<E, N, T>(cur, pt, a.se, a.sj, a.E, median, y, rv);
      step(t, y, rv);
      if constexpr (E > 0) {
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int j = 0; j < N; ++j) cur[e][j] = nxt[e][j];
      }
    }
  }
  if (a.nll) a.nll[b] = acc.value((double)TT * N);
  if (!a.out) {  // filter only
    if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
    return;
  }
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
// Lane mapping: a 256-thread block covers 256 consecutive trajectories of ONE
// chunk, so the chunk index (and with it every time index and plane offset)
// is wave-uniform and lives in SGPRs; the only per-lane address term is the
// 32-bit trajectory index b (global_load saddr + voffset).
constexpr int kBlock = 256;

inline long long blocks_per_chunk(long long B) { return (B + kBlock - 1) / kBlock; }

// UNI (many trajectories): every block lies in one chunk, so c is uniform.
// !UNI (few trajectories, B << 256): lanes are (chunk, trajectory) pairs in
// chunk-major order, so one wave spans several chunks and no lane idles.
template <bool UNI>
struct Lane {
  long long c;
  unsigned b;
  EKS_DEV bool init(long long B, long long NC) {
    if constexpr (UNI) {
      const long long bpc = (B + kBlock - 1) / kBlock;
      c = blockIdx.x / bpc;
      b = (unsigned)((blockIdx.x - c * bpc) * kBlock + threadIdx.x);
      return c < NC && (long long)b < B;
    } else {
      const long long lane = blockIdx.x * (long long)kBlock + threadIdx.x;
      if (lane >= NC * B) return false;
      c = lane / B;
      b = (unsigned)(lane - c * B);
      return true;
    }
  }
};

inline bool uniform_lanes(long long B) {
  const long long cap = blocks_per_chunk(B) * kBlock;
  return (cap - B) * 8 <= cap;  // at most 1/8 of the lanes idle
}

// element `plane` of a time-major plane array (B values per plane): uniform
// 64-bit plane base + 32-bit per-lane byte offset, which hipcc lowers to the
// global_load/store saddr + voffset form (no per-lane 64-bit address math).
template <typename T>
EKS_DEV T &pl(T *base, long long plane, long long B, unsigned b) {
  char *pb = (char *)(base + plane * B);
  const unsigned off = b * (unsigned)sizeof(T);
  return *(T *)(pb + off);
}

template <int R>
EKS_DEV void store_state_pl(double *base, long long plane0, long long B, unsigned b,
                            const double (&m)[R], const double (&P)[R][R]) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) pl(base, plane0 + (k++), B, b) = m[i];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = i; j < R; ++j) pl(base, plane0 + (k++), B, b) = P[i][j];
}

template <int R>
EKS_DEV void load_state_pl(const double *base, long long plane0, long long B, unsigned b,
                           double (&m)[R], double (&P)[R][R]) {
  int k = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) m[i] = pl(base, plane0 + (k++), B, b);
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = i; j < R; ++j) P[i][j] = P[j][i] = pl(base, plane0 + (k++), B, b);
}

// Per-trajectory model in plane form (ParamLayout field k of trajectory b in
// plane k): the streaming passes of algo 3 load the model once per
// (chunk, trajectory) lane, and the caller's row layout (param_len doubles
// per trajectory, 160 B at r = n = 2) makes every lane touch two cache lines
// of which it uses a few fields -- at config 4 about 5 B per keypoint-timestep
// re-fetched from HBM once the streaming data has evicted them from L2.  In
// planes a wave's load of one field is one 512-byte segment, and a structure
// the kernel is compiled for (A = I, C = I) is not read at all: k_model_planes
// checks it once per trajectory instead.
template <int R, int N, int AI, int CI>
EKS_DEV void load_model_pl(const double *base, long long B, unsigned b, bool with_prior,
                           Model<R, N> &md) {
  using L = ParamLayout<R, N>;
  if (with_prior) {
#pragma unroll
    for (int i = 0; i < R; ++i) md.m0[i] = pl(base, L::m0 + i, B, b);
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) md.S0[i][j] = pl(base, L::S0 + i * R + j, B, b);
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      md.A[i][j] = AI == kAId ? (i == j ? 1.0 : 0.0) : pl(base, L::A + i * R + j, B, b);
      md.Q[i][j] = pl(base, L::Q + i * R + j, B, b);
    }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j)
      md.C[i][j] = CI == kCId ? (i == j ? 1.0 : 0.0) : pl(base, L::C + i * R + j, B, b);
#pragma unroll
  for (int i = 0; i < N; ++i) md.off[i] = pl(base, L::off + i, B, b);
}

// one thread per trajectory: params rows -> planes, model structure check;
// and the call's chain sync block (tickets, flags: `zw` 16-byte words) zeroed
// on the way, so a graph step has no memset node in front of the passes
template <int R, int N, int AI, int CI>
__global__ __launch_bounds__(256) void k_model_planes(const double *params, long long B,
                                                      double *planes, int32_t *status,
                                                      uint4 *zero, long long zw) {
  using L = ParamLayout<R, N>;
  const long long b = (long long)blockIdx.x * 256 + threadIdx.x;
  for (long long i = b; i < zw; i += (long long)gridDim.x * 256) zero[i] = make_uint4(0u, 0u, 0u, 0u);
  if (b >= B) return;
  const double *pp = params + b * L::len;
#pragma unroll
  for (int k = 0; k < L::len; ++k) planes[(long long)k * B + b] = pp[k];
  Model<R, N> md;
  md.load(pp, false);
  if (!md.template valid<AI, CI>()) flag(status, b, EKS_STATUS_BAD_MODEL);
}

// Stream the chunk's member predictions once: ensemble each step, store the
// raw average and the variance for K3/K5, and feed the step to `absorb`
// (the plain filter for chunk 0, the element build otherwise).
template <int E, int N, typename T, typename YT, int D, typename Absorb>
EKS_DEV void c1_stream(const SmoothArgs &a, const ChunkPlan &p, long long s, long long e,
                       unsigned b, const double (&off)[N], Absorb &&absorb) {
  const long long B = a.B;
  if constexpr (is_yev<T>::value) {
    // the ensemble is already in the caller's planes: stream y / ev
    // ring loads are unconditional (step index clamped to the chunk's last:
    // a cache-hit re-read), so they stay in flight: a load under a
    // lane-divergent `if` is merged into its slot by a copy that waits for it
    constexpr int DY = 2;
    if (p.ywave) {
      // every lane of the wave reads the same step of the single-column
      // planes (members shared by all trajectories, e.g. the pupil sweep's
      // candidate models): scalar loads into SGPRs through the constant
      // address space, so the ring costs no VGPRs (K1 of the sweep is bound
      // by its FP64 chains at the waves per SIMD its VGPRs allow)
      using CY = const __attribute__((address_space(4))) YT;
      using CE = const __attribute__((address_space(4))) double;
      CY *yp = (CY *)p.ysrc;
      CE *ep = (CE *)p.evsrc;
      const int su = __builtin_amdgcn_readfirstlane((int)s);
      const int eu = __builtin_amdgcn_readfirstlane((int)e);
      YT ys[DY][N];
      double es[DY][N];
      auto sfetch = [&](int q, int t) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          ys[q][j] = yp[t * N + j];
          es[q][j] = ep[t * N + j];
        }
      };
#pragma unroll
      for (int q = 0; q < DY; ++q) sfetch(q, min(su + q, eu - 1));
      for (int t0 = su; t0 < eu; t0 += DY) {
#pragma unroll
        for (int q = 0; q < DY; ++q) {
          const int t = t0 + q;
          double y[N], rv[N];
#pragma unroll
          for (int j = 0; j < N; ++j) {
            y[j] = (double)ys[q][j] - off[j];
            rv[j] = es[q][j];
          }
          sfetch(q, min(t + DY, eu - 1));
          if (t < eu) absorb((long long)t, y, rv);
        }
      }
      return;
    }
    YT yr[DY][N];
    double er[DY][N];
    auto fetch = [&](int q, long long t) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        yr[q][j] = pl((const YT *)p.ysrc, t * N + j, p.yB, p.ylane(b));
        er[q][j] = pl((const double *)p.evsrc, t * N + j, p.yB, p.ylane(b));
      }
    };
#pragma unroll
    for (int q = 0; q < DY; ++q) fetch(q, min(s + q, e - 1));
    for (long long t0 = s; t0 < e; t0 += DY) {
#pragma unroll
      for (int q = 0; q < DY; ++q) {
        const long long t = t0 + q;
        double y[N], rv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
          y[j] = (double)yr[q][j] - off[j];
          rv[j] = er[q][j];
        }
        fetch(q, min(t + DY, e - 1));
        if (t < e) absorb(t, y, rv);
      }
    }
    return;
  } else {
  constexpr int EE = E > 0 ? E : 1;
  const bool median = a.median != 0;
  YT *ybuf = (YT *)(a.ws + p.y_off);
  double *evbuf = (double *)(a.ws + p.ev_off);
  const T *ob = (const T *)a.obs + (long long)b * a.sb;
  T ring[D][EE][N];
  if constexpr (E > 0) {  // unconditional clamped ring loads, as above
#pragma unroll
    for (int q = 0; q < D; ++q) load_step<E, N, T>(ob + min(s + q, e - 1) * a.st, a.se, a.sj, ring[q]);
  }
  for (long long t0 = s; t0 < e; t0 += D) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const long long t = t0 + q;
      T cur[EE][N];
      if constexpr (E > 0) {
#pragma unroll
        for (int u = 0; u < E; ++u)
#pragma unroll
          for (int j = 0; j < N; ++j) cur[u][j] = ring[q][u][j];
        load_step<E, N, T>(ob + min(t + D, e - 1) * a.st, a.se, a.sj, ring[q]);
      }
      if (t < e) {
        const T *pt = ob + t * a.st;
        double avg[N], rv[N], y[N];
        reduce_step<E, N, T>(cur, pt, a.se, a.sj, a.E, median, avg, rv);
#pragma unroll
        for (int j = 0; j < N; ++j) {
          if (p.yB != 1 || b == 0) {
            pl(ybuf, t * N + j, p.yB, p.ylane(b)) = (YT)avg[j];
            pl(evbuf, t * N + j, p.yB, p.ylane(b)) = rv[j];
          }
          y[j] = avg[j] - off[j];
        }
        absorb(t, y, rv);
      }
    }
  }
  }
}

// Members shared by every trajectory (batch stride 0: candidate models of one
// recording, the pupil NLL sweep): the ensemble of each step is computed ONCE
// here, one lane per step, into the single-column y / ev planes (yB = 1) that
// K1 (as YevIn input), K3 and K5 then read for every trajectory, instead of
// every (chunk, trajectory) lane re-reducing the same members.
template <int E, int N, typename T, typename YT>
__global__ __launch_bounds__(kBlock) void k_c0_shared(SmoothArgs a, ChunkPlan p) {
  const long long t = blockIdx.x * (long long)kBlock + threadIdx.x;
  constexpr int EE = E > 0 ? E : 1;
  const T *pt = (const T *)a.obs + t * a.st;
  T cur[EE][N];
  // a step's E x N members contiguous and 16-byte aligned (the pupil sweep's
  // (T, E, 8) float32 layout): 16-byte loads, a quarter of the requests
  constexpr bool kVec = E > 0 && (E * N) % 4 == 0 && std::is_same<T, float>::value;
  constexpr int Q = kVec ? EE * N / 4 : 1;  // 16-byte words per step
  const bool vec = kVec && a.sj == 1 && a.se == N && (((uintptr_t)a.obs | (uintptr_t)(a.st * 4)) & 15) == 0;
  // consecutive steps contiguous too: the block's 256 steps are one run of
  // 256 Q words, loaded word-per-lane (every wave instruction one contiguous
  // 1 KB) and handed to the step lanes through LDS -- a lane reading its own
  // step's Q words directly puts 64 lanes 16 Q bytes apart on every load
  // (config 5: 160 MB of members at ~1.7 TB/s)
  __shared__ float4 stage[kVec ? kBlock * Q : 1];
  const bool staged = vec && a.st == (long long)E * N;
  if constexpr (kVec) {
    if (staged) {
      const long long tb = blockIdx.x * (long long)kBlock;
      const int nq = (int)(min((long long)kBlock, a.T - tb) * Q);
      const float4 *src = reinterpret_cast<const float4 *>((const float *)a.obs + tb * a.st);
      float4 r[Q];
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        const int i = threadIdx.x + k * kBlock;
        r[k] = i < nq ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < Q; ++k) stage[threadIdx.x + k * kBlock] = r[k];
      __syncthreads();
    }
  }
  if (t >= a.T) return;
  if constexpr (kVec) {
    if (vec) {
      float4 q[EE * N / 4];
      if (staged) {
#pragma unroll
        for (int k = 0; k < EE * N / 4; ++k) q[k] = stage[threadIdx.x * Q + k];
      } else {
#pragma unroll
        for (int k = 0; k < EE * N / 4; ++k) q[k] = reinterpret_cast<const float4 *>(pt)[k];
      }
#pragma unroll
      for (int k = 0; k < EE * N / 4; ++k) {
        const float w[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[(4 * k + u) / N][(4 * k + u) % N] = w[u];
      }
    } else {
      load_step<E, N, T>(pt, a.se, a.sj, cur);
    }
  } else if constexpr (E > 0) {
    load_step<E, N, T>(pt, a.se, a.sj, cur);
  }
  double avg[N], rv[N];
  reduce_step<E, N, T>(cur, pt, a.se, a.sj, a.E, a.median != 0, avg, rv);
  YT *ybuf = (YT *)(a.ws + p.y_off);
  double *evbuf = (double *)(a.ws + p.ev_off);
  if constexpr (N % 4 == 0 && std::is_same<YT, float>::value) {  // 16-byte stores
#pragma unroll
    for (int j = 0; j < N; j += 4)
      *reinterpret_cast<float4 *>(ybuf + t * N + j) =
          make_float4((float)avg[j], (float)avg[j + 1], (float)avg[j + 2], (float)avg[j + 3]);
#pragma unroll
    for (int j = 0; j < N; j += 2)
      *reinterpret_cast<double2 *>(evbuf + t * N + j) = make_double2(rv[j], rv[j + 1]);
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      ybuf[t * N + j] = (YT)avg[j];
      evbuf[t * N + j] = rv[j];
    }
  }
}

// K1 for chunk c of trajectory b
template <int R, int N, int E, typename T, typename YT, int AI, int CI, bool UNI>
EKS_DEV void c1_chunk(const SmoothArgs &a, const ChunkPlan &p, long long c, unsigned b,
                      Elem<R> &El) {
  // member prefetch distance (steps); few-trajectory lanes (!UNI: < 1 wave per
  // SIMD, nothing else to hide the HBM latency behind) keep more in flight
  constexpr int D = (E > 0 && E * N <= 16) ? (UNI ? 2 : kC1Dnu) : 1;
  const long long B = a.B, TT = a.T;
  Model<R, N> md;
  const bool first = c == 0 && a.t_base == 0;  // the globally first chunk starts at the prior
  md.load(a.params + (long long)b * ParamLayout<R, N>::len, first);
  const long long s = c * p.L, e = min(TT, s + p.L);
  bool ok = true;
  if (c == 0 && !md.template valid<AI, CI>()) flag(a.status, b, EKS_STATUS_BAD_MODEL);
  if (first) {
    // chunk 0: the plain filter from the prior; summarised as the known
    // filtered state (Ab = 0, bb = m, Cb = P, no likelihood terms)
    double m[R], P[R][R];
    NllAcc acc;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = md.m0[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = md.S0[i][j];
    }
    c1_stream<E, N, T, YT, D>(a, p, s, e, b, md.off, [&](long long t, const double (&y)[N],
                                                          const double (&rv)[N]) {
      if (t > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
      kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
    });
    if (p.nll_closed) pl((double *)(a.ws + p.nllp_off), c, B, b) = acc.value((double)(e - s) * N);
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
  } else {
    El.set_identity();
    NllAcc acc;
    c1_stream<E, N, T, YT, D>(a, p, s, e, b, md.off, [&](long long, const double (&y)[N],
                                                          const double (&rv)[N]) {
      elem_absorb<R, N, AI, CI>(El, md.A, md.Q, md.C, y, rv, ok, &acc);
    });
    if (p.nll_closed) pl((double *)(a.ws + p.nllp_off), c, B, b) = acc.value((double)(e - s) * N);
  }
  if (!ok) flag(a.status, b, first ? EKS_STATUS_SINGULAR : EKS_STATUS_SCAN);
}

// zero the chained scans' sync words for K2 / K4 of this call (block 0 of K1:
// stream order makes them visible to the scans without a memset launch)
EKS_DEV void zero_scan_sync(const SmoothArgs &a, const ChunkPlan &p) {
  if (blockIdx.x != 0 || p.sync_bytes == 0) return;
  unsigned *z = p.sync(a.ws);
  for (size_t i = threadIdx.x; i < p.sync_bytes / 4; i += blockDim.x) z[i] = 0u;
}

template <int R, int N, int E, typename T, typename YT, int AI, int CI, bool UNI>
EKS_DEV void c1_elem_body(const SmoothArgs &a, const ChunkPlan &p) {
  zero_scan_sync(a, p);
  Lane<UNI> ln;
  const bool valid = ln.init(a.B, p.NC);
  double *eplane = (double *)(a.ws + p.elem_off);
  constexpr int EL = Elem<R>::len;
  if constexpr (UNI) {
    if (!valid) return;
    Elem<R> El;
    c1_chunk<R, N, E, T, YT, AI, CI, UNI>(a, p, ln.c, ln.b, El);
    El.store(eplane + ((long long)ln.b * p.NC + ln.c) * EL, 1);
  } else {
    Elem<R> El;
    if (valid)
      c1_chunk<R, N, E, T, YT, AI, CI, UNI>(a, p, ln.c, ln.b, El);
    else
      El.set_identity();
    if (p.grp) {
      // group mode: inclusive scan over this trajectory's chunks in the block
      // (lanes B apart), Hillis-Steele through LDS (dynamic: EL x 256 doubles)
      extern __shared__ double dsh[];
      const int tid = threadIdx.x, Bi = (int)a.B;
      bool ok = true;
      for (int k = 1; k * Bi < kBlock; k <<= 1) {
        El.store(dsh + tid, kBlock);
        __syncthreads();
        const int j = tid - k * Bi;
        Elem<R> o;
        if (j >= 0) o.load(dsh + j, kBlock);
        __syncthreads();
        if (j >= 0 && valid) {
          Elem<R> t;
          ok = compose_elem<R>(o, El, t) && ok;
          El = t;
        }
      }
      if (valid) {
        if (!ok) flag(a.status, ln.b, EKS_STATUS_SCAN);
        if (tid + Bi >= kBlock || ln.c + 1 == p.NC)  // the group's last chunk: the group total
          El.store((double *)(a.ws + p.gagg_off) + ((long long)ln.b * p.NG + blockIdx.x) * EL, 1);
      }
    }
    if (valid) El.store(eplane + ((long long)ln.b * p.NC + ln.c) * EL, 1);
  }
}

template <int R, int N, int E, typename T, typename YT, int AI, int CI, bool UNI>
__global__ __launch_bounds__(kBlock) void k_c1_elem(SmoothArgs a, ChunkPlan p) {
  c1_elem_body<R, N, E, T, YT, AI, CI, UNI>(a, p);
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
  Elem<R> El, Nx;
  // elements are stored trajectory-major: row (b, c) of Elem<R>::len doubles
  const double *erow = elem + b * p.NC * Elem<R>::len;
  bool ok = true;
  if (a.t_base == 0) {
    using L = ParamLayout<R, N>;
    const double *pp = a.params + b * param_stride<R, N>(a.n);
    load_vec<R>(pp + L::m0, m);
    load_mat<R, R>(pp + L::S0, P);
    store_state<R>(cst + b, B, m, P);  // chunk 0 starts from the prior
    El.load(erow, 1);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = El.bb[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = El.Cb[i][j];
    }
  } else {
    // a later time segment: chunk 0 starts from the filtered state handed
    // over by the earlier segments, and its element is a regular one
    load_state<R>(a.seg_in + b * (R + Sym<R>::len), 1, m, P);
    store_state<R>(cst + b, B, m, P);
    El.load(erow, 1);
    ok = compose_state<R>(m, P, El) && ok;
  }
  // software pipelined: the element of chunk c+1 is in flight while chunk c
  // is composed (the chain is latency bound, not bandwidth bound)
  double *np_ = (double *)(a.ws + p.nllp_off);
  const bool nllc = p.nll_closed && a.t_base == 0;
  if (p.NC > 1) El.load(erow + Elem<R>::len, 1);
  for (long long c = 1; c < p.NC; ++c) {
    store_state<R>(cst + (c * KS) * B + b, B, m, P);
    if (c + 1 < p.NC && (nllc || c + 2 < p.NC)) Nx.load(erow + (c + 1) * Elem<R>::len, 1);
    if (nllc) np_[c * B + b] = elem_nll_share<R>(m, P, El, np_[c * B + b], ok);
    if (c + 1 < p.NC) {
      ok = compose_state<R>(m, P, El) && ok;
      El = Nx;
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SCAN);
}

// Per-thread runs of the parallel chunk scans: PD element / map loads in
// flight while one is composed.  The chain is bound by the latency of these
// loads (K1's / K3's rows live in other XCDs' L2s or HBM, ~1-2 us), not by the
// compositions, so a depth-1 prefetch pays one load latency per chunk.  Ring
// loads are unconditional (index clamped into the run: a cache-hit re-read at
// the tail), so the compiler cannot merge a divergent load into its slot with
// a copy that waits for it.
template <int R>
constexpr int scan_pd() { return R <= 2 ? kScanPd : 1; }  // r = 3: 27-double elements, 2 would spill at 512 threads

// fn(c, element c) for c = c0 .. c1-1 in order; rows of Elem<R>::len doubles
template <int R, typename F>
EKS_DEV void elem_run(const double *rows, long long c0, long long c1, F &&fn) {
  constexpr int PD = scan_pd<R>();
  if (c0 >= c1) return;
  Elem<R> ring[PD];
#pragma unroll
  for (int k = 0; k < PD; ++k) ring[k].load(rows + min(c0 + k, c1 - 1) * Elem<R>::len, 1);
  for (long long c = c0; c < c1; c += PD) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const Elem<R> e = ring[k];
      ring[k].load(rows + min(c + k + PD, c1 - 1) * Elem<R>::len, 1);
      if (c + k < c1) fn(c + k, e);
    }
  }
}

// whole elements through the hand-off primitives (handoff.hpp)
template <int R>
EKS_DEV void elem_store_wt(const Elem<R> &E, double *p) {
  double v[Elem<R>::len];
  E.store(v, 1);
#pragma unroll
  for (int k = 0; k < Elem<R>::len; ++k) st_wt(p + k, v[k]);
}
template <int R>
EKS_DEV void elem_load_wt(Elem<R> &E, const double *p) {
  double v[Elem<R>::len];
#pragma unroll
  for (int k = 0; k < Elem<R>::len; ++k) v[k] = ld_wt(p + k);
  E.load(v, 1);
}

// K2, chained form (many chunks per trajectory): G blocks of 4 waves per
// trajectory, taken from a ticket counter so that the blocks of trajectory
// b hold consecutive tickets and a block only ever waits for blocks with
// smaller tickets (already running or done: every wait ends).
//  1. thread tid of block g owns chunks [c0, c1) (q = CPB / 256, ~1): it
//     composes their elements; each wave scans its 64 aggregates
//     (Hillis-Steele, 6 compositions); the wave totals are combined in LDS;
//     the block total is published (write-through stores + flag);
//  2. wave 0 gathers the totals of blocks 0..g-1 (one per lane) and scans
//     them with the same Hillis-Steele tree: lane g-1 holds the block's
//     exclusive prefix;
//  3. each thread walks its chunks from its exclusive prefix, writing the
//     chunk start states (and, filter-only calls, the closed-form NLL
//     shares; fused: per-block sums, added in block order by block G-1).
// The association order of every composition depends on (NC, G) alone, so
// results are deterministic.  Latency: ~2q + 6 + 3 + 6 compositions and two
// hand-offs whatever NC (the single-block form was ~2 NC / 256 chunk loads
// in sequence: config 2's K2 31.8 us).
template <int R, int N>
__global__ __launch_bounds__(256) void k_c2_fscan_g(SmoothArgs a, ChunkPlan p) {
  constexpr int W = 4, EL = Elem<R>::len, KS = R + Sym<R>::len;
  __shared__ double tot[W][EL];
  __shared__ double bpre[EL];
  __shared__ double ns[W];
  __shared__ unsigned tk;
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned *sync = p.sync(a.ws);
  if (tid == 0) tk = atomicAdd(sync, 1u);
  __syncthreads();
  const long long B = a.B, NC = p.NC;
  const int G = p.G;
  const unsigned t = __builtin_amdgcn_readfirstlane(tk);
  const long long b = t / (unsigned)G;
  const int g = (int)(t - (unsigned)b * (unsigned)G);
  if (b >= B) return;
  const double *elem = (const double *)(a.ws + p.elem_off);
  const double *erow = elem + b * NC * EL;
  double *cst = (double *)(a.ws + p.cstart_off);
  unsigned *fl_tot = p.flags(a.ws, 0, B) + b * G, *fl_nll = p.flags(a.ws, 1, B) + b * G;
  double *aggs = (double *)(a.ws + p.agg_off) + b * G * EL;
  double *parts = (double *)(a.ws + p.part_off) + b * G;
  const long long NCb = p.count_of(b, B);  // NC, or this trajectory's group count
  const long long cb0 = min(NCb, (long long)g * p.CPB), cb1 = min(NCb, cb0 + p.CPB);
  const long long q = (p.CPB + 255) / 256;
  const long long c0 = min(cb1, cb0 + tid * q), c1 = min(cb1, c0 + q);
  bool ok = true;
  Elem<R> agg;
  agg.set_identity();
  elem_run<R>(erow, c0, c1, [&](long long c, const Elem<R> &e) {
    if (c == c0) {
      agg = e;
    } else {
      Elem<R> tt;
      ok = compose_elem<R>(agg, e, tt) && ok;
      agg = tt;
    }
  });
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const Elem<R> o = shfl_elem<R, true>(agg, k);
    if (l >= k) {
      Elem<R> tt;
      ok = compose_elem<R>(o, agg, tt) && ok;
      agg = tt;
    }
  }
  Elem<R> ex = shfl_elem<R, true>(agg, 1);
  if (l == 0) ex.set_identity();
  if (l == 63) agg.store(tot[w], 1);
  __syncthreads();
  Elem<R> pre;  // the totals of the block's earlier waves, in order
  if (w > 0) {
    pre.load(tot[0], 1);
    for (int v = 1; v < w; ++v) {
      Elem<R> tv, tt;
      tv.load(tot[v], 1);
      ok = compose_elem<R>(pre, tv, tt) && ok;
      pre = tt;
    }
    if (l == 0) {
      ex = pre;
    } else {
      Elem<R> tt;
      ok = compose_elem<R>(pre, ex, tt) && ok;
      ex = tt;
    }
  }
  if (w == W - 1 && g + 1 < G) {  // the block total, for the later blocks
    Elem<R> tv, bt;
    tv.load(tot[W - 1], 1);
    ok = compose_elem<R>(pre, tv, bt) && ok;
    if (l == 0) elem_store_wt<R>(bt, aggs + (long long)g * EL);
    publish_flag(fl_tot + g, l);
  }
  if (g > 0) {  // the totals of blocks 0..g-1
    if (w == 0) {
      Elem<R> e;
      e.set_identity();
      if (!wait_flag_lanes(fl_tot + l, l < g, a.wait_ticks)) ok = false;
      if (l < g) elem_load_wt<R>(e, aggs + (long long)l * EL);
      for (int k = 1; k < g; k <<= 1) {  // levels past g - 1 leave lanes < g alone
        const Elem<R> o = shfl_elem<R, true>(e, k);
        if (l >= k) {
          Elem<R> tt;
          ok = compose_elem<R>(o, e, tt) && ok;
          e = tt;
        }
      }
      if (l == g - 1) e.store(bpre, 1);
    }
    __syncthreads();
    Elem<R> bp;
    bp.load(bpre, 1);
    if (tid == 0) {
      ex = bp;
    } else {
      Elem<R> tt;
      ok = compose_elem<R>(bp, ex, tt) && ok;
      ex = tt;
    }
  }
  const bool first = g == 0 && tid == 0;  // owns chunk 0
  double nsum = 0.0;  // this thread's NLL shares (nll_fused)
  if (c0 < c1 && a.t_base > 0) {
    // a later time segment: every thread starts from the handed-over state
    // composed with the elements before its first chunk
    double m[R], P[R][R];
    load_state<R>(a.seg_in + b * KS, 1, m, P);
    if (!first) ok = compose_state<R>(m, P, ex) && ok;
    for (long long c = c0; c < c1; ++c) {
      store_state<R>(cst + (c * KS) * B + b, B, m, P);
      if (c + 1 < c1) {
        Elem<R> e;
        e.load(erow + c * EL, 1);
        ok = compose_state<R>(m, P, e) && ok;
      }
    }
  } else if (c0 < c1) {
    double m[R], P[R][R];
    long long c = c0;
    if (first) {
      using L = ParamLayout<R, N>;
      const double *pp = a.params + b * param_stride<R, N>(a.n);
      load_vec<R>(pp + L::m0, m);
      load_mat<R, R>(pp + L::S0, P);
      store_state<R>(cst + b, B, m, P);  // chunk 0 starts from the prior
      Elem<R> e0;
      e0.load(erow, 1);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        m[i] = e0.bb[i];
#pragma unroll
        for (int j = 0; j < R; ++j) P[i][j] = e0.Cb[i][j];
      }
      c = 1;
    } else {
      // chunk 0's element is the filtered state itself (Ab = 0), so the
      // prefix is the state entering c0
#pragma unroll
      for (int i = 0; i < R; ++i) {
        m[i] = ex.bb[i];
#pragma unroll
        for (int j = 0; j < R; ++j) P[i][j] = ex.Cb[i][j];
      }
    }
    double *np_ = (double *)(a.ws + p.nllp_off);
    const bool need = !p.nll_closed;  // the start states feed K3 / K5 (not a closed-form NLL call)
    elem_run<R>(erow, c, c1, [&](long long c, const Elem<R> &e) {
      if (need) store_state<R>(cst + (c * KS) * B + b, B, m, P);
      if (p.nll_closed) {
        const double sh = elem_nll_share<R>(m, P, e, np_[c * B + b], ok);
        if (p.nll_fused) nsum += sh;
        else np_[c * B + b] = sh;
      }
      if (c + 1 < c1) ok = compose_state<R>(m, P, e) && ok;
    });
    if (first && p.nll_fused) nsum += np_[b];  // chunk 0's share: the plain filter's (K1)
  }
  if (p.nll_fused) {  // per thread in chunk order, the block (fixed order), then the blocks in order
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) nsum += __shfl_xor(nsum, k, 64);
    if (l == 0) ns[w] = nsum;
    __syncthreads();
    double s = ns[0];
    for (int v = 1; v < W; ++v) s += ns[v];
    if (G == 1) {
      if (tid == 0) a.nll[b] = s;
    } else if (w == 0) {
      if (g + 1 < G) {
        if (l == 0) st_wt(parts + g, s);
        publish_flag(fl_nll + g, l);
      } else {  // the last block adds the partial sums in block order
        if (!wait_flag_lanes(fl_nll + l, l < g, a.wait_ticks)) ok = false;
        if (l == 0) {
          double tsum = 0.0;
          for (int v = 0; v < g; ++v) tsum += ld_wt(parts + v);
          a.nll[b] = tsum + s;
        }
      }
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SCAN);
}

template <int R>
struct Affine {
  double G[R][R], g[R];
  EKS_DEV void set_identity() {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      g[i] = 0.0;
#pragma unroll
      for (int j = 0; j < R; ++j) G[i][j] = (i == j) ? 1.0 : 0.0;
    }
  }
  // (this o h)(x) = G (Gh x + gh) + g
  EKS_DEV Affine after(const Affine &h) const {
    Affine o;
    matmul<R, R, R>(G, h.G, o.G);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double t = g[i];
#pragma unroll
      for (int k = 0; k < R; ++k) t = fma(G[i][k], h.g[k], t);
      o.g[i] = t;
    }
    return o;
  }
  EKS_DEV Affine shfl_down(int delta) const {
    Affine o;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      o.g[i] = __shfl_down(g[i], delta, 64);
#pragma unroll
      for (int j = 0; j < R; ++j) o.G[i][j] = __shfl_down(G[i][j], delta, 64);
    }
    return o;
  }
};

template <int R>
EKS_DEV void map_store_wt(const Affine<R> &F, double *p) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    st_wt(p + R * R + i, F.g[i]);
#pragma unroll
    for (int j = 0; j < R; ++j) st_wt(p + i * R + j, F.G[i][j]);
  }
}
template <int R>
EKS_DEV void map_load_wt(Affine<R> &F, const double *p) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    F.g[i] = ld_wt(p + R * R + i);
#pragma unroll
    for (int j = 0; j < R; ++j) F.G[i][j] = ld_wt(p + i * R + j);
  }
}

// K4, chained form: chunk maps ms_start[c] = G_c ms_start[c+1] + g_c, G
// blocks of 4 waves per trajectory as in K2 but in reverse: the tickets of
// trajectory b go to its blocks g = G-1 .. 0, and a block waits only for the
// later blocks' totals.  Each thread composes its chunks' maps right to
// left, each wave suffix-scans its lanes, the wave totals are combined in
// LDS, the block total (and the block's NLL partial sum) is published; wave
// 0 then suffix-scans the totals of blocks g+1..G-1 and each thread walks
// its chunks from the smoothed mean entering its last one.  Block 0, which
// waits for every other block, adds the NLL partial sums in block order.
template <int R>
__global__ __launch_bounds__(256) void k_c4_bscan_g(SmoothArgs a, ChunkPlan p) {
  constexpr int W = 4, MR = R * R + R;
  __shared__ double tot[W][MR];
  __shared__ double bsuf[MR];
  __shared__ double nsum[W];
  __shared__ unsigned tk;
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned *sync = p.sync(a.ws);
  if (tid == 0) tk = atomicAdd(sync + 32, 1u);
  __syncthreads();
  const long long B = a.B, NC = p.NC;
  const int G = p.G;
  const unsigned t = __builtin_amdgcn_readfirstlane(tk);
  const long long b = t / (unsigned)G;
  const int g = G - 1 - (int)(t - (unsigned)b * (unsigned)G);
  if (b >= B) return;
  const double *bw = (const double *)(a.ws + p.bwd_off);
  double *msend = (double *)(a.ws + p.msend_off);
  unsigned *fl = p.flags(a.ws, 2, B) + b * G;
  double *maggs = (double *)(a.ws + p.magg_off) + b * G * MR;
  double *parts = (double *)(a.ws + p.part_off) + B * G + b * G;
  const long long NCb = p.count_of(b, B);  // NC, or this trajectory's group count
  const long long cb0 = min(NCb, (long long)g * p.CPB), cb1 = min(NCb, cb0 + p.CPB);
  const long long q = (p.CPB + 255) / 256;
  const long long c0 = min(cb1, cb0 + tid * q), c1 = min(cb1, c0 + q);
  auto load_map = [&](const double *s) {
    Affine<R> f;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      f.g[i] = s[R * R + i];
#pragma unroll
      for (int j = 0; j < R; ++j) f.G[i][j] = s[i * R + j];
    }
    return f;
  };
  auto map_of = [&](long long c) { return load_map(bw + (b * NC + c) * MR); };
  // fn(c, map c) for c = c1-1 down to c0, PD maps in flight (see elem_run)
  auto map_run = [&](auto &&fn) {
    constexpr int PD = 2 * scan_pd<R>();
    if (c0 >= c1) return;
    Affine<R> ring[PD];
#pragma unroll
    for (int k = 0; k < PD; ++k) ring[k] = map_of(max(c1 - 1 - k, c0));
    for (long long c = c1 - 1; c >= c0; c -= PD) {
#pragma unroll
      for (int k = 0; k < PD; ++k) {
        const Affine<R> f = ring[k];
        ring[k] = map_of(max(c - k - PD, c0));
        if (c - k >= c0) fn(c - k, f);
      }
    }
  };
  Affine<R> F;
  F.set_identity();
  map_run([&](long long, const Affine<R> &f) { F = f.after(F); });
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const Affine<R> o = F.shfl_down(k);
    if (l + k < 64) F = F.after(o);
  }
  Affine<R> X = F.shfl_down(1);
  if (l == 63) X.set_identity();
  double s = 0.0;  // NLL shares of this thread's chunks, then of the wave
  if (a.nll) {
    const double *np_ = (const double *)(a.ws + p.nllp_off);
    for (long long c = c0; c < c1; ++c) s += np_[c * B + b];
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) s += __shfl_xor(s, k, 64);
  }
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      tot[w][R * R + i] = F.g[i];
#pragma unroll
      for (int j = 0; j < R; ++j) tot[w][i * R + j] = F.G[i][j];
    }
    nsum[w] = s;
  }
  __syncthreads();
  Affine<R> S;  // the later waves' totals
  S.set_identity();
  if (w + 1 < W) {
    S = load_map(tot[W - 1]);
    for (int v = W - 2; v > w; --v) S = load_map(tot[v]).after(S);
    X = X.after(S);
  }
  double part = nsum[0];  // the block's NLL partial, waves in order
  for (int v = 1; v < W; ++v) part += nsum[v];
  bool ok = true;
  if (w == 0 && g > 0) {  // the block total (and partial), for the earlier blocks
    const Affine<R> T0 = load_map(tot[0]).after(S);
    if (l == 0) {
      map_store_wt<R>(T0, maggs + (long long)g * MR);
      st_wt(parts + g, part);
    }
    publish_flag(fl + g, l);
  }
  if (g + 1 < G) {  // the totals of blocks g+1..G-1
    if (w == 0) {
      Affine<R> e;
      e.set_identity();
      const bool need = l > g && l < G;
      if (!wait_flag_lanes(fl + l, need, a.wait_ticks)) ok = false;
      if (need) map_load_wt<R>(e, maggs + (long long)l * MR);
      for (int k = 1; k < G - 1 - g; k <<= 1) {  // lane g+1 needs G-1-g lanes
        const Affine<R> o = e.shfl_down(k);
        if (l + k < 64) e = e.after(o);
      }
      if (l == g + 1) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          bsuf[R * R + i] = e.g[i];
#pragma unroll
          for (int j = 0; j < R; ++j) bsuf[i * R + j] = e.G[i][j];
        }
      }
      if (a.nll && g == 0 && l == 0) {  // every other block's partial is visible now
        double tsum = part;
        for (int v = 1; v < G; ++v) tsum += ld_wt(parts + v);
        a.nll[b] = tsum;
      }
    }
    __syncthreads();
    X = X.after(load_map(bsuf));
  } else if (a.nll && G == 1 && tid == 0) {
    a.nll[b] = part;
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SCAN);
  double ms[R];
  // X maps the value entering the last chunk (none for the globally last
  // segment: its map is constant; the next segment's ms otherwise)
#pragma unroll
  for (int i = 0; i < R; ++i) {
    double t = X.g[i];
    if (a.seg_in)
#pragma unroll
      for (int k = 0; k < R; ++k) t = fma(X.G[i][k], a.seg_in[b * R + k], t);
    ms[i] = t;
  }
  map_run([&](long long c, const Affine<R> &f) {
    if (c + 1 < NCb || a.seg_in) {
#pragma unroll
      for (int i = 0; i < R; ++i) msend[(c * R + i) * B + b] = ms[i];
    }
    double nx[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double t = f.g[i];
#pragma unroll
      for (int k = 0; k < R; ++k) t = fma(f.G[i][k], ms[k], t);
      nx[i] = t;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = nx[i];
  });
}

// Time-sharded smoothing (eks_smooth_seg): the aggregate of a segment's
// chunk elements (phase 1) and of its chunk RTS maps (phase 2), one wave per
// trajectory, lanes composing contiguous chunk ranges then an ordered
// in-wave scan.  Elements compose left to right, maps right to left.
// Time segments, phase 1: the segment's aggregate filtering element = the
// ordered composition of its chunk elements (one block of W waves per
// trajectory: per-thread runs of chunks, an in-order tree over the lanes of
// each wave, then the W wave totals in order).
template <int R, int W>
__global__ __launch_bounds__(64 * W) void k_seg_elems(SmoothArgs a, ChunkPlan p) {
  __shared__ double tot[W][Elem<R>::len];
  const long long b = blockIdx.x;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const long long NC = p.NC;
  if (b >= a.B) return;
  const double *elem = (const double *)(a.ws + p.elem_off);
  const long long q = (NC + 64 * W - 1) / (64 * W);
  const long long c0 = min(NC, (long long)tid * q), c1 = min(NC, c0 + q);
  bool ok = true;
  Elem<R> agg;
  agg.set_identity();
  for (long long c = c0; c < c1; ++c) {
    Elem<R> e, t;
    e.load(elem + (b * NC + c) * Elem<R>::len, 1);
    ok = compose_elem<R>(agg, e, t) && ok;
    agg = t;
  }
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {  // lane l: lanes [l, l + 2k) in order
    const Elem<R> o = shfl_elem<R, false>(agg, k);
    if (l + k < 64) {
      Elem<R> t;
      ok = compose_elem<R>(agg, o, t) && ok;
      agg = t;
    }
  }
  if (l == 0) agg.store(tot[w], 1);
  __syncthreads();
  if (tid == 0) {
    for (int v = 1; v < W; ++v) {
      Elem<R> e, t;
      e.load(tot[v], 1);
      ok = compose_elem<R>(agg, e, t) && ok;
      agg = t;
    }
    agg.store(a.seg_out + b * Elem<R>::len, 1);
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SCAN);
}

// Time segments, phase 2: the segment's aggregate smoothing map (the chunk
// maps composed right to left), same block shape as k_seg_elems.
template <int R, int W>
__global__ __launch_bounds__(64 * W) void k_seg_maps(SmoothArgs a, ChunkPlan p) {
  __shared__ double tot[W][R * R + R];
  const long long b = blockIdx.x;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const long long NC = p.NC;
  if (b >= a.B) return;
  const double *bw = (const double *)(a.ws + p.bwd_off);
  const long long q = (NC + 64 * W - 1) / (64 * W);
  const long long c0 = min(NC, (long long)tid * q), c1 = min(NC, c0 + q);
  auto load_map = [&](const double *sp) {
    Affine<R> f;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      f.g[i] = sp[R * R + i];
#pragma unroll
      for (int j = 0; j < R; ++j) f.G[i][j] = sp[i * R + j];
    }
    return f;
  };
  Affine<R> F;
  F.set_identity();
  for (long long c = c1 - 1; c >= c0; --c) F = load_map(bw + (b * NC + c) * (R * R + R)).after(F);
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const Affine<R> o = F.shfl_down(k);
    if (l + k < 64) F = F.after(o);
  }
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      tot[w][R * R + i] = F.g[i];
#pragma unroll
      for (int j = 0; j < R; ++j) tot[w][i * R + j] = F.G[i][j];
    }
  }
  __syncthreads();
  if (tid == 0) {
    for (int v = 1; v < W; ++v) F = F.after(load_map(tot[v]));
    double *o = a.seg_out + b * (R * R + R);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      o[R * R + i] = F.g[i];
#pragma unroll
      for (int j = 0; j < R; ++j) o[i * R + j] = F.G[i][j];
    }
  }
}

// Combine the all-gathered segment aggregates of every rank (one thread per
// trajectory).  kind 0: the filtered state entering segment `self` = the
// first segment's element (a state: Ab = 0) composed with the elements of
// segments 1 .. self-1.  kind 1: the smoothed mean entering segment self + 1
// = the maps of segments nseg-1 .. self+1 applied right to left (the last
// segment's map is constant).
template <int R>
__global__ __launch_bounds__(64) void k_seg_combine(int kind, long long B, int nseg, int self,
                                                    const double *__restrict__ in,
                                                    double *__restrict__ out,
                                                    int32_t *__restrict__ status) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (b >= B) return;
  bool ok = true;
  if (kind == 0) {
    constexpr int EL = Elem<R>::len;
    Elem<R> e0;
    e0.load(in + b * EL, 1);
    double m[R], P[R][R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      m[i] = e0.bb[i];
#pragma unroll
      for (int j = 0; j < R; ++j) P[i][j] = e0.Cb[i][j];
    }
    for (int sg = 1; sg < self; ++sg) {
      Elem<R> e;
      e.load(in + ((long long)sg * B + b) * EL, 1);
      ok = compose_state<R>(m, P, e) && ok;
    }
    store_state<R>(out + b * (R + Sym<R>::len), 1, m, P);
  } else {
    constexpr int ML = R * R + R;
    double ms[R];
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = 0.0;
    for (int sg = nseg - 1; sg > self; --sg) {
      const double *f = in + ((long long)sg * B + b) * ML;
      double nx[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        double t = f[R * R + i];
#pragma unroll
        for (int k = 0; k < R; ++k) t = fma(f[i * R + k], ms[k], t);
        nx[i] = t;
      }
#pragma unroll
      for (int i = 0; i < R; ++i) ms[i] = nx[i];
    }
#pragma unroll
    for (int i = 0; i < R; ++i) out[b * R + i] = ms[i];
  }
  if (!ok && status) atomicOr(status + b, EKS_STATUS_SCAN);
}

// RTS gain (J_t, d_t) of step t in the (J, d) planes: R*R + R planes per step
template <int R>
EKS_DEV void store_jd(double *base, long long t, long long B, unsigned b, const double (&J)[R][R],
                      const double (&d)[R]) {
  constexpr int MR = R * R + R;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    pl(base, t * MR + R * R + i, B, b) = d[i];
#pragma unroll
    for (int j = 0; j < R; ++j) pl(base, t * MR + i * R + j, B, b) = J[i][j];
  }
}

// y / ev of step t (time-major planes), raw
template <int N, typename YT>
EKS_DEV void load_yev(const YT *ybuf, const double *evbuf, long long t, long long B, unsigned b,
                      YT (&y)[N], double (&rv)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    y[j] = pl(ybuf, t * N + j, B, b);
    rv[j] = pl(evbuf, t * N + j, B, b);
  }
}

template <int R, int N, typename YT, int AI, int CI, int LS, bool UNI>
__global__ __launch_bounds__(kBlock) void k_c3_rerun(SmoothArgs a, ChunkPlan p) {
  // y / ev prefetch distance (steps; divides LS): 2 keeps the (2, 2) kernel at
  // 3 waves/SIMD (160 VGPRs), measured 3 % faster than 4 (174 VGPRs, 2 waves)
  constexpr int D = (R <= 2 && N <= 2) ? (UNI ? 2 : kC3Dnu) : (LS < 4 ? LS : 4);
  static_assert(LS % D == 0, "prefetch distance must divide the checkpoint interval");
  Lane<UNI> ln;
  const long long B = a.B, TT = a.T;
  const bool valid = ln.init(B, p.NC);
  if (UNI || !p.grp) {
    if (!valid) return;
  }
  constexpr int KS = R + Sym<R>::len, MR = R * R + R;
  double G[R][R], g[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    g[i] = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) G[i][j] = (i == j) ? 1.0 : 0.0;
  }
  double share = 0.0;  // the chunk's NLL share
  if (valid) {
  const long long c = ln.c;
  const unsigned b = ln.b;
  Model<R, N> md;
  md.load(a.params + (long long)b * ParamLayout<R, N>::len, false);
  const YT *ybuf = (const YT *)p.ysrc;
  const double *evbuf = (const double *)p.evsrc;
  double *ckpt = (double *)(a.ws + p.ckpt_off);
  double *jdp = (double *)(a.ws + p.jd_off);
  double m[R], P[R][R];
  bool ok = true;
  if (!UNI && p.grp) {
    // group mode: the group's start state (K2) composed with the inclusive
    // prefix K1 stored for the chunk before (same block: lane - B)
    const double *gst = (const double *)(a.ws + p.gst_off);
    if (threadIdx.x >= B) {
      Elem<R> pe;
      pe.load((const double *)(a.ws + p.elem_off) + ((long long)b * p.NC + c - 1) * Elem<R>::len, 1);
      if (blockIdx.x == 0) {  // group 0 holds chunk 0, a filtered state (Ab = 0)
#pragma unroll
        for (int i = 0; i < R; ++i) {
          m[i] = pe.bb[i];
#pragma unroll
          for (int j = 0; j < R; ++j) P[i][j] = pe.Cb[i][j];
        }
      } else {
        load_state_pl<R>(gst, (long long)blockIdx.x * KS, B, b, m, P);
        ok = compose_state<R>(m, P, pe) && ok;
      }
    } else {
      load_state_pl<R>(gst, (long long)blockIdx.x * KS, B, b, m, P);
    }
    if (!ok) flag(a.status, b, EKS_STATUS_SCAN);
  } else {
    load_state_pl<R>((const double *)(a.ws + p.cstart_off), c * KS, B, b, m, P);
  }
  const long long s = c * p.L, e = min(TT, s + p.L);
  NllAcc acc;
  YT yr[D][N];
  double er[D][N];
  // unconditional ring loads, step clamped to the chunk's last (see c1_stream)
#pragma unroll
  for (int q = 0; q < D; ++q) load_yev<N, YT>(ybuf, evbuf, min(s + q, e - 1), p.yB, p.ylane(b), yr[q], er[q]);
  long long k = 0;
  for (long long t0 = s; t0 < e; t0 += LS, ++k) {
    if (p.smooth && !p.jd) store_state_pl<R>(ckpt, (c * p.NSUB + k) * KS, B, b, m, P);  // state before t0
#pragma unroll
    for (int q = 0; q < LS; ++q) {
      const long long t = t0 + q;
      double y[N], rv[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        y[j] = (double)yr[q % D][j] - md.off[j];
        rv[j] = er[q % D][j];
      }
      load_yev<N, YT>(ybuf, evbuf, min(t + D, e - 1), p.yB, p.ylane(b), yr[q % D], er[q % D]);
      if (t < e) {
        if (t + a.t_base > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
        kf_update<R, N, CI>(m, P, md.C, y, rv, acc, ok);
        if (!p.smooth) continue;
        if (t + a.t_base + 1 < a.T_total) {
          double J[R][R], d[R], GJ[R][R];
          ok = rts_gain<R, AI>(m, P, md.A, md.Q, J, d) && ok;
          if (p.jd) store_jd<R>(jdp, t, B, b, J, d);
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
            for (int j = 0; j < R; ++j) G[i][j] = GJ[i][j];
        } else {  // ms[T-1] = mf[T-1]: the map ends in a constant
          if (p.jd) {
            double Z[R][R] = {};
            store_jd<R>(jdp, t, B, b, Z, m);
          }
#pragma unroll
          for (int i = 0; i < R; ++i) {
            double sg = g[i];
#pragma unroll
            for (int u = 0; u < R; ++u) sg = fma(G[i][u], m[u], sg);
            g[i] = sg;
          }
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int j = 0; j < R; ++j) G[i][j] = 0.0;
        }
      }
    }
  }
  share = acc.value((double)(e - s) * N);
  pl((double *)(a.ws + p.nllp_off), c, B, b) = share;
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
  }  // valid
  if (!p.smooth) return;
  if constexpr (!UNI) {
    if (p.grp) {
      // group mode: suffix scan of the maps over this trajectory's chunks in
      // the block (lanes B apart, right to left) and of the NLL shares, in
      // LDS (dynamic: MR + 1 planes of 256 doubles)
      extern __shared__ double dsh[];
      const int tid = threadIdx.x, Bi = (int)B;
      Affine<R> F;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        F.g[i] = g[i];
#pragma unroll
        for (int j = 0; j < R; ++j) F.G[i][j] = G[i][j];
      }
      for (int k = 1; k * Bi < kBlock; k <<= 1) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          dsh[(R * R + i) * kBlock + tid] = F.g[i];
#pragma unroll
          for (int j = 0; j < R; ++j) dsh[(i * R + j) * kBlock + tid] = F.G[i][j];
        }
        dsh[MR * kBlock + tid] = share;
        __syncthreads();
        const int j2 = tid + k * Bi;
        const bool has = j2 < kBlock && valid && ln.c + k < p.NC;
        Affine<R> o;
        double os = 0.0;
        if (has) {
#pragma unroll
          for (int i = 0; i < R; ++i) {
            o.g[i] = dsh[(R * R + i) * kBlock + j2];
#pragma unroll
            for (int j = 0; j < R; ++j) o.G[i][j] = dsh[(i * R + j) * kBlock + j2];
          }
          os = dsh[MR * kBlock + j2];
        }
        __syncthreads();
        if (has) {
          F = F.after(o);
          share += os;
        }
      }
      if (!valid) return;
      const unsigned b = ln.b;
      if (tid < Bi) {  // the group's first chunk: the group totals
        double *gm = (double *)(a.ws + p.gmap_off) + ((long long)b * p.NG + blockIdx.x) * MR;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          gm[R * R + i] = F.g[i];
#pragma unroll
          for (int j = 0; j < R; ++j) gm[i * R + j] = F.G[i][j];
        }
        pl((double *)(a.ws + p.gnll_off), (long long)blockIdx.x, B, b) = share;
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        g[i] = F.g[i];
#pragma unroll
        for (int j = 0; j < R; ++j) G[i][j] = F.G[i][j];
      }
    }
  }
  // chunk maps are stored trajectory-major: row (b, c) = [G (R*R) | g (R)]
  // (group mode: the suffix through the group's last chunk)
  double *bw = (double *)(a.ws + p.bwd_off) + ((long long)ln.b * p.NC + ln.c) * MR;
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) bw[i * R + j] = G[i][j];
#pragma unroll
  for (int i = 0; i < R; ++i) bw[R * R + i] = g[i];
}

template <int R>
__global__ __launch_bounds__(64) void k_c4_bscan(SmoothArgs a, ChunkPlan p) {
  const long long b = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long B = a.B;
  if (b >= B) return;
  const double *bw = (const double *)(a.ws + p.bwd_off);
  double *msend = (double *)(a.ws + p.msend_off);
  const double *np_ = (const double *)(a.ws + p.nllp_off);
  auto load_map = [&](long long c, double (&G)[R][R], double (&g)[R]) {
    const double *q = bw + (b * p.NC + c) * (R * R + R);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      g[i] = q[R * R + i];
#pragma unroll
      for (int j = 0; j < R; ++j) G[i][j] = q[i * R + j];
    }
  };
  double ms[R], G[R][R], g[R], Gn[R][R], gn[R];
  // the value entering the last chunk: none for the globally last segment
  // (its map is constant), the next segment's ms otherwise
#pragma unroll
  for (int i = 0; i < R; ++i) ms[i] = a.seg_in ? a.seg_in[b * R + i] : 0.0;
  if (a.seg_in)
#pragma unroll
    for (int i = 0; i < R; ++i) msend[((p.NC - 1) * R + i) * B + b] = ms[i];
  load_map(p.NC - 1, G, g);
  for (long long c = p.NC - 1; c >= 0; --c) {
    if (c >= 1) load_map(c - 1, Gn, gn);  // next map in flight during this one
    double nx[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = g[i];
#pragma unroll
      for (int j = 0; j < R; ++j) s = fma(G[i][j], ms[j], s);
      nx[i] = s;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = nx[i];
    if (c >= 1) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        msend[((c - 1) * R + i) * B + b] = ms[i];
        g[i] = gn[i];
#pragma unroll
        for (int j = 0; j < R; ++j) G[i][j] = Gn[i][j];
      }
    }
  }
  if (a.nll) {
    double s = 0.0;
    for (long long c = 0; c < p.NC; ++c) s += np_[c * B + b];
    a.nll[b] = s;
  }
}

// filter-only calls (no `out`): the NLL of each trajectory is the sum of its
// chunks' shares; one wave per trajectory, lane l sums chunks l, l+64, ...,
// then a fixed-order shuffle tree (deterministic)
template <int R>
__global__ __launch_bounds__(64) void k_c4_nll(SmoothArgs a, ChunkPlan p) {
  const long long b = blockIdx.x;
  const int l = threadIdx.x;
  if (b >= a.B || !a.nll) return;
  const double *np_ = (const double *)(a.ws + p.nllp_off);
  double s = 0.0;
  for (long long c = l; c < p.NC; c += 64) s += np_[c * a.B + b];
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) s += __shfl_xor(s, k, 64);
  if (l == 0) a.nll[b] = s;
}

// the smoothed mean entering chunk c of trajectory b from the right (K5)
template <int R, bool UNI>
EKS_DEV void c5_ms_in(const SmoothArgs &a, const ChunkPlan &p, long long c, unsigned b,
                      double (&ms)[R]) {
  const long long B = a.B, TT = a.T;
  // ms entering the chunk from the right: from K4, or for the globally last
  // chunk unused (its map ends in the constant mf[T-1]); the last chunk of an
  // earlier time segment gets it from the next segment (eks_smooth_seg)
  if (!UNI && p.grp) {
    // group mode: the mean entering the group from the right (K4) through
    // the suffix of the maps after this chunk (K3, same block: lane + B);
    // the trajectory's last group ends in a constant map (no mean enters)
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = 0.0;
    if (c + 1 < p.NC) {
      const long long blk = blockIdx.x;
      const bool last_group = ((p.NC - 1) * B + b) / kBlock == blk;
      double mg[R];
#pragma unroll
      for (int i = 0; i < R; ++i)
        mg[i] = last_group ? 0.0 : pl((const double *)(a.ws + p.gms_off), blk * R + i, B, b);
      if (threadIdx.x + B < kBlock) {
        const double *f = (const double *)(a.ws + p.bwd_off) + ((long long)b * p.NC + c + 1) * (R * R + R);
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double t = f[R * R + i];
          if (!last_group)
#pragma unroll
            for (int k = 0; k < R; ++k) t = fma(f[i * R + k], mg[k], t);
          ms[i] = t;
        }
      } else {
#pragma unroll
        for (int i = 0; i < R; ++i) ms[i] = mg[i];
      }
    }
  } else if (c + 1 < p.NC || a.t_base + TT < a.T_total) {
    const double *me = (const double *)(a.ws + p.msend_off);
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = pl(me, c * R + i, B, b);
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) ms[i] = 0.0;
  }
}

template <int R, int N, typename YT, int AI, int CI, int LS, bool UNI>
__global__ __launch_bounds__(kBlock) void k_c5_final(SmoothArgs a, ChunkPlan p) {
  Lane<UNI> ln;
  const long long B = a.B, TT = a.T;
  if (!ln.init(B, p.NC)) return;
  const long long c = ln.c;
  const unsigned b = ln.b;
  constexpr int KS = R + Sym<R>::len;
  Model<R, N> md;
  md.load(a.params + (long long)b * ParamLayout<R, N>::len, false);
  const YT *ybuf = (const YT *)p.ysrc;
  const double *evbuf = (const double *)p.evsrc;
  const double *ckpt = (const double *)(a.ws + p.ckpt_off);
  double ms[R];
  c5_ms_in<R, UNI>(a, p, c, b, ms);
  const long long s = c * p.L, e = min(TT, s + p.L);
  const long long nsub = (e - s + LS - 1) / LS;
  bool ok = true;
  NllAcc dummy;
  double *outb = a.out + (long long)b * a.ob;
  for (long long k = nsub - 1; k >= 0; --k) {
    const long long t0 = s + k * LS;
    double m[R], P[R][R];
    load_state_pl<R>(ckpt, (c * p.NSUB + k) * KS, B, b, m, P);
    YT yr[LS][N];
    double er[LS][N];
    // unconditional loads (step clamped to the chunk's last): a divergent
    // `if` around each would serialise them (see c1_stream)
#pragma unroll
    for (int j = 0; j < LS; ++j) load_yev<N, YT>(ybuf, evbuf, min(t0 + j, e - 1), p.yB, p.ylane(b), yr[j], er[j]);
    double Jr[LS][R][R], dr[LS][R];
#pragma unroll
    for (int j = 0; j < LS; ++j) {
      const long long t = t0 + j;
      if (t < e) {
        double y[N], rv[N];
#pragma unroll
        for (int q = 0; q < N; ++q) {
          y[q] = (double)yr[j][q] - md.off[q];
          rv[q] = er[j][q];
        }
        if (t + a.t_base > 0) kf_predict<R, AI>(m, P, md.A, md.Q);
        kf_update<R, N, CI>(m, P, md.C, y, rv, dummy, ok);
        if (t + a.t_base + 1 < a.T_total) {
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
      const long long t = t0 + j;
      if (t < e) {
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
        if (a.ms) store_vec<R>(a.ms + ((long long)b * TT + t) * R, ms);
      }
    }
  }
  if (!ok) flag(a.status, b, EKS_STATUS_SINGULAR);
}

// K5 of (J, d) mode: the backward mean recursion ms_t = J_t ms_{t+1} + d_t
// over the chunk from the stored gains (K3), D steps of gains in flight
template <int R, int N, int CI, bool UNI>
__global__ __launch_bounds__(kBlock) void k_c5_jd(SmoothArgs a, ChunkPlan p) {
  constexpr int D = 2, MR = R * R + R;
  Lane<UNI> ln;
  const long long B = a.B, TT = a.T;
  if (!ln.init(B, p.NC)) return;
  const long long c = ln.c;
  const unsigned b = ln.b;
  Model<R, N> md;
  md.load(a.params + (long long)b * ParamLayout<R, N>::len, false);
  double ms[R];
  c5_ms_in<R, UNI>(a, p, c, b, ms);
  const double *jdp = (const double *)(a.ws + p.jd_off);
  const long long s = c * p.L, e = min(TT, s + p.L);
  double *outb = a.out + (long long)b * a.ob;
  double ring[D][MR];
  auto fetch = [&](int q, long long t) {
#pragma unroll
    for (int k = 0; k < MR; ++k) ring[q][k] = pl(jdp, t * MR + k, B, b);
  };
  // unconditional loads, step clamped to the chunk's first (see c1_stream)
#pragma unroll
  for (int q = 0; q < D; ++q) fetch(q, max(e - 1 - q, s));
  for (long long t0 = e - 1; t0 >= s; t0 -= D) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const long long t = t0 - q;
      double f[MR];
#pragma unroll
      for (int k = 0; k < MR; ++k) f[k] = ring[q][k];
      fetch(q, max(t - D, s));
      if (t >= s) {
        double nx[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          double sm = f[R * R + i];
#pragma unroll
          for (int k = 0; k < R; ++k) sm = fma(f[i * R + k], ms[k], sm);
          nx[i] = sm;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) ms[i] = nx[i];
        project_store<R, N, CI>(outb + t * a.ot, a.oj, md.C, ms, md.off);
        if (a.ms) store_vec<R>(a.ms + ((long long)b * TT + t) * R, ms);
      }
    }
  }
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

#include "two_pass.hpp"

template <int R, int N, int AI, int CI>
int launch_shape(const SmoothArgs &a, int algo, long long L) {
  if (algo == 3) return launch_algo3<R, N, AI, CI>(a);
  const bool f32 = a.dtype == EKS_F32;
  const bool yev = a.dtype == EKS_YEV32 || a.dtype == EKS_YEV64;
  if (algo == 1) {
    if (yev) {
      auto go_yev = [&](auto ytag) -> int {
        using YT = decltype(ytag);
        prof_call_begin();
        prof_mark(a.stream, "k_smooth_seq");
        hipLaunchKernelGGL((k_smooth_seq<R, N, 0, YevIn<YT>, AI, CI>), dim3(grid_for(a.B, 64)),
                           dim3(64), 0, a.stream, a);
        prof_call_end(a.stream);
        return check_launch("k_smooth_seq");
      };
      return a.dtype == EKS_YEV32 ? go_yev(float{}) : go_yev(double{});
    }
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
  ChunkPlan p = make_plan(a.B, a.T, R, N, L);
  p.smooth = a.out != nullptr;
  p.nll_closed = (!p.smooth && a.phase == 0 && a.nll) ? 1 : 0;
  p.nll_fused = (p.nll_closed && p.NC > wave_scan_chunks()) ? 1 : 0;
  const bool shared = !yev && a.sb == 0 && a.B > 1;
  p.yB = shared ? 1 : a.B;
  // (int step indices in the scalar path: T < 2^31 / N)
  p.ywave = (shared && (uniform_lanes(a.B) || a.B % 64 == 0) && a.T * N < (1LL << 31)) ? 1 : 0;
  const bool uni = uniform_lanes(a.B);
  // group mode: few trajectories, smoothing, whole pipeline, chained scans
  // (B <= 256: every block but the last holds chunks of every trajectory)
  p.grp = (!uni && a.B <= kBlock && p.smooth && a.phase == 0 && p.NC > wave_scan_chunks() &&
           p.NG > 0) ? 1 : 0;
  const size_t lds1 = p.grp ? (size_t)Elem<R>::len * kBlock * 8 : 0;  // K1's group scan
  const size_t lds3 = p.grp ? (size_t)(R * R + R + 1) * kBlock * 8 : 0;  // K3's
  p.jd = (p.jd_off && p.smooth && a.phase == 0) ? 1 : 0;
  ChunkPlan pg = p, p4 = p;  // K2 / K4 over the group totals
  if (p.grp) {
    pg.NC = p4.NC = p.NG;
    pg.G = p4.G = p.GG;
    pg.CPB = p4.CPB = p.CPBG;
    pg.gnc = p4.gnc = p.NC;
    pg.elem_off = p.gagg_off;
    pg.cstart_off = p.gst_off;
    p4.bwd_off = p.gmap_off;
    p4.msend_off = p.gms_off;
    p4.nllp_off = p.gnll_off;
  }
  const unsigned gch = uni ? (unsigned)(p.NC * blocks_per_chunk(a.B))
                           : grid_for(p.NC * a.B, kBlock);
  const unsigned g64 = grid_for(a.B, 64);
  // y is stored as float when it is exactly a member value (odd-E median of f32)
  const bool y32 = yev ? a.dtype == EKS_YEV32 : (f32 && a.median && (a.E == 3 || a.E == 5));
  if (yev) {
    p.ysrc = (const char *)a.obs;
    p.evsrc = p.ysrc + yev_ev_offset(a.B, a.T, N, y32 ? sizeof(float) : sizeof(double));
  } else {
    p.ysrc = a.ws + p.y_off;
    p.evsrc = a.ws + p.ev_off;
  }
  bool begun = false;  // the profiler's call already opened (k_c0_shared)
  auto run = [&](auto tag, auto ytag, auto unitag) -> int {
    using Tp = decltype(tag);
    using YT = decltype(ytag);
    constexpr bool U = decltype(unitag)::value;
    constexpr int LS = sub_len_c(R, N);
    const int ph = a.phase;  // 0: whole pipeline; 1 / 2 / 3: time-segment phases
    if (!begun) prof_call_begin();
    int rc;
    if (ph == 0 || ph == 1) {
      auto k1 = [&](auto Ec) {
        constexpr int EE = decltype(Ec)::value;
        prof_mark(a.stream, "k_c1_elem");
        hipLaunchKernelGGL((k_c1_elem<R, N, EE, Tp, YT, AI, CI, U>), dim3(gch), dim3(kBlock), lds1,
                           a.stream, a, p);
        return check_launch("k_c1_elem");
      };
      if constexpr (is_yev<Tp>::value)
        rc = k1(ic<0>{});  // the members are not read: E does not matter
      else
        rc = dispatch_members_c(a.E, k1);
      if (rc) return rc;
      if (ph == 1) {  // the segment's aggregate element
        prof_mark(a.stream, "k_seg_elems");
        const int sw1 = scan_waves(p.NC);
        if (sw1 == 8)
          hipLaunchKernelGGL((k_seg_elems<R, 8>), dim3((unsigned)a.B), dim3(512), 0, a.stream, a,
                             p);
        else if (sw1 == 4)
          hipLaunchKernelGGL((k_seg_elems<R, 4>), dim3((unsigned)a.B), dim3(256), 0, a.stream, a,
                             p);
        else
          hipLaunchKernelGGL((k_seg_elems<R, 1>), dim3((unsigned)a.B), dim3(64), 0, a.stream, a,
                             p);
        prof_call_end(a.stream);
        return check_launch("k_seg_elems");
      }
    }
    // the chunk scans: one lane per trajectory while the chain is short, one
    // wave per trajectory (log-depth scan) when it is long
    const bool wave_scan = p.NC > wave_scan_chunks();
    const int sw = scan_waves(p.NC);
    // the chained scans' sync words: zeroed by K1 in a whole-pipeline call
    auto zero_sync = [&]() -> int {
      if (hipMemsetAsync(a.ws + p.sync_off, 0, p.sync_bytes, a.stream) != hipSuccess)
        return set_err(EKS_ERR_HIP, "eks_smooth: hipMemsetAsync failed");
      return 0;
    };
    if (ph == 0 || ph == 2) {
      if (ph == 2 && wave_scan && (rc = zero_sync())) return rc;
      prof_mark(a.stream, "k_c2_fscan");
      if (!wave_scan)
        hipLaunchKernelGGL((k_c2_fscan<R, N>), dim3(g64), dim3(64), 0, a.stream, a, p);
      else
        hipLaunchKernelGGL((k_c2_fscan_g<R, N>), dim3((unsigned)(a.B * pg.G)), dim3(256), 0,
                           a.stream, a, pg);
      if ((rc = check_launch("k_c2_fscan"))) return rc;
      if (p.nll_fused) {  // K2 summed the closed-form NLL shares: done
        prof_call_end(a.stream);
        return 0;
      }
      if (!p.nll_closed) {
        prof_mark(a.stream, "k_c3_rerun");
        hipLaunchKernelGGL((k_c3_rerun<R, N, YT, AI, CI, LS, U>), dim3(gch), dim3(kBlock), lds3,
                           a.stream, a, p);
        if ((rc = check_launch("k_c3_rerun"))) return rc;
      }
      if (ph == 2 && p.smooth) {  // the segment's aggregate RTS map
        prof_mark(a.stream, "k_seg_maps");
        if (sw == 8)
          hipLaunchKernelGGL((k_seg_maps<R, 8>), dim3((unsigned)a.B), dim3(512), 0, a.stream, a,
                             p);
        else if (sw == 4)
          hipLaunchKernelGGL((k_seg_maps<R, 4>), dim3((unsigned)a.B), dim3(256), 0, a.stream, a,
                             p);
        else
          hipLaunchKernelGGL((k_seg_maps<R, 1>), dim3((unsigned)a.B), dim3(64), 0, a.stream, a,
                             p);
        prof_call_end(a.stream);
        return check_launch("k_seg_maps");
      }
      if (!p.smooth) {  // filter only: sum the NLL shares, no backward pass
        prof_mark(a.stream, "k_c4_nll");
        hipLaunchKernelGGL((k_c4_nll<R>), dim3((unsigned)a.B), dim3(64), 0, a.stream, a, p);
        prof_call_end(a.stream);
        return check_launch("k_c4_nll");
      }
    }
    if (ph == 3 && wave_scan && (rc = zero_sync())) return rc;
    prof_mark(a.stream, "k_c4_bscan");
    if (!wave_scan)
      hipLaunchKernelGGL((k_c4_bscan<R>), dim3(g64), dim3(64), 0, a.stream, a, p);
    else
      hipLaunchKernelGGL((k_c4_bscan_g<R>), dim3((unsigned)(a.B * p4.G)), dim3(256), 0, a.stream,
                         a, p4);
    if ((rc = check_launch("k_c4_bscan"))) return rc;
    if (p.jd) {
      prof_mark(a.stream, "k_c5_jd");
      hipLaunchKernelGGL((k_c5_jd<R, N, CI, U>), dim3(gch), dim3(kBlock), 0, a.stream, a, p);
      prof_call_end(a.stream);
      return check_launch("k_c5_jd");
    }
    prof_mark(a.stream, "k_c5_final");
    hipLaunchKernelGGL((k_c5_final<R, N, YT, AI, CI, LS, U>), dim3(gch), dim3(kBlock), 0,
                       a.stream, a, p);
    prof_call_end(a.stream);
    return check_launch("k_c5_final");
  };
  auto with_uni = [&](auto tag, auto ytag) -> int {
    return uni ? run(tag, ytag, std::true_type{}) : run(tag, ytag, std::false_type{});
  };
  if (yev) return y32 ? with_uni(YevIn<float>{}, float{}) : with_uni(YevIn<double>{}, double{});
  if (shared) {
    // the ensemble once (k_c0_shared), then the pipeline on those planes
    if (a.phase == 0 || a.phase == 1) {
      auto k0 = [&](auto tag, auto ytag) -> int {
        using Tp = decltype(tag);
        using YT = decltype(ytag);
        return dispatch_members_c(a.E, [&](auto Ec) {
          constexpr int EE = decltype(Ec)::value;
          prof_mark(a.stream, "k_c0_shared");
          hipLaunchKernelGGL((k_c0_shared<EE, N, Tp, YT>), dim3(grid_for(a.T, kBlock)),
                             dim3(kBlock), 0, a.stream, a, p);
          return check_launch("k_c0_shared");
        });
      };
      prof_call_begin();
      begun = true;
      const int rc = y32 ? k0(float{}, float{}) : f32 ? k0(float{}, double{}) : k0(double{}, double{});
      if (rc) return rc;
    }
    return y32 ? with_uni(YevIn<float>{}, float{}) : with_uni(YevIn<double>{}, double{});
  }
  if (y32) return with_uni(float{}, float{});
  return f32 ? with_uni(float{}, double{}) : with_uni(double{}, double{});
}

template <int R>
int launch_seg_combine(int kind, long long B, int nseg, int self, const double *in, double *out,
                       int32_t *status, hipStream_t s) {
  hipLaunchKernelGGL((k_seg_combine<R>), dim3(grid_for(B, 64)), dim3(64), 0, s, kind, B, nseg,
                     self, in, out, status);
  return check_launch("k_seg_combine");
}

// the runtime-n smoother (eks_shape_rt.hip)
int launch_rt(const SmoothArgs &a);
size_t rt_workspace_bytes(long long B, long long T, int n, int r);

// per-shape entry points (defined in eks_shape_*.hip)
int launch_22(const SmoothArgs &a, int algo, long long L);
int launch_34(const SmoothArgs &a, int algo, long long L);
int launch_36(const SmoothArgs &a, int algo, long long L);
int launch_38(const SmoothArgs &a, int algo, long long L);
int launch_312(const SmoothArgs &a, int algo, long long L);
int launch_316(const SmoothArgs &a, int algo, long long L);

}  // namespace eks
