// C ABI of the fused smoother: eks_smooth, eks_smooth_workspace_bytes,
// eks_smooth_chunk_len (include/eks_hip.h).  Validates arguments, zeroes the
// status array, picks the algorithm and dispatches to the per-shape
// launchers of eks_shape_*.hip.
#include "smooth_impl.hpp"

using namespace eks;

namespace {

// automatic choice: the sequential algorithm when one chunk covers the
// trajectory (B alone fills the GPU); the two-pass algorithm 3 for the
// (r, n) = (2, 2) single-view shape with many trajectories (whole 256-lane
// blocks per chunk) and compile-time member counts; else the three-pass
// time-parallel scan.  A requested algo 2 with a single chunk runs
// sequentially; a requested algo 3 runs at any T (compiled E).
int pick_algo(long long B, long long T, int n, int r, int E, int algo) {
  const long long L = chunk_len(B, T, r);
  if (algo == 1) return 1;
  const bool a3_ok = E >= 3 && E <= 5;  // compiled member counts; any T
  if (algo == 3 && a3_ok) return 3;
  if (L >= T) return 1;
  if (algo == 3) return 2;
  if (algo == 2) return 2;
  const bool many = uniform_lanes(B) && B >= 2048;
  return (a3_ok && many && r == 2 && n == 2 && T >= 2 * fine_len3(r, n)) ? 3 : 2;
}

bool shape_compiled(int r, int n) {
  return (r == 2 && n == 2) || (r == 3 && (n == 4 || n == 6 || n == 8 || n == 12 || n == 16));
}

// the runtime-n kernel (one lane per trajectory, any n <= kMaxObsRt): shapes
// without compiled kernels, or any shape with algo = 4
bool use_rt(int r, int n, int algo) {
  return (r == 2 || r == 3) && n <= kMaxObsRt && (algo == 4 || !shape_compiled(r, n));
}

}  // namespace

namespace eks {
long long g_wait_ticks = kDefaultWaitTicks;
long long g_a3_slice_bytes = 0;
long long g_a3_mode = 0;
long long g_a3_lb = 0;
long long g_rt_form = 0;
extern long long g_fit_select;  // eks_fit.hip
}

extern "C" {

int64_t eks_smooth_chunk_len(int64_t B, int64_t T, int r) {
  if (B <= 0 || T <= 0 || r < 1) return 0;
  const long long L = chunk_len(B, T, r);
  return L >= T ? 0 : L;
}

int eks_smooth_algo(int64_t B, int64_t T, int n, int r, int E, int algo) {
  if (B <= 0 || T <= 0 || r < 1 || n < 1 || algo < 0 || algo > 4) return 0;
  if (use_rt(r, n, algo)) return 4;
  return pick_algo(B, T, n, r, E, algo);
}

size_t eks_smooth_workspace_bytes(int64_t B, int64_t T, int n, int r, int E, int algo) {
  (void)E;
  if (B <= 0 || T <= 0 || r < 1 || n < 1) return 0;
  if (use_rt(r, n, algo)) return rt_workspace_bytes(B, T, n, r);
  const int al = pick_algo(B, T, n, r, E, algo);
  if (al == 1) return seq_workspace_bytes(B, T, r);
  // smoothing calls of few trajectories use shorter chunks than filter-only ones
  const size_t p2 = std::max(make_plan(B, T, r, n, chunk_len(B, T, r)).total,
                             make_plan(B, T, r, n, chunk_len_smooth(B, T, r)).total);
  // algo 3 smooths only: a filter-only (NLL) call of the same shape runs algo 2
  return al == 3 ? std::max(p2, make_plan3(B, T, r, n).total) : p2;
}

// shared validation and dispatch of eks_smooth / eks_smooth_seg
static int smooth_call(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
                       int64_t sb, int64_t st, int64_t se, int64_t sj, int mode,
                       const double *params, double *out, int64_t ob, int64_t ot, int64_t oj,
                       double *ms, double *nll, void *workspace, size_t workspace_bytes,
                       int model_flags, int algo, int32_t *status, void *stream, int64_t t_base,
                       int64_t T_total, int phase, const double *seg_in, double *seg_out) {
  if (!obs || !params || !status) return set_err(EKS_ERR_ARG, "eks_smooth: NULL pointer");
  if (!out && (!nll || ms) && (phase == 0 || phase == 3))
    return set_err(EKS_ERR_ARG, "eks_smooth: out may be NULL only for a filter-only (nll) call");
  if (B < 0 || T < 1 || E < 1) return set_err(EKS_ERR_ARG, "eks_smooth: need B>=0, T>=1, E>=1");
  if (E > kMaxMembers) return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth: E=%d > %d", E, kMaxMembers);
  if (mode != EKS_MEDIAN && mode != EKS_MEAN)
    return set_err(EKS_ERR_ARG, "%d averaging not supported", mode);
  if (obs_dtype != EKS_F32 && obs_dtype != EKS_F64 && obs_dtype != EKS_YEV32 &&
      obs_dtype != EKS_YEV64)
    return set_err(EKS_ERR_ARG, "bad dtype");
  if (algo < 0 || algo > 4) return set_err(EKS_ERR_ARG, "eks_smooth: algo %d unknown", algo);
  const bool rt = use_rt(r, n, algo);
  if (!rt && !shape_compiled(r, n))
    return set_err(EKS_ERR_UNSUPPORTED,
                   "eks_smooth: (r=%d, n=%d) not supported (compiled: (2,2) (3,4) (3,6) (3,8) "
                   "(3,12) (3,16); any n <= %d for r = 2, 3)", r, n, kMaxObsRt);
  if (rt && phase)
    return set_err(EKS_ERR_UNSUPPORTED, "eks_smooth_seg: (r=%d, n=%d) has no time-parallel kernels", r, n);
  if ((model_flags & EKS_MODEL_C_IDENTITY) && r != n)
    return set_err(EKS_ERR_ARG, "eks_smooth: C = I needs r == n");
  if ((model_flags & EKS_MODEL_PUPIL) && (r != 3 || n != 8))
    return set_err(EKS_ERR_ARG, "eks_smooth: EKS_MODEL_PUPIL needs r = 3, n = 8");
  if (B == 0) return EKS_OK;
  // (the runtime-n kernels: algo 1 picks their sequential form)
  int al = rt ? (algo == 1 ? 1 : 4) : phase ? 2 : pick_algo(B, T, n, r, E, algo);
  const size_t need = phase ? make_plan(B, T, r, n, chunk_len(B, T, r)).total
                            : eks_smooth_workspace_bytes(B, T, n, r, E, al);
  if (!workspace || workspace_bytes < need)
    return set_err(EKS_ERR_ARG, "eks_smooth: workspace of %zu bytes needed", need);
  if (al == 3 && !out) al = 2;  // filter only: algo 3 has no NLL-only mode
  // algo 3 addresses members as unsigned 32-bit offsets within a step
  if (al == 3 && (sb < 0 || se < 0 || sj < 0 || ((int64_t)(E - 1) * se + (int64_t)(n - 1) * sj) * 8 >= (1LL << 31)))
    al = 2;
  hipStream_t s = (hipStream_t)stream;
  if (phase <= 1 && hipMemsetAsync(status, 0, (size_t)B * sizeof(int32_t), s) != hipSuccess)
    return set_err(EKS_ERR_HIP, "eks_smooth: hipMemsetAsync(status) failed");
  SmoothArgs a{obs,    obs_dtype, B,  T,  E,         n,     r,  sb,      st,    se,
               sj,     mode == EKS_MEDIAN ? 1 : 0,  params, out, ob, ot, oj, ms,    nll,
               (char *)workspace, workspace_bytes, model_flags, al, status, s};
  a.t_base = t_base;
  a.T_total = T_total;
  a.phase = phase;
  a.seg_in = seg_in;
  a.seg_out = seg_out;
  a.wait_ticks = g_wait_ticks;
  if (rt) return launch_rt(a);  // model_flags are promises only: the general kernel serves all
  long long L = (out && phase == 0) ? chunk_len_smooth(B, T, r) : chunk_len(B, T, r);
  if (L >= T) L = (T + 7) / 8 * 8;
  if (r == 2 && n == 2) return launch_22(a, al, L);
  if (n == 4) return launch_34(a, al, L);
  if (n == 6) return launch_36(a, al, L);
  if (n == 12) return launch_312(a, al, L);
  if (n == 16) return launch_316(a, al, L);
  return launch_38(a, al, L);
}

int eks_smooth(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
               int64_t sb, int64_t st, int64_t se, int64_t sj, int mode, const double *params,
               double *out, int64_t ob, int64_t ot, int64_t oj, double *ms, double *nll,
               void *workspace, size_t workspace_bytes, int model_flags, int algo,
               int32_t *status, void *stream) {
  clear_err();
  return smooth_call(obs, obs_dtype, B, T, E, n, r, sb, st, se, sj, mode, params, out, ob, ot,
                     oj, ms, nll, workspace, workspace_bytes, model_flags, algo, status, stream,
                     0, T, 0, nullptr, nullptr);
}

size_t eks_smooth_seg_workspace_bytes(int64_t B, int64_t T, int n, int r) {
  if (B <= 0 || T <= 0 || r < 1 || n < 1) return 0;
  return make_plan(B, T, r, n, chunk_len(B, T, r)).total;
}

int eks_smooth_seg(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
                   int64_t sb, int64_t st, int64_t se, int64_t sj, int mode,
                   const double *params, double *out, int64_t ob, int64_t ot, int64_t oj,
                   double *ms, double *nll, void *workspace, size_t workspace_bytes,
                   int model_flags, int32_t *status, int64_t t_base, int64_t T_total, int phase,
                   const double *seg_in, double *seg_out, void *stream) {
  clear_err();
  if (phase < 1 || phase > 3) return set_err(EKS_ERR_ARG, "eks_smooth_seg: phase must be 1..3");
  if (t_base < 0 || t_base + T > T_total)
    return set_err(EKS_ERR_ARG, "eks_smooth_seg: frames [%lld, %lld) outside [0, %lld)",
                   (long long)t_base, (long long)(t_base + T), (long long)T_total);
  if ((phase == 1 || (phase == 2 && out)) && !seg_out)
    return set_err(EKS_ERR_ARG, "eks_smooth_seg: seg_out needed");
  if (phase == 2 && !out && !nll)
    return set_err(EKS_ERR_ARG, "eks_smooth_seg: phase 2 needs out (smooth) or nll (filter only)");
  if (phase == 2 && t_base > 0 && !seg_in)
    return set_err(EKS_ERR_ARG, "eks_smooth_seg: phase 2 of a later segment needs the state");
  if (phase == 3 && t_base + T < T_total && !seg_in)
    return set_err(EKS_ERR_ARG, "eks_smooth_seg: phase 3 of an earlier segment needs the mean");
  if (phase == 3 && !out) return set_err(EKS_ERR_ARG, "eks_smooth_seg: phase 3 needs out");
  return smooth_call(obs, obs_dtype, B, T, E, n, r, sb, st, se, sj, mode, params, out, ob, ot,
                     oj, phase == 3 ? ms : nullptr, nll, workspace, workspace_bytes,
                     model_flags, 2, status,
                     stream, t_base, T_total, phase,
                     phase == 2 && t_base == 0 ? nullptr
                     : (phase == 3 && t_base + T == T_total ? nullptr : seg_in),
                     seg_out);
}

int64_t eks_debug_set(int key, int64_t value) {
  clear_err();
  switch (key) {
    case EKS_DBG_WAIT_US: {
      const long long prev = g_wait_ticks < 0 ? -1 : g_wait_ticks / (kWallHz / 1000000);
      g_wait_ticks = value == 0 ? kDefaultWaitTicks : value < 0 ? -1 : value * (kWallHz / 1000000);
      return prev;
    }
    case EKS_DBG_A3_SLICE_BYTES: {
      const long long prev = g_a3_slice_bytes;
      g_a3_slice_bytes = value > 0 ? value : 0;
      return prev;
    }
    case EKS_DBG_A3_MODE: {
      const long long prev = g_a3_mode;
      g_a3_mode = value > 0 ? value : 0;
      return prev;
    }
    case EKS_DBG_A3_LB: {
      const long long prev = g_a3_lb;
      g_a3_lb = value == 1 || value == 2 ? value : 0;
      return prev;
    }
    case EKS_DBG_RT_FORM: {
      const long long prev = g_rt_form;
      g_rt_form = value == 1 || value == 2 ? value : 0;
      return prev;
    }
    case EKS_DBG_FIT_SELECT: {
      const long long prev = g_fit_select;
      g_fit_select = value == 1 || value == 2 ? value : 0;
      return prev;
    }
    default: return set_err(EKS_ERR_ARG, "eks_debug_set: unknown key %d", key), -1;
  }
}

int eks_seg_combine(int kind, int64_t B, int nseg, int self, int r, const double *in,
                    double *out, int32_t *status, void *stream) {
  clear_err();
  if (!in || !out) return set_err(EKS_ERR_ARG, "eks_seg_combine: NULL pointer");
  if (kind != 0 && kind != 1) return set_err(EKS_ERR_ARG, "eks_seg_combine: kind 0 or 1");
  if (nseg < 1 || self < 0 || self >= nseg) return set_err(EKS_ERR_ARG, "eks_seg_combine: bad self");
  if (B <= 0) return EKS_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (r) {
    case 2: return launch_seg_combine<2>(kind, B, nseg, self, in, out, status, s);
    case 3: return launch_seg_combine<3>(kind, B, nseg, self, in, out, status, s);
    default: return set_err(EKS_ERR_UNSUPPORTED, "eks_seg_combine: r=%d not compiled in", r);
  }
}

}  // extern "C"
