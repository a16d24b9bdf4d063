/*
 * eks_hip.h -- C ABI of libeks_hip.so, the MI355X (gfx950) ensemble Kalman
 * smoother.  Plain pointers and sizes only: no torch or numpy types.
 *
 * The reference (erialc-cal/eks, Python) has no FFI; its boundary is the four
 * Python functions of eks/ensemble_kalman.py.  Each entry point below states
 * which of them it replaces.  The Python package eks_amd binds these symbols
 * with ctypes (see INTEGRATION.md for the binding a maintainer of the
 * reference would add).
 *
 * Conventions
 *   - Every array argument is a DEVICE pointer (hipMalloc'd / torch cuda
 *     memory) unless the comment says otherwise.  Calls are stream-ordered on
 *     `stream` (a hipStream_t passed as void*; NULL = the null stream) and do
 *     not synchronise; they never allocate, so they can be captured in a
 *     hipGraph.
 *   - Floating point is float64 ("f64") throughout the recursions; member
 *     observations may be f32 or f64 (EKS_F32 / EKS_F64).
 *   - Matrices are row-major.  Batched arrays carry a leading trajectory
 *     index b in [0, B); a "trajectory" is one (video, keypoint) series.
 *   - Return value: EKS_OK or an error code; eks_last_error() gives the text
 *     (thread-local).  Numerical failures are reported per trajectory in the
 *     optional int32 `status` array (device, length B), a bit mask:
 *       0 = ok
 *       EKS_STATUS_SINGULAR   a matrix the reference would hand to
 *                             np.linalg.solve was singular (the reference
 *                             raises LinAlgError there)
 *       EKS_STATUS_BAD_MODEL  a model_flags promise (A or C = identity, the
 *                             pupil structure) does not hold for this
 *                             trajectory's parameters
 *       EKS_STATUS_SCAN       the time-parallel scan could not form a chunk
 *                             summary (singular Q with exact observations);
 *                             rerun that batch with algo = 1
 *     NaNs propagate exactly as in numpy and are not an error.
 */
#ifndef EKS_HIP_H
#define EKS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  EKS_OK = 0,
  EKS_ERR_ARG = 1,         /* bad size / NULL pointer / bad mode */
  EKS_ERR_UNSUPPORTED = 2, /* (r, n, E) combination not compiled in */
  EKS_ERR_HIP = 4          /* a HIP runtime call failed */
};

/* per-trajectory status bits */
enum { EKS_STATUS_SINGULAR = 1, EKS_STATUS_BAD_MODEL = 2, EKS_STATUS_SCAN = 4 };

/* model structure promises for eks_smooth (verified per trajectory) */
enum { EKS_MODEL_A_IDENTITY = 1, EKS_MODEL_C_IDENTITY = 2, EKS_MODEL_PUPIL = 4 };

enum { EKS_F32 = 0, EKS_F64 = 1 };
/* eks_smooth input that is not member predictions but the ensemble output
 * itself, as written by eks_fit (yev != NULL): y / ev planes, y float32
 * (EKS_YEV32) or float64 (EKS_YEV64); see eks_yev_bytes. */
enum { EKS_YEV32 = 2, EKS_YEV64 = 3 };
enum { EKS_MEDIAN = 0, EKS_MEAN = 1 };

/* Last error message of the calling thread ("" if none). */
const char *eks_last_error(void);

/* Library ABI version (major*100 + minor). */
int eks_version(void);

/* Largest state / observation / ensemble sizes the kernels accept. */
int eks_max_latent(void);
int eks_max_obs(void);
int eks_max_members(void);

/*
 * eks_ensemble -- replaces eks/ensemble_kalman.py:4-57 `ensemble()`.
 *
 * Member observation x(b, t, e, j) is read from
 *     obs[b*sb + t*st + e*se + j*sj]      (strides in ELEMENTS, any layout)
 * for b < B, t < T, e < E, j < n.  For every (b, t, j):
 *     preds = median_e x   (mode EKS_MEDIAN; mean of the two middle values
 *                            for even E, as np.median)  or  mean_e x
 *     vars  = var_e(x, ddof=0) / E     (in both modes, quirk of :46)
 * A NaN among the members makes both outputs NaN (np.median / np.var).
 * preds / vars: (B, T, n) contiguous f64.
 */
int eks_ensemble(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n,
                 int64_t sb, int64_t st, int64_t se, int64_t sj, int mode,
                 double *preds, double *vars, void *stream);

/*
 * eks_forward -- replaces eks/ensemble_kalman.py:59-107 `filtering_pass()`
 * (and the kalman_dot calls it makes, :110-117), batched over B trajectories.
 *
 * Inputs (all f64, contiguous):
 *   y  (B, T, n)   observations        ev (B, T, n)  ensemble variances
 *   m0 (B, r)      S0 (B, r, r)        A (B, r, r)   Q (B, r, r)   C (B, n, r)
 *   R  (B, n, n) or NULL: the caller's R matrix.  As in the reference its
 *      diagonal is replaced by ev[t] at every step; NULL means R is diagonal.
 *      This function does not write R (the Python shim reproduces the
 *      in-place mutation on the host).
 *   params_shared: if nonzero, m0/S0/A/Q/C/R hold ONE trajectory's values
 *      used for all b (batch stride 0).
 * Outputs (any may be NULL):
 *   mf (B, T, r)   Vf (B, T, r, r)   S (B, T, r, r) -- S[t] = A Vf[t] A^T + Q,
 *      the covariance predicted for step t+1; S[T-1] = 0 as in the reference.
 *   nll (B) -- the Gaussian innovation negative log-likelihood
 *      (the reference has no counterpart).
 *   status (B) int32 -- see above.
 */
int eks_forward(int64_t B, int64_t T, int n, int r, const double *y, const double *ev,
                const double *m0, const double *S0, const double *A, const double *Q,
                const double *C, const double *R, int params_shared, double *mf, double *Vf,
                double *S, double *nll, int32_t *status, void *stream);

/*
 * eks_backward -- replaces eks/ensemble_kalman.py:120-164 `smooth_backward()`.
 *   mf (B,T,r), Vf (B,T,r,r), S (B,T,r,r), A (B,r,r) (shared if params_shared)
 *   -> ms (B,T,r), Vs (B,T,r,r), CV (B,T-1,r,r); any output may be NULL.
 * J_t = solve(S[t], A Vf[t])^T, exactly as :158 (Q, C and y are unused by
 * the reference and are not arguments here).
 */
int eks_backward(int64_t B, int64_t T, int r, const double *mf, const double *Vf,
                 const double *S, const double *A, int params_shared, double *ms, double *Vs,
                 double *CV, int32_t *status, void *stream);

/*
 * eks_kalman_dot -- replaces eks/ensemble_kalman.py:110-117 `kalman_dot()`:
 *   out (r, k) = V C^T (R + C V C^T)^{-1} x,  x (n, k), V (r, r), C (n, r), R (n, n).
 * k = 1 for the vector form.  Single problem, f64.
 */
int eks_kalman_dot(int n, int r, int k, const double *x, const double *V, const double *C,
                   const double *R, double *out, int32_t *status, void *stream);

/*
 * Packed per-trajectory model for the fused smoother: for each b, P doubles
 *   [ m0 (r) | S0 (r*r) | A (r*r) | Q (r*r) | C (n*r) | offset (n) ]
 * with P = eks_param_len(n, r).  `offset` is added to C ms[t] on output (the
 * camera / keypoint means the wrappers subtract before filtering and add back
 * after: eks/multiview_pca_smoother.py:698-700, :756-765;
 * eks/pupil_smoother.py:158-172, :197).
 */
int64_t eks_param_len(int n, int r);

/*
 * eks_smooth -- the fused hot path: ensemble (eks_ensemble) -> centre
 * (y = preds - offset) -> forward filter -> RTS backward -> projection
 * out = C ms + offset, i.e. eks/ensemble_kalman.py:4-164 plus
 * eks/multiview_pca_smoother.py:745 / eks/pupil_smoother.py:190, in one call
 * for B trajectories with R diagonal (R_t = diag(ev[t])).
 *
 *   obs      member observations, strides as eks_ensemble
 *   params   (B, P) f64 packed models (see eks_param_len)
 *   out      smoothed observations out(b,t,j) = out[b*ob + t*ot + j*oj] (f64);
 *            NULL = filter only: just the NLL (requires nll, ms must be NULL),
 *            e.g. to score candidate models in a parameter sweep
 *   ms       (B, T, r) contiguous smoothed latents, or NULL
 *   nll      (B) or NULL
 *   model_flags  EKS_MODEL_A_IDENTITY / EKS_MODEL_C_IDENTITY: the caller
 *            promises A = I (and C = I, r = n) for every trajectory, which
 *            selects kernels that skip those products (single-view: both;
 *            multi-camera: A).  EKS_MODEL_PUPIL (r = 3, n = 8): C is the
 *            pupil measurement matrix of eks/pupil_smoother.py:150-153 (rows
 *            in the order top x, y, bottom x, y, right x, y, left x, y) and A,
 *            Q are diagonal (:140-147): sparse updates, the two pairs of
 *            equal rows folded into one observation each.  Violations are
 *            flagged in `status` by the compiled kernels (algos 1-3).  The
 *            runtime-n kernel (algo 4) runs the general model whatever the
 *            flags say: it neither uses nor checks them, so it never sets
 *            EKS_STATUS_BAD_MODEL (its results are those of the general
 *            model, i.e. correct for any A, C).
 *   workspace / workspace_bytes: device scratch of at least
 *            eks_smooth_workspace_bytes(...) bytes (not zeroed by caller).
 *   algo     0 = automatic, 1 = sequential (one lane per trajectory),
 *            2 = time-parallel chunked scan, three passes,
 *            3 = time-parallel, two passes over the members (chunk-level RTS
 *            maps; smoothing only: a filter-only call runs algo 2; needs
 *            E in 3..5 or y / ev planes, else algo 2),
 *            4 = the runtime-n kernels (any n <= 64, r = 2 or 3, members or
 *            y / ev planes): what every (r, n) without compiled kernels runs --
 *            (2, 2) and (3, 4|6|8|12|16) are compiled; e.g. the multi-camera model
 *            with V = 5, 7 or V > 8 cameras, n = 2V (the reference accepts any V:
 *            eks/multiview_pca_smoother.py:641-666).  eks_smooth_algo
 *            reports 4 for those shapes.  Many trajectories: one GPU lane
 *            per trajectory, sequential in time; few long ones: algo 2's
 *            time-parallel chunk scan with the n observation rows streamed
 *            one at a time (EKS_DBG_RT_FORM below).
 *   status   (B) int32, REQUIRED; zeroed by the call, then bit flags as above.
 */
size_t eks_smooth_workspace_bytes(int64_t B, int64_t T, int n, int r, int E, int algo);
int eks_smooth(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
               int64_t sb, int64_t st, int64_t se, int64_t sj, int mode, const double *params,
               double *out, int64_t ob, int64_t ot, int64_t oj, double *ms, double *nll,
               void *workspace, size_t workspace_bytes, int model_flags, int algo,
               int32_t *status, void *stream);

/* Chunk length the time-parallel algorithm uses for (B, T, r) (0 if algo 1
 * would be chosen automatically).  Exposed for tests and DESIGN.md. */
int64_t eks_smooth_chunk_len(int64_t B, int64_t T, int r);

/* The algorithm (1, 2 or 3) an eks_smooth call with these arguments runs
 * (smoothing calls; a filter-only call that resolves to 3 runs 2).  Exposed
 * for the bench line and tests. */
int eks_smooth_algo(int64_t B, int64_t T, int n, int r, int E, int algo);

/*
 * Time-sharded smoothing (SURVEY.md §8(e) "shard the time axis"): the frames
 * of every trajectory are split into nseg contiguous segments, segment k on
 * rank k, and the chunked scan of eks_smooth runs per segment in three
 * phases with two exchanges of per-trajectory aggregates between them (the
 * reference has no equivalent: its smoother is one sequential loop,
 * eks/ensemble_kalman.py:59-164).  Per segment of T frames starting at t_base of
 * T_total, with the arguments of eks_smooth (obs/out point at the segment's
 * own frames):
 *   phase 1: seg_out (B, EL), EL = R*R + 2R + R(R+1) <- the segment's aggregate
 *            filtering element (A, b, C, eta, J; C and J packed) (zeroes status);
 *   -> all-gather the elements, eks_seg_combine(kind 0) -> state (B, R+R(R+1)/2)
 *   phase 2: seg_in = that state (NULL on segment 0); seg_out (B, R*R + R) <-
 *            the segment's aggregate smoothing map ms_in -> ms_first;
 *   -> all-gather the maps, eks_seg_combine(kind 1) -> mean (B, R)
 *            (filter only: out = NULL, nll != NULL -> nll = the segment's share,
 *            no map, no phase 3)
 *   phase 3: seg_in = the smoothed mean entering the next segment (NULL on
 *            the last); writes out, ms (B, T, r) if not NULL, and nll = the
 *            segment's share, whose sum over segments is eks_smooth's nll.
 * The workspace (eks_smooth_seg_workspace_bytes) must survive phases 1..3.
 * Results equal eks_smooth's to rounding (different association order).
 */
size_t eks_smooth_seg_workspace_bytes(int64_t B, int64_t T, int n, int r);
int eks_smooth_seg(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
                   int64_t sb, int64_t st, int64_t se, int64_t sj, int mode,
                   const double *params, double *out, int64_t ob, int64_t ot, int64_t oj,
                   double *ms, double *nll, void *workspace, size_t workspace_bytes,
                   int model_flags, int32_t *status, int64_t t_base, int64_t T_total, int phase,
                   const double *seg_in, double *seg_out, void *stream);
/* kind 0: in = nseg gathered elements (nseg, B, EL) -> out = state entering
 * segment `self`; kind 1: in = gathered maps (nseg, B, R*R+R) -> out = mean
 * entering segment self+1 (zeros when self is last).  status may be NULL. */
int eks_seg_combine(int kind, int64_t B, int nseg, int self, int r, const double *in,
                    double *out, int32_t *status, void *stream);

/*
 * eks_newton_filter -- replaces eks/newton_eks.py:115-148
 * `kalman_newton_recursive(y, mu0, S0, A, B, ensemble_vars, E, max_iter)`
 * for B trajectories (one lane each): information-form filter with
 * q[0] = mu0, P0 = inv(S0), D_t = diag(ensemble_vars[t]), P carried over
 * between the max_iter iterations, q updated in place.
 *   y, ev   (B, T, n) f64 contiguous (centred observations, ensemble variances)
 *   mu0 (r), S0 (r, r), A (r, r), Bm (n, r), E (r, r): per trajectory
 *           (b-strided) or, with params_shared = 1, one model for all
 *   q       (B, T, r) f64 output
 *   status  (B) int32 or NULL: EKS_STATUS_SINGULAR where the reference's
 *           np.linalg.inv would raise (zero variance, singular S0 / info).
 * The reference's loss vector is identically 0 (q is updated in place), so
 * it is not produced here.
 */
int eks_newton_filter(int64_t B, int64_t T, int n, int r, const double *y, const double *ev,
                      const double *mu0, const double *S0, const double *A, const double *Bm,
                      const double *E, int params_shared, int max_iter, double *q,
                      int32_t *status, void *stream);

/*
 * eks_fit -- batched model fit (F2), replacing the per-keypoint host fit of
 * eks/multiview_pca_smoother.py:684-731 (kind EKS_FIT_MULTICAM: PCA with r
 * axes, r = 3 there) and the single-view model of SURVEY.md §8 A6 (kind
 * EKS_FIT_SINGLEVIEW, r == n): good frames = max_j ensemble variance <=
 * np.percentile(., quantile_keep); offset = mean of their ensemble
 * predictions; S0 = diag(var of the good latents); Q = smooth_param *
 * cov(diff(good latents)) (ddof 1); A = I; C = I or the principal axes.
 * Writes params (B, eks_param_len(n, r)) for eks_smooth.  obs and strides
 * as eks_smooth (T >= 2).  status (B) or NULL: EKS_STATUS_SINGULAR where no
 * frame was kept (NaN threshold).  workspace: eks_fit_workspace_bytes.
 * n even, 2 <= n <= 16 (coordinate pairs: single view, or 2V for V <= 8
 * cameras; n > 8 runs the wide kernels and needs EKS_FIT_MULTICAM with
 * r = 3; the per-keypoint multi-camera wrappers fit on the host for any V).
 */
enum { EKS_FIT_SINGLEVIEW = 1, EKS_FIT_MULTICAM = 2 };
size_t eks_fit_workspace_bytes(int64_t B, int64_t T, int n);
int eks_fit(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
            int64_t sb, int64_t st, int64_t se, int64_t sj, int mode, int kind,
            double smooth_param, double quantile_keep, double *params, void *workspace,
            size_t workspace_bytes, int32_t *status, void *yev, void *stream);

/*
 * Ensemble hand-off from eks_fit to eks_smooth (fit + smooth reading the
 * member predictions once): with yev != NULL (eks_yev_bytes(B, T, n,
 * obs_dtype, E, mode) bytes of device memory) eks_fit also writes the
 * ensemble output -- y planes [t*n + j][b] (float32 when every y is a member
 * value: float32 members, median, E in {3, 5}; else float64), then ev planes
 * (float64) at a 256-byte aligned offset -- and eks_smooth called with
 * obs = yev and obs_dtype = eks_yev_dtype(obs_dtype, E, mode)
 * (EKS_YEV32 / EKS_YEV64; strides ignored) smooths from it.  Results are
 * bit-identical to eks_smooth on the members.
 */
int eks_yev_dtype(int obs_dtype, int E, int mode);
size_t eks_yev_bytes(int64_t B, int64_t T, int n, int obs_dtype, int E, int mode);

/*
 * eks_interp1d -- linear resampling for the asynchronous two-camera paw
 * smoother (F4), replacing the scipy.interpolate.interp1d(kind='linear')
 * calls of eks/multiview_pca_smoother.py:86-96 (which delegate to np.interp
 * for 1-D float64 columns): out(q, c) = y interpolated at xq[q] for each of
 * the ncol columns of y (element (k, c) at y[k*sy_row + c*sy_col]), sample
 * times x (nx, ascending).  Bit-identical to np.interp.  status (nq) or NULL:
 * EKS_STATUS_BAD_MODEL for queries outside [x[0], x[nx-1]] (interp1d raises
 * there; the output is NaN).  Device pointers, f64.
 */
int eks_interp1d(const double *x, int64_t nx, const double *y, int64_t ncol, int64_t sy_row,
                 int64_t sy_col, const double *xq, int64_t nq, double *out, int64_t so_row,
                 int64_t so_col, int32_t *status, void *stream);

/*
 * Test and fault-injection settings (process-wide, not part of the
 * smoother's semantics; tests only).  Returns the previous value.
 *   EKS_DBG_WAIT_US        bound of every in-launch chain wait of the
 *                          time-parallel passes, in microseconds of wall-clock
 *                          time (0 = the default, 1 s).  A wait that reaches
 *                          it gives up, flags its trajectories EKS_STATUS_SCAN
 *                          and lets the launch finish.  -1 = every wait gives
 *                          up at once (drives the time-out path).
 *   EKS_DBG_A3_SLICE_BYTES largest member byte offset span of one algo-3
 *                          launch (0 = 4 GB, the buffer descriptor's range);
 *                          a smaller span forces the batch slicing.
 *   EKS_DBG_FIT_SELECT     eks_fit's percentile selection: 0 = automatic
 *                          (split over row segments for B < 512 rows), 1 =
 *                          one block per row, 2 = split (both must give the
 *                          same threshold and kept-frame mask).  The
 *                          workspace size follows the setting.
 *   EKS_DBG_A3_MODE        retired (round 5): algo 3 has one launch form,
 *                          the forward pass then the backward pass; the key
 *                          still round-trips its value and changes nothing.
 *   EKS_DBG_A3_LB          algo 3's backward look-back: 0 = automatic (batches
 *                          of at most 48 64-trajectory groups), 1 = never,
 *                          2 = always.  Results are bit-identical.
 *   EKS_DBG_RT_FORM        the runtime-n smoother (algo 4): 0 = automatic
 *                          (time-parallel when the trajectories alone do not
 *                          fill the GPU), 1 = one lane per trajectory, 2 =
 *                          time-parallel.  Results agree to rounding; set it
 *                          before eks_smooth_workspace_bytes.
 */
enum { EKS_DBG_WAIT_US = 1, EKS_DBG_A3_SLICE_BYTES = 2, EKS_DBG_FIT_SELECT = 3,
       EKS_DBG_A3_MODE = 4, EKS_DBG_A3_LB = 5, EKS_DBG_RT_FORM = 6 };
int64_t eks_debug_set(int key, int64_t value);

/*
 * Profiling aid (not part of the smoother's semantics).  After
 * eks_profile_begin(max_calls), each eks_smooth call on this thread records
 * a hipEvent on its stream before each of its kernels and after the last one
 * (at most max_calls calls).  eks_profile_end synchronises on those events,
 * writes the per-kernel average milliseconds over the recorded calls into
 * kernel_ms[0..k) and the kernel names into names[k * name_len] (host
 * buffers), switches profiling off and returns k (kernels per call).
 */
int eks_profile_begin(int max_calls);
int eks_profile_end(double *kernel_ms, char *names, int max_kernels, int name_len);

#ifdef __cplusplus
}
#endif
#endif /* EKS_HIP_H */
