// F2: batched model fit on the device -- the step before the smoother.
//
// Replaces the per-keypoint host fit of
//   eks/multiview_pca_smoother.py:684-731   (multi-camera PCA model)
//   SURVEY.md §8 A6                         (single-view model, same template
//                                            without the PCA)
// for B trajectories at once:
//   good   = frames whose max_j ensemble variance <= np.percentile(., q)
//   offset = mean of the good ensemble predictions            (:698-700)
//   single-view: S0 = diag(var(good y)), Q = s cov(diff(good y)), A = C = I
//   multicam:    W = top-r principal axes of the good y       (:708)
//                S0 = diag(var(good y W^T)), Q = s W cov(diff(good y)) W^T,
//                A = I, C = W^T                               (:722-730)
// written straight into the packed parameter rows eks_smooth reads.
//
// Kernels (all f64):
//   k_fit_worst   one lane per (trajectory, chunk of frames): ensemble of
//                 every frame (same code as eks_ensemble), v_t = max_j var
//                 stored trajectory-major
//   k_fit_select  one 256-thread block per trajectory: exact order
//                 statistics v_(lo), v_(lo+1) by MSD radix select on the
//                 IEEE bit patterns (12-bit digits, LDS histograms, early
//                 exit once the candidate is unique), then numpy's linear
//                 interpolation -> threshold, and the kept-frame bit mask
//   k_fit_accum   one lane per (trajectory, chunk): ensemble again (or the y
//                 hand-off plane + the frame mask), keep frames with
//                 v_t <= threshold, chunk sums of y - K and its outer
//                 products (K = the trajectory's frame-0 ensemble, a shift
//                 that keeps the one-pass sums well conditioned), of the
//                 differences between consecutive kept frames and their
//                 outer products, first / last kept y
//   k_fit_merge   sums of the chunk partials in order (plain additions; the
//                 kept-frame pair straddling two chunks added where they meet)
//   k_fit_final   one wave per trajectory: means / scatter matrices from the
//                 sums, PCA by cyclic Jacobi on the n x n scatter matrix,
//                 parameter rows
// The results agree with the numpy fit to rounding (different summation
// order), which moves the smoothed outputs by ~1e-12 px.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "../../include/eks_hip.h"
#include "eks_common.hpp"
#include "ensemble.hpp"
#include "tuning.hpp"

namespace eks {

namespace {

constexpr int kDigitBits = 12;
constexpr int kBins = 1 << kDigitBits;

// ensemble of one frame: y[j] = median/mean, v = max_j var (NaN-propagating
// like np.max)
template <int E, int N, typename T>
EKS_DEV void frame_ensemble(const T *p, long long se, long long sj, int Ert, bool median,
                            double (&y)[N], double (&ev)[N], double &v) {
  v = -1.0;
  bool nan = false;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double avg, var;
    if constexpr (E > 0) {
      T raw[E];
#pragma unroll
      for (int e = 0; e < E; ++e) raw[e] = p[j * sj + e * se];
      ensemble_reduce<E, T>(raw, median, avg, var);
    } else {
      ensemble_reduce_rt<T>(p + j * sj, se, Ert, median, avg, var);
    }
    y[j] = avg;
    ev[j] = var;
    nan |= (var != var);
    v = var > v ? var : v;
  }
  if (nan) v = __builtin_nan("");
}

template <int E, int N, typename T>
EKS_DEV void frame_ensemble(const T *p, long long se, long long sj, int Ert, bool median,
                            double (&y)[N], double &v) {
  double ev[N];
  frame_ensemble<E, N, T>(p, se, sj, Ert, median, y, ev, v);
}

// y / ev hand-off planes (eks_smooth EKS_YEV32 / EKS_YEV64 input):
// time-major [t*N + j][b], y of type YT then ev (f64) 256-byte aligned
struct YevOut {
  void *y = nullptr;
  double *ev = nullptr;
};

struct FitShape {
  long long B, T;
  int NC;          // chunks per trajectory
  long long Lc;    // frames per chunk
};

// the shift K of trajectory b (its frame-0 ensemble y, n values), written by
// k_fit_accum's chunk-0 lanes for k_fit_final
struct FitShift {
  double *K;
};

// words the worst pass zeroes on the side (the split selection's histograms
// and row states: no memset launch before k_sel_hist)
struct ZeroSpan {
  unsigned *p = nullptr;
  long long n = 0;
  EKS_DEV void run() const {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
      p[i] = 0u;
  }
};

constexpr int kTile = 16;  // frames per register tile: one 128-byte row segment per lane

// the same from E x N member values already in registers (raw[j][e])
template <int E, int N, typename T>
EKS_DEV void frame_ensemble_raw(const T (&raw)[N][E], bool median, double (&y)[N],
                                double (&ev)[N], double &v) {
  v = -1.0;
  bool nan = false;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double avg, var;
    ensemble_reduce<E, T>(raw[j], median, avg, var);
    y[j] = avg;
    ev[j] = var;
    nan |= (var != var);
    v = var > v ? var : v;
  }
  if (nan) v = __builtin_nan("");
}

// frames of member loads in flight per lane in k_fit_worst (compiled E: a
// register ring; 4 x 10 loads at E = 5, n = 2.  Round 4's form loaded one
// column of E members and waited for it: 5 loads in flight per wave, 4.2 TB/s)
// The depth follows the frame's size (round 6, advisor finding): ~160 bytes
// of member values per lane in flight (4 frames at n = 2 float32, 2 at
// n = 4, 1 at n >= 6 or E x n x 8 > 80 bytes) -- a fixed depth of 4 held
// 4 E n values in registers and spilled every n >= 4 instantiation into
// AGPRs at one wave per SIMD (n = 8, E = 5: 256 VGPRs + 101 AGPRs).
#ifndef EKS_WORST_D  // A/B builds only (tools/build_cur.sh): the n = 2 depth
#define EKS_WORST_D 4
#endif
template <int E, int N, typename T>
constexpr int worst_depth() {
  constexpr int bytes = (E > 0 ? E : 1) * N * (int)sizeof(T);
  constexpr int d = 160 / bytes;
  return d >= EKS_WORST_D ? EKS_WORST_D : d >= 2 ? 2 : 1;
}
static_assert(16 % EKS_WORST_D == 0, "the ring slots repeat every register tile");

template <int E, int N, typename T, typename YT>
__global__ __launch_bounds__(256) void k_fit_worst(const T *__restrict__ obs, FitShape sh,
                                                   long long sb, long long st, long long se,
                                                   long long sj, int Ert, int median,
                                                   double *__restrict__ worst, YevOut yo,
                                                   FitShift ks, ZeroSpan zs) {
  zs.run();
  // each lane computes kTile consecutive frames of its (trajectory, chunk)
  // into LDS; the block then writes the trajectory-major rows as whole
  // 128-byte segments (16 lanes per segment) instead of one 8-byte store
  // per lane per frame
  __shared__ double tile[256][kTile + 1];
  __shared__ long long base[256];
  const long long lane = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const bool active = lane < sh.B * sh.NC;
  long long b = 0, t0 = 0, t1 = 0;
  if (active) {
    b = lane % sh.B;
    t0 = (lane / sh.B) * sh.Lc;
    t1 = t0 + sh.Lc < sh.T ? t0 + sh.Lc : sh.T;
  }
  const T *pb = obs + b * sb;
  const long long ntiles = sh.Lc / kTile;  // Lc is a multiple of kTile
  // one frame's outputs: the y / ev hand-off planes, the trajectory's shift K
  auto frame_out = [&](long long u, const double (&y)[N], const double (&ev)[N]) {
    if (u == 0)  // the trajectory's shift for the accumulation (frame 0's ensemble)
#pragma unroll
      for (int j = 0; j < N; ++j) ks.K[b * N + j] = y[j];
    if (yo.y)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        ((YT *)yo.y)[(u * N + j) * sh.B + b] = (YT)y[j];
        yo.ev[(u * N + j) * sh.B + b] = ev[j];
      }
  };
  // compiled E: the lane's frames stream through a ring kWorstD frames deep
  // (reads past the lane's last frame are clamped to it: cache hits)
  constexpr int RE = E > 0 ? E : 1;
  constexpr int kWorstD = worst_depth<E, N, T>();
  T ring[kWorstD][N][RE];
  auto fetch = [&](int slot, long long u) {
    u = u < t1 ? u : t1 - 1;
    const T *p = pb + u * st;
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int e = 0; e < RE; ++e) ring[slot][j][e] = p[j * sj + e * se];
  };
  if constexpr (E > 0)
    if (active && t1 > t0)
#pragma unroll
      for (int q = 0; q < kWorstD; ++q) fetch(q, t0 + q);
  for (long long kt = 0; kt < ntiles; ++kt) {
    const long long t = t0 + kt * kTile;
    if (active && t + kTile <= t1) {
#pragma unroll
      for (int k = 0; k < kTile; ++k) {
        double y[N], ev[N];
        if constexpr (E > 0) {
          const int slot = k % kWorstD;
          T raw[N][RE];
#pragma unroll
          for (int j = 0; j < N; ++j)
#pragma unroll
            for (int e = 0; e < RE; ++e) raw[j][e] = ring[slot][j][e];
          fetch(slot, t + k + kWorstD);
          frame_ensemble_raw<RE, N, T>(raw, median != 0, y, ev, tile[threadIdx.x][k]);
        } else {
          frame_ensemble<E, N, T>(pb + (t + k) * st, se, sj, Ert, median != 0, y, ev,
                                  tile[threadIdx.x][k]);
        }
        frame_out(t + k, y, ev);
      }
      base[threadIdx.x] = b * sh.T + t;
    } else {
      base[threadIdx.x] = -1;
      if (active)
        for (long long u = t; u < t1; ++u) {  // ragged end of the last chunk
          double y[N], ev[N], v;
          frame_ensemble<E, N, T>(pb + u * st, se, sj, Ert, median != 0, y, ev, v);
          worst[b * sh.T + u] = v;
          frame_out(u, y, ev);
        }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 256 / 16; ++p) {
      const int r = p * 16 + (threadIdx.x >> 4), k = threadIdx.x & 15;
      const long long o = base[r];
      if (o >= 0) worst[o + k] = tile[r][k];
    }
    __syncthreads();
  }
}

// Apply f(key, index) to every key of a row, BLK threads, kSelU
// independent loads in flight per thread (memory-level parallelism for the global-memory
// passes).  The 64 lanes of a wave always hold 64 consecutive, 64-aligned
// indices, so a ballot inside f is one word of a frame bit mask -- as long as
// the whole wave runs the same loop: the unrolled loop's condition tests the
// wave's LAST index (i | 63), so near the end of a row a wave never splits
// between the unrolled body and the tail loop (a split wave would ballot in
// two halves, and the two writers of the mask word would overwrite each
// other's frames).
template <int BLK, int U = kSelU, typename K, typename F>
EKS_DEV void for_keys(const K *keys, long long n, F &&f) {
  static_assert(BLK % 64 == 0, "whole waves");
  long long i = threadIdx.x;
  for (; (i | 63) + (U - 1) * BLK < n; i += U * BLK) {
    K x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = keys[i + u * BLK];
#pragma unroll
    for (int u = 0; u < U; ++u) f(x[u], i + u * BLK);
  }
  for (; i < n; i += BLK) f(keys[i], i);
}

// Jacobi rotation (c, s) of the pair p < q that zeroes a_pq:
//   t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)), theta = (a_qq - a_pp) / (2 a_pq)
//     = sgn(theta) |h| / (|d| + sqrt(d^2 + h^2)),  d = a_qq - a_pp, h = 2 a_pq,
//   c = 1 / sqrt(t^2 + 1), s = t c,
// from the hardware reciprocal / reciprocal square root plus Newton steps
// (~22 dependent VALU ops; the IEEE form's three divisions and two square
// roots were ~700 cycles per round of the PCA's Jacobi -- k_fitw_final
// 0.100 ms at 6 cameras).  The rotation is exact to a few ulp; Jacobi's
// convergence does not depend on it.
EKS_DEV double nr_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
EKS_DEV double nr_rsq(double x) {  // x > 0
  double y = __builtin_amdgcn_rsq(x);
  double hx = 0.5 * x;
  y = y * fma(-hx * y, y, 1.5);
  return y * fma(-hx * y, y, 1.5);
}
// the PCA Jacobi's convergence bound on (off-diagonal / diagonal) squared
// mass: 1e-30 ~ n eps^2, the level rounding leaves (round 4: 1e-34)
#ifndef EKS_JACOBI_TOL
#define EKS_JACOBI_TOL 1e-30
#endif
constexpr double kJacobiTol = EKS_JACOBI_TOL;
EKS_DEV void jacobi_cs(double app, double aqq, double apq, double &c, double &s) {
  c = 1.0;
  s = 0.0;
  if (apq == 0.0) return;
  double d = aqq - app, h = 2.0 * apq;
  double x = fma(d, d, h * h);
  if (!(x >= 0x1p-1000 && x <= 0x1p1000)) {
    // |d|, |h| below ~1e-151 or above ~1e150: x under- / overflows and r
    // would be 0 * inf.  t is invariant under a common scaling of d and h,
    // so rescale both by the power of two of the larger (exact; the
    // matrices are pre-scaled by pca_scale, so this is a backstop)
    int e;
    (void)frexp(fmax(fabs(d), fabs(h)), &e);
    d = ldexp(d, -e);
    h = ldexp(h, -e);
    x = fma(d, d, h * h);
  }
  const double r = x * nr_rsq(x);  // sqrt(d^2 + h^2)
  double t = fabs(h) * nr_rcp(fabs(d) + r);
  if (d != 0.0 && ((d < 0.0) != (h < 0.0))) t = -t;  // theta < 0
  c = nr_rsq(fma(t, t, 1.0));
  s = t * c;
}

// The power of two 2^-e that brings the largest |entry| of the PCA's scatter
// matrix into [0.5, 1): the Jacobi then runs on exactly scaled entries (the
// rotations and the eigenvalue order are invariant under it; without it the
// squared off-diagonal mass of a matrix with entries below ~1e-154
// underflows to 0 and the sweeps stop before rotating).  m: the max |entry|
EKS_DEV int pca_scale(double m) {
  int e = 0;
  if (m > 0.0 && m <= __DBL_MAX__) (void)frexp(m, &e);
  return e;
}

// lane 0 of the wave's active lanes (the writer of a ballot word)
EKS_DEV bool first_active_lane() {
  return (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1;
}

// block-wide exclusive prefix sum of one value per thread (BLK threads)
template <int BLK>
EKS_DEV long long block_excl_scan(long long x, long long *tmp, long long &total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  long long inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) tmp[wave] = inc;
  __syncthreads();
  long long base = 0, tot = 0;
  for (int w = 0; w < BLK / 64; ++w) {
    base += w < wave ? tmp[w] : 0;
    tot += tmp[w];
  }
  __syncthreads();
  total = tot;
  return base + inc - x;
}

// k-th smallest (0-based) key of the row, MSD radix select over the bits
// below `top` (the keys' common prefix above it is `prefix`).  All threads
// call it and get the same result.  DB-bit digits: `hist` holds 2^DB bins.
template <class X>
struct nodeduce {
  using type = X;
};

template <int BLK, int DB = kDigitBits, typename K = uint64_t>
EKS_DEV K block_select(const K *keys, long long n, long long k, int top,
                       typename nodeduce<K>::type prefix,
                       unsigned *hist, uint64_t *su, long long *si) {
  constexpr int kBitsK = 8 * sizeof(K);
  K mask = top >= kBitsK - 1 ? K(0) : K(~((K(2) << top) - K(1)));  // bits above `top` fixed
  for (int hi_bit = top; hi_bit >= 0; hi_bit -= DB) {
    const int lo_bit = hi_bit - DB + 1 > 0 ? hi_bit - DB + 1 : 0;
    const int bits = hi_bit - lo_bit + 1;
    const unsigned nb = 1u << bits;
    for (unsigned i = threadIdx.x; i < nb; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for_keys<BLK>(keys, n, [&](K x, long long) {
      if ((x & mask) == prefix) atomicAdd(&hist[(x >> lo_bit) & (nb - 1)], 1u);
    });
    __syncthreads();
    // parallel scan of the histogram: thread i owns bins [i*per, (i+1)*per)
    const unsigned per = (nb + BLK - 1) / BLK;
    long long mine = 0;
    for (unsigned d = threadIdx.x * per; d < (threadIdx.x + 1) * per && d < nb; ++d)
      mine += hist[d];
    long long total;
    long long acc = block_excl_scan<BLK>(mine, si + 2, total);
    if (k >= acc && k < acc + mine) {  // exactly one thread
      unsigned d = threadIdx.x * per;
      while (acc + hist[d] <= k) acc += hist[d++];
      su[0] = (uint64_t)(prefix | (K(d) << lo_bit));
      si[0] = k - acc;
      si[1] = hist[d];
    }
    __syncthreads();
    prefix = (K)su[0];
    k = si[0];
    const long long left = si[1];
    mask |= K(nb - 1) << lo_bit;
    __syncthreads();
    if (left == 1 && lo_bit > 0) {  // the candidate is unique: find it
      if (threadIdx.x == 0) su[1] = ~0ull;
      __syncthreads();
      for_keys<BLK>(keys, n, [&](K x, long long) {
        if ((x & mask) == prefix) atomicMin((unsigned long long *)&su[1], (unsigned long long)x);
      });
      __syncthreads();
      const K r = (K)su[1];
      __syncthreads();
      return r;
    }
  }
  return prefix;
}

// One block per trajectory.  Pass 1 histograms the top digit (bits 50-62:
// exponent and first two mantissa bits; variances are >= 0 so bit patterns sort
// like values) over the row in global memory; pass 2 compacts the keys of
// the bin holding rank `lo` into LDS (with their frame indices) and sets the
// kept-frame bits of every frame below that bin; the remaining digits and the
// neighbouring order statistic are then resolved in LDS, and the bin's own
// frames are marked against the threshold there.  The frame mask
// (`kept`, 64 frames per word, trajectory-major, W words per row) is what
// k_fit_accum reads instead of the ev plane.  A bin larger than the LDS
// buffer falls back to selecting over the global row, and a row too long for
// 16-bit indices (or a threshold equal to a key above the bin) marks the
// frames in one more pass over the row.
//
// LDS (round 6): the top digit is 13 bits (bits 50-62) and the bin's
// candidates are compacted into the histogram's own LDS once the bin is
// known, so a 256-thread block needs ~20 KB instead of ~39 KB and a CU holds
// twice the rows in flight (the passes are latency bound per row: round 5's
// 512-thread and register-resident forms, with fewer rows per CU, were
// slower in proportion).  EKS_SEL_COMPACT=0 builds round 5's layout (12-bit
// digit, 3 072 candidates beside the histogram) for A/B runs.
#ifndef EKS_SEL_COMPACT
#define EKS_SEL_COMPACT 1
#endif
constexpr bool kSelCompact = EKS_SEL_COMPACT != 0;
constexpr int kSelTopBits = kSelCompact ? 13 : 12;  // top digit: bits 63-kSelTopBits .. 62
constexpr int kSelBins = 1 << kSelTopBits;
constexpr int kCand = kSelCompact ? 1536 : 3072;    // LDS candidates (+ 16-bit indices)
constexpr int kSelDigit = 8;       // digits of the in-LDS select (1 KB histogram)
// rows with 16-bit frame indices and an LDS frame mask (2 KB / 8 KB)
constexpr long long kLdsMaskT = kSelCompact ? 16384 : 65536;

// KPT > 0 (rows of at most BLK * KPT frames): the row is read ONCE, into
// KPT registers per thread, and both passes (histogram, compaction + mask)
// run over the registers -- round 4's form read the row from memory twice
// (1.93x the worst plane's bytes at config 4).  KPT = 0: the passes read
// the row from memory (longer rows).
// waves per SIMD the selection is compiled for (its VGPR budget: 64 at 8):
// the compact layout's ~20 KB of LDS allows 8 blocks of 256 threads per CU.
// Config 4 (17 408 rows of 10 000 frames), alternated on one box:
// k_fit_select 0.765-0.771 ms (round 5's layout, 4 blocks per CU) -> 0.565
// (compact, 6) -> 0.504-0.511 (compact, 8); profiles/r06/ab_fit/README.md
#ifndef EKS_SEL_WPE
#define EKS_SEL_WPE (EKS_SEL_COMPACT ? 8 : 1)
#endif
// key loads in flight per thread of the selection's row passes (compact
// layout: twice the blocks per CU, so half of kSelU keeps the bytes in flight)
#ifndef EKS_SEL_U
#define EKS_SEL_U 8
#endif
constexpr int kSelRowU = kSelCompact ? EKS_SEL_U : kSelU;
// The register-row form (KPT > 0: rows <= 4 096 frames read once into 16 keys
// per thread) is off by default since the compact layout: at T = 4 000 and
// 17 408 rows the two-read form at 8 rows per CU selects in 0.30 ms, the
// register form 0.33 ms at its own register budget (0.56 at 64 VGPRs, where
// it spills), round 5's 0.40 (profiles/r06/ab_fit/ab_short_rows.txt).
// EKS_SEL_REGROWS=1 builds it back for A/B runs.
#ifndef EKS_SEL_KPT_WPE
#define EKS_SEL_KPT_WPE 1
#endif
#ifndef EKS_SEL_REGROWS
#define EKS_SEL_REGROWS 0
#endif
template <int BLK, int KPT = 0>
__global__ __launch_bounds__(BLK, KPT > 0 ? EKS_SEL_KPT_WPE : EKS_SEL_WPE) void k_fit_select(const double *__restrict__ worst,
                                                    long long TT, long long lo, long long hi,
                                                    double g, double *__restrict__ thr,
                                                    uint64_t *__restrict__ kept, long long W) {
  // the top-digit histogram; after the bin is found the same LDS holds the
  // bin's candidates (compact layout) or the row's frame mask (round 5's).
  // Rows shorter than 65 536 frames (the 256-thread kernel) count in 16-bit
  // halves of the words.
  constexpr bool kPacked = BLK == 256 || BLK == 512;
  constexpr int kHistWords = kPacked ? kSelBins / 2 : kSelBins;
  constexpr int kCandBytes = kCand * (int)(sizeof(uint64_t) + sizeof(uint16_t));
  // compact layout: the candidates (keys, then 16-bit frame indices) reuse
  // the histogram's words once the bin is found; the frame mask has its own
  constexpr int kHistAlloc =
      kSelCompact && kCandBytes > kHistWords * 4 ? (kCandBytes + 3) / 4 : kHistWords;
  __shared__ __attribute__((aligned(16))) unsigned hist[kHistAlloc];
  auto hcount = [&](unsigned d) -> unsigned {
    return kPacked ? (hist[d >> 1] >> ((d & 1u) << 4)) & 0xffffu : hist[d];
  };
  __shared__ unsigned hsel[1 << kSelDigit];
  __shared__ uint64_t su[4];
  __shared__ long long si[2 + BLK / 64];
  __shared__ double sthr;
  __shared__ unsigned ncand;
  __shared__ int any_nan;
  uint64_t *cand;
  uint16_t *cidx;
  uint64_t *smask;
  if constexpr (kSelCompact) {
    static_assert(kCandBytes <= (int)sizeof(hist), "candidates fit the histogram's LDS");
    __shared__ uint64_t smask_own[kLdsMaskT / 64];
    cand = reinterpret_cast<uint64_t *>(hist);
    cidx = reinterpret_cast<uint16_t *>(cand + kCand);
    smask = smask_own;
  } else {
    __shared__ uint64_t cand_own[kCand];
    __shared__ uint16_t cidx_own[kCand];
    static_assert(kLdsMaskT / 64 * sizeof(uint64_t) <= sizeof(hist), "mask fits the histogram");
    cand = cand_own;
    cidx = cidx_own;
    smask = reinterpret_cast<uint64_t *>(hist);
  }
  const long long b = blockIdx.x;
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(worst + b * TT);
  uint64_t *krow = kept ? kept + b * W : nullptr;
  constexpr int lo_bit = 63 - kSelTopBits;
  // the row's keys in registers (KPT > 0): key threadIdx.x + u * BLK in
  // xr[u]; every load issued at once.  Past the row: +inf bit patterns
  // above every variance (never counted: the loops below test the index).
  constexpr int KR = KPT > 0 ? KPT : 1;
  uint64_t xr[KR];
  if constexpr (KPT > 0) {
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const long long i = threadIdx.x + (long long)u * BLK;
      xr[u] = i < TT ? keys[i] : ~0ull;
    }
  }
  // f(key, index) over the row: from the registers, or from memory
  auto row_keys = [&](auto &&f) {
    if constexpr (KPT > 0) {
#pragma unroll
      for (int u = 0; u < KPT; ++u) {
        const long long i = threadIdx.x + (long long)u * BLK;
        // whole waves run each u (indices of a wave are 64-aligned): the
        // ballots inside f see the wave's 64 frames, past-the-row lanes false
        if ((long long)(threadIdx.x & ~63u) + (long long)u * BLK < TT) f(xr[u], i, i < TT);
      }
    } else {
      for_keys<BLK, kSelRowU>(keys, TT, [&](uint64_t x, long long i) { f(x, i, true); });
    }
  };
  for (unsigned i = threadIdx.x; i < (unsigned)kHistWords; i += BLK) hist[i] = 0;
  if (threadIdx.x == 0) {
    any_nan = 0;
    ncand = 0;
  }
  __syncthreads();
  // pass 1: NaN check + top-digit histogram
  bool nan = false;
  row_keys([&](uint64_t x, long long, bool valid) {
    if (!valid) return;
    nan |= (x & 0x7fffffffffffffffull) > 0x7ff0000000000000ull;
    const unsigned d = (unsigned)(x >> lo_bit) & (kSelBins - 1);
    if constexpr (kPacked)
      atomicAdd(&hist[d >> 1], 1u << ((d & 1u) << 4));  // counts <= T < 65 536
    else
      atomicAdd(&hist[d], 1u);
  });
  if (nan) any_nan = 1;
  __syncthreads();
  if (any_nan) {  // np.percentile of an array holding NaN is NaN: no frame kept
    if (threadIdx.x == 0) thr[b] = __builtin_nan("");
    if (krow)
      for (long long w = threadIdx.x; w < W; w += BLK) krow[w] = 0ull;
    return;
  }
  // bin of rank lo (parallel scan over the histogram)
  {
    constexpr unsigned per = kSelBins / BLK;
    long long mine = 0;
    for (unsigned d = threadIdx.x * per; d < (threadIdx.x + 1) * per; ++d) mine += hcount(d);
    long long total;
    long long acc = block_excl_scan<BLK>(mine, si + 2, total);
    if (lo >= acc && lo < acc + mine) {
      unsigned d = threadIdx.x * per;
      while (acc + hcount(d) <= lo) acc += hcount(d++);
      su[0] = (uint64_t)d << lo_bit;
      si[0] = lo - acc;
      si[1] = hcount(d);
    }
    __syncthreads();
  }
  const uint64_t binpfx = su[0];
  const long long kin = si[0], cnt_bin = si[1];
  const uint64_t binmask = ~((1ull << lo_bit) - 1);
  __syncthreads();
  const bool in_lds = cnt_bin <= kCand;
  const bool lds_mask = krow && in_lds && TT <= kLdsMaskT;
  uint64_t ka;
  long long le_in_bin = -1;  // keys of the bin <= ka (when resolved in LDS)
  uint64_t above_in_bin = ~0ull;
  if (in_lds) {
    // pass 2: compact the bin into LDS; mask words of the frames below it
    // wave-aggregated slot allocation: one LDS atomic per wave and key batch
    row_keys([&](uint64_t x, long long i, bool valid) {
      if (lds_mask) {
        const uint64_t mb = __ballot(valid && x < binpfx);  // below the bin: kept
        if (first_active_lane()) smask[i >> 6] = mb;
      }
      const bool in = valid && (x & binmask) == binpfx;
      const uint64_t m = __ballot(in);
      if (m == 0) return;
      const int lane = threadIdx.x & 63;
      const unsigned below = (unsigned)__popcll(m & ((1ull << lane) - 1));
      unsigned base = 0;
      if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&ncand, (unsigned)__popcll(m));
      base = __shfl(base, __ffsll((long long)m) - 1, 64);
      if (in) {
        cand[base + below] = x;
        cidx[base + below] = (uint16_t)i;
      }
    });
    __syncthreads();
    ka = block_select<BLK, kSelDigit>(cand, cnt_bin, kin, lo_bit - 1, binpfx, hsel, su, si);
    if (hi != lo) {
      if (threadIdx.x == 0) {
        su[1] = ~0ull;
        si[0] = 0;
      }
      __syncthreads();
      unsigned long long c = 0, ab = ~0ull;
      for (long long i = threadIdx.x; i < cnt_bin; i += BLK) {
        const uint64_t x = cand[i];
        c += x <= ka;
        if (x > ka && x < ab) ab = x;
      }
      atomicAdd((unsigned long long *)&si[0], c);
      atomicMin((unsigned long long *)&su[1], ab);
      __syncthreads();
      le_in_bin = si[0];
      above_in_bin = su[1];
      __syncthreads();
    }
  } else if constexpr (kPacked) {  // the 8 KB histogram holds 2 048 bins: 8-bit digits
    ka = block_select<BLK, kSelDigit>(keys, TT, lo, 62, 0ull, hsel, su, si);
  } else {
    ka = block_select<BLK>(keys, TT, lo, 62, 0ull, hist, su, si);
  }
  uint64_t kb = ka;
  if (hi != lo) {
    if (le_in_bin >= 0 && le_in_bin >= kin + 2) {
      kb = ka;                      // ka repeats at rank lo + 1
    } else if (le_in_bin >= 0 && above_in_bin != ~0ull) {
      kb = above_in_bin;            // next key of the same bin
    } else {
      // rank lo + 1 lies above ka: v_(lo+1) = ka if ka repeats, else the least
      // key above ka (one pass over the global row)
      if (threadIdx.x == 0) {
        su[1] = ~0ull;
        si[0] = 0;
      }
      __syncthreads();
      unsigned long long c = 0, ab = ~0ull;
      for_keys<BLK, kSelRowU>(keys, TT, [&](uint64_t x, long long) {
        c += x <= ka;
        if (x > ka && x < ab) ab = x;
      });
      atomicAdd((unsigned long long *)&si[0], c);
      atomicMin((unsigned long long *)&su[1], ab);
      __syncthreads();
      kb = si[0] >= hi + 1 ? ka : su[1];
    }
  }
  if (threadIdx.x == 0) {
    const double a = __longlong_as_double((long long)ka);
    const double bb = __longlong_as_double((long long)kb);
    const double d = bb - a;  // numpy's _lerp
    const double t = g >= 0.5 ? bb - d * (1.0 - g) : a + d * g;
    thr[b] = t;
    sthr = t;
  }
  if (!krow) return;
  __syncthreads();
  const double th = sthr;
  // every key above the bin is >= kb >= th: kept only when equal to th, which
  // needs kb above the bin and th == kb (then mark from the global row)
  const bool amb = (kb & binmask) != binpfx && th >= __longlong_as_double((long long)kb);
  if (lds_mask && !amb) {
    for (long long i = threadIdx.x; i < cnt_bin; i += BLK)
      if (__longlong_as_double((long long)cand[i]) <= th)
        atomicOr((unsigned long long *)&smask[cidx[i] >> 6], 1ull << (cidx[i] & 63));
    __syncthreads();
    for (long long w = threadIdx.x; w < W; w += BLK) krow[w] = smask[w];
  } else {
    for_keys<BLK, kSelRowU>(keys, TT, [&](uint64_t x, long long i) {
      const uint64_t m = __ballot(__longlong_as_double((long long)x) <= th);
      if (first_active_lane()) krow[i >> 6] = m;
    });
  }
}

// ---------------------------------------------------------------------------
// The same selection for FEW long rows (sel_split_auto below): one
// block per row leaves most of the chip idle (config 2: 17 blocks), so each
// row is cut into segments of kSegKeys keys, one block per (row, segment),
// in four launches:
//   k_sel_hist   top-digit histogram of the segment in LDS, added to the
//                row's global histogram (no-return atomics), NaN flag
//   k_sel_bin    one block per row: the bin of rank lo (scan of the global
//                histogram), zeroes the row's candidate counter
//   k_sel_cand   per segment: kept-frame mask words of the frames below the
//                bin (ballot), the bin's keys and frame indices appended to
//                the row's candidate buffer (wave-aggregated slots; their
//                order varies, the order statistics do not), the least key
//                above the bin (atomicMin)
//   k_sel_final  one block per row: MSD radix select of ranks lo / lo + 1
//                among the candidates (LDS when they fit, else in place),
//                numpy's _lerp, the bin's kept frames marked in the mask
// Same threshold and mask bits as k_fit_select (tests/test_gpu_fit_mask.py).
// ---------------------------------------------------------------------------
// The automatic choice (EKS_DBG_FIT_SELECT 0): the split for fewer than 64
// rows, and for rows too long for the one-block kernel's LDS mask (the
// whole-row marking pass, bins beyond its candidate buffer) up to 1 023 rows;
// one block per row otherwise.  Whole device fits (tools/sel_split_timing.py,
// profiles/r06/ab_fit/split_timing.txt), one block per row vs split:
// T = 10 000, B = 64 / 512: 0.102 vs 0.118 / 0.188 vs 0.238 ms; T = 50 000,
// B = 64 / 512: 0.256 vs 0.175 / 0.800 vs 0.672 ms.  (Round 5: split below
// 512 rows whatever the length.)  Large B x T keeps one block per row: the
// split's candidate buffers take B T 12 bytes.
constexpr long long kSelSplitB = 64, kSelSplitLongB = 1024;
bool sel_split_auto(long long B, long long T) {
  return B < kSelSplitB || (T > kLdsMaskT && B < kSelSplitLongB);
}
// threads of the one-block-per-row selection for rows of 4 097 .. 65 535
// frames (A/B builds: -DEKS_SEL_BLK=512)
#ifndef EKS_SEL_BLK
#define EKS_SEL_BLK 256
#endif
constexpr int kSelBlk = EKS_SEL_BLK;
}  // namespace
// eks_debug_set(EKS_DBG_FIT_SELECT): 0 automatic, 1 one block per row, 2 split
long long g_fit_select = 0;
namespace {
constexpr long long kSegKeys = 2048;
// k_sel_hist's segments: 8 x longer, because each block zeroes and flushes
// a 16 384-bin LDS histogram (at 1 024 keys per block that cost 3x the keys:
// config 2 k_sel_hist 0.010 -> 0.033 ms with the 14-bit digit)
constexpr long long kHistSeg = 8192;
// the split path's top digit: 14 bits (exponent + 3 mantissa bits; 64 KB LDS
// histograms): a 4x narrower bin than k_fit_select's 12 bits, so k_sel_final
// selects among ~4x fewer candidates (config 2: ~18 k -> ~4.5 k keys)
constexpr int kSplitBits = 14, kSplitBins = 1 << kSplitBits, kSplitLo = 63 - kSplitBits;

struct SelRow {  // per-row state of the split selection (zeroed by a memset)
  unsigned nan, ncand;
  unsigned long long binpfx, kin, cnt_bin, above;  // above: least key above the bin
};

__global__ __launch_bounds__(256) void k_sel_hist(const double *__restrict__ worst, long long TT,
                                                  int G, unsigned *__restrict__ ghist,
                                                  SelRow *__restrict__ rows) {
  __shared__ unsigned hist[kSplitBins];
  constexpr int lo_bit = kSplitLo;
  const long long b = blockIdx.x / G, g = blockIdx.x % G;
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(worst + b * TT);
  const long long k0 = g * kHistSeg, k1 = k0 + kHistSeg < TT ? k0 + kHistSeg : TT;
  for (int i = threadIdx.x; i < kSplitBins; i += 256) hist[i] = 0;
  __syncthreads();
  bool nan = false;
  constexpr int U = 8;  // independent key loads in flight per thread
  for (long long i0 = k0 + threadIdx.x; i0 < k1; i0 += 256 * U) {
    uint64_t x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = i0 + u * 256 < k1 ? keys[i0 + u * 256] : 0ull;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * 256 < k1) {
        nan |= (x[u] & 0x7fffffffffffffffull) > 0x7ff0000000000000ull;
        atomicAdd(&hist[(unsigned)(x[u] >> lo_bit) & (kSplitBins - 1)], 1u);
      }
  }
  if (__any(nan) && (threadIdx.x & 63) == 0) atomicOr(&rows[b].nan, 1u);
  __syncthreads();
  unsigned *gh = ghist + b * kSplitBins;
  for (int i = threadIdx.x; i < kSplitBins; i += 256)
    if (hist[i]) atomicAdd(&gh[i], hist[i]);
}

__global__ __launch_bounds__(256) void k_sel_bin(const unsigned *__restrict__ ghist, long long lo,
                                                 SelRow *__restrict__ rows) {
  // the row's histogram staged in LDS with 16-byte loads (all in flight at
  // once), then per-thread sums, a block scan and the owner's walk in LDS
  __shared__ uint4 hs[kSplitBins / 4];
  __shared__ long long si[2 + 4];
  const long long b = blockIdx.x;
  const uint4 *h4 = reinterpret_cast<const uint4 *>(ghist + b * kSplitBins);
  constexpr int per4 = kSplitBins / 4 / 256;
  uint4 v[per4];
#pragma unroll
  for (int k = 0; k < per4; ++k) v[k] = h4[k * 256 + threadIdx.x];
#pragma unroll
  for (int k = 0; k < per4; ++k) hs[k * 256 + threadIdx.x] = v[k];
  __syncthreads();
  const unsigned *h = reinterpret_cast<const unsigned *>(hs);
  constexpr unsigned per = kSplitBins / 256;
  long long mine = 0;
  for (unsigned d = threadIdx.x * per; d < (threadIdx.x + 1) * per; ++d) mine += h[d];
  long long total;
  long long acc = block_excl_scan<256>(mine, si + 2, total);
  if (lo >= acc && lo < acc + mine) {  // exactly one thread
    unsigned d = threadIdx.x * per;
    while (acc + h[d] <= (unsigned long long)lo) acc += h[d++];
    rows[b].binpfx = (unsigned long long)d << kSplitLo;
    rows[b].kin = lo - acc;
    rows[b].cnt_bin = h[d];
  }
  if (threadIdx.x == 0) {
    rows[b].ncand = 0;
    rows[b].above = ~0ull;
  }
}

__global__ __launch_bounds__(256) void k_sel_cand(const double *__restrict__ worst, long long TT,
                                                  int G, SelRow *__restrict__ rows,
                                                  uint64_t *__restrict__ ckey,
                                                  unsigned *__restrict__ cidx,
                                                  uint64_t *__restrict__ kept, long long W) {
  const long long b = blockIdx.x / G, g = blockIdx.x % G;
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(worst + b * TT);
  const long long k0 = g * kSegKeys, k1 = k0 + kSegKeys < TT ? k0 + kSegKeys : TT;
  SelRow &row = rows[b];
  const bool nan = row.nan != 0;
  const uint64_t binpfx = row.binpfx, binmask = ~((1ull << kSplitLo) - 1);
  uint64_t *krow = kept ? kept + b * W : nullptr;
  uint64_t *ck = ckey + b * TT;
  unsigned *ci = cidx + b * TT;
  unsigned long long above = ~0ull;
  // the segment's bin keys are staged in LDS and appended with ONE global
  // atomic per block (per-wave atomics on the row's counter serialised: ~400
  // per row at config 2)
  __shared__ uint64_t sk[kSegKeys];
  __shared__ unsigned sidx[kSegKeys];
  __shared__ unsigned scount, sbase;
  if (threadIdx.x == 0) scount = 0;
  __syncthreads();
  // whole waves per 64-key word: k0 is a multiple of 64 and every wave of the
  // loop runs the same iterations (the index test is on the wave's last lane).
  // The segment's kSegKeys / 256 keys per thread are loaded up front (all in
  // flight at once), then classified.
  constexpr int KP = (int)(kSegKeys / 256);
  uint64_t xs[KP];
#pragma unroll
  for (int u = 0; u < KP; ++u) {
    const long long i = k0 + (threadIdx.x & ~63) + u * 256 + (threadIdx.x & 63);
    xs[u] = i < k1 ? keys[i] : ~0ull;
  }
#pragma unroll
  for (int u = 0; u < KP; ++u) {
    const long long i0 = k0 + (threadIdx.x & ~63) + u * 256;
    if (i0 >= k1) break;  // wave-uniform
    const long long i = i0 + (threadIdx.x & 63);
    const bool in_row = i < k1;
    const uint64_t x = xs[u];
    if (krow) {
      const uint64_t mb = __ballot(in_row && !nan && x < binpfx);  // below the bin: kept
      if ((threadIdx.x & 63) == 0) krow[i0 >> 6] = mb;
    }
    if (nan) continue;
    const bool in = in_row && (x & binmask) == binpfx;
    if (in_row && (x & binmask) > binpfx && x < above) above = x;
    const uint64_t m = __ballot(in);
    if (m == 0) continue;
    const int lane = threadIdx.x & 63;
    const unsigned below = (unsigned)__popcll(m & ((1ull << lane) - 1));
    unsigned base = 0;
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&scount, (unsigned)__popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1, 64);
    if (in) {
      sk[base + below] = x;
      sidx[base + below] = (unsigned)i;
    }
  }
  // the least key above the bin: wave minimum, then one atomic per wave
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long other = __shfl_xor(above, o, 64);
    above = other < above ? other : above;
  }
  if (!nan && (threadIdx.x & 63) == 0 && above != ~0ull) atomicMin(&row.above, above);
  __syncthreads();
  const unsigned cnt = scount;
  if (cnt == 0) return;
  if (threadIdx.x == 0) sbase = atomicAdd(&row.ncand, cnt);
  __syncthreads();
  const unsigned base = sbase;
  for (unsigned k = threadIdx.x; k < cnt; k += 256) {
    ck[base + k] = sk[k];
    ci[base + k] = sidx[k];
  }
}

// candidates of the split selection held in LDS (156 KB: the kernel runs one
// 1024-thread block per row, few rows)
constexpr int kCandBig = 19968;  // 156 KB

template <int BLK>
__global__ __launch_bounds__(BLK) void k_sel_final(const double *__restrict__ worst, long long TT,
                                                   long long hi_minus_lo, double g,
                                                   const SelRow *__restrict__ rows,
                                                   const uint64_t *__restrict__ ckey,
                                                   const unsigned *__restrict__ cidx,
                                                   double *__restrict__ thr,
                                                   uint64_t *__restrict__ kept, long long W) {
  __shared__ unsigned hsel[1 << kSelDigit];
  __shared__ uint64_t cand[kCandBig];
  __shared__ uint64_t su[4];
  __shared__ long long si[2 + BLK / 64];
  const long long b = blockIdx.x;
  const SelRow row = rows[b];
  uint64_t *krow = kept ? kept + b * W : nullptr;
  if (row.nan) {  // np.percentile of an array holding NaN is NaN: no frame kept
    if (threadIdx.x == 0) thr[b] = __builtin_nan("");
    return;  // (k_sel_cand wrote zero mask words)
  }
  const uint64_t binpfx = row.binpfx;
  const long long kin = (long long)row.kin, cnt = (long long)row.cnt_bin;
  const uint64_t *ck = ckey + b * TT;
  const unsigned *ci = cidx + b * TT;
  constexpr int lo_bit = kSplitLo;
  uint64_t ka;
  const uint64_t *src = ck;
  if (cnt <= kCandBig) {
    for (long long i = threadIdx.x; i < cnt; i += BLK) cand[i] = ck[i];
    __syncthreads();
    src = cand;
  }
  ka = block_select<BLK, kSelDigit>(src, cnt, kin, lo_bit - 1, binpfx, hsel, su, si);
  uint64_t kb = ka;
  if (hi_minus_lo) {
    // rank lo + 1: ka again if it repeats in the bin, else the next key of the
    // bin, else the least key above the bin
    if (threadIdx.x == 0) {
      su[1] = ~0ull;
      si[0] = 0;
    }
    __syncthreads();
    unsigned long long c = 0, ab = ~0ull;
    for (long long i = threadIdx.x; i < cnt; i += BLK) {
      const uint64_t x = src[i];
      c += x <= ka;
      if (x > ka && x < ab) ab = x;
    }
    atomicAdd((unsigned long long *)&si[0], c);
    atomicMin((unsigned long long *)&su[1], ab);
    __syncthreads();
    const long long le = si[0];
    const unsigned long long nxt = su[1];
    kb = le >= kin + 2 ? ka : nxt != ~0ull ? nxt : row.above;
  }
  __shared__ double sthr;
  if (threadIdx.x == 0) {
    const double a = __longlong_as_double((long long)ka);
    const double bb = __longlong_as_double((long long)kb);
    const double d = bb - a;  // numpy's _lerp
    const double t = g >= 0.5 ? bb - d * (1.0 - g) : a + d * g;
    thr[b] = t;
    sthr = t;
  }
  if (!krow) return;
  __syncthreads();
  const double th = sthr;
  // the bin's kept frames; keys above the bin are >= kb >= th: kept only
  // when equal to th, i.e. th == kb with kb above the bin (then the keys
  // equal to kb, all outside the candidates, are marked from the row).
  // When the row's mask fits in LDS after the candidates, the bits are
  // gathered there (LDS atomics) and each touched word is OR-ed into the
  // mask once, instead of one global atomic per kept frame.
  if (src == cand && cnt + W <= kCandBig) {
    uint64_t *lm = cand + cnt;
    for (long long w = threadIdx.x; w < W; w += BLK) lm[w] = 0;
    __syncthreads();
    for (long long i = threadIdx.x; i < cnt; i += BLK)
      if (__longlong_as_double((long long)src[i]) <= th)
        atomicOr((unsigned long long *)&lm[ci[i] >> 6], 1ull << (ci[i] & 63));
    __syncthreads();
    for (long long w = threadIdx.x; w < W; w += BLK)
      if (lm[w]) atomicOr((unsigned long long *)&krow[w], (unsigned long long)lm[w]);
  } else {
    for (long long i = threadIdx.x; i < cnt; i += BLK)
      if (__longlong_as_double((long long)src[i]) <= th)
        atomicOr((unsigned long long *)&krow[ci[i] >> 6], 1ull << (ci[i] & 63));
  }
  const bool amb = (kb & ~((1ull << lo_bit) - 1)) != binpfx &&
                   th >= __longlong_as_double((long long)kb);
  if (amb) {
    const uint64_t *keys = reinterpret_cast<const uint64_t *>(worst + b * TT);
    for (long long i = threadIdx.x; i < TT; i += BLK)
      if (keys[i] == kb) atomicOr((unsigned long long *)&krow[i >> 6], 1ull << (i & 63));
  }
}

// per-chunk statistics, packed symmetric matrices (upper triangle, row-major):
// kept-frame count, sum of z = y - K and of z z^T, kept-pair count, sum of
// the pair differences d and of d d^T, first / last kept y
template <int N>
struct ChunkStats {
  static constexpr int kTri = N * (N + 1) / 2;
  // [cnt | S1 N | S2 tri | npair | D1 N | D2 tri | first N | last N]
  static constexpr int cnt = 0, mean = 1, M = 1 + N;
  static constexpr int npair = 1 + N + kTri, dmean = npair + 1, dM = dmean + N;
  static constexpr int first = dM + kTri, last = first + N;
  static constexpr int kLen = last + N;
};

template <int N>
EKS_DEV constexpr int tri(int i, int j) {  // i <= j
  return i * N - i * (i - 1) / 2 + (j - i);
}

// the same layout for a runtime n (the wide fit; k_fit_merge<0>)
struct CsRt {
  int n, kTri, cnt, mean, M, npair, dmean, dM, first, last, kLen;
  EKS_DEV explicit CsRt(int n_)
      : n(n_), kTri(n_ * (n_ + 1) / 2), cnt(0), mean(1), M(1 + n_), npair(1 + n_ + kTri),
        dmean(npair + 1), dM(dmean + n_), first(dM + kTri), last(first + n_), kLen(last + n_) {}
  EKS_DEV int tri(int i, int j) const { return i * n - i * (i - 1) / 2 + (j - i); }
};

// the sums of a frame range, merged as  L (+) R  (R the later frames)
template <int N>
struct Partial {
  static constexpr int kTri = N * (N + 1) / 2;
  double cnt, S1[N], S2[kTri], np, D1[N], D2[kTri], first[N], last[N];
  EKS_DEV void merge_right(const Partial &R) {
    if (R.cnt == 0.0) return;
    if (cnt == 0.0) {
      *this = R;
      return;
    }
    // the kept pair where the ranges meet, then the right range's own sums
    // (k_fit_merge adds in the same order)
    double d[N];
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = R.first[i] - last[i];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      D1[i] += d[i];
#pragma unroll
      for (int j = i; j < N; ++j) D2[tri<N>(i, j)] = fma(d[i], d[j], D2[tri<N>(i, j)]);
    }
    np += 1.0;
    cnt += R.cnt;
#pragma unroll
    for (int i = 0; i < N; ++i) S1[i] += R.S1[i];
#pragma unroll
    for (int i = 0; i < kTri; ++i) S2[i] += R.S2[i];
    np += R.np;
#pragma unroll
    for (int i = 0; i < N; ++i) D1[i] += R.D1[i];
#pragma unroll
    for (int i = 0; i < kTri; ++i) D2[i] += R.D2[i];
#pragma unroll
    for (int i = 0; i < N; ++i) last[i] = R.last[i];
  }
  EKS_DEV Partial shfl_down(int delta) const {
    Partial o;
    auto mv = [&](double x) { return __shfl_down(x, delta, 64); };
    o.cnt = mv(cnt);
    o.np = mv(np);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      o.S1[i] = mv(S1[i]);
      o.D1[i] = mv(D1[i]);
      o.first[i] = mv(first[i]);
      o.last[i] = mv(last[i]);
    }
#pragma unroll
    for (int i = 0; i < kTri; ++i) {
      o.S2[i] = mv(S2[i]);
      o.D2[i] = mv(D2[i]);
    }
    return o;
  }
};

// Lane mappings: trajectory-fastest (many trajectories: coalesced plane
// loads, a few chunks per trajectory) or, with WAVE_MERGE (few long
// trajectories), 64 consecutive chunks of one trajectory per wave, whose
// partials the wave merges by a shuffle tree into one (fixed order): the
// merge kernel then sees T / (64 Lc) partials per trajectory instead of
// T / Lc.
template <int E, int N, typename T, typename YT, bool FROM_YEV, bool WAVE_MERGE>
__global__ __launch_bounds__(256) void k_fit_accum(const T *__restrict__ obs, FitShape sh,
                                                   long long sb, long long st, long long se,
                                                   long long sj, int Ert, int median,
                                                   const double *__restrict__ thr,
                                                   const uint64_t *__restrict__ kept,
                                                   long long W, double *__restrict__ part,
                                                   YevOut yi, FitShift ks) {
  using CS = ChunkStats<N>;
  const long long lane = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long NCp = WAVE_MERGE ? (sh.NC + 63) / 64 * 64 : sh.NC;  // chunks per trajectory, padded
  if (!WAVE_MERGE && lane >= sh.B * sh.NC) return;
  if (WAVE_MERGE && lane >= sh.B * NCp) return;  // (whole waves: NCp is a multiple of 64)
  const long long b = WAVE_MERGE ? lane / NCp : lane % sh.B;
  const long long c = WAVE_MERGE ? lane % NCp : lane / sh.B;
  const long long t0 = c * sh.Lc < sh.T ? c * sh.Lc : sh.T;
  const long long t1 = t0 + sh.Lc < sh.T ? t0 + sh.Lc : sh.T;
  const T *pb = obs + b * sb;
  const double th = thr[b];
  const uint64_t *krow = FROM_YEV ? kept + b * W : nullptr;
  auto y_of = [&](long long t, double (&y)[N]) {
    if constexpr (FROM_YEV) {
#pragma unroll
      for (int j = 0; j < N; ++j) y[j] = (double)((const YT *)yi.y)[(t * N + j) * sh.B + b];
    } else {
      double v;
      frame_ensemble<E, N, T>(pb + t * st, se, sj, Ert, median != 0, y, v);
    }
  };
  // the trajectory's shift: its frame-0 ensemble, written by k_fit_worst (a
  // NaN there means a NaN variance, hence a NaN threshold: no kept frame)
  double K[N];
#pragma unroll
  for (int j = 0; j < N; ++j) K[j] = ks.K[b * N + j];
  double S1[N], S2[CS::kTri], D1[N], D2[CS::kTri], first[N], last[N];
  double cnt = 0.0, npair = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) S1[i] = D1[i] = first[i] = last[i] = 0.0;
#pragma unroll
  for (int i = 0; i < CS::kTri; ++i) S2[i] = D2[i] = 0.0;
  auto take = [&](const double (&y)[N]) {  // one kept frame, in frame order
    if (cnt == 0.0) {
#pragma unroll
      for (int i = 0; i < N; ++i) first[i] = y[i];
    } else {
      double d[N];
#pragma unroll
      for (int i = 0; i < N; ++i) d[i] = y[i] - last[i];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        D1[i] += d[i];
#pragma unroll
        for (int j = i; j < N; ++j) D2[tri<N>(i, j)] = fma(d[i], d[j], D2[tri<N>(i, j)]);
      }
      npair += 1.0;
    }
    double z[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      z[i] = y[i] - K[i];
      last[i] = y[i];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      S1[i] += z[i];
#pragma unroll
      for (int j = i; j < N; ++j) S2[tri<N>(i, j)] = fma(z[i], z[j], S2[tri<N>(i, j)]);
    }
    cnt += 1.0;
  };
  if constexpr (FROM_YEV && !WAVE_MERGE) {
    // Trajectory-fastest lanes: the wave's 64 trajectories read the SAME
    // frame at each step, so every frame's y is one coalesced row segment;
    // the y plane streams through a ring kAccD frames deep and the kept bit
    // of k_fit_select's mask decides which frames are summed.  (Round 4
    // gathered only the kept frames, four at a time: each lane a different
    // frame, so every 4-byte load was its own 64-byte request -- 1.79 GB
    // fetched for the 0.35 GB kept, 3.8 TB/s.)  Frame order is kept: the
    // sums are those of the member path.
    constexpr int kAccD = 8;
    YT ring[kAccD][N];
    const YT *yb = (const YT *)yi.y;
    auto fetch = [&](int q, long long t) {
      t = t < t1 ? t : t1 - 1;
#pragma unroll
      for (int j = 0; j < N; ++j) ring[q][j] = yb[(t * N + j) * sh.B + b];
    };
    if (t1 > t0)
#pragma unroll
      for (int q = 0; q < kAccD; ++q) fetch(q, t0 + q);
    // whole blocks of kAccD frames as straight-line code (no per-frame
    // guard: the waitcnt pass then counts the ring's loads exactly instead of
    // draining them at every frame).  t0 is a multiple of 16, so a block never
    // straddles a mask word; the word of the NEXT block is loaded at the top
    // of each block, ahead of that block's ring loads (vmcnt counts in issue
    // order: a word loaded just before its use would drain the ring)
    const long long wl = (t1 - 1) >> 6;  // the chunk's last mask word
    uint64_t m = krow[t0 >> 6];
    long long tb = t0;
    // (unrolled 8 x: the waitcnt pass loses count of the ring at a loop
    // back-edge and drains it there, so take one back-edge per 64 frames)
#pragma unroll 8
    for (; tb + kAccD <= t1; tb += kAccD) {
      const long long wn = (tb + kAccD) >> 6;
      const uint64_t mnext = krow[wn < wl ? wn : wl];
#pragma unroll
      for (int q = 0; q < kAccD; ++q) {
        double y[N];
#pragma unroll
        for (int j = 0; j < N; ++j) y[j] = (double)ring[q][j];
        fetch(q, tb + q + kAccD);
        if ((m >> ((tb + q) & 63)) & 1ull) take(y);
      }
      m = mnext;
    }
    if (tb < t1) {  // the chunk's last frames (fewer than kAccD)
#pragma unroll
      for (int q = 0; q < kAccD; ++q)
        if (tb + q < t1) {
          double y[N];
#pragma unroll
          for (int j = 0; j < N; ++j) y[j] = (double)ring[q][j];
          if ((m >> ((tb + q) & 63)) & 1ull) take(y);
        }
    }
  } else if constexpr (FROM_YEV) {
    // WAVE_MERGE (few long trajectories, a wave = 64 chunks of one
    // trajectory): the kept frames are taken from the mask words KB at a
    // time with their y loads in flight together (a loop over every frame
    // with a branch per frame had one load round trip per kept frame);
    // frame order is kept, so the sums are those of the member path.
    constexpr int KB = 4;
    for (long long wb = t0 & ~63LL; wb < t1; wb += 64) {
      uint64_t m = krow[wb >> 6];
      if (wb < t0) m &= ~0ull << (t0 - wb);
      if (t1 - wb < 64) m &= (1ull << (t1 - wb)) - 1;
      while (m) {
        long long ts[KB];
        int k = 0;
#pragma unroll
        for (int u = 0; u < KB; ++u) {
          if (m) {
            ts[u] = wb + __ffsll((long long)m) - 1;
            m &= m - 1;
            k = u + 1;
          } else {
            ts[u] = ts[0];  // padding: a cache-hit re-load, not taken
          }
        }
        double ys[KB][N];
#pragma unroll
        for (int u = 0; u < KB; ++u) y_of(ts[u], ys[u]);
#pragma unroll
        for (int u = 0; u < KB; ++u)
          if (u < k) take(ys[u]);
      }
    }
  } else {
    for (long long t = t0; t < t1; ++t) {
      double y[N], v;
      frame_ensemble<E, N, T>(pb + t * st, se, sj, Ert, median != 0, y, v);
      if (v <= th) take(y);
    }
  }
  Partial<N> pt;
  pt.cnt = cnt;
  pt.np = npair;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    pt.S1[i] = S1[i];
    pt.D1[i] = D1[i];
    pt.first[i] = first[i];
    pt.last[i] = last[i];
  }
#pragma unroll
  for (int i = 0; i < CS::kTri; ++i) {
    pt.S2[i] = S2[i];
    pt.D2[i] = D2[i];
  }
  long long slot = lane;  // partial row: (chunk, trajectory) -> c * B + b
  if constexpr (WAVE_MERGE) {
    // tree over the wave's 64 chunks: lane l merges lane l + 2^k at level k
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const Partial<N> r = pt.shfl_down(k);
      if ((threadIdx.x & (2 * k - 1)) == 0) pt.merge_right(r);
    }
    if ((threadIdx.x & 63) != 0) return;
    slot = (c / 64) * sh.B + b;
  }
  double *o = part + slot * (long long)CS::kLen;
  o[CS::cnt] = pt.cnt;
  o[CS::npair] = pt.np;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    o[CS::mean + i] = pt.S1[i];
    o[CS::dmean + i] = pt.D1[i];
    o[CS::first + i] = pt.first[i];
    o[CS::last + i] = pt.last[i];
#pragma unroll
    for (int j = i; j < N; ++j) {
      o[CS::M + tri<N>(i, j)] = pt.S2[tri<N>(i, j)];
      o[CS::dM + tri<N>(i, j)] = pt.D2[tri<N>(i, j)];
    }
  }
}

// Merge F consecutive chunk partials of one trajectory into one, in order:
// the sums add, and where two non-empty ranges meet the kept pair straddling
// them (first kept y of the right minus last kept y of the left) adds one
// difference.  One thread per (trajectory, group, packed matrix element);
// every thread reads the counts and the first / last values it needs, so
// there is no cross-thread dependence.  The F partials' loads are issued
// kMergeUnroll at a time ahead of the (sequential, fixed-order) additions.
constexpr int kMergeUnroll = 4;
template <int N>  // N = 0: n = nrt (the wide fit)
__global__ __launch_bounds__(256) void k_fit_merge(long long B, int nc_in, int F,
                                                   const double *__restrict__ in,
                                                   double *__restrict__ out, int nrt) {
  const CsRt CS(N > 0 ? N : nrt);  // compile-time constants for N > 0
  const int nc_out = (nc_in + F - 1) / F;
  const long long gid = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long total = B * nc_out * CS.kTri;
  if (gid >= total) return;
  const int e = (int)(gid % CS.kTri);
  const long long bg = gid / CS.kTri;
  const long long b = bg % B, g = bg / B;
  int i = 0;
  while (CS.tri(i, CS.n - 1) < e) ++i;  // element e = (i, j), i <= j
  const int j = i + (e - CS.tri(i, i));
  double n = 0.0, si = 0.0, s2 = 0.0, np_ = 0.0, di = 0.0, dj = 0.0, d2 = 0.0;
  double fi = 0.0, li = 0.0, lj = 0.0;
  bool have = false;
  const int c0 = (int)g * F, c1 = c0 + F < nc_in ? c0 + F : nc_in;
  for (int cb = c0; cb < c1; cb += kMergeUnroll) {
    double v[kMergeUnroll][11];
#pragma unroll
    for (int u = 0; u < kMergeUnroll; ++u) {
      const int c = cb + u < c1 ? cb + u : c1 - 1;  // clamped: a re-read, not used
      const double *o = in + ((long long)c * B + b) * CS.kLen;
      v[u][0] = o[CS.cnt];
      v[u][1] = o[CS.first + i];
      v[u][2] = o[CS.first + j];
      v[u][3] = o[CS.mean + i];
      v[u][4] = o[CS.M + e];
      v[u][5] = o[CS.npair];
      v[u][6] = o[CS.dmean + i];
      v[u][7] = o[CS.dmean + j];
      v[u][8] = o[CS.dM + e];
      v[u][9] = o[CS.last + i];
      v[u][10] = o[CS.last + j];
    }
#pragma unroll
    for (int u = 0; u < kMergeUnroll; ++u) {
      if (cb + u >= c1 || v[u][0] == 0.0) continue;
      if (have) {  // the pair (last kept of the ranges before, first kept of this one)
        const double xi = v[u][1] - li, xj = v[u][2] - lj;
        di += xi;
        dj += xj;
        d2 = fma(xi, xj, d2);
        np_ += 1.0;
      } else {
        fi = v[u][1];
      }
      n += v[u][0];
      si += v[u][3];
      s2 += v[u][4];
      np_ += v[u][5];
      di += v[u][6];
      dj += v[u][7];
      d2 += v[u][8];
      li = v[u][9];
      lj = v[u][10];
      have = true;
    }
  }
  double *w = out + ((long long)g * B + b) * CS.kLen;
  w[CS.M + e] = s2;
  w[CS.dM + e] = d2;
  if (i == j) {
    w[CS.mean + i] = si;
    w[CS.dmean + i] = di;
    w[CS.first + i] = fi;
    w[CS.last + i] = li;
  }
  if (e == 0) {
    w[CS.cnt] = n;
    w[CS.npair] = np_;
  }
}

// Parameter rows from the fully merged statistics (one partial per
// trajectory): one wavefront per trajectory, lane L = i N + j owning entry
// (i, j) of the n x n matrices.  The PCA axes come from a cyclic Jacobi
// eigen-decomposition done across the wave: each rotation is three
// broadcasts and two lane shuffles, no matrix leaves the registers.
template <int R, int N>
__global__ __launch_bounds__(64) void k_fit_final(long long B, const double *__restrict__ part,
                                                  FitShift ks, int kind, double smooth_param,
                                                  double *__restrict__ params,
                                                  int32_t *__restrict__ status) {
  using CS = ChunkStats<N>;
  __shared__ double sV[N * N], sM[N * N], sD[N * N], sEv[N];
  const long long b = blockIdx.x;
  const int L = threadIdx.x;
  const int i = L / N, j = L % N;
  const bool own = L < N * N;
  const double *o = part + b * CS::kLen;
  const double n = o[CS::cnt];
  double np_ = o[CS::npair];
  if (np_ < 1.0) np_ = __builtin_nan("");  // np.cov of no pairs is NaN
  const int ti = own ? (i <= j ? tri<N>(i, j) : tri<N>(j, i)) : 0;
  // centred scatter matrices from the shifted sums: sum z z^T - S1 S1^T / n
  // (good frames; z = y - K) and sum d d^T - D1 D1^T / np (kept-pair
  // differences)
  const double s1i = own ? o[CS::mean + i] : 0.0, s1j = own ? o[CS::mean + j] : 0.0;
  const double d1i = own ? o[CS::dmean + i] : 0.0, d1j = own ? o[CS::dmean + j] : 0.0;
  const double Mij = own ? o[CS::M + ti] - s1i * (s1j / n) : 0.0;
  const double Dij = own ? o[CS::dM + ti] - d1i * (d1j / np_) : 0.0;
  ParamLayout<R, N> P;
  double *pr = params + b * (long long)P.len;
  if (L < R) pr[P.m0 + L] = 0.0;
  if (L < R * R) pr[P.A + L] = (L / R == L % R) ? 1.0 : 0.0;
  if (L < N) pr[P.off + L] = ks.K[b * N + L] + o[CS::mean + L] / n;  // mean of the good y
  if (kind == EKS_FIT_SINGLEVIEW) {
    // S0 = diag(var(good y)) (ddof 0), Q = s cov(diff) (ddof 1), A = C = I
    if (own && i < R && j < R) {
      pr[P.S0 + i * R + j] = i == j ? Mij / n : 0.0;
      pr[P.Q + i * R + j] = smooth_param * (Dij / (np_ - 1.0));
    }
    if (own && j < R) pr[P.C + i * R + j] = i == j ? 1.0 : 0.0;
  } else {
    // principal axes of the good-frame scatter matrix (sklearn's PCA axes
    // up to sign; outputs do not depend on the sign)
    double a = Mij, v = (own && i == j) ? 1.0 : 0.0;
    {
      double m = own ? fabs(a) : 0.0;
#pragma unroll
      for (int w = 32; w >= 1; w >>= 1) m = fmax(m, __shfl_xor(m, w, 64));
      a = ldexp(a, -pca_scale(m));
    }
    // parallel cyclic Jacobi (round-robin ordering): each sweep is N - 1
    // rounds of N / 2 disjoint rotations, applied at once as A <- J^T A J,
    // V <- V J (lane (i, j) combines the entries of its row pair x column
    // pair: four reads, no dependence on the other rotations of the round)
    const int Nm = N - 1;
    auto slot_of = [&](int x, int k) { return x == 0 ? 0 : 1 + (x - 1 + Nm - (k % Nm)) % Nm; };
    auto idx_at = [&](int pos, int k) { return pos == 0 ? 0 : 1 + (pos - 1 + k) % Nm; };
    double off_prev = __builtin_inf();
    for (int sweep = 0; sweep < 60; ++sweep) {
      double off = (own && i < j) ? a * a : 0.0, dia = (own && i == j) ? a * a : 0.0;
#pragma unroll
      for (int w = 32; w >= 1; w >>= 1) {
        off += __shfl_xor(off, w, 64);
        dia += __shfl_xor(dia, w, 64);
      }
      // converged: the off-diagonal mass at the rounding level of the
      // diagonal, or no longer shrinking (FMA-rounded rotations can leave
      // it hovering just above a tighter bound for the remaining sweeps)
      if (off == 0.0 || off <= kJacobiTol * dia || off >= off_prev) break;
      off_prev = off;
      for (int k = 0; k < Nm; ++k) {
        // the partner of index x in round k: positions pos and N-1-pos pair up
        auto partner = [&](int x) { return idx_at(Nm - slot_of(x, k), k); };
        const int pi = partner(i), pj = partner(j);
        // rotation of the pair {x, partner}: J_pp = c, J_pq = s, J_qp = -s,
        // J_qq = c with p < q; returns (J_xx, J_partner,x)
        auto rot = [&](int x, int px, double &jxx, double &jpx) {
          const int p = x < px ? x : px, q = x < px ? px : x;
          const double apq = __shfl(a, p * N + q, 64);
          const double app = __shfl(a, p * N + p, 64), aqq = __shfl(a, q * N + q, 64);
          double c, sn;
          jacobi_cs(app, aqq, apq, c, sn);
          jxx = c;
          jpx = x == p ? -sn : sn;  // J_qp = -s (x = p), J_pq = s (x = q)
        };
        double ji, jpi_i, jj, jpj_j;
        rot(own ? i : 0, own ? pi : partner(0), ji, jpi_i);
        rot(own ? j : 0, own ? pj : partner(0), jj, jpj_j);
        const int li = own ? i : 0, lj = own ? j : 0, lpi = own ? pi : 0, lpj = own ? pj : 0;
        const double a_ipj = __shfl(a, li * N + lpj, 64);
        const double a_pij = __shfl(a, lpi * N + lj, 64);
        const double a_pipj = __shfl(a, lpi * N + lpj, 64);
        const double v_ipj = __shfl(v, li * N + lpj, 64);
        if (own) {
          // A'_ij = sum_{k in {i, pi}, l in {j, pj}} J_ki A_kl J_lj
          const double r0 = a * jj + a_ipj * jpj_j;       // (A J)_ij
          const double r1 = a_pij * jj + a_pipj * jpj_j;  // (A J)_{pi j}
          a = ji * r0 + jpi_i * r1;
          v = v * jj + v_ipj * jpj_j;
        }
      }
    }
    if (own) {
      sV[L] = v;
      sM[L] = Mij;
      sD[L] = Dij;
      if (i == j) sEv[i] = a;
    }
    __syncthreads();
    // lane (k, l) < R x R: S0 = diag(W (M / n) W^T), Q = s W (DM / (np - 1)) W^T
    // with W's rows the eigenvectors of the R largest eigenvalues
    int order[R];
    unsigned used = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {  // k-th largest eigenvalue (first index on ties)
      int best = -1;
      for (int e = 0; e < N; ++e)
        if (!((used >> e) & 1u) && (best < 0 || sEv[e] > sEv[best])) best = e;
      order[k] = best;
      used |= 1u << best;
    }
    if (L < R * R) {
      const int k = L / R, l = L % R;
      int ok_ = 0, ol = 0;
#pragma unroll
      for (int u = 0; u < R; ++u) {
        ok_ = u == k ? order[u] : ok_;
        ol = u == l ? order[u] : ol;
      }
      double s0 = 0.0, q = 0.0;
      for (int x = 0; x < N; ++x)
        for (int y = 0; y < N; ++y) {
          const double w = sV[x * N + ok_] * sV[y * N + ol];
          s0 = fma(w, sM[x * N + y], s0);
          q = fma(w, sD[x * N + y], q);
        }
      pr[P.S0 + L] = k == l ? s0 / n : 0.0;
      pr[P.Q + L] = smooth_param * (q / (np_ - 1.0));
    }
    if (own && j < R) {
      int oj = 0;
#pragma unroll
      for (int u = 0; u < R; ++u) oj = u == j ? order[u] : oj;
      pr[P.C + i * R + j] = sV[i * N + oj];
    }
  }
  if (status && L == 0) status[b] = n > 0.0 ? 0 : EKS_STATUS_SINGULAR;
}

// ---------------------------------------------------------------------------
// Wide models: n = 10..16 observed coordinates (5-8 cameras; the reference
// fits any camera count, eks/multiview_pca_smoother.py:684-731).  k_fit_accum
// keeps both packed scatter sums per lane, 2 n (n + 1) / 2 doubles (272 at
// n = 16: far past the register file), so here each (trajectory, chunk) is
// served by a group of kNW = 16 lanes, lane i owning column i: its ensemble,
// S1_i, D1_i and ROW i of the two scatter sums; the other columns of a frame
// arrive by shuffles inside the group.  The partial rows have k_fit_accum's
// layout, so k_fit_merge (N = 0: runtime n) merges them; k_fitw_final does
// the PCA of the n x n matrix with one 256-thread block (lane (i, j), LDS).
// ---------------------------------------------------------------------------
constexpr int kNW = 16;

// Broadcast of lane J of each 16-lane DPP row to the whole row: the groups
// of kNW = 16 lanes are exactly the wave's DPP rows, so one v_mov_b64_dpp
// row_newbcast:J (gfx950's 64-bit DPP broadcast) replaces a __shfl (two
// ds_bpermute_b32 through the LDS crossbar plus their waits).  The row is
// active or idle as a whole (the kept decision is uniform over a group).
template <int J>
EKS_DEV double row_bcast(double x) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass only parses device code)
  const long v = __builtin_bit_cast(long, x);
  const long r = __builtin_amdgcn_update_dpp(0L, v, 0x150 + J, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
#else
  return x;
#endif
}
// acc[j] += x * (x of column j) for the group's kNW columns
template <int... J>
EKS_DEV void row_outer(double x, double (&acc)[kNW], std::integer_sequence<int, J...>) {
  ((acc[J] = fma(x, row_bcast<J>(x), acc[J])), ...);
}

// k_fit_worst's lanes and tiles (trajectory-fastest lanes over chunks of
// frames: the hand-off planes' rows, B values each, are written by
// consecutive lanes; the worst rows leave through an LDS tile) with the
// frame's n columns reduced in a runtime loop (runtime E)
template <typename T, typename YT, int E>
__global__ __launch_bounds__(256) void k_fitw_worst(const T *__restrict__ obs, FitShape sh,
                                                    long long sb, long long st, long long se,
                                                    long long sj, int Ert, int n, int median,
                                                    double *__restrict__ worst, YevOut yo,
                                                    FitShift ks, ZeroSpan zs) {
  zs.run();
  __shared__ double tile[256][kTile + 1];
  __shared__ long long base[256];
  const long long lane = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const bool active = lane < sh.B * sh.NC;
  long long b = 0, t0 = 0, t1 = 0;
  if (active) {
    b = lane % sh.B;
    t0 = (lane / sh.B) * sh.Lc;
    t1 = t0 + sh.Lc < sh.T ? t0 + sh.Lc : sh.T;
  }
  const T *pb = obs + b * sb;
  // the frames [fa, fe) column by column (kRtDP columns' member loads in
  // flight for compiled E); put(t, v_t) receives each frame's worst variance
  double v = -1.0;
  bool nan = false;
  auto col_done = [&](long long t, int j, double avg, double var) {
    nan |= (var != var);
    v = var > v ? var : v;
    if (t == 0) ks.K[b * n + j] = avg;
    if (yo.y) {
      ((YT *)yo.y)[(t * n + j) * sh.B + b] = (YT)avg;
      yo.ev[(t * n + j) * sh.B + b] = var;
    }
  };
  auto frames = [&](long long fa, long long fe, auto &&put) {
    auto begin = [&](long long) {
      v = -1.0;
      nan = false;
    };
    auto end = [&](long long t) { put(t, nan ? __builtin_nan("") : v); };
    if constexpr (E > 0) {
      T ring[kRtDP][E];
      auto fetch = [&](int k, long long t, int j) {
        const T *pc = pb + t * st + j * sj;
#pragma unroll
        for (int u = 0; u < E; ++u) ring[k][u] = pc[u * se];
      };
      auto col = [&](int k, long long t, int j) {
        double avg, var;
        ensemble_reduce<E, T>(ring[k], median != 0, avg, var);
        col_done(t, j, avg, var);
      };
      rt_columns(fa, fe, n, fetch, col, begin, end);
    } else {
      for (long long t = fa; t < fe; ++t) {
        begin(t);
        for (int j = 0; j < n; ++j) {
          double avg, var;
          column_reduce<0, T>(pb + t * st + j * sj, se, Ert, median != 0, avg, var);
          col_done(t, j, avg, var);
        }
        end(t);
      }
    }
  };
  const long long ntiles = sh.Lc / kTile;  // Lc is a multiple of kTile
  for (long long kt = 0; kt < ntiles; ++kt) {
    const long long t = t0 + kt * kTile;
    if (active && t + kTile <= t1) {
      frames(t, t + kTile, [&](long long u, double w) { tile[threadIdx.x][u - t] = w; });
      base[threadIdx.x] = b * sh.T + t;
    } else {
      base[threadIdx.x] = -1;
      if (active)  // ragged end
        frames(t, t1, [&](long long u, double w) { worst[b * sh.T + u] = w; });
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 256 / 16; ++p) {
      const int r = p * 16 + (threadIdx.x >> 4), k = threadIdx.x & 15;
      const long long o = base[r];
      if (o >= 0) worst[o + k] = tile[r][k];
    }
    __syncthreads();
  }
}

template <typename T, typename YT, bool FROM_YEV, int E>
__global__ __launch_bounds__(256) void k_fitw_accum(const T *__restrict__ obs, FitShape sh,
                                                    long long sb, long long st, long long se,
                                                    long long sj, int Ert, int n, int median,
                                                    const double *__restrict__ thr,
                                                    const uint64_t *__restrict__ kept,
                                                    long long W, double *__restrict__ part,
                                                    YevOut yi, FitShift ks) {
  const long long gl = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long pc = gl / kNW;  // (chunk, trajectory) pair: c * B + b
  if (pc >= sh.B * sh.NC) return;  // whole groups (B NC kNW lanes)
  const int i = (int)(gl % kNW);  // column; the group is the lane's DPP row
  const bool own = i < n;
  const int ic = own ? i : n - 1;  // idle lanes shadow the last column (never stored)
  const long long b = pc % sh.B, c = pc / sh.B;
  const long long t0 = c * sh.Lc < sh.T ? c * sh.Lc : sh.T;
  const long long t1 = t0 + sh.Lc < sh.T ? t0 + sh.Lc : sh.T;
  const T *pb = obs + b * sb + ic * sj;
  const double th = thr[b];
  const uint64_t *krow = FROM_YEV ? kept + b * W : nullptr;
  const double K = ks.K[b * n + ic];
  double S2[kNW], D2[kNW];
#pragma unroll
  for (int j = 0; j < kNW; ++j) S2[j] = D2[j] = 0.0;
  double cnt = 0.0, npair = 0.0, S1 = 0.0, D1 = 0.0, first = 0.0, last = 0.0;
  auto take = [&](double y) {  // one kept frame
    if (cnt == 0.0) {
      first = y;
    } else {
      const double d = y - last;
      D1 += d;
      row_outer(d, D2, std::make_integer_sequence<int, kNW>{});
      npair += 1.0;
    }
    const double z = y - K;
    last = y;
    S1 += z;
    row_outer(z, S2, std::make_integer_sequence<int, kNW>{});
    cnt += 1.0;
  };
  // a frame is kept when v = max over the group's columns <= th (uniform over
  // the group; a NaN variance made the threshold NaN: nothing is kept)
  auto kept_v = [&](double var) {
    double v = var;
#pragma unroll
    for (int w = kNW / 2; w >= 1; w >>= 1) {
      const double o = __shfl_xor(v, w, 64);
      v = o > v ? o : v;
    }
    return v <= th;
  };
  // DF frames' loads in flight (unconditional, index clamped into the chunk)
  constexpr int DF = 4;
  auto cl = [&](long long t) { return t < t1 ? t : t1 - 1; };
  if (t0 < t1) {
    if constexpr (FROM_YEV) {
      const YT *yp = (const YT *)yi.y;
      auto ld = [&](long long t) { return yp[(cl(t) * n + ic) * sh.B + b]; };
      YT ring[DF];
#pragma unroll
      for (int q = 0; q < DF; ++q) ring[q] = ld(t0 + q);
      uint64_t kw = krow[t0 >> 6];
      for (long long tb = t0; tb < t1; tb += DF) {
#pragma unroll
        for (int q = 0; q < DF; ++q) {
          const long long t = tb + q;
          const YT yv = ring[q];
          ring[q] = ld(t + DF);
          if (t < t1) {
            if ((t & 63) == 0) kw = krow[t >> 6];
            if ((kw >> (t & 63)) & 1ull) take((double)yv);
          }
        }
      }
    } else if constexpr (E > 0) {
      T ring[DF][E];
      auto ld = [&](int q, long long t) {
        const T *pt = pb + cl(t) * st;
#pragma unroll
        for (int u = 0; u < E; ++u) ring[q][u] = pt[u * se];
      };
#pragma unroll
      for (int q = 0; q < DF; ++q) ld(q, t0 + q);
      for (long long tb = t0; tb < t1; tb += DF) {
#pragma unroll
        for (int q = 0; q < DF; ++q) {
          const long long t = tb + q;
          T cur[E];
#pragma unroll
          for (int u = 0; u < E; ++u) cur[u] = ring[q][u];
          ld(q, t + DF);
          if (t < t1) {
            double y, var;
            ensemble_reduce<E, T>(cur, median != 0, y, var);
            if (kept_v(var)) take(y);
          }
        }
      }
    } else {
      for (long long t = t0; t < t1; ++t) {
        double y, var;
        column_reduce<0, T>(pb + t * st, se, Ert, median != 0, y, var);
        if (kept_v(var)) take(y);
      }
    }
  }
  const CsRt CS(n);
  double *o = part + pc * (long long)CS.kLen;
  if (i == 0) {
    o[CS.cnt] = cnt;
    o[CS.npair] = npair;
  }
  if (!own) return;
  o[CS.mean + i] = S1;
  o[CS.dmean + i] = D1;
  o[CS.first + i] = first;
  o[CS.last + i] = last;
#pragma unroll
  for (int j = 0; j < kNW; ++j)
    if (j >= i && j < n) {
      o[CS.M + CS.tri(i, j)] = S2[j];
      o[CS.dM + CS.tri(i, j)] = D2[j];
    }
}

// k_fit_final's PCA model for n = 10..16 (even): one 256-thread block per
// trajectory, thread (i, j) = (L / 16, L % 16) owning entry (i, j); the
// round-robin Jacobi's cross-entry reads go through LDS
template <int R>
__global__ __launch_bounds__(256) void k_fitw_final(long long B, const double *__restrict__ part,
                                                    FitShift ks, int n, double smooth_param,
                                                    double *__restrict__ params,
                                                    int32_t *__restrict__ status) {
  // sA / sV double-buffered by round parity: a round's reads of one buffer
  // are ordered before the next write of it by the following round's
  // barrier, so one barrier per round
  __shared__ double sA2[2][kNW * kNW], sV2[2][kNW * kNW];
  __shared__ double sM[kNW * kNW], sD[kNW * kNW], sEv[kNW];
  double *sV = sV2[0];
  __shared__ double sRed[2][4];
  // the round-robin schedule, partner of index x in round k, tabulated once
  // (runtime n: each entry takes three integer divisions, which on every
  // thread's path of every round cost more than the rotation itself)
  __shared__ unsigned char sPart[kNW - 1][kNW];
  const CsRt CS(n);
  const long long b = blockIdx.x;
  const int L = threadIdx.x, i = L / kNW, j = L % kNW;
  const bool own = i < n && j < n;
  const double *o = part + b * CS.kLen;
  const double cnt = o[CS.cnt];
  double np_ = o[CS.npair];
  if (np_ < 1.0) np_ = __builtin_nan("");
  const int ti = own ? (i <= j ? CS.tri(i, j) : CS.tri(j, i)) : 0;
  const double s1i = own ? o[CS.mean + i] : 0.0, s1j = own ? o[CS.mean + j] : 0.0;
  const double d1i = own ? o[CS.dmean + i] : 0.0, d1j = own ? o[CS.dmean + j] : 0.0;
  const double Mij = own ? o[CS.M + ti] - s1i * (s1j / cnt) : 0.0;
  const double Dij = own ? o[CS.dM + ti] - d1i * (d1j / np_) : 0.0;
  // packed row [m0 | S0 | A | Q | C (n x R) | offset (n)]
  const int pS0 = R, pA = R + R * R, pQ = R + 2 * R * R, pC = R + 3 * R * R, pOff = pC + n * R;
  double *pr = params + b * (long long)(pOff + n);
  if (L < R) pr[L] = 0.0;
  if (L < R * R) pr[pA + L] = (L / R == L % R) ? 1.0 : 0.0;
  if (L < n) pr[pOff + L] = ks.K[b * n + L] + o[CS.mean + L] / cnt;
  double a = Mij, v = (own && i == j) ? 1.0 : 0.0;
  {  // the exact power-of-two pre-scaling of k_fit_final (pca_scale)
    double m = own ? fabs(a) : 0.0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) m = fmax(m, __shfl_xor(m, w, 64));
    if ((L & 63) == 0) sRed[0][L >> 6] = m;
    __syncthreads();
    m = fmax(fmax(sRed[0][0], sRed[0][1]), fmax(sRed[0][2], sRed[0][3]));
    __syncthreads();
    a = ldexp(a, -pca_scale(m));
  }
  const int Nm = n - 1;
  auto slot_of = [&](int x, int k) { return x == 0 ? 0 : 1 + (x - 1 + Nm - (k % Nm)) % Nm; };
  auto idx_at = [&](int pos, int k) { return pos == 0 ? 0 : 1 + (pos - 1 + k) % Nm; };
  if (i < Nm && j < n) sPart[i][j] = (unsigned char)idx_at(Nm - slot_of(j, i), i);
  __syncthreads();
  double off_prev = __builtin_inf();
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = (own && i < j) ? a * a : 0.0, dia = (own && i == j) ? a * a : 0.0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
      off += __shfl_xor(off, w, 64);
      dia += __shfl_xor(dia, w, 64);
    }
    if ((L & 63) == 0) {
      sRed[0][L >> 6] = off;
      sRed[1][L >> 6] = dia;
    }
    __syncthreads();
    off = sRed[0][0] + sRed[0][1] + sRed[0][2] + sRed[0][3];
    dia = sRed[1][0] + sRed[1][1] + sRed[1][2] + sRed[1][3];
    __syncthreads();
    if (off == 0.0 || off <= kJacobiTol * dia || off >= off_prev) break;  // block-uniform
    off_prev = off;
    for (int k = 0; k < Nm; ++k) {
      const int pb = k & 1;
      double *sA = sA2[pb], *sVb = sV2[pb];
      sA[L] = a;
      sVb[L] = v;
      __syncthreads();
      const int li = own ? i : 0, lj = own ? j : 0;
      const int pi = sPart[k][li], pj = sPart[k][lj];
      auto rot = [&](int x, int px, double &jxx, double &jpx) {
        const int p = x < px ? x : px, q = x < px ? px : x;
        const double apq = sA[p * kNW + q], app = sA[p * kNW + p], aqq = sA[q * kNW + q];
        double cs, sn;
        jacobi_cs(app, aqq, apq, cs, sn);
        jxx = cs;
        jpx = x == p ? -sn : sn;
      };
      double ji, jpi_i, jj, jpj_j;
      rot(li, pi, ji, jpi_i);
      rot(lj, pj, jj, jpj_j);
      const double a_ipj = sA[li * kNW + pj], a_pij = sA[pi * kNW + lj];
      const double a_pipj = sA[pi * kNW + pj], v_ipj = sVb[li * kNW + pj];
      if (own) {
        const double r0 = a * jj + a_ipj * jpj_j;
        const double r1 = a_pij * jj + a_pipj * jpj_j;
        a = ji * r0 + jpi_i * r1;
        v = v * jj + v_ipj * jpj_j;
      }
    }
  }
  __syncthreads();  // (the sweep cap: the last round's reads of sV2[0])
  sV[L] = v;
  sM[L] = Mij;
  sD[L] = Dij;
  if (own && i == j) sEv[i] = a;
  __syncthreads();
  int order[R];
  unsigned used = 0;
#pragma unroll
  for (int k = 0; k < R; ++k) {  // k-th largest eigenvalue (first index on ties)
    int best = -1;
    for (int e = 0; e < n; ++e)
      if (!((used >> e) & 1u) && (best < 0 || sEv[e] > sEv[best])) best = e;
    order[k] = best;
    used |= 1u << best;
  }
  if (L < R * R) {
    const int k = L / R, l = L % R;
    int ok_ = 0, ol = 0;
#pragma unroll
    for (int u = 0; u < R; ++u) {
      ok_ = u == k ? order[u] : ok_;
      ol = u == l ? order[u] : ol;
    }
    double s0 = 0.0, q = 0.0;
    for (int x = 0; x < n; ++x)
      for (int y = 0; y < n; ++y) {
        const double w = sV[x * kNW + ok_] * sV[y * kNW + ol];
        s0 = fma(w, sM[x * kNW + y], s0);
        q = fma(w, sD[x * kNW + y], q);
      }
    pr[pS0 + L] = k == l ? s0 / cnt : 0.0;
    pr[pQ + L] = smooth_param * (q / (np_ - 1.0));
  }
  if (own && j < R) {
    int oj = 0;
#pragma unroll
    for (int u = 0; u < R; ++u) oj = u == j ? order[u] : oj;
    pr[pC + i * R + j] = sV[i * kNW + oj];
  }
  if (status && L == 0) status[b] = cnt > 0.0 ? 0 : EKS_STATUS_SINGULAR;
}

// chunks per trajectory (k_fit_worst's and k_fit_accum's lanes): enough
// lanes to fill the chip (~256k; the wide fit's groups of kNW lanes count
// kNW each), chunks of >= kTile frames, a multiple of kTile frames each
void fit_chunks(long long B, long long T, int &nc, long long &lc, int n = 0) {
  const long long target = n > kMaxObs ? 262144 / kNW : 262144;
  long long nn = (target + B - 1) / (B > 0 ? B : 1);
  const long long cap = T / kTile > 1 ? T / kTile : 1;
  if (nn > cap) nn = cap;
  if (nn < 1) nn = 1;
  lc = (T + nn - 1) / nn;
  lc = (lc + kTile - 1) / kTile * kTile;
  nc = (int)((T + lc - 1) / lc);
}

// (at six cameras' 782 partials, 28 per thread in two launches measured
// slower than 16 in three: 0.031 -> 0.036 ms, profiles/r05/ab14)
constexpr int kMergeFan = 16;

// few long trajectories (B < 64: a trajectory-fastest wave would span
// several chunks of short row segments): k_fit_accum merges each wave's 64
// chunks itself.  From 64 trajectories on, the lanes stay trajectory-fastest
// (one coalesced row segment per frame and wave; the 8-GPU shard of config
// 4, B = 2 176, nc = 105: the wave-merge form's lanes 96 frames apart in the
// time-major y plane fetched 1.18 GB for its 0.17 GB) and k_fit_merge
// reduces the nc partials.
bool fit_wave_merge(long long B, int nc, int n = 0) { return n <= kMaxObs && nc >= 64 && B < 64; }
int fit_partials(long long B, int nc, int n = 0) {
  return fit_wave_merge(B, nc, n) ? (nc + 63) / 64 : nc;
}
constexpr int kMaxObsFit = kNW;  // n of eks_fit (even; n > kMaxObs: the wide kernels)

}  // namespace

}  // namespace eks

using namespace eks;

extern "C" size_t eks_fit_workspace_bytes(int64_t B, int64_t T, int n) {
  if (B <= 0 || T <= 0 || n < 1 || n > kMaxObsFit) return 0;
  int nc;
  long long lc;
  fit_chunks(B, T, nc, lc, n);
  const long long len = 2 + 4LL * n + (long long)n * (n + 1);
  const long long np = fit_partials(B, nc, n);
  const long long nc2 = (np + kMergeFan - 1) / kMergeFan;
  const long long W = (T + 63) / 64;  // frame-mask words per trajectory
  // worst plane, thresholds, chunk partials, kept-frame mask, shifts K
  size_t bytes = (size_t)(B * T + B + B * (np + nc2) * len + B * W + B * n) * sizeof(double);
  // split selection: histograms, row states, candidate keys + indices
  if (sel_split_auto(B, T) || g_fit_select == 2)
    bytes += (size_t)B * kSplitBins * 4 + (size_t)B * sizeof(SelRow) + (size_t)B * T * 12 + 512;
  return bytes;
}

// y of the hand-off planes is float32 exactly when it is a member value:
// float32 members, median mode, odd E the smoother specialises (3, 5)
static bool yev_float(int obs_dtype, int E, int mode) {
  return obs_dtype == EKS_F32 && mode == EKS_MEDIAN && (E == 3 || E == 5);
}

extern "C" int eks_yev_dtype(int obs_dtype, int E, int mode) {
  return yev_float(obs_dtype, E, mode) ? EKS_YEV32 : EKS_YEV64;
}

extern "C" size_t eks_yev_bytes(int64_t B, int64_t T, int n, int obs_dtype, int E, int mode) {
  if (B <= 0 || T <= 0 || n < 1) return 0;
  const size_t ys = yev_float(obs_dtype, E, mode) ? 4 : 8;
  return yev_ev_offset(B, T, n, ys) + (size_t)B * T * n * 8;
}

extern "C" int eks_fit(const void *obs, int obs_dtype, int64_t B, int64_t T, int E, int n, int r,
                       int64_t sb, int64_t st, int64_t se, int64_t sj, int mode, int kind,
                       double smooth_param, double quantile_keep, double *params,
                       void *workspace, size_t workspace_bytes, int32_t *status, void *yev,
                       void *stream) {
  clear_err();
  if (!obs || !params || !workspace) return set_err(EKS_ERR_ARG, "eks_fit: NULL pointer");
  if (B < 0 || T < 2 || E < 1 || n < 1) return set_err(EKS_ERR_ARG, "eks_fit: bad sizes");
  if (B == 0) return EKS_OK;
  if (E > kMaxMembers) return set_err(EKS_ERR_UNSUPPORTED, "eks_fit: E=%d > %d", E, kMaxMembers);
  if (mode != EKS_MEDIAN && mode != EKS_MEAN)
    return set_err(EKS_ERR_ARG, "%d averaging not supported", mode);
  if (obs_dtype != EKS_F32 && obs_dtype != EKS_F64) return set_err(EKS_ERR_ARG, "bad dtype");
  if (kind != EKS_FIT_SINGLEVIEW && kind != EKS_FIT_MULTICAM)
    return set_err(EKS_ERR_ARG, "eks_fit: unknown model kind %d", kind);
  if (kind == EKS_FIT_SINGLEVIEW && r != n)
    return set_err(EKS_ERR_ARG, "eks_fit: single-view model needs r == n");
  if (kind == EKS_FIT_MULTICAM && (r > n || r < 1))
    return set_err(EKS_ERR_ARG, "eks_fit: PCA model needs 1 <= r <= n");
  if (!(quantile_keep >= 0.0 && quantile_keep <= 100.0))
    return set_err(EKS_ERR_ARG, "eks_fit: quantile_keep must be in [0, 100]");
  if (workspace_bytes < eks_fit_workspace_bytes(B, T, n))
    return set_err(EKS_ERR_ARG, "eks_fit: workspace too small (%zu < %zu)", workspace_bytes,
                   eks_fit_workspace_bytes(B, T, n));
  hipStream_t s = (hipStream_t)stream;
  FitShape sh{B, T, 0, 0};
  fit_chunks(B, T, sh.NC, sh.Lc, n);
  const long long len = 2 + 4LL * n + (long long)n * (n + 1);
  double *worst = (double *)workspace;
  double *thr = worst + B * T;
  const int npart = fit_partials(B, sh.NC, n);
  const bool wave_merge = fit_wave_merge(B, sh.NC, n);
  double *partA = thr + B;
  double *partB = partA + B * (long long)npart * len;
  const long long W = (T + 63) / 64;
  uint64_t *kept = reinterpret_cast<uint64_t *>(
      partB + B * (long long)((npart + kMergeFan - 1) / kMergeFan) * len);
  FitShift ks{reinterpret_cast<double *>(kept + B * W)};
  // split selection (few rows): its buffers after the shifts
  const bool split_sel = g_fit_select == 1 ? false : g_fit_select == 2 ? true : sel_split_auto(B, T);
  const int G = (int)((T + kSegKeys - 1) / kSegKeys);
  char *sel_base = reinterpret_cast<char *>(
      (reinterpret_cast<uintptr_t>(ks.K + B * n) + 255) / 256 * 256);  // 16-byte loads in k_sel_bin
  unsigned *ghist = reinterpret_cast<unsigned *>(sel_base);
  SelRow *rows = reinterpret_cast<SelRow *>(sel_base + (size_t)B * kSplitBins * 4);
  uint64_t *ckey = reinterpret_cast<uint64_t *>(
      (reinterpret_cast<uintptr_t>(rows + B) + 255) / 256 * 256);
  unsigned *cidx = reinterpret_cast<unsigned *>(ckey + B * T);
  // np.percentile 'linear': virtual index (T - 1) q / 100
  const double vi = (double)(T - 1) * (quantile_keep / 100.0);
  const long long lo = (long long)floor(vi);
  const long long hi = lo + 1 < T ? lo + 1 : T - 1;
  const double g = vi - (double)lo;
  const int median = mode == EKS_MEDIAN ? 1 : 0;
  const unsigned grid = grid_for(B * sh.NC, 256);
  const bool y32 = yev_float(obs_dtype, E, mode);
  YevOut yo;
  if (yev) {
    yo.y = yev;
    yo.ev = (double *)((char *)yev + yev_ev_offset(B, T, n, y32 ? 4 : 8));
  }
  ZeroSpan zs;
  if (split_sel) {
    zs.p = ghist;
    zs.n = (long long)(((size_t)B * kSplitBins * 4 + (size_t)B * sizeof(SelRow)) / 4);
  }
  // the order statistics, the threshold and (with the hand-off planes
  // written) the kept-frame mask k_fit_accum reads instead of the ev plane
  auto select = [&]() -> int {
    prof_mark(s, "k_fit_select");
    if (split_sel) {
      // few long rows: one block per (row, segment) in four launches
      // (ghist and the row states were zeroed by the worst pass: zs)
      const unsigned gs = (unsigned)(B * G);
      prof_mark(s, "k_sel_hist");
      const int GH = (int)((T + kHistSeg - 1) / kHistSeg);
      hipLaunchKernelGGL(k_sel_hist, dim3((unsigned)(B * GH)), dim3(256), 0, s, worst, T, GH,
                         ghist, rows);
      prof_mark(s, "k_sel_bin");
      hipLaunchKernelGGL(k_sel_bin, dim3((unsigned)B), dim3(256), 0, s, ghist, lo, rows);
      prof_mark(s, "k_sel_cand");
      hipLaunchKernelGGL(k_sel_cand, dim3(gs), dim3(256), 0, s, worst, T, G, rows, ckey, cidx,
                         yev ? kept : nullptr, W);
      prof_mark(s, "k_sel_final");
      hipLaunchKernelGGL(k_sel_final<1024>, dim3((unsigned)B), dim3(1024), 0, s, worst, T,
                         hi - lo, g, rows, ckey, cidx, thr, yev ? kept : nullptr, W);
    } else if (T >= 65536) {
      hipLaunchKernelGGL(k_fit_select<1024>, dim3((unsigned)B), dim3(1024), 0, s, worst, T,
                         lo, hi, g, thr, yev ? kept : nullptr, W);
    } else if (EKS_SEL_REGROWS && T <= 256 * 16) {  // the row read once, into registers
      hipLaunchKernelGGL((k_fit_select<256, 16>), dim3((unsigned)B), dim3(256), 0, s, worst, T, lo,
                         hi, g, thr, yev ? kept : nullptr, W);
    } else {
      hipLaunchKernelGGL(k_fit_select<kSelBlk>, dim3((unsigned)B), dim3(kSelBlk), 0, s, worst, T,
                         lo, hi, g, thr, yev ? kept : nullptr, W);
    }
    return check_launch("k_fit_select");
  };
  // merge the chunk partials in order, kMergeFan at a time, ping-pong
  auto merge = [&](auto Nc, int npart_) -> double * {
    constexpr int NN = decltype(Nc)::value;
    double *src = partA, *dst = partB;
    int nc = npart_;
    const long long tri = (long long)n * (n + 1) / 2;
    while (nc > 1) {
      const int nout = (nc + kMergeFan - 1) / kMergeFan;
      prof_mark(s, "k_fit_merge");
      hipLaunchKernelGGL((k_fit_merge<NN>), dim3(grid_for(B * (long long)nout * tri, 256)),
                         dim3(256), 0, s, B, nc, kMergeFan, src, dst, n);
      if (check_launch("k_fit_merge")) return nullptr;
      double *t = src;
      src = dst;
      dst = t;
      nc = nout;
    }
    return src;
  };
  // keypoint observations come in (x, y) pairs: n = 2 (single view) or 2V
  // (V cameras); the odd n are not compiled (they doubled this unit's code)
  if (n % 2 != 0 || n > kMaxObsFit)
    return set_err(EKS_ERR_UNSUPPORTED, "eks_fit: n=%d not supported (even, <= %d)", n, kMaxObsFit);
  if (n > kMaxObs) {  // 5-8 cameras: the wide kernels (runtime n, runtime E)
    if (kind != EKS_FIT_MULTICAM || r != 3)
      return set_err(EKS_ERR_UNSUPPORTED, "eks_fit: n=%d needs the PCA model with r = 3", n);
    auto wide_e = [&](auto tag, auto ytag, auto Ec) -> int {
      using Tp = decltype(tag);
      using YT = decltype(ytag);
      constexpr int EE = decltype(Ec)::value;
      prof_call_begin();
      prof_mark(s, "k_fitw_worst");
      int ncw;
      long long lcw;
      fit_chunks(B, T, ncw, lcw);  // k_fit_worst's lanes (one per (trajectory, chunk))
      const FitShape shw{B, T, ncw, lcw};
      hipLaunchKernelGGL((k_fitw_worst<Tp, YT, EE>), dim3(grid_for(B * (long long)ncw, 256)), dim3(256), 0, s,
                         (const Tp *)obs, shw, sb, st, se, sj, E, n, median, worst, yo, ks, zs);
      int rc = check_launch("k_fitw_worst");
      if (rc || (rc = select())) return rc;
      prof_mark(s, "k_fitw_accum");
      const unsigned ga = grid_for(B * (long long)sh.NC * kNW, 256);
      if (yev)
        hipLaunchKernelGGL((k_fitw_accum<Tp, YT, true, 0>), dim3(ga), dim3(256), 0, s,
                           (const Tp *)obs, sh, sb, st, se, sj, E, n, median, thr, kept, W, partA,
                           yo, ks);
      else
        hipLaunchKernelGGL((k_fitw_accum<Tp, YT, false, EE>), dim3(ga), dim3(256), 0, s,
                           (const Tp *)obs, sh, sb, st, se, sj, E, n, median, thr, kept, W, partA,
                           yo, ks);
      if ((rc = check_launch("k_fitw_accum"))) return rc;
      double *src = merge(ic<0>{}, npart);
      if (!src) return EKS_ERR_HIP;
      prof_mark(s, "k_fitw_final");
      hipLaunchKernelGGL((k_fitw_final<3>), dim3((unsigned)B), dim3(256), 0, s, B, src, ks, n,
                         smooth_param, params, status);
      prof_call_end(s);
      return check_launch("k_fitw_final");
    };
    auto wide = [&](auto tag, auto ytag) -> int {
      switch (E) {
        case 3: return wide_e(tag, ytag, ic<3>{});
        case 4: return wide_e(tag, ytag, ic<4>{});
        case 5: return wide_e(tag, ytag, ic<5>{});
        default: return wide_e(tag, ytag, ic<0>{});
      }
    };
    if (y32) return wide(float{}, float{});
    return obs_dtype == EKS_F32 ? wide(float{}, double{}) : wide(double{}, double{});
  }
  auto dispatch_even = [&](auto &&f) -> int {
    switch (n) {
      case 2: return f(ic<2>{});
      case 4: return f(ic<4>{});
      case 6: return f(ic<6>{});
      default: return f(ic<8>{});
    }
  };
  return dispatch_even([&](auto Nc) {
    constexpr int NN = decltype(Nc)::value;
    auto by_type = [&](auto tag, auto ytag) -> int {
      using Tp = decltype(tag);
      using YT = decltype(ytag);
      auto by_e = [&](auto Ec) -> int {
        constexpr int EE = decltype(Ec)::value;
        prof_call_begin();
        prof_mark(s, "k_fit_worst");
        hipLaunchKernelGGL((k_fit_worst<EE, NN, Tp, YT>), dim3(grid), dim3(256), 0, s,
                           (const Tp *)obs, sh, sb, st, se, sj, E, median, worst, yo, ks, zs);
        int rc = check_launch("k_fit_worst");
        if (rc) return rc;
        if ((rc = select())) return rc;
        prof_mark(s, "k_fit_accum");
        // with the hand-off planes written, the second pass reads the y plane
        // and the frame mask (8 B per frame for n = 2 with float32 y) instead
        // of the members (40 B) and skips the sort
        auto accum = [&](auto from_yev, auto wm) {
          constexpr bool FY = decltype(from_yev)::value != 0, WM = decltype(wm)::value != 0;
          const long long lanes = WM ? B * (long long)npart * 64 : B * (long long)sh.NC;
          // the plane path never reads the members: one instantiation per (n,
          // y type), not per member count and type
          constexpr int EA = FY ? 0 : EE;
          using TA = typename std::conditional<FY, float, Tp>::type;
          hipLaunchKernelGGL((k_fit_accum<EA, NN, TA, YT, FY, WM>), dim3(grid_for(lanes, 256)),
                             dim3(256), 0, s, (const TA *)obs, sh, sb, st, se, sj, E, median, thr,
                             kept, W, partA, yo, ks);
        };
        if (yev) {
          if (wave_merge) accum(ic<1>{}, ic<1>{});
          else accum(ic<1>{}, ic<0>{});
        } else {
          if (wave_merge) accum(ic<0>{}, ic<1>{});
          else accum(ic<0>{}, ic<0>{});
        }
        if ((rc = check_launch("k_fit_accum"))) return rc;
        double *src = merge(Nc, npart);
        if (!src) return EKS_ERR_HIP;
        prof_mark(s, "k_fit_final");
        rc = dispatch_r(r, [&](auto Rc) {
          constexpr int RR = decltype(Rc)::value;
          if constexpr (RR > NN) {
            return set_err(EKS_ERR_ARG, "eks_fit: r > n");
          } else {
            hipLaunchKernelGGL((k_fit_final<RR, NN>), dim3((unsigned)B), dim3(64), 0, s, B, src,
                               ks, kind, smooth_param, params, status);
            return check_launch("k_fit_final");
          }
        });
        prof_call_end(s);
        return rc;
      };
      switch (E) {
        case 3: return by_e(ic<3>{});
        case 4: return by_e(ic<4>{});
        case 5: return by_e(ic<5>{});
        default: return by_e(ic<0>{});
      }
    };
    if (y32) return by_type(float{}, float{});
    return obs_dtype == EKS_F32 ? by_type(float{}, double{}) : by_type(double{}, double{});
  });
}
