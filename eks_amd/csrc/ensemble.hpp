// Ensemble reduction over E members (eks/ensemble_kalman.py:34-46), in
// registers, the one arithmetic every kernel uses (eks_ensemble, the fit,
// every smoother), so hand-offs between them are bit-identical:
//   mean = sum(x) * (1/E)    (numpy's summation order; the division as a
//                             product by the reciprocal: <= 1 ulp from
//                             numpy's x / E, exact for E a power of two)
//   var  = sum((x - mean)^2) * (1/E^2)   (np.var ddof=0, then / E; <= 2 ulp)
//   median: middle order statistic, or (lo + hi) / 2 for even E
// and propagates NaN as np.median / np.var do.
#pragma once
#include <type_traits>

#include "small_linalg.hpp"

namespace eks {

template <typename T>
EKS_DEV double to_f64(T v) { return static_cast<double>(v); }

// A rounded product the compiler may not fuse into its consumers (x - mean,
// P + var, ...): with fp-contract the fusion would depend on where the
// function is inlined, and a kernel reading y / ev from the fit's planes must
// see the same bits as one computing them itself.
EKS_DEV double rounded(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

// numpy-order summation of a register array: numpy's pairwise_sum rule for
// n <= 128 (sequential below 8 elements, 8 interleaved partial sums above).
template <int E>
EKS_DEV double np_sum(const double (&x)[E]) {
  if constexpr (E < 8) {
    double s = x[0];
#pragma unroll
    for (int i = 1; i < E; ++i) s += x[i];
    return s;
  } else {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = x[j];
    constexpr int full = E - (E % 8);
#pragma unroll
    for (int i = 8; i < full; i += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += x[i + j];
    double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int k = full; k < E; ++k) s += x[k];
    return s;
  }
}

// Sorting network (odd-even transposition) on E values of the input type:
// min/max on the raw member values is exact, the median is converted after.
template <int E, typename T>
EKS_DEV void sort_net(T (&v)[E]) {
#pragma unroll
  for (int p = 0; p < E; ++p)
#pragma unroll
    for (int i = p & 1; i + 1 < E; i += 2) {
      const T a = v[i], b = v[i + 1];
      v[i] = a < b ? a : b;
      v[i + 1] = a < b ? b : a;
    }
}

// min / max of floats as one v_med3_f32 each: med3(a, b, -inf) = min(a, b).
// The infinities go through an empty asm so the compiler cannot turn the med3
// back into a v_min/v_max, which in IEEE mode costs a canonicalisation of
// every input (NaN members are handled by the caller's flag, not here).
struct F32MinMax {
  float ninf = -__builtin_inff(), pinf = __builtin_inff();
  EKS_DEV F32MinMax() {
    asm volatile("" : "+s"(ninf));
    asm volatile("" : "+s"(pinf));
  }
  EKS_DEV float mn(float a, float b) const { return __builtin_amdgcn_fmed3f(a, b, ninf); }
  EKS_DEV float mx(float a, float b) const { return __builtin_amdgcn_fmed3f(a, b, pinf); }
};

// the median of E member values (exact: a selection, or the mean of the two
// middle ones for even E)
template <int E, typename T>
EKS_DEV double median_of(const T (&raw)[E]) {
  if constexpr (std::is_same<T, float>::value && (E == 3 || E == 4 || E == 5)) {
    if constexpr (E == 3) {  // 1 v_med3_f32
      return (double)__builtin_amdgcn_fmed3f(raw[0], raw[1], raw[2]);
    } else if constexpr (E == 4) {
      // the two middle values of four are {max(p, q), min(P, Q)} for the
      // pairs' minima p, q and maxima P, Q (4 med3 + 2 instead of a sorting
      // network); numpy's mean of the two, (s1 + s2) / 2 (the addition
      // commutes, so their order does not matter)
      const F32MinMax f;
      const float a = f.mx(f.mn(raw[0], raw[1]), f.mn(raw[2], raw[3]));
      const float b = f.mn(f.mx(raw[0], raw[1]), f.mx(raw[2], raw[3]));
      return ((double)a + (double)b) / 2.0;
    } else {  // 7: drop the min and max of s0..s3, then the median of 3
      const F32MinMax f;
      const float lo = f.mx(f.mn(raw[0], raw[1]), f.mn(raw[2], raw[3]));
      const float hi = f.mn(f.mx(raw[0], raw[1]), f.mx(raw[2], raw[3]));
      return (double)__builtin_amdgcn_fmed3f(lo, hi, raw[4]);
    }
  } else {
    T v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = raw[e];
    sort_net<E, T>(v);
    if constexpr (E % 2 == 1)
      return to_f64(v[E / 2]);
    else
      return (to_f64(v[E / 2 - 1]) + to_f64(v[E / 2])) / 2.0;
  }
}

// Reduce one column of E member values (compile-time E).
template <int E, typename T>
EKS_DEV void ensemble_reduce(const T (&raw)[E], bool median, double &avg, double &var) {
  constexpr double invE = 1.0 / (double)E, invE2 = 1.0 / ((double)E * (double)E);
  double x[E];
#pragma unroll
  for (int e = 0; e < E; ++e) x[e] = to_f64(raw[e]);
  const double mean = rounded(np_sum<E>(x) * invE);
  double d[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const double t = x[e] - mean;
    d[e] = t * t;
  }
  var = rounded(np_sum<E>(d) * invE2);  // NaN members make it NaN by themselves
  if (median) {
    avg = median_of<E, T>(raw);
    // a NaN member makes the sum NaN, so only a NaN mean (a NaN member, or
    // +inf and -inf members) needs the per-member test: one compare per
    // column on the common path instead of E.  The selection would skip NaN
    // members; np.median returns NaN.
    const bool mnan = mean != mean;
    if (__builtin_amdgcn_ballot_w64(mnan) != 0) {  // wave-uniform: skipped as a whole
      asm volatile("");  // not speculated: the common path runs none of this
      bool has_nan = false;
#pragma unroll
      for (int e = 0; e < E; ++e) has_nan |= (raw[e] != raw[e]);
      if (mnan && has_nan) avg = __builtin_nan("");
    }
  } else {
    avg = mean;
  }
}

// Runtime-E reduction (E up to EKS_MAX_MEMBERS) reading members straight from
// memory: O(E^2) rank selection for the median.  Used only when E has no
// compiled-in specialisation.
template <typename T>
EKS_DEV void ensemble_reduce_rt(const T *p, long long se, int E, bool median, double &avg,
                                double &var) {
  bool has_nan = false;
  // numpy pairwise_sum order over f(0..E-1)
  auto np_sum_rt = [&](auto f) {
    if (E < 8) {
      double s = f(0);
      for (int i = 1; i < E; ++i) s += f(i);
      return s;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f(j);
    const int full = E - (E % 8);
    for (int i = 8; i < full; i += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += f(i + j);
    double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (int k = full; k < E; ++k) s += f(k);
    return s;
  };
  // the compiled path's arithmetic (products by the reciprocals)
  const double invE = 1.0 / (double)E, invE2 = 1.0 / ((double)E * (double)E);
  const double mean = rounded(np_sum_rt([&](int i) { return to_f64(p[(long long)i * se]); }) * invE);
  var = rounded(np_sum_rt([&](int i) {
          const double t = to_f64(p[(long long)i * se]) - mean;
          return t * t;
        }) * invE2);
  for (int e = 0; e < E; ++e) {
    const double v = to_f64(p[(long long)e * se]);
    has_nan |= (v != v);
  }
  if (median) {
    // order statistics k_lo, k_hi (equal for odd E)
    const int k_hi = E / 2, k_lo = (E % 2) ? E / 2 : E / 2 - 1;
    double v_lo = 0.0, v_hi = 0.0;
    for (int i = 0; i < E; ++i) {
      const T xi = p[(long long)i * se];
      int less = 0, eq = 0;
      for (int j = 0; j < E; ++j) {
        const T xj = p[(long long)j * se];
        less += (xj < xi);
        eq += (xj == xi);
      }
      if (less <= k_lo && k_lo < less + eq) v_lo = to_f64(xi);
      if (less <= k_hi && k_hi < less + eq) v_hi = to_f64(xi);
    }
    avg = (E % 2) ? v_hi : (v_lo + v_hi) / 2.0;
  } else {
    avg = mean;
  }
  if (has_nan) {
    avg = __builtin_nan("");
    var = __builtin_nan("");
  }
}

// One coordinate's ensemble from memory (members se apart): the compiled-E
// reduction on registers when E > 0, else the runtime-E one.  The
// runtime-n kernels use it so that the common member counts (3, 4, 5) do not
// pay the runtime reduction's O(E^2) memory reads.
template <int E, typename T>
EKS_DEV void column_reduce(const T *p, long long se, int Ert, bool median, double &avg,
                           double &var) {
  if constexpr (E > 0) {
    T raw[E];
#pragma unroll
    for (int e = 0; e < E; ++e) raw[e] = p[(long long)e * se];
    ensemble_reduce<E, T>(raw, median, avg, var);
  } else {
    ensemble_reduce_rt<T>(p, se, Ert, median, avg, var);
  }
}

// A run of (step, column) pairs -- steps [s, e), n columns each -- as one
// flattened stream with the loads of the next DP columns in flight (the
// runtime-n kernels: eks_shape_rt.hip, the wide fit): the column's observation (members or
// plane values) and its row of C with the offset.  One lane walks one
// trajectory's chunk sequentially, so without this every column paid a full
// load latency (n = 12: 12 round trips per step).  fetch(k, t, j) loads
// column (t, j) into ring slot k (indices clamped into the chunk: a cache-hit
// re-read past its end keeps the loads unconditional); col(k, t, j) consumes
// slot k; begin(t) / end(t) bracket each step.
constexpr int kRtDP = 4;
template <typename Fetch, typename Col, typename Begin, typename End>
EKS_DEV void rt_columns(long long s, long long e, int n, Fetch &&fetch, Col &&col, Begin &&begin,
                        End &&end) {
  constexpr int DP = kRtDP;
  const long long Q = (e - s) * n;
  long long tf = s;  // next column to fetch: (tf, jf)
  int jf = 0;
  auto fetch_next = [&](int k) {
    if (tf < e) fetch(k, tf, jf);
    else fetch(k, e - 1, n - 1);
    if (++jf == n) {
      jf = 0;
      ++tf;
    }
  };
#pragma unroll
  for (int k = 0; k < DP; ++k) fetch_next(k);
  long long t = s;
  int j = 0;
  for (long long q = 0; q < Q; q += DP) {
#pragma unroll
    for (int k = 0; k < DP; ++k) {
      if (q + k < Q) {
        if (j == 0) begin(t);
        col(k, t, j);  // consumes slot k
        fetch_next(k);
        if (++j == n) {
          j = 0;
          end(t);
          ++t;
        }
      }
    }
  }
}

}  // namespace eks
