// F4: linear resampling of one camera's member predictions onto another
// camera's timestamps -- the scipy.interpolate.interp1d(kind="linear") calls
// of the asynchronous paw smoother (eks/multiview_pca_smoother.py:82-99).
//
//   k_interp1d   one thread per (query, column): binary search of the
//                query in the ascending sample times, then the arithmetic
//                interp1d delegates to for 1-D float64 data (np.interp):
//                  j with x[j] <= xq < x[j+1]; exact hits return y[j]
//                  slope = (y[j+1] - y[j]) / (x[j+1] - x[j])
//                  out   = slope * (xq - x[j]) + y[j]   (NaN: from the right)
//                with each operation rounded separately (no FMA
//                contraction), so the result is bit-identical to numpy's.
// Queries outside [x[0], x[nx-1]] are flagged (scipy raises ValueError); the
// reference only evaluates inside that range.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/eks_hip.h"
#include "eks_common.hpp"

namespace eks {
namespace {

__global__ __launch_bounds__(256) void k_interp1d(const double *__restrict__ x, long long nx,
                                                  const double *__restrict__ y, long long ncol,
                                                  long long sy_row, long long sy_col,
                                                  const double *__restrict__ xq, long long nq,
                                                  double *__restrict__ out, long long so_row,
                                                  long long so_col, int32_t *__restrict__ status) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= nq * ncol) return;
  const long long q = i / ncol, c = i - q * ncol;
  const double v = xq[q];
  if (!(v >= x[0] && v <= x[nx - 1])) {
    if (status && c == 0) status[q] = EKS_STATUS_BAD_MODEL;
    out[q * so_row + c * so_col] = __builtin_nan("");
    return;
  }
  // j with x[j] <= v < x[j+1] (count of x[k] <= v, minus one)
  long long lo = 0, hi = nx;
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if (x[mid] <= v)
      lo = mid + 1;
    else
      hi = mid;
  }
  const long long j = lo - 1;
  const double *yc = y + c * sy_col;
  double r;
  if (v == x[nx - 1]) {
    r = yc[(nx - 1) * sy_row];  // right edge
  } else if (x[j] == v) {
    r = yc[j * sy_row];         // exact sample time
  } else {
#pragma clang fp contract(off)
    const double y0 = yc[j * sy_row], y1 = yc[(j + 1) * sy_row];
    const double slope = (y1 - y0) / (x[j + 1] - x[j]);
    r = slope * (v - x[j]) + y0;
    if (r != r) {  // NaN from one side: try the other (numpy's rule)
      r = slope * (v - x[j + 1]) + y1;
      if (r != r && y0 == y1) r = y0;
    }
  }
  out[q * so_row + c * so_col] = r;
  if (status && c == 0) status[q] = 0;
}

}  // namespace
}  // namespace eks

using namespace eks;

extern "C" int eks_interp1d(const double *x, int64_t nx, const double *y, int64_t ncol,
                            int64_t sy_row, int64_t sy_col, const double *xq, int64_t nq,
                            double *out, int64_t so_row, int64_t so_col, int32_t *status,
                            void *stream) {
  clear_err();
  if (!x || !y || !xq || !out) return set_err(EKS_ERR_ARG, "eks_interp1d: NULL pointer");
  if (nx < 2 || ncol < 0 || nq < 0) return set_err(EKS_ERR_ARG, "eks_interp1d: need nx >= 2");
  if (nq == 0 || ncol == 0) return EKS_OK;
  hipLaunchKernelGGL(k_interp1d, dim3(grid_for(nq * ncol, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, nx, y, ncol, sy_row, sy_col, xq, nq, out, so_row,
                     so_col, status);
  return check_launch("k_interp1d");
}
