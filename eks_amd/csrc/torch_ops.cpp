// torch.ops.eks.*: the C ABI of libeks_hip.so registered as PyTorch operators
// in C++ ("the torch extension wraps the same functions as
// torch.ops.eks.*"; BASELINE north star: ensemble() / forward_pass() /
// backward_pass() / compute_nll() as a PyTorch-ROCm C++/HIP extension).
//
// Built by eks_amd/build.py into eks_amd/lib/libeks_torch.so (linked against
// libtorch and libeks_hip.so) and loaded by eks_amd/ops.py with
// torch.ops.load_library: the operators' dispatch has no Python frame.  Each
// operator has a CUDA-key kernel (the HIP device: on ROCm builds of PyTorch
// the GPU dispatch key is CUDA) that launches on the current stream, and a
// Meta kernel that only computes shapes (FakeTensor / torch.compile tracing).
// There is no CPU kernel: a CPU tensor is a dispatch error.
//
//   eks::ensemble(obs, mode)                       eks/ensemble_kalman.py:4-57
//   eks::forward(y, ev, m0, S0, A, Q, C)           :59-117  (filtering_pass)
//   eks::backward(mf, Vf, S, A)                    :120-164 (smooth_backward)
//   eks::nll(obs, params, n, r, mode, flags)       compute_nll
//   eks::smooth(obs, params, n, r, mode, flags, algo)  the fused hot path
//   eks::fit(obs, kind, n, r, s, q, mode)          eks/multiview_pca_smoother.py:684-731
//   eks::newton_filter(y, ev, mu0, S0, A, Bm, E, max_iter)  eks/newton_eks.py:115-148
//   eks::interp1d(x, y, xq)                        eks/multiview_pca_smoother.py:86-96
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <initializer_list>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/eks_hip.h"

namespace {

using at::Tensor;

// (ROCm PyTorch: the HIP device is the "cuda" device type; its streams and
// guard are the masquerading ones)
void* cur_stream(const Tensor& t) {
  return (void*)at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check(int rc, const char* what) {
  TORCH_CHECK(rc == EKS_OK, what, " failed (code ", rc, "): ", eks_last_error());
}

int mode_code(const std::string& mode) {
  TORCH_CHECK(mode == "median" || mode == "mean", mode, " averaging not supported");
  return mode == "median" ? EKS_MEDIAN : EKS_MEAN;
}

int obs_dtype(const Tensor& obs) {
  TORCH_CHECK(obs.scalar_type() == at::kFloat || obs.scalar_type() == at::kDouble,
              "obs must be float32 or float64");
  return obs.scalar_type() == at::kFloat ? EKS_F32 : EKS_F64;
}

void need_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "eks ops run on the GPU only (no CPU fallback): ", name,
              " is a ", t.device().str(), " tensor");
}

at::TensorOptions f64(const Tensor& like) { return like.options().dtype(at::kDouble); }
at::TensorOptions i32(const Tensor& like) { return like.options().dtype(at::kInt); }

Tensor contiguous_f64(const Tensor& t) { return t.to(at::kDouble).contiguous(); }

// an argument of the call's device: moved there (float64, contiguous) when it
// is a host / numpy-derived tensor, so no host pointer reaches a kernel
Tensor on_dev_f64(const Tensor& t, const Tensor& like) {
  return t.to(like.device(), at::kDouble).contiguous();
}

// model argument `t` must be lead + shp: per trajectory (lead = {B}) or
// shared by every trajectory (lead = {}), as the Python shims check
// (eks_amd/newton_eks.py: newton_filter_batch)
void check_shape(const Tensor& t, const char* name, bool shared, int64_t B,
                 std::initializer_list<int64_t> shp) {
  std::vector<int64_t> want;
  if (!shared) want.push_back(B);
  want.insert(want.end(), shp.begin(), shp.end());
  TORCH_CHECK(t.sizes().vec() == want, name, " has shape ", t.sizes(), ", expected ",
              at::IntArrayRef(want));
}

// ---------------------------------------------------------------- ensemble
std::tuple<Tensor, Tensor> ensemble_gpu(const Tensor& obs, const std::string& mode) {
  need_gpu(obs, "obs");
  TORCH_CHECK(obs.dim() == 4, "obs must be viewed as (B, T, E, n)");
  const c10::DeviceGuard g(obs.device());
  const int64_t B = obs.size(0), T = obs.size(1), E = obs.size(2), n = obs.size(3);
  Tensor preds = at::empty({B, T, n}, f64(obs));
  Tensor vars = at::empty({B, T, n}, f64(obs));
  check(eks_ensemble(obs.data_ptr(), obs_dtype(obs), B, T, (int)E, (int)n, obs.stride(0),
                     obs.stride(1), obs.stride(2), obs.stride(3), mode_code(mode),
                     preds.data_ptr<double>(), vars.data_ptr<double>(), cur_stream(obs)),
        "eks_ensemble");
  return {preds, vars};
}
std::tuple<Tensor, Tensor> ensemble_meta(const Tensor& obs, const std::string&) {
  TORCH_CHECK(obs.dim() == 4, "obs must be viewed as (B, T, E, n)");
  auto o = obs.options().dtype(at::kDouble);
  return {at::empty({obs.size(0), obs.size(1), obs.size(3)}, o),
          at::empty({obs.size(0), obs.size(1), obs.size(3)}, o)};
}

// ----------------------------------------------------------------- forward
// y, ev (B, T, n); m0 (B, r); S0, A, Q (B, r, r); C (B, n, r) -- or, with no
// leading B, one model shared by every trajectory.  R is diagonal = ev[t]
// (the reference overwrites R's diagonal every step and never reads the rest
// unless the caller's R has off-diagonal entries: the Python shim passes R).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> forward_gpu(const Tensor& y, const Tensor& ev,
                                                               const Tensor& m0, const Tensor& S0,
                                                               const Tensor& A, const Tensor& Q,
                                                               const Tensor& C) {
  need_gpu(y, "y");
  TORCH_CHECK(y.dim() == 3 && ev.sizes() == y.sizes(), "y and ev must both be (B, T, n)");
  TORCH_CHECK(m0.dim() == 1 || m0.dim() == 2, "m0 must be (r,) or (B, r)");
  const c10::DeviceGuard g(y.device());
  const int64_t B = y.size(0), T = y.size(1), n = y.size(2), r = m0.size(-1);
  const bool sh = m0.dim() == 1;
  const int shared = sh ? 1 : 0;
  check_shape(m0, "m0", sh, B, {r});
  check_shape(S0, "S0", sh, B, {r, r});
  check_shape(A, "A", sh, B, {r, r});
  check_shape(Q, "Q", sh, B, {r, r});
  check_shape(C, "C", sh, B, {n, r});
  Tensor y_ = contiguous_f64(y), ev_ = on_dev_f64(ev, y);
  Tensor m0_ = on_dev_f64(m0, y), S0_ = on_dev_f64(S0, y), A_ = on_dev_f64(A, y);
  Tensor Q_ = on_dev_f64(Q, y), C_ = on_dev_f64(C, y);
  Tensor mf = at::empty({B, T, r}, f64(y));
  Tensor Vf = at::empty({B, T, r, r}, f64(y));
  Tensor S = at::empty({B, T, r, r}, f64(y));
  Tensor nll = at::empty({B}, f64(y));
  Tensor status = at::zeros({B}, i32(y));
  check(eks_forward(B, T, (int)n, (int)r, y_.data_ptr<double>(), ev_.data_ptr<double>(),
                    m0_.data_ptr<double>(), S0_.data_ptr<double>(), A_.data_ptr<double>(),
                    Q_.data_ptr<double>(), C_.data_ptr<double>(), nullptr, shared,
                    mf.data_ptr<double>(), Vf.data_ptr<double>(), S.data_ptr<double>(),
                    nll.data_ptr<double>(), status.data_ptr<int32_t>(), cur_stream(y)),
        "eks_forward");
  return {mf, Vf, S, nll, status};
}
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> forward_meta(const Tensor& y, const Tensor&,
                                                                const Tensor& m0, const Tensor&,
                                                                const Tensor&, const Tensor&,
                                                                const Tensor&) {
  const int64_t B = y.size(0), T = y.size(1), r = m0.size(-1);
  auto o = y.options().dtype(at::kDouble);
  return {at::empty({B, T, r}, o), at::empty({B, T, r, r}, o), at::empty({B, T, r, r}, o),
          at::empty({B}, o), at::empty({B}, y.options().dtype(at::kInt))};
}

// ---------------------------------------------------------------- backward
std::tuple<Tensor, Tensor, Tensor, Tensor> backward_gpu(const Tensor& mf, const Tensor& Vf,
                                                        const Tensor& S, const Tensor& A) {
  need_gpu(mf, "mf");
  TORCH_CHECK(mf.dim() == 3, "mf must be (B, T, r)");
  TORCH_CHECK(A.dim() == 2 || A.dim() == 3, "A must be (r, r) or (B, r, r)");
  const c10::DeviceGuard g(mf.device());
  const int64_t B = mf.size(0), T = mf.size(1), r = mf.size(2);
  const bool sh = A.dim() == 2;
  const int shared = sh ? 1 : 0;
  TORCH_CHECK(Vf.sizes() == at::IntArrayRef({B, T, r, r}), "Vf has shape ", Vf.sizes(),
              ", expected (", B, ", ", T, ", ", r, ", ", r, ")");
  TORCH_CHECK(S.sizes() == at::IntArrayRef({B, T, r, r}), "S has shape ", S.sizes(),
              ", expected (", B, ", ", T, ", ", r, ", ", r, ")");
  check_shape(A, "A", sh, B, {r, r});
  Tensor mf_ = contiguous_f64(mf), Vf_ = on_dev_f64(Vf, mf), S_ = on_dev_f64(S, mf);
  Tensor A_ = on_dev_f64(A, mf);
  Tensor ms = at::empty({B, T, r}, f64(mf));
  Tensor Vs = at::empty({B, T, r, r}, f64(mf));
  Tensor CV = at::empty({B, T > 1 ? T - 1 : 0, r, r}, f64(mf));
  Tensor status = at::zeros({B}, i32(mf));
  check(eks_backward(B, T, (int)r, mf_.data_ptr<double>(), Vf_.data_ptr<double>(),
                     S_.data_ptr<double>(), A_.data_ptr<double>(), shared, ms.data_ptr<double>(),
                     Vs.data_ptr<double>(), T > 1 ? CV.data_ptr<double>() : nullptr,
                     status.data_ptr<int32_t>(), cur_stream(mf)),
        "eks_backward");
  return {ms, Vs, CV, status};
}
std::tuple<Tensor, Tensor, Tensor, Tensor> backward_meta(const Tensor& mf, const Tensor&,
                                                         const Tensor&, const Tensor&) {
  const int64_t B = mf.size(0), T = mf.size(1), r = mf.size(2);
  auto o = mf.options().dtype(at::kDouble);
  return {at::empty({B, T, r}, o), at::empty({B, T, r, r}, o),
          at::empty({B, T > 1 ? T - 1 : 0, r, r}, o), at::empty({B}, mf.options().dtype(at::kInt))};
}

// --------------------------------------------------------- smooth / nll
// workspace: a fresh byte tensor from PyTorch's caching allocator (stream
// ordered on the current stream, so reuse across calls is free)
std::tuple<Tensor, Tensor, Tensor> smooth_impl(const Tensor& obs, const Tensor& params, int64_t n,
                                               int64_t r, const std::string& mode, int64_t flags,
                                               int64_t algo, bool want_out) {
  need_gpu(obs, "obs");
  need_gpu(params, "params");
  TORCH_CHECK(params.device() == obs.device(), "params is on ", params.device().str(),
              ", obs on ", obs.device().str());
  TORCH_CHECK(obs.dim() == 4 && obs.size(3) == n, "obs must be viewed as (B, T, E, n) with n=", n);
  const c10::DeviceGuard g(obs.device());
  const int64_t B = obs.size(0), T = obs.size(1), E = obs.size(2);
  Tensor prm = params.contiguous();
  TORCH_CHECK(prm.scalar_type() == at::kDouble && prm.dim() == 2 && prm.size(0) == B &&
                  prm.size(1) == eks_param_len((int)n, (int)r),
              "params must be a (", B, ", ", eks_param_len((int)n, (int)r), ") float64 tensor");
  // time-major output buffer (coalesced stores), returned as a (B, T, n) view
  Tensor out_tm = want_out ? at::empty({T, B, n}, f64(obs)) : Tensor();
  Tensor nll = want_out ? Tensor() : at::empty({B}, f64(obs));
  Tensor status = at::empty({B}, i32(obs));
  const size_t wsb = eks_smooth_workspace_bytes(B, T, (int)n, (int)r, (int)E, (int)algo);
  Tensor ws = at::empty({(int64_t)std::max<size_t>(wsb, 1)}, obs.options().dtype(at::kByte));
  check(eks_smooth(obs.data_ptr(), obs_dtype(obs), B, T, (int)E, (int)n, (int)r, obs.stride(0),
                   obs.stride(1), obs.stride(2), obs.stride(3), mode_code(mode),
                   prm.data_ptr<double>(), want_out ? out_tm.data_ptr<double>() : nullptr,
                   want_out ? n : 0, want_out ? B * n : 0, 1, nullptr,
                   want_out ? nullptr : nll.data_ptr<double>(), ws.data_ptr(), (size_t)ws.numel(),
                   (int)flags, (int)algo, status.data_ptr<int32_t>(), cur_stream(obs)),
        "eks_smooth");
  Tensor out = want_out ? out_tm.permute({1, 0, 2}).contiguous() : Tensor();
  return {out, nll, status};
}
std::tuple<Tensor, Tensor> smooth_gpu(const Tensor& obs, const Tensor& params, int64_t n,
                                      int64_t r, const std::string& mode, int64_t flags,
                                      int64_t algo) {
  auto res = smooth_impl(obs, params, n, r, mode, flags, algo, true);
  return {std::get<0>(res), std::get<2>(res)};
}
std::tuple<Tensor, Tensor> smooth_meta(const Tensor& obs, const Tensor&, int64_t n, int64_t,
                                       const std::string&, int64_t, int64_t) {
  return {at::empty({obs.size(0), obs.size(1), n}, obs.options().dtype(at::kDouble)),
          at::empty({obs.size(0)}, obs.options().dtype(at::kInt))};
}
// compute_nll: the filter-only pass; raises where the reference's solve would
// (singular system) or when a model promise does not hold
Tensor nll_gpu(const Tensor& obs, const Tensor& params, int64_t n, int64_t r,
               const std::string& mode, int64_t flags) {
  auto res = smooth_impl(obs, params, n, r, mode, flags, 0, false);
  Tensor st = std::get<2>(res);
  const int64_t bad = st.ne(0).sum().item<int64_t>();
  if (bad) {
    // a chain breakdown (EKS_STATUS_SCAN) is retried with the sequential algorithm
    if (st.bitwise_and(EKS_STATUS_SCAN).ne(0).any().item<bool>())
      res = smooth_impl(obs, params, n, r, mode, flags, 1, false);
    st = std::get<2>(res);
    TORCH_CHECK(!st.bitwise_and(EKS_STATUS_BAD_MODEL).ne(0).any().item<bool>(),
                "eks::nll: a model_flags promise does not hold");
    TORCH_CHECK(!st.ne(0).any().item<bool>(), "eks::nll: singular system (LinAlgError)");
  }
  return std::get<1>(res);
}
Tensor nll_meta(const Tensor& obs, const Tensor&, int64_t, int64_t, const std::string&, int64_t) {
  return at::empty({obs.size(0)}, obs.options().dtype(at::kDouble));
}

// --------------------------------------------------------------------- fit
std::tuple<Tensor, Tensor> fit_gpu(const Tensor& obs, const std::string& kind, int64_t n, int64_t r,
                                   double smooth_param, double quantile_keep,
                                   const std::string& mode) {
  need_gpu(obs, "obs");
  TORCH_CHECK(obs.dim() == 4 && obs.size(3) == n, "obs must be viewed as (B, T, E, n) with n=", n);
  TORCH_CHECK(kind == "singleview" || kind == "multicam", "kind must be singleview or multicam");
  const c10::DeviceGuard g(obs.device());
  const int64_t B = obs.size(0), T = obs.size(1), E = obs.size(2);
  Tensor params = at::empty({B, eks_param_len((int)n, (int)r)}, f64(obs));
  Tensor status = at::empty({B}, i32(obs));
  const size_t wsb = eks_fit_workspace_bytes(B, T, (int)n);
  Tensor ws = at::empty({(int64_t)std::max<size_t>(wsb, 1)}, obs.options().dtype(at::kByte));
  check(eks_fit(obs.data_ptr(), obs_dtype(obs), B, T, (int)E, (int)n, (int)r, obs.stride(0),
                obs.stride(1), obs.stride(2), obs.stride(3), mode_code(mode),
                kind == "singleview" ? EKS_FIT_SINGLEVIEW : EKS_FIT_MULTICAM, smooth_param,
                quantile_keep, params.data_ptr<double>(), ws.data_ptr(), (size_t)ws.numel(),
                status.data_ptr<int32_t>(), nullptr, cur_stream(obs)),
        "eks_fit");
  return {params, status};
}
std::tuple<Tensor, Tensor> fit_meta(const Tensor& obs, const std::string&, int64_t n, int64_t r,
                                    double, double, const std::string&) {
  return {at::empty({obs.size(0), eks_param_len((int)n, (int)r)}, obs.options().dtype(at::kDouble)),
          at::empty({obs.size(0)}, obs.options().dtype(at::kInt))};
}

// ---------------------------------------------------------- newton_filter
std::tuple<Tensor, Tensor> newton_gpu(const Tensor& y, const Tensor& ev, const Tensor& mu0,
                                      const Tensor& S0, const Tensor& A, const Tensor& Bm,
                                      const Tensor& E, int64_t max_iter) {
  need_gpu(y, "y");
  TORCH_CHECK(y.dim() == 3 && ev.sizes() == y.sizes(), "y and ev must both be (B, T, n)");
  TORCH_CHECK(mu0.dim() == 1 || mu0.dim() == 2, "mu0 must be (r,) or (B, r)");
  const c10::DeviceGuard g(y.device());
  const int64_t B = y.size(0), T = y.size(1), n = y.size(2), r = mu0.size(-1);
  const bool sh = mu0.dim() == 1;
  const int shared = sh ? 1 : 0;
  check_shape(mu0, "mu0", sh, B, {r});
  check_shape(S0, "S0", sh, B, {r, r});
  check_shape(A, "A", sh, B, {r, r});
  check_shape(Bm, "B", sh, B, {n, r});
  check_shape(E, "E", sh, B, {r, r});
  Tensor y_ = contiguous_f64(y), ev_ = on_dev_f64(ev, y), mu0_ = on_dev_f64(mu0, y);
  Tensor S0_ = on_dev_f64(S0, y), A_ = on_dev_f64(A, y), B_ = on_dev_f64(Bm, y),
         E_ = on_dev_f64(E, y);
  Tensor q = at::empty({B, T, r}, f64(y));
  Tensor status = at::zeros({B}, i32(y));
  check(eks_newton_filter(B, T, (int)n, (int)r, y_.data_ptr<double>(), ev_.data_ptr<double>(),
                          mu0_.data_ptr<double>(), S0_.data_ptr<double>(), A_.data_ptr<double>(),
                          B_.data_ptr<double>(), E_.data_ptr<double>(), shared, (int)max_iter,
                          q.data_ptr<double>(), status.data_ptr<int32_t>(), cur_stream(y)),
        "eks_newton_filter");
  return {q, status};
}
std::tuple<Tensor, Tensor> newton_meta(const Tensor& y, const Tensor&, const Tensor& mu0,
                                       const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                                       int64_t) {
  return {at::empty({y.size(0), y.size(1), mu0.size(-1)}, y.options().dtype(at::kDouble)),
          at::empty({y.size(0)}, y.options().dtype(at::kInt))};
}

// --------------------------------------------------------------- interp1d
Tensor interp_gpu(const Tensor& x, const Tensor& y, const Tensor& xq) {
  need_gpu(x, "x");
  TORCH_CHECK(y.dim() == 2 && x.dim() == 1 && xq.dim() == 1 && y.size(0) == x.size(0),
              "x (n,), y (n, C), xq (q,)");
  const c10::DeviceGuard g(x.device());
  Tensor x_ = contiguous_f64(x), y_ = y.to(x.device(), at::kDouble), xq_ = on_dev_f64(xq, x);
  const int64_t n = x_.size(0), C = y_.size(1), q = xq_.size(0);
  Tensor out = at::empty({q, C}, f64(x));
  Tensor status = at::zeros({q}, i32(x));
  check(eks_interp1d(x_.data_ptr<double>(), n, y_.data_ptr<double>(), C, y_.stride(0),
                     y_.stride(1), xq_.data_ptr<double>(), q, out.data_ptr<double>(), out.stride(0),
                     out.stride(1), status.data_ptr<int32_t>(), cur_stream(x)),
        "eks_interp1d");
  TORCH_CHECK(!status.ne(0).any().item<bool>(),
              "A value in x_new is outside the interpolation range.");
  return out;
}
Tensor interp_meta(const Tensor&, const Tensor& y, const Tensor& xq) {
  return at::empty({xq.size(0), y.size(1)}, y.options().dtype(at::kDouble));
}

}  // namespace

TORCH_LIBRARY(eks, m) {
  m.def("ensemble(Tensor obs, str mode) -> (Tensor, Tensor)");
  m.def("forward(Tensor y, Tensor ev, Tensor m0, Tensor S0, Tensor A, Tensor Q, Tensor C) -> "
        "(Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("backward(Tensor mf, Tensor Vf, Tensor S, Tensor A) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("smooth(Tensor obs, Tensor params, int n, int r, str mode, int flags, int algo) -> "
        "(Tensor, Tensor)");
  m.def("nll(Tensor obs, Tensor params, int n, int r, str mode, int flags) -> Tensor");
  m.def("fit(Tensor obs, str kind, int n, int r, float smooth_param, float quantile_keep, "
        "str mode) -> (Tensor, Tensor)");
  m.def("newton_filter(Tensor y, Tensor ev, Tensor mu0, Tensor S0, Tensor A, Tensor Bm, "
        "Tensor E, int max_iter) -> (Tensor, Tensor)");
  m.def("interp1d(Tensor x, Tensor y, Tensor xq) -> Tensor");
}

TORCH_LIBRARY_IMPL(eks, CUDA, m) {
  m.impl("ensemble", &ensemble_gpu);
  m.impl("forward", &forward_gpu);
  m.impl("backward", &backward_gpu);
  m.impl("smooth", &smooth_gpu);
  m.impl("nll", &nll_gpu);
  m.impl("fit", &fit_gpu);
  m.impl("newton_filter", &newton_gpu);
  m.impl("interp1d", &interp_gpu);
}

TORCH_LIBRARY_IMPL(eks, Meta, m) {
  m.impl("ensemble", &ensemble_meta);
  m.impl("forward", &forward_meta);
  m.impl("backward", &backward_meta);
  m.impl("smooth", &smooth_meta);
  m.impl("nll", &nll_meta);
  m.impl("fit", &fit_meta);
  m.impl("newton_filter", &newton_meta);
  m.impl("interp1d", &interp_meta);
}
