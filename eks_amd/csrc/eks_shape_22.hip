// Fused-smoother kernels instantiated for latent r = 2, observations n = 2
// (one translation unit per shape so hipcc compiles them in parallel).
#include "smooth_impl.hpp"

namespace eks {

int launch_22(const SmoothArgs &a, int algo, long long L) {
  const int flags = a.flags;
  if ((flags & EKS_MODEL_A_IDENTITY) && (flags & EKS_MODEL_C_IDENTITY))
    return launch_shape<2, 2, kAId, kCId>(a, algo, L);
  return launch_shape<2, 2, kAGen, kCGen>(a, algo, L);
}

}  // namespace eks

#if EKS_STAMPS
// profiling builds only (-DEKS_STAMPS=1): copy algo 3's phase stamps to the host
extern "C" int eks_dbg_stamps(void *dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(eks::g_stamps), bytes);
}
#endif
