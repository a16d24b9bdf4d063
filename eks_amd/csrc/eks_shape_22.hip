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
