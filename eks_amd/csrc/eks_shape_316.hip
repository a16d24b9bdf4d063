// Fused-smoother kernels instantiated for latent r = 3, observations n = 16
// (eight cameras; one translation unit per shape so hipcc compiles them in
// parallel).
#include "smooth_impl.hpp"

namespace eks {

int launch_316(const SmoothArgs &a, int algo, long long L) {
  const int flags = a.flags;
  if (flags & EKS_MODEL_A_IDENTITY) return launch_shape<3, 16, kAId, kCGen>(a, algo, L);
  return launch_shape<3, 16, kAGen, kCGen>(a, algo, L);
}

}  // namespace eks
