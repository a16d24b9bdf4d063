// In-launch hand-off primitives shared by the chained passes of algo 3
// (two_pass.hpp) and algo 2's chained chunk scans (smooth_impl.hpp).
// Agent scope, global address space: payloads are stored write-through
// (relaxed agent-scope atomic stores, `sc1`) by the wave that publishes,
// which drains (`s_waitcnt vmcnt(0)`) before one agent-scope flag store; the
// consumer polls the flag with agent-scope loads and reads the payload with
// agent-scope (`sc1`, L1-bypassing) loads.
#pragma once
#include <hip/hip_runtime.h>

#include "eks_common.hpp"

namespace eks {

typedef __attribute__((address_space(1))) unsigned k3_gu32;
typedef __attribute__((address_space(1))) unsigned long long k3_gu64;

EKS_DEV void st_wt(double *p, double v) {  // write-through (sc1) store
  __hip_atomic_store((k3_gu64 *)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
EKS_DEV double ld_wt(const double *p) {  // L1-bypassing (sc1) load
  return __builtin_bit_cast(double, __hip_atomic_load((k3_gu64 *)p, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}
// publish: every payload store of this wave drained, then one flag store
EKS_DEV void publish_flag(unsigned *flag, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store((k3_gu32 *)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wait for a flag (the whole wave polls the one word); false on timeout
// (~0.1 s: only a bug could get there, and then the call must still end)
#ifndef EKS_K3_NOWAIT
#define EKS_K3_NOWAIT 0  // 1: tuning experiment only -- skip the chain waits (wrong results)
#endif
EKS_DEV bool wait_flag(const unsigned *flag) {
  if (EKS_K3_NOWAIT) return true;
  unsigned spins = 0;
  while (__hip_atomic_load((k3_gu32 *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
    if (++spins > (1u << 16)) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
  return true;
}

// every lane with `need` polls its own flag word; returns once all of them
// are set (false on timeout, as wait_flag)
EKS_DEV bool wait_flag_lanes(const unsigned *flag, bool need) {
  if (EKS_K3_NOWAIT) return true;
  bool ready = !need;
  unsigned spins = 0;
  while (true) {
    if (!ready)
      ready = __hip_atomic_load((k3_gu32 *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    if (__all(ready)) break;
    if (++spins > (1u << 16)) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return true;
}

}  // namespace eks
