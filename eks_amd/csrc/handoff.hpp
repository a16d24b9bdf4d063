// In-launch hand-off primitives shared by the chained passes of algo 3
// (two_pass.hpp) and algo 2's chained chunk scans (smooth_impl.hpp).
// Agent scope, global address space: payloads are stored write-through
// (relaxed agent-scope atomic stores, `sc1`) by the wave that publishes,
// which drains (`s_waitcnt vmcnt(0)`) before one agent-scope flag store; the
// consumer polls the flag with agent-scope loads and reads the payload with
// agent-scope (`sc1`, L1-bypassing) loads.
//
// Every wait is bounded in wall-clock time (the 100 MHz constant clock read
// by wall_clock64, independent of the shader clock and of s_sleep's length):
// a wait that gives up returns false, the caller flags its trajectories
// EKS_STATUS_SCAN and still publishes, so nothing behind it hangs.  The bound
// is a kernel argument (SmoothArgs::wait_ticks, default 1 s;
// eks_debug_set(EKS_DBG_WAIT_US) changes it).  A negative bound is the
// fault-injection mode of the tests: every wait that would have to poll gives
// up at once.
#pragma once
#include <hip/hip_runtime.h>

#include "eks_common.hpp"
#include "tuning.hpp"

namespace eks {

typedef __attribute__((address_space(1))) unsigned k3_gu32;
typedef __attribute__((address_space(1))) unsigned long long k3_gu64;

constexpr long long kWallHz = 100000000LL;  // wall_clock64 rate on gfx950 (hipDeviceAttributeWallClockRate)
constexpr long long kDefaultWaitTicks = kWallHz;  // 1 s

EKS_DEV void st_wt(double *p, double v) {  // write-through (sc1) store
  __hip_atomic_store((k3_gu64 *)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
EKS_DEV double ld_wt(const double *p) {  // L1-bypassing (sc1) load
  return __builtin_bit_cast(double, __hip_atomic_load((k3_gu64 *)p, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}
EKS_DEV unsigned ld_flag(const unsigned *p) {
  return __hip_atomic_load((k3_gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// publish: every payload store of this wave drained, then one flag store of
// value v (1 unless the flag has several states).  kHandoffFences: every lane
// issues an agent-scope release fence (its payload stores made visible at
// agent scope before anything after the fence), then lane 0 stores the flag.
EKS_DEV void publish_flag(unsigned *flag, int lane, unsigned v = 1u) {
  if constexpr (kHandoffFences) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (lane == 0) __hip_atomic_store((k3_gu32 *)flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// after a poll that saw a published flag: the payload loads below it
// (kHandoffFences: an agent-scope acquire fence; else a compiler-level one,
// the payload being read with L1- and L2-bypassing agent-scope loads)
EKS_DEV void acquire_after_poll() {
  if constexpr (kHandoffFences)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a wall-clock deadline for one wait
struct Deadline {
  unsigned long long t0 = 0;
  long long ticks;
  EKS_DEV explicit Deadline(long long wait_ticks) : ticks(wait_ticks) {}
  // true once the bound has passed (the first call starts the clock)
  EKS_DEV bool expired() {
    if (ticks < 0) return true;
    const unsigned long long now = wall_clock64();
    if (t0 == 0) t0 = now;
    return (long long)(now - t0) > ticks;
  }
};

// wait until a flag word is >= v (the whole wave polls the one word);
// false on timeout
EKS_DEV bool wait_flag(const unsigned *flag, long long wait_ticks, unsigned v = 1u) {
  if (wait_ticks < 0) return false;  // fault injection (tests)
  Deadline dl(wait_ticks);
  while ((unsigned)__builtin_amdgcn_readfirstlane(ld_flag(flag)) < v) {
    if (dl.expired()) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  acquire_after_poll();  // the payload loads below the poll
  return true;
}

// every lane with `need` polls its own flag word; returns once all of them
// are set (false on timeout, as wait_flag)
EKS_DEV bool wait_flag_lanes(const unsigned *flag, bool need, long long wait_ticks) {
  if (wait_ticks < 0) return false;  // fault injection (tests)
  bool ready = !need;
  Deadline dl(wait_ticks);
  while (true) {
    if (!ready) ready = ld_flag(flag) != 0u;
    if (__all(ready)) break;
    if (dl.expired()) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  acquire_after_poll();
  return true;
}

// Decoupled look-back over a chain of units (flag states: 0 = nothing yet,
// kAggReady = the unit's own aggregate published, kIncReady = its inclusive
// value published).  Starting at unit `j` and stepping by `step` (-1: towards
// earlier units), returns the first unit whose inclusive value is published;
// every unit passed on the way has its aggregate published.  The 64 lanes of
// the wave read 64 consecutive flags of the walk at once (one load round
// trip per window instead of one per unit: a poll waits behind the CU's
// streaming loads); units that have published nothing yet are polled again.
// On timeout `ok` is cleared and the search stops (the caller's value is
// then stale and flagged, not used).  Units with smaller tickets publish
// their aggregate before they wait for anything, and the first unit of the
// chain publishes its inclusive value directly, so the search ends.
constexpr unsigned kAggReady = 1u, kIncReady = 2u;
// the fast path: is unit j's inclusive value already published?
EKS_DEV bool inc_ready(const unsigned *flag, long long wait_ticks) {
  if (wait_ticks < 0) return false;  // fault injection: always look back
  if ((unsigned)__builtin_amdgcn_readfirstlane(ld_flag(flag)) < kIncReady) return false;
  acquire_after_poll();
  return true;
}
// the same with a flag word polled earlier (v, any lane's copy: the word is
// wave-uniform); false when it did not say "inclusive published" yet
EKS_DEV bool inc_ready_early(unsigned v, long long wait_ticks) {
  if (wait_ticks < 0) return false;  // fault injection: always look back
  if ((unsigned)__builtin_amdgcn_readfirstlane(v) < kIncReady) return false;
  acquire_after_poll();
  return true;
}
EKS_DEV long long look_back(const unsigned *flags, long long j, long long stride, int step,
                            long long nunits, long long wait_ticks, bool &ok) {
  if (wait_ticks < 0) {  // fault injection (tests): give up at once
    ok = false;
    return j;
  }
  const int l = threadIdx.x & 63;
  Deadline dl(wait_ticks);
  long long base = j;
  while (true) {
    const long long u = base + (long long)step * l;
    const bool valid = u >= 0 && u < nunits;
    const unsigned f = valid ? ld_flag(flags + u * stride) : 0u;
    const unsigned long long inc = __ballot(valid && f >= kIncReady);
    const unsigned long long none = __ballot(valid && f == 0u);
    const unsigned long long all = __ballot(valid);
    if (inc) {
      const int k0 = __ffsll((long long)inc) - 1;  // the nearest inclusive value
      const unsigned long long before = k0 == 0 ? 0ull : ((1ull << k0) - 1ull);
      if ((none & before) == 0ull) {
        acquire_after_poll();
        return base + (long long)step * k0;
      }
    } else if (none == 0ull && all == ~0ull) {
      base += (long long)step * 64;  // 64 aggregates: look further
      continue;
    }
    if (dl.expired()) {
      ok = false;
      return base;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

}  // namespace eks
