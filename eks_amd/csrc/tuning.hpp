// Compile-time tuning constants of the kernels: the measured choices, one
// place.  A few knobs take a -D override for A/B variant builds
// (tools/build_cur.sh NAME -DKNOB=v unit.hip); the defaults are what ships.
#pragma once

namespace eks {

// algo 3's member passes stream ~7 GB (config 4) that no cache holds between
// the two passes: member loads and output stores are non-temporal there
// (config 4: k3_elem 1.67 -> 1.62, k3_final 1.93 -> 1.87 ms, profiles/r02/nt).
// Algo 2 keeps cached loads: its few-trajectory shapes re-read members from
// the Infinity Cache (config 2 K1 0.046 -> 0.061 ms with non-temporal loads).
constexpr bool kNtLoad = true;
constexpr bool kNtOut = true;

// In-launch hand-offs (handoff.hpp): false = the ISA protocol (payload
// stores write-through at agent scope, s_waitcnt vmcnt(0), flag store;
// consumer: flag poll, compiler-level acquire, L2-bypassing payload loads);
// true = the HIP memory model's agent-scope release / acquire fences around
// the same accesses (buffer_wbl2 sc1 before the flag, buffer_inv sc1 after
// the poll).  Both are measured in DESIGN.md.
#ifndef EKS_HANDOFF_FENCES
#define EKS_HANDOFF_FENCES 0
#endif
constexpr bool kHandoffFences = EKS_HANDOFF_FENCES != 0;

// member prefetch distance (steps) of both algo-3 passes; k3_bwd its own
// (config 4, one box: k3_bwd 1.858 / 1.801 / 1.848 ms at 2 / 3 / 4 steps,
// profiles/r05/ab2; k3_fwd 1.397 / 1.408 / 1.412 ms, profiles/r05/ab7)
#ifndef EKS_K3F_D
#define EKS_K3F_D 2
#endif
constexpr int kK3D = EKS_K3F_D;
#ifndef EKS_K3B_D
#define EKS_K3B_D 3
#endif
constexpr int kK3BD = EKS_K3B_D;
// the same from the fit's y / ev hand-off planes (f32 y, f64 ev: 24 B per
// step and lane instead of 40): a deeper ring keeps the bytes in flight
#ifndef EKS_K3_YEV_D
#define EKS_K3_YEV_D 4
#endif
constexpr int kK3YevD = EKS_K3_YEV_D;

// algo 3's chains: every unit publishes its aggregate (k3_fwd: its element,
// k3_bwd: its map) as soon as it has it, before looking at its neighbour, so
// a later unit never waits for an earlier one's own chain wait -- only for
// its stream to end (0: only a unit that finds its neighbour not ready
// publishes one, round 4's rule)
#ifndef EKS_EAGER_AGG
#define EKS_EAGER_AGG 0
#endif
constexpr bool kEagerAgg = EKS_EAGER_AGG != 0;
// k3_bwd's look-back instantiation for every batch of the single-view shape
// (0: only for batches of at most kLbGroups groups, round 4's rule)
#ifndef EKS_A3_LB_ALL
#define EKS_A3_LB_ALL 0
#endif
constexpr bool kLbAll = EKS_A3_LB_ALL != 0;

// algo 3's chains: wave 0 issues the poll of its neighbour's flag as soon as
// its own stream ends (before the unit's element / map composition and its
// barrier), and uses the word at the chain point when it already says
// "published" -- one load round trip off the chain (0: poll at the chain point)
#ifndef EKS_EARLY_POLL
#define EKS_EARLY_POLL 1
#endif
constexpr bool kEarlyPoll = EKS_EARLY_POLL != 0;

// k3_bwd's whole-chunk loop: a scheduling barrier after every step (one
// step's registers live at a time); A/B with -DEKS_K3B_SCHED=0
#ifndef EKS_K3B_SCHED
#define EKS_K3B_SCHED 1
#endif
constexpr bool kK3BSched = EKS_K3B_SCHED != 0;

// few-trajectory prefetch distances of algo 2's K1 / K3 (config 2: 2 / 4 / 8
// steps all within 2 %, tools/c2_dsweep.sh -- these lanes are bound by the
// per-step FP64 dependency chain, not by the load latency)
constexpr int kC1Dnu = 2;
constexpr int kC3Dnu = 2;

// element / map loads in flight per thread of the chained chunk scans
// (config 2, B = 17, T = 1e5: depth 1 / 2 / 4 -> K2 35 / 39 / 41 us)
constexpr int kScanPd = 1;

// independent key loads in flight per thread in eks_fit's selection passes
// (8 / 16 / 32: 0.91 / 0.85 / 0.86 ms at config 4)
constexpr int kSelU = 16;

}  // namespace eks
