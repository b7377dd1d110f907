// Last-arriving-workgroup epilogues: a reduction that used to be its own (latency-bound, ~5 us)
// launch after a producer kernel runs instead in the producer's last workgroup of a group.
//
// Protocol (the pattern of grid_sync.h, without the wait): every workgroup of the group writes its
// partial row with plain stores, drains them, meets at the workgroup barrier; thread 0 publishes
// with an agent-scope release (this XCD's L2 written back) and takes a ticket with an agent-scope
// atomic.  The workgroup drawing the last ticket acquires (agent scope: stale lines of its CU and
// L2 invalidated), resets the counter to zero for the next launch (counters are zero at rest: they live
// in the per-call workspace, zeroed at the start of each forward), and alone reads every partial row in a fixed order
// -- so the result does not depend on which workgroup arrives last (bit-reproducible).  Nobody
// waits: the other workgroups leave, so the grid need not be co-resident.
#pragma once
#include <hip/hip_runtime.h>

namespace dfd {

// DFD_TAIL_WT (A/B build switch, default 0): the partial rows are written and read with agent-scope
// atomic stores / loads (coherent at the device level without an L2 write-back or invalidate) and the
// arrival carries no release / acquire fence -- measures what the fences cost
#ifndef DFD_TAIL_WT
#define DFD_TAIL_WT 0
#endif

template <typename V>
__device__ __forceinline__ void tail_store(V* p, V v) {
  if constexpr (DFD_TAIL_WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <typename V>
__device__ __forceinline__ V tail_load(const V* p) {
  if constexpr (DFD_TAIL_WT) return __hip_atomic_load(const_cast<V*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// true in every thread of the last-arriving workgroup of the `expected` workgroups sharing `ctr`
__device__ __forceinline__ bool tail_arrive(unsigned* ctr, unsigned expected) {
  __shared__ int tail_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (!DFD_TAIL_WT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == expected - 1;
    if (last) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (!DFD_TAIL_WT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    tail_last = last;
  }
  __syncthreads();
  return tail_last != 0;
}

// Where a timed-out barrier is reported.  `dev`: a device word every waiter polls, so one timeout
// releases the whole grid at once; `host`: a word in coherent pinned host memory the plan checks on
// every later call (sticky until the host clears it), so a launch whose outputs are invalid can never
// go unnoticed -- no host synchronisation on the normal path.  Either may be null.
// `budget`: wall-clock ticks (wall_clock64) a waiter polls before it gives up -- the launcher sizes it
// to ~2 s from the device's wall-clock rate (sync_budget_ticks); a group that is not co-resident within
// it (e.g. another stream's kernels hold the CUs) gives up instead of hanging.
struct SyncAbort {
  int* dev;
  int* host;
  unsigned long long budget;
};

// fallback budget when the launcher passes none: 2 s at a 100 MHz wall clock
constexpr unsigned long long kSyncBudgetTicks = 200000000ull;

// host side: `seconds` of the current device's wall clock (hipDeviceAttributeWallClockRate, kHz)
inline unsigned long long sync_budget_ticks(double seconds) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      khz <= 0)
    khz = 100000;
  return (unsigned long long)(seconds * 1e3 * (double)khz);
}

__device__ __forceinline__ void sync_abort_raise(const SyncAbort& ab) {
  if (ab.dev) __hip_atomic_store(ab.dev, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ab.host) __hip_atomic_store(ab.host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The n workgroups sharing `arrive` / `depart` (all co-resident) wait for each other: every one's
// prior global writes are visible to all after the call (agent-scope release before arriving, acquire
// after the wait).  The last to leave zeroes both counters for the next launch (zero at rest).
// Bounded: a group that could not be co-resident raises the abort words after kSyncBudgetTicks and
// every waiter that sees the device word leaves; the call returns false and the launch's outputs are
// invalid (the host reports it: SyncAbort).  Callers launch this form only when the grid fits the
// device at once.
__device__ __forceinline__ bool group_sync(unsigned* arrive, unsigned* depart, unsigned n, SyncAbort ab = {}) {
  __shared__ int group_sync_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    const unsigned long long t0 = wall_clock64(), budget = ab.budget ? ab.budget : kSyncBudgetTicks;
    unsigned spins = 0;
    while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255u) != 0) continue;  // the slow checks every 256 polls
      if (ab.dev && __hip_atomic_load(ab.dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { ok = 0; break; }
      if (wall_clock64() - t0 > budget || spins > (1u << 27)) {  // (a poll count too, never unbounded)
        sync_abort_raise(ab);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (__hip_atomic_fetch_add(depart, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1) {
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(depart, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    group_sync_ok = ok;
  }
  __syncthreads();
  return group_sync_ok != 0;
}

}  // namespace dfd
