// Grid-wide barrier for persistent launches whose whole grid is co-resident (one workgroup per CU
// or fewer; the launchers check the occupancy).  Monotonic counter: the caller passes the count the
// counter reaches at this barrier (k-th barrier of a G-workgroup grid: k * G); the counter and the
// abort flag are zeroed by the launcher before the launch.
//
// Every storing wave drains its stores, the workgroup meets, lane 0 publishes with an agent-scope
// release (writes back this XCD's L2) and arrives with a relaxed agent-scope atomic, then polls
// with relaxed agent-scope loads and s_sleep; an agent-scope acquire (invalidates this XCD's L2)
// makes the other workgroups' stores visible.  Bounded: a grid that is not co-resident raises the
// abort flag instead of spinning forever, and every workgroup that sees the flag leaves (the
// launch's outputs are then invalid and the host reports it).
#pragma once
#include <hip/hip_runtime.h>

namespace dfd {

__device__ __forceinline__ bool grid_sync(unsigned* bar, unsigned target, int* abort_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int grid_sync_ok;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    unsigned spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { ok = 0; break; }
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 22)) {
        __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    grid_sync_ok = ok;
  }
  __syncthreads();
  return grid_sync_ok != 0;
}

}  // namespace dfd
