// Test seam (dfd_test_occupy): workgroups that hold whole CUs for a bounded wall-clock time, so a GPU
// test can run the B0 plan while another stream's kernel denies it most of the device (the split SE
// excitation's slice barrier must then either complete or fail loudly, tail.h SyncAbort).
#include "kernels.h"
#include "tail.h"

namespace dfd {

constexpr int kOccupyLds = 160 * 1024 - 64;  // the whole CU's LDS: no other workgroup with LDS fits beside it

__global__ __launch_bounds__(1024) void occupy_kernel(unsigned long long ticks, int* sink) {
  __shared__ char hold[kOccupyLds];
  volatile char* h = hold;
  h[threadIdx.x * 64] = (char)threadIdx.x;  // the allocation is live (not optimised away)
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  unsigned spins = 0;
  // bounded twice: the wall clock, and a poll count in case the clock does not advance
  while (wall_clock64() - t0 < ticks && ++spins < (1u << 28)) __builtin_amdgcn_s_sleep(32);
  __syncthreads();
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = h[64];
}

int launch_occupy(hipStream_t s, int workgroups, int64_t microseconds) {
  if (workgroups < 1 || workgroups > 4096 || microseconds < 0 || microseconds > 10000000) {
    set_error("occupy: 1..4096 workgroups for at most 10 s", __FILE__, __LINE__);
    return -1;
  }
  const unsigned long long ticks = sync_budget_ticks((double)microseconds * 1e-6);  // the device's wall-clock rate
  hipLaunchKernelGGL(occupy_kernel, dim3((unsigned)workgroups), dim3(1024), 0, s, ticks, nullptr);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd

#include "test_seams.h"

namespace dfd {

__global__ __launch_bounds__(256) void group_sync_test_kernel(int expected, unsigned long long budget, int* scratch,
                                                              int* host_word) {
  unsigned* ctr = reinterpret_cast<unsigned*>(scratch);
  const bool ok = group_sync(ctr, ctr + 1, (unsigned)expected, SyncAbort{scratch + 2, host_word, budget});
  if (threadIdx.x == 0) scratch[3 + blockIdx.x] = ok ? 1 : 2;
}

int launch_group_sync_test(hipStream_t s, int workgroups, int expected, double seconds, int* scratch, int* host_word) {
  int dev = 0, cus = 0;
  DFD_HIP_CHECK(hipGetDevice(&dev));
  DFD_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // a co-resident grid (the barrier's precondition) and a bounded wait
  if (workgroups < 1 || workgroups > cus || expected < 1 || seconds <= 0.0 || seconds > 10.0 || !scratch) {
    set_error("group_sync test: 1..CUs workgroups, 0 < seconds <= 10", __FILE__, __LINE__);
    return -1;
  }
  hipLaunchKernelGGL(group_sync_test_kernel, dim3((unsigned)workgroups), dim3(256), 0, s, expected,
                     sync_budget_ticks(seconds), scratch, host_word);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
