// Launchers of the test-only kernels (k_test.hip) behind the dfd_test_* C entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfd {
// `workgroups` workgroups meet at one group_sync (tail.h) that expects `expected` arrivals, with a
// budget of `seconds`; scratch: >= 3 + workgroups zeroed ints ([arrive, depart, device abort word,
// per-workgroup result 1 = passed / 2 = gave up]); host_word: the sticky host word the barrier raises
int launch_group_sync_test(hipStream_t s, int workgroups, int expected, double seconds, int* scratch, int* host_word);
}  // namespace dfd
