// Concurrency probe (development tool): does a late-stage 1x1 weight gradient overlap with the data
// gradient it is independent of?  For each late-stage pair, the average time per iteration of
//   serial : dgrad then wgrad on one stream,
//   2q     : dgrad on stream 1 and wgrad on stream 2 (fork / join events every iteration, the plan's
//            wgrad_stream pattern),
// over back-to-back iterations with HIP events.  build: make -C tools pair_probe (KB_T=f16)
#include <cstdio>
#include <cstdlib>
#include <functional>

#include "../deepfake-video-detection_amd/csrc/kernels.h"
#include "../include/dfd_hip.h"

using namespace dfd;
#ifndef KB_T
#define KB_T f16
#endif
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

int main() {
  const int F = 256, iters = 40;
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, f0, f1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&f0, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&f1, hipEventDisableTiming));
  const int64_t big = (int64_t)F * 14 * 14 * 1152;
  KB_T *A, *B, *C, *D, *X;
  float *slab, *slab2, *dW, *dW2, *sc, *sh, *gate;
  for (KB_T** p : {&A, &B, &C, &D, &X}) { CK(hipMalloc(p, big * 2)); CK(hipMemset(*p, 0x1c, big * 2)); }
  const int64_t slab_cap = 16ll << 20;
  CK(hipMalloc(&slab, slab_cap * 4)); CK(hipMalloc(&slab2, slab_cap * 4));
  CK(hipMalloc(&dW, 8 << 20)); CK(hipMalloc(&dW2, 8 << 20));
  CK(hipMalloc(&sc, 1 << 16)); CK(hipMalloc(&sh, 1 << 16)); CK(hipMalloc(&gate, (int64_t)F * 2048 * 4));
  CK(hipMemset(sc, 0, 1 << 16)); CK(hipMemset(sh, 0, 1 << 16)); CK(hipMemset(gate, 0, (int64_t)F * 2048 * 4));
  struct Case { const char* name; int64_t M; int cout, mid, hw; bool pwl, gated_mat; };
  const Case cases[] = {
      {"7x7 pwl 192<-1152", F * 49, 192, 1152, 49, true, true},
      {"7x7 pw 1152<-192", F * 49, 192, 1152, 49, false, false},
      {"6.0 pwl 320<-1152", F * 49, 320, 1152, 49, true, true},
      {"14x14 pwl 112<-672", F * 196, 112, 672, 196, true, false},
      {"14x14 pw 672<-112", F * 196, 112, 672, 196, false, false},
      {"14x14 pwl 80<-480", F * 196, 80, 480, 196, true, false},
  };
  auto time_it = [&](const std::function<void()>& f) {
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3 * ms / iters;
  };
  for (const Case& c : cases) {
    Pro pn{}, pg{sc, sh, gate, c.hw, c.mid};
    // dgrad: pwl: gs[M x cout] . W -> [M x mid]; pw: ge1[M x mid] . W1t -> [M x cout] (+ skip)
    auto dgrad = [&](hipStream_t s) {
      if (c.pwl) return launch_pw_gemm<KB_T>(s, A, B, C, nullptr, c.M, c.mid, c.cout, PRO_NONE, pn, nullptr, nullptr);
      return launch_pw_gemm<KB_T>(s, A, B, C, D, c.M, c.cout, c.mid, PRO_NONE, pn, nullptr, nullptr);
    };
    auto wgrad = [&](hipStream_t s) {
      if (c.pwl)
        return launch_pw_wgrad<KB_T>(s, A, X, c.M, c.cout, c.mid, c.gated_mat ? PRO_GATE : PRO_BN_SILU_G, pg, slab2,
                                     slab_cap, dW2, false);
      return launch_pw_wgrad<KB_T>(s, A, X, c.M, c.mid, c.cout, PRO_NONE, pn, slab2, slab_cap, dW2, false);
    };
    const double td = time_it([&] { dgrad(s1); });
    const double tw = time_it([&] { wgrad(s1); });
    const double ts = time_it([&] { dgrad(s1); wgrad(s1); });
    const double t2 = time_it([&] {
      CK(hipEventRecord(f0, s1));
      CK(hipStreamWaitEvent(s2, f0, 0));
      wgrad(s2);
      dgrad(s1);
      CK(hipEventRecord(f1, s2));
      CK(hipStreamWaitEvent(s1, f1, 0));
    });
    // both queues free-running (no per-iteration fork/join): overlap without the event cost
    wgrad(s2); dgrad(s1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s1));
    CK(hipStreamWaitEvent(s2, e0, 0));
    for (int i = 0; i < iters; ++i) { wgrad(s2); dgrad(s1); }
    CK(hipEventRecord(f1, s2));
    CK(hipStreamWaitEvent(s1, f1, 0));
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double tf = 1e3 * ms / iters;
    // events alone: fork / join around nothing on s2
    const double te = time_it([&] {
      CK(hipEventRecord(f0, s1));
      CK(hipStreamWaitEvent(s2, f0, 0));
      dgrad(s1);
      CK(hipEventRecord(f1, s2));
      CK(hipStreamWaitEvent(s1, f1, 0));
    });
    // fork only (the side stream waits for the main one; the main stream never waits): the plan form with
    // per-block scratch, joined once at the end of the backward
    wgrad(s2); dgrad(s1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i) {
      CK(hipEventRecord(f0, s1));
      CK(hipStreamWaitEvent(s2, f0, 0));
      wgrad(s2);
      dgrad(s1);
    }
    CK(hipEventRecord(f1, s2));
    CK(hipStreamWaitEvent(s1, f1, 0));
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double tk = 1e3 * ms / iters;
    printf("fork-only %6.1f | ", tk);
    printf("%-22s dgrad %6.1f  wgrad(+reduce) %6.1f  serial %6.1f  2q %6.1f  2q-free %6.1f  dgrad+events %6.1f us\n",
           c.name, td, tw, ts, t2, tf, te);
  }
  return 0;
}
