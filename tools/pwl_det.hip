// Determinism harness of the fused projection backward (k_pwl_bwd.hip) per storage type: the same
// inputs twice (output buffers pre-filled with different patterns), every output compared bitwise.
// Links the library objects (tools/Makefile: make pwl_det).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../deepfake-video-detection_amd/csrc/kernels.h"

using namespace dfd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

static float hrand(uint64_t i, uint64_t salt) {  // uniform [-1, 1)
  uint64_t z = i * 0x9E3779B97F4A7C15ull + salt * 0xBF58476D1CE4E5B9ull;
  z ^= z >> 31; z *= 0x94D049BB133111EBull; z ^= z >> 29;
  return (float)((z >> 40) & 0xffffff) / 8388608.f - 1.f;
}
static uint16_t to16(float f, bool half) {
  if (half) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; }
  uint32_t u; memcpy(&u, &f, 4); u += 0x7fff + ((u >> 16) & 1); return (uint16_t)(u >> 16);
}

template <typename T>
static int run(bool half, int F, int hw, int N, int K, bool bn3) {
  const int64_t HW = (int64_t)hw * hw, M = F * HW;
  std::vector<uint16_t> hgs(M * N), hy3(M * N), hy2(M * K), hwt((int64_t)K * N);
  for (int64_t i = 0; i < M * N; ++i) { hgs[i] = to16(hrand(i, 1) * 32.f, half); hy3[i] = to16(hrand(i, 2) * 2.f, half); }
  for (int64_t i = 0; i < M * K; ++i) hy2[i] = to16(hrand(i, 3) * 3.f, half);
  for (int64_t i = 0; i < (int64_t)K * N; ++i) hwt[i] = to16(hrand(i, 4) * 0.3f, half);
  std::vector<float> hco(3 * N), hk(4 * K), hg((int64_t)F * K);
  for (int i = 0; i < 3 * N; ++i) hco[i] = hrand(i, 5);
  for (int i = 0; i < K; ++i) { hk[i] = 0.5f + 0.5f * hrand(i, 6); hk[K + i] = hrand(i, 7) * 0.2f; hk[2 * K + i] = hrand(i, 8); hk[3 * K + i] = 1.f + 0.3f * hrand(i, 9); }
  for (int64_t i = 0; i < (int64_t)F * K; ++i) hg[i] = 0.5f + 0.5f * hrand(i, 10);
  T *gs, *y3, *y2, *wt, *ge2;
  float *co, *kk, *gate, *slab, *dW, *part;
  const int64_t slab_cap = 1ll << 24, part_cap = 5ll * 16 * F * K;
  CK(hipMalloc(&gs, M * N * 2)); CK(hipMalloc(&y3, M * N * 2)); CK(hipMalloc(&y2, M * K * 2));
  CK(hipMalloc(&wt, (int64_t)K * N * 2)); CK(hipMalloc(&ge2, M * K * 2));
  CK(hipMalloc(&co, 3 * N * 4)); CK(hipMalloc(&kk, 4 * K * 4)); CK(hipMalloc(&gate, (int64_t)F * K * 4));
  CK(hipMalloc(&slab, slab_cap * 4)); CK(hipMalloc(&dW, (int64_t)N * K * 4)); CK(hipMalloc(&part, part_cap * 4));
  CK(hipMemcpy(gs, hgs.data(), M * N * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(y3, hy3.data(), M * N * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(y2, hy2.data(), M * K * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(wt, hwt.data(), (int64_t)K * N * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(co, hco.data(), 3 * N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(kk, hk.data(), 4 * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(gate, hg.data(), (int64_t)F * K * 4, hipMemcpyHostToDevice));
  std::vector<uint16_t> oge[2];
  std::vector<float> odw[2], opart[2];
  int hs = 1;
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipMemset(ge2, rep ? 0x7f : 0, M * K * 2));
    CK(hipMemset(part, rep ? 0x7f : 0, part_cap * 4));
    CK(hipMemset(slab, rep ? 0x7f : 0, slab_cap * 4));
    const int rc = launch_pwl_bwd<T>(0, gs, bn3 ? y3 : nullptr, bn3 ? co : nullptr, wt, y2, kk, kk + K, kk + 2 * K,
                                     kk + 3 * K, gate, F, (int)HW, N, K, ge2, slab, slab_cap, dW, false, part,
                                     part_cap, &hs);
    CK(hipDeviceSynchronize());
    if (rc != 0) { printf("launch rc %d\n", rc); return 1; }
    oge[rep].resize(M * K); odw[rep].resize((int64_t)N * K); opart[rep].resize(5ll * hs * F * K);
    CK(hipMemcpy(oge[rep].data(), ge2, M * K * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(odw[rep].data(), dW, (int64_t)N * K * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(opart[rep].data(), part, 5ll * hs * F * K * 4, hipMemcpyDeviceToHost));
  }
  int64_t dge = 0, ddw = 0, dpart[5] = {0, 0, 0, 0, 0};
  int64_t first_ge = -1;
  for (int64_t i = 0; i < M * K; ++i)
    if (oge[0][i] != oge[1][i]) { if (first_ge < 0) first_ge = i; ++dge; }
  for (int64_t i = 0; i < (int64_t)N * K; ++i) ddw += memcmp(&odw[0][i], &odw[1][i], 4) != 0;
  const int64_t pq = (int64_t)hs * F * K;
  int64_t first_p = -1;
  for (int q = 0; q < 5; ++q)
    for (int64_t i = 0; i < pq; ++i)
      if (memcmp(&opart[0][q * pq + i], &opart[1][q * pq + i], 4) != 0) { ++dpart[q]; if (first_p < 0) first_p = q * pq + i; }
  printf("%s F%d %dx%d K%d->N%d bn3 %d hsplit %d: ge2 diff %lld (first row %lld ch %lld), dW diff %lld, part diff %lld %lld %lld %lld %lld",
         half ? "f16 " : "bf16", F, hw, hw, K, N, bn3, hs, (long long)dge, (long long)(first_ge < 0 ? -1 : first_ge / K),
         (long long)(first_ge < 0 ? -1 : first_ge % K), (long long)ddw, (long long)dpart[0], (long long)dpart[1],
         (long long)dpart[2], (long long)dpart[3], (long long)dpart[4]);
  if (first_p >= 0) {
    const int64_t q = first_p / pq, r = first_p % pq;
    printf(" (first part q %lld h %lld f %lld c %lld: %g vs %g)", (long long)q, (long long)(r / ((int64_t)F * K)),
           (long long)(r / K % F), (long long)(r % K), opart[0][first_p], opart[1][first_p]);
  }
  printf("\n");
  hipFree(gs); hipFree(y3); hipFree(y2); hipFree(wt); hipFree(ge2); hipFree(co); hipFree(kk); hipFree(gate);
  hipFree(slab); hipFree(dW); hipFree(part);
  return 0;
}

int main() {
  struct S { int hw, N, K; } shapes[3] = {{112, 16, 32}, {56, 24, 96}, {56, 24, 144}};
  for (int F : {32, 8}) {
    for (auto& q : shapes) {
      for (int bn3 = 0; bn3 < 2; ++bn3) {
        if (run<bf16>(false, F, q.hw, q.N, q.K, bn3)) return 1;
        if (run<f16>(true, F, q.hw, q.N, q.K, bn3)) return 1;
      }
    }
  }
  return 0;
}
