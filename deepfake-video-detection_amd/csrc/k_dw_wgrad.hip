// Depthwise conv weight-gradient:
//   dW[c][kh][kw] = sum_{f,oy,ox} dY[f,oy,ox,c] * silu(bn(y))[f, oy*S-pad+kh, ox*S-pad+kw, c]
// Per workgroup: output tiles of one channel group; thread (vec, tap, sub) accumulates its tap
// over pixels p = sub (mod 64/K^2) of every tile in registers; one slab row per workgroup row,
// summed by the deterministic slab reducer.
#include "dw_common.h"

namespace dfd {

template <typename T, int TH, int TW, int K, int S>
__global__ __launch_bounds__(256, 2) void dw_wgrad_kernel(DwGeom g, const T* __restrict__ dY, const T* __restrict__ X,
                                                       Pro pro, float* __restrict__ slab, int ntiles, int groups,
                                                       int tiles_x, int tiles_y) {
  using D = DwT<TH, TW, K, S>;
  constexpr int KK = K * K;
  constexpr int NSUB = 64 / KK;
  __shared__ __attribute__((aligned(16))) float tin[D::NIN * DCG];
  __shared__ __attribute__((aligned(16))) float tg[D::NPX * DCG];
  const int tid = threadIdx.x, vec = tid & 3, tl = tid >> 2;
  const int tap = tl % KK, sub = tl / KK;
  const int kh = tap / K, kw = tap - (tap / K) * K;
  const bool active = sub < NSUB;
  const int grp = blockIdx.x % groups;
  const int c0 = grp * DCG, C = g.C;
  const int c = c0 + vec * 8;
  const bool cok = c < C;
  float sc[8], sh[8];
  if (cok) {
    ld8f(pro.scale + c, sc);
    ld8f(pro.shift + c, sh);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = 1.f; sh[j] = 0.f; }
  }
  const float one[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  const float zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const int tpf = tiles_x * tiles_y;
  for (int t = blockIdx.x / groups; t < ntiles; t += gridDim.x / groups) {
    const int f = t / tpf, r = t - (t / tpf) * tpf;
    const int ty = r / tiles_x, tx = r - (r / tiles_x) * tiles_x;
    const int oy0 = ty * TH, ox0 = tx * TW;
    lds_barrier();
    stage_tile<T, PRO_BN_SILU, D::IH, D::IW>(tin, X, f, oy0 * S - g.pad, ox0 * S - g.pad, g.H, g.W, C, c, cok, sc,
                                             sh);
    stage_tile<T, PRO_NONE, TH, TW>(tg, dY, f, oy0, ox0, g.Ho, g.Wo, C, c, cok, one, zero);
    lds_barrier();
    if (active) {
#pragma unroll 4
      for (int p = sub; p < D::NPX; p += NSUB) {
        const int py = p / TW, px = p - (p / TW) * TW;
        float gy[8], xv[8];
        ld8(tg + p * DCG + vec * 8, gy);
        ld8(tin + ((py * S + kh) * D::IW + (px * S + kw)) * DCG + vec * 8, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(gy[j], xv[j], acc[j]);
      }
    }
  }
  lds_barrier();
  float* red = tin;  // [NSUB][KK][32] <= NIN*32
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(sub * KK + tap) * DCG + vec * 8 + j] = acc[j];
  }
  lds_barrier();
  float* out = slab + (int64_t)(blockIdx.x / groups) * C * KK;
  for (int i = tid; i < KK * DCG; i += 256) {
    const int tp2 = i / DCG, cl = i - tp2 * DCG;
    float a = 0.f;
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb) a += red[(sb * KK + tp2) * DCG + cl];
    if (c0 + cl < C) out[(int64_t)(c0 + cl) * KK + tp2] = a;
  }
}

template <typename T, int TH, int TW, int K, int S>
static int wgrad_launch(hipStream_t s, const DwGeom& g, const T* dY, const T* X, const Pro& pro, float* slab,
                        int64_t slab_cap, float* dW, bool accumulate) {
  if constexpr (!DwT<TH, TW, K, S>::wgrad_ok) {
    set_error("dw wgrad: tile does not fit", __FILE__, __LINE__);
    return -1;
  } else {
    static_assert((64 / (K * K)) * K * K * DCG <= DwT<TH, TW, K, S>::NIN * DCG, "reduce buffer");
    const int tiles_x = cdiv(g.Wo, TW), tiles_y = cdiv(g.Ho, TH);
    const int ntiles = g.frames * tiles_x * tiles_y;
    const int groups = cdiv(g.C, DCG);
    const int64_t per = (int64_t)g.C * K * K;
    int64_t rows = std::min<int64_t>(ntiles, std::max<int64_t>(1, 1024 / groups));
    rows = std::max<int64_t>(1, std::min<int64_t>(rows, slab_cap / per));
    const int gx = (int)(rows * groups);
    hipLaunchKernelGGL((dw_wgrad_kernel<T, TH, TW, K, S>), dim3(gx), dim3(256), 0, s, g, dY, X, pro, slab, ntiles,
                       groups, tiles_x, tiles_y);
    DFD_HIP_CHECK(hipGetLastError());
    return launch_reduce_slabs(s, slab, (int)rows, per, dW, accumulate);
  }
}

template <typename T, int K, int S>
static int wgrad_ks(hipStream_t s, const DwGeom& g, const T* dY, const T* X, const Pro& pro, float* slab,
                    int64_t slab_cap, float* dW, bool accumulate) {
  const bool ok[kNumDwTiles] = {DwT<16, 16, K, S>::wgrad_ok, DwT<8, 28, K, S>::wgrad_ok, DwT<14, 14, K, S>::wgrad_ok,
                                DwT<14, 7, K, S>::wgrad_ok, DwT<8, 8, K, S>::wgrad_ok, DwT<7, 7, K, S>::wgrad_ok};
  int pick = -1;
  for (int i = 0; i < kNumDwTiles && pick < 0; ++i)
    if (ok[i] && g.Ho % kDwTiles[i].th == 0 && g.Wo % kDwTiles[i].tw == 0) pick = i;
  if (pick < 0) pick = kDwFallback;
  switch (pick) {
    case 0: return wgrad_launch<T, 16, 16, K, S>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
    case 1: return wgrad_launch<T, 8, 28, K, S>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
    case 2: return wgrad_launch<T, 14, 14, K, S>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
    case 3: return wgrad_launch<T, 14, 7, K, S>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
    case 4: return wgrad_launch<T, 8, 8, K, S>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
    default: return wgrad_launch<T, 7, 7, K, S>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
  }
}

template <typename T>
int launch_dw_wgrad(hipStream_t s, const DwGeom& g, const T* dY, const T* X, const Pro& pro, int pro_mode, float* slab,
                    int64_t slab_cap, float* dW, bool accumulate) {
  if (pro_mode != PRO_BN_SILU) { set_error("dw wgrad: input must be a BN+SiLU producer", __FILE__, __LINE__); return -1; }
  if (g.k == 3 && g.s == 1) return wgrad_ks<T, 3, 1>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
  if (g.k == 3 && g.s == 2) return wgrad_ks<T, 3, 2>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
  if (g.k == 5 && g.s == 1) return wgrad_ks<T, 5, 1>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
  if (g.k == 5 && g.s == 2) return wgrad_ks<T, 5, 2>(s, g, dY, X, pro, slab, slab_cap, dW, accumulate);
  set_error("dw: unsupported kernel/stride", __FILE__, __LINE__);
  return -1;
}

template int launch_dw_wgrad<float>(hipStream_t, const DwGeom&, const float*, const float*, const Pro&, int, float*,
                                    int64_t, float*, bool);
template int launch_dw_wgrad<bf16>(hipStream_t, const DwGeom&, const bf16*, const bf16*, const Pro&, int, float*,
                                   int64_t, float*, bool);
template int launch_dw_wgrad<f16>(hipStream_t, const DwGeom&, const f16*, const f16*, const Pro&, int, float*,
                                   int64_t, float*, bool);

}  // namespace dfd
