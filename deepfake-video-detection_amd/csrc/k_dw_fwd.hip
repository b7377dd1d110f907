// Depthwise conv forward (timm conv_dw; src/pretrained_detector.py:116): NHWC, k = 3/5,
// s = 1/2, pad k//2, producer BN+SiLU fused into staging, BN-stat partials in the epilogue.
#include "dw_common.h"

// bit mask of the tile shapes whose kernel prefetches the next tile's input window while it computes
// the current one (A/B knob): 1 = 16x16, 2 = 8x28, 4 = 14x14, 8 = 14x7, 16 = 8x8, 32 = 7x7
#ifndef DFD_DWF_PF
#define DFD_DWF_PF 0
#endif

// 1: the stride-2 bf16 kernels stage the producer's SiLU output as bf16 in LDS (half the window:
// twice the co-resident workgroups) instead of fp32
#ifndef DFD_DWF_BF16LDS
#define DFD_DWF_BF16LDS 0
#endif

namespace dfd {

template <int TH, int TW> constexpr bool dwf_pf() {
  return (DFD_DWF_PF & ((TH == 16) ? 1 : (TH == 8 && TW == 28) ? 2 : (TH == 14 && TW == 14) ? 4
                        : (TH == 14) ? 8 : (TH == 8) ? 16 : 32)) != 0;
}

template <typename T, int TH, int TW, int K, int S, bool STATS, bool PF = dwf_pf<TH, TW>()>
__global__ __launch_bounds__(256, 2) void dw_fwd_kernel(DwGeom g, const T* __restrict__ X, const float* __restrict__ w,
                                                     T* __restrict__ Y, Pro pro, float* __restrict__ stats, int ntiles,
                                                     int groups, int tiles_x, int tiles_y) {
  using D = DwT<TH, TW, K, S>;
  using LT = std::conditional_t<(DFD_DWF_BF16LDS != 0 && S == 2 && sizeof(T) == 2), T, float>;
  __shared__ __attribute__((aligned(16))) LT tin[D::NIN * DCG];
  __shared__ __attribute__((aligned(16))) float wts[K * K * DCG];
  const int tid = threadIdx.x, vec = tid & 3, tp = tid >> 2;
  const int grp = blockIdx.x % groups;
  const int c0 = grp * DCG, C = g.C;
  const int c = c0 + vec * 8;
  const bool cok = c < C;
  for (int i = tid; i < K * K * DCG; i += 256) {
    const int tap = i / DCG, cl = i - tap * DCG;
    wts[i] = (c0 + cl < C) ? w[(int64_t)(c0 + cl) * K * K + tap] : 0.f;
  }
  float sc[8], sh[8];
  if (cok) {
    ld8f(pro.scale + c, sc);
    ld8f(pro.shift + c, sh);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = 1.f; sh[j] = 0.f; }
  }
  int lofs[D::P], ly[D::P], lx[D::P];
#pragma unroll
  for (int i = 0; i < D::P; ++i) {
    const int p = tp + 64 * i;
    ly[i] = p / TW;
    lx[i] = p - (p / TW) * TW;
    lofs[i] = ((ly[i] * S) * D::IW + (S == 2 ? lx[i] : lx[i] * S)) * DCG + vec * 8;  // S == 2: de-interleaved
  }
  float st_s[8], st_q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
  const int tpf = tiles_x * tiles_y;
  const int tstep = gridDim.x / groups;
  StageRegs<T, D::IH, D::IW> sr;
  auto issue = [&](int t) {  // input window of tile t (nothing when t is past the end)
    const int f = t / tpf, r = t - (t / tpf) * tpf;
    const int ty = r / tiles_x, tx = r - (r / tiles_x) * tiles_x;
    stage_issue<T, D::IH, D::IW>(sr, X, f, ty * TH * S - g.pad, tx * TW * S - g.pad, g.H, g.W, C, c, cok, t < ntiles);
  };
  if (PF) issue(blockIdx.x / groups);
  for (int t = blockIdx.x / groups; t < ntiles; t += tstep) {
    const int f = t / tpf, r = t - (t / tpf) * tpf;
    const int ty = r / tiles_x, tx = r - (r / tiles_x) * tiles_x;
    const int oy0 = ty * TH, ox0 = tx * TW;
    if (!PF) issue(t);
    lds_barrier();
    stage_commit<T, PRO_BN_SILU, D::IH, D::IW, S == 2>(tin, sr, sc, sh);
    lds_barrier();
    if (PF && t + tstep < ntiles) issue(t + tstep);  // in flight while this tile computes
    float acc[D::P][8];
#pragma unroll
    for (int i = 0; i < D::P; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
    // taps: one kernel row per iteration (not unrolled) keeps the live registers to
    // P x 8 accumulators + one row of inputs; every weight read is a 16-lane LDS broadcast
#pragma unroll 1
    for (int kh = 0; kh < K; ++kh) {
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        float wv[8];
        ld8(wts + (kh * K + kw) * DCG + vec * 8, wv);
#pragma unroll
        for (int i = 0; i < D::P; ++i) {
          if (i == D::P - 1 && tp + 64 * i >= D::NPX) continue;
          float x[8];
          ld8(tin + lofs[i] + (kh * D::IW + (S == 2 ? di_col<D::IW, true>(kw) : kw)) * DCG, x);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(x[j], wv[j], acc[i][j]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < D::P; ++i) {
      const int oy = oy0 + ly[i], ox = ox0 + lx[i];
      if (tp + 64 * i < D::NPX && oy < g.Ho && ox < g.Wo && cok) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = Tr<T>::round(acc[i][j]);
        st8(Y + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * C + c, acc[i]);
        if constexpr (STATS) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { st_s[j] += acc[i][j]; st_q[j] += acc[i][j] * acc[i][j]; }
        }
      }
    }
  }
  if constexpr (STATS) reduce_write_stats(st_s, st_q, reinterpret_cast<float*>(tin), stats + (int64_t)(blockIdx.x / groups) * 2 * C, C, c0);
}

template <typename T, int TH, int TW, int K, int S>
static int fwd_launch(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                      int* stat_rows) {
  if constexpr (!DwT<TH, TW, K, S>::fwd_ok) {
    set_error("dw fwd: tile does not fit", __FILE__, __LINE__);
    return -1;
  } else {
    const int tiles_x = cdiv(g.Wo, TW), tiles_y = cdiv(g.Ho, TH);
    const int ntiles = g.frames * tiles_x * tiles_y;
    const int groups = cdiv(g.C, DCG);
    // persistent grid: the co-resident workgroups, at most 1024 (stat rows)
    const int res = stats ? resident_wgs<dw_fwd_kernel<T, TH, TW, K, S, true>, 256>()
                          : resident_wgs<dw_fwd_kernel<T, TH, TW, K, S, false>, 256>();
    const int gx = (int)(std::min<int64_t>(ntiles, std::max(1, std::min(res, 1024) / groups)) * groups);
    if (stats)
      hipLaunchKernelGGL((dw_fwd_kernel<T, TH, TW, K, S, true>), dim3(gx), dim3(256), 0, s, g, X, w, Y, pro, stats,
                         ntiles, groups, tiles_x, tiles_y);
    else
      hipLaunchKernelGGL((dw_fwd_kernel<T, TH, TW, K, S, false>), dim3(gx), dim3(256), 0, s, g, X, w, Y, pro, stats,
                         ntiles, groups, tiles_x, tiles_y);
    if (stat_rows) *stat_rows = gx / groups;
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
}

template <typename T, int K, int S>
static int fwd_ks(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                  int* stat_rows) {
  const bool ok[kNumDwTiles] = {DwT<16, 16, K, S>::fwd_ok, DwT<8, 28, K, S>::fwd_ok, DwT<14, 14, K, S>::fwd_ok,
                                DwT<14, 7, K, S>::fwd_ok, DwT<8, 8, K, S>::fwd_ok, DwT<7, 7, K, S>::fwd_ok};
  int pick = -1;
  // stride 2: the 8x8 tile first where it divides the map -- its 17x17 fp32 input window lets
  // 4 workgroups share a CU (14x7's 29x15 window: 2), measured 231 -> 213 us on blocks.1.0
  if (S == 2 && ok[4] && g.Ho % 8 == 0 && g.Wo % 8 == 0) pick = 4;
  for (int i = 0; i < kNumDwTiles && pick < 0; ++i)
    if (ok[i] && g.Ho % kDwTiles[i].th == 0 && g.Wo % kDwTiles[i].tw == 0) pick = i;
  if (pick < 0) pick = kDwFallback;  // 8x8 with masked partial tiles
  switch (pick) {
    case 0: return fwd_launch<T, 16, 16, K, S>(s, g, X, w, Y, pro, stats, stat_rows);
    case 1: return fwd_launch<T, 8, 28, K, S>(s, g, X, w, Y, pro, stats, stat_rows);
    case 2: return fwd_launch<T, 14, 14, K, S>(s, g, X, w, Y, pro, stats, stat_rows);
    case 3: return fwd_launch<T, 14, 7, K, S>(s, g, X, w, Y, pro, stats, stat_rows);
    case 4: return fwd_launch<T, 8, 8, K, S>(s, g, X, w, Y, pro, stats, stat_rows);
    default: return fwd_launch<T, 7, 7, K, S>(s, g, X, w, Y, pro, stats, stat_rows);
  }
}

template <typename T>
int launch_dw_fwd(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, int pro_mode,
                  float* stats, int* stat_rows, const BnFwdFin* fin) {
  if (g.C & 7) { set_error("dw: C must be a multiple of 8", __FILE__, __LINE__); return -1; }
  if (pro_mode != PRO_BN_SILU) { set_error("dw fwd: input must be a BN+SiLU producer", __FILE__, __LINE__); return -1; }
  // the input BN's finalize inside the channel-pair kernel where it applies (few stat rows), else its
  // own launch first (pro.scale / pro.shift are that launch's outputs)
  const bool embed = fin && fin->rows > 0 && fin->rows <= kBnFinRowsMax;
  if (fin && fin->rows > 0 && !embed) DFD_TRY(launch_bn_finalize_fin(s, *fin, g.C));
  {
    const int rc = try_dw_fwd1<T>(s, g, X, w, Y, pro, stats, stat_rows, embed ? fin : nullptr);
    if (rc < 0) return -1;
    if (rc > 0) return 0;
  }
  if (embed) DFD_TRY(launch_bn_finalize_fin(s, *fin, g.C));  // the channel-pair kernel does not cover this shape
  if (g.s == 1 && dw_strip_enabled()) {
    const int rc = try_dw_fwd_strip<T>(s, g, X, w, Y, pro, stats, stat_rows);
    if (rc != 0) return rc > 0 ? 0 : -1;
  }
  if (g.k == 3 && g.s == 1) return fwd_ks<T, 3, 1>(s, g, X, w, Y, pro, stats, stat_rows);
  if (g.k == 3 && g.s == 2) return fwd_ks<T, 3, 2>(s, g, X, w, Y, pro, stats, stat_rows);
  if (g.k == 5 && g.s == 1) return fwd_ks<T, 5, 1>(s, g, X, w, Y, pro, stats, stat_rows);
  if (g.k == 5 && g.s == 2) return fwd_ks<T, 5, 2>(s, g, X, w, Y, pro, stats, stat_rows);
  set_error("dw: unsupported kernel/stride", __FILE__, __LINE__);
  return -1;
}

template int launch_dw_fwd<float>(hipStream_t, const DwGeom&, const float*, const float*, float*, const Pro&, int,
                                  float*, int*, const BnFwdFin*);
template int launch_dw_fwd<bf16>(hipStream_t, const DwGeom&, const bf16*, const float*, bf16*, const Pro&, int,
                                 float*, int*, const BnFwdFin*);
template int launch_dw_fwd<f16>(hipStream_t, const DwGeom&, const f16*, const float*, f16*, const Pro&, int,
                                 float*, int*, const BnFwdFin*);

}  // namespace dfd
