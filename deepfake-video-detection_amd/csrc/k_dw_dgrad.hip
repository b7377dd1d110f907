// Depthwise conv input-gradient, fused with the backward reduction of the producer's BN+SiLU:
//   dA[f,iy,ix,c] = sum_{kh,kw} dY[f,(iy+pad-kh)/S,(ix+pad-kw)/S,c] * w[c][kh][kw]   (exact divisions only)
//   out = g = dA * silu'(y*scale+shift)  (y = producer's pre-BN output at the same pixel)
//   stats rows += [sum g, sum g*(y-mean)*invstd]  -> bn_bwd_finalize / bn_bwd_apply
// so the 6x-expanded tensor is read once here instead of again by a separate BN reduction.
#include "dw_common.h"

namespace dfd {

template <typename T, int TH, int TW, int K, int S>
__global__ __launch_bounds__(256, 2) void dw_dgrad_kernel(DwGeom g, const T* __restrict__ dY, const float* __restrict__ w,
                                                       T* __restrict__ out, const T* __restrict__ Yp, BnBwdIn bn,
                                                       float* __restrict__ stats, int ntiles, int groups, int tiles_x,
                                                       int tiles_y) {
  using D = DwT<TH, TW, K, S>;
  __shared__ __attribute__((aligned(16))) float tg[D::NG * DCG];
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
  float sc[8], sh[8], mu[8], is[8];
  if (cok) {
    ld8f(bn.scale + c, sc); ld8f(bn.shift + c, sh); ld8f(bn.mean + c, mu); ld8f(bn.invstd + c, is);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = 1.f; sh[j] = 0.f; mu[j] = 0.f; is[j] = 1.f; }
  }
  const float one[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  const float zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int ly[D::P], lx[D::P];
#pragma unroll
  for (int i = 0; i < D::P; ++i) {
    const int p = tp + 64 * i;
    ly[i] = p / TW;
    lx[i] = p - (p / TW) * TW;
  }
  float st_s[8], st_q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
  const int tpf = tiles_x * tiles_y;
  for (int t = blockIdx.x / groups; t < ntiles; t += gridDim.x / groups) {
    const int f = t / tpf, r = t - (t / tpf) * tpf;
    const int ty = r / tiles_x, tx = r - (r / tiles_x) * tiles_x;
    const int iy0 = ty * TH, ix0 = tx * TW;
    const int gy0 = floordiv(iy0 + g.pad - (K - 1), S), gx0 = floordiv(ix0 + g.pad - (K - 1), S);
    lds_barrier();
    stage_tile<T, PRO_NONE, D::GH, D::GW>(tg, dY, f, gy0, gx0, g.Ho, g.Wo, C, c, cok, one, zero);
    // producer pre-BN values of this thread's pixels (masked loads, in flight during the taps)
    Raw8<T> ryp[D::P];
#pragma unroll
    for (int i = 0; i < D::P; ++i) {
      const int iy = iy0 + ly[i], ix = ix0 + lx[i];
      const bool ok = tp + 64 * i < D::NPX && iy < g.H && ix < g.W && cok;
      raw_ld(ryp[i], Yp + (((int64_t)f * g.H + iy) * g.W + ix) * C + c, Yp, ok);
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < D::P; ++i) {
      const int iy = iy0 + ly[i], ix = ix0 + lx[i];
      if (!(tp + 64 * i < D::NPX && iy < g.H && ix < g.W && cok)) continue;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll 1
      for (int kh = 0; kh < K; ++kh) {
        const int tyv = iy + g.pad - kh;
        if (S == 2 && (tyv & 1)) continue;
        const int gyl = (S == 2 ? (tyv >> 1) : tyv) - gy0;
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
          const int txv = ix + g.pad - kw;
          if (S == 2 && (txv & 1)) continue;
          const int gxl = (S == 2 ? (txv >> 1) : txv) - gx0;
          float x[8], wv[8];
          ld8(tg + (gyl * D::GW + gxl) * DCG + vec * 8, x);
          ld8(wts + (kh * K + kw) * DCG + vec * 8, wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(x[j], wv[j], acc[j]);
        }
      }
      const int64_t o = (((int64_t)f * g.H + iy) * g.W + ix) * C + c;
      float y[8];
      raw_to_f(ryp[i], y);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gg = Tr<T>::round(acc[j] * dsiluf_(y[j] * sc[j] + sh[j]));
        acc[j] = gg;
        st_s[j] += gg;
        st_q[j] += gg * (y[j] - mu[j]) * is[j];
      }
      st8(out + o, acc);
    }
  }
  reduce_write_stats(st_s, st_q, tg, stats + (int64_t)(blockIdx.x / groups) * 2 * C, C, c0);
}

template <typename T, int TH, int TW, int K, int S>
static int dgrad_launch(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* out, const T* Yp,
                        const BnBwdIn& bn, float* stats, int* stat_rows) {
  if constexpr (!DwT<TH, TW, K, S>::dgrad_ok) {
    set_error("dw dgrad: tile does not fit", __FILE__, __LINE__);
    return -1;
  } else {
    const int tiles_x = cdiv(g.W, TW), tiles_y = cdiv(g.H, TH);
    const int ntiles = g.frames * tiles_x * tiles_y;
    const int groups = cdiv(g.C, DCG);
    const int gx = dw_grid(ntiles, groups);
    hipLaunchKernelGGL((dw_dgrad_kernel<T, TH, TW, K, S>), dim3(gx), dim3(256), 0, s, g, dY, w, out, Yp, bn, stats,
                       ntiles, groups, tiles_x, tiles_y);
    if (stat_rows) *stat_rows = gx / groups;
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
}

template <typename T, int K, int S>
static int dgrad_ks(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* out, const T* Yp,
                    const BnBwdIn& bn, float* stats, int* stat_rows) {
  const bool ok[kNumDwTiles] = {DwT<16, 16, K, S>::dgrad_ok, DwT<8, 28, K, S>::dgrad_ok, DwT<14, 14, K, S>::dgrad_ok,
                                DwT<14, 7, K, S>::dgrad_ok, DwT<8, 8, K, S>::dgrad_ok, DwT<7, 7, K, S>::dgrad_ok};
  int pick = -1;
  for (int i = 0; i < kNumDwTiles && pick < 0; ++i)
    if (ok[i] && g.H % kDwTiles[i].th == 0 && g.W % kDwTiles[i].tw == 0) pick = i;
  if (pick < 0) pick = kDwFallback;
  switch (pick) {
    case 0: return dgrad_launch<T, 16, 16, K, S>(s, g, dY, w, out, Yp, bn, stats, stat_rows);
    case 1: return dgrad_launch<T, 8, 28, K, S>(s, g, dY, w, out, Yp, bn, stats, stat_rows);
    case 2: return dgrad_launch<T, 14, 14, K, S>(s, g, dY, w, out, Yp, bn, stats, stat_rows);
    case 3: return dgrad_launch<T, 14, 7, K, S>(s, g, dY, w, out, Yp, bn, stats, stat_rows);
    case 4: return dgrad_launch<T, 8, 8, K, S>(s, g, dY, w, out, Yp, bn, stats, stat_rows);
    default: return dgrad_launch<T, 7, 7, K, S>(s, g, dY, w, out, Yp, bn, stats, stat_rows);
  }
}

template <typename T>
int launch_dw_dgrad(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* out, const T* Yp,
                    const BnBwdIn* bn, float* stats, int* stat_rows) {
  if (!bn || !Yp || !stats) { set_error("dw dgrad: the fused BN-backward inputs are required", __FILE__, __LINE__); return -1; }
  if (g.k == 3 && g.s == 1) return dgrad_ks<T, 3, 1>(s, g, dY, w, out, Yp, *bn, stats, stat_rows);
  if (g.k == 3 && g.s == 2) return dgrad_ks<T, 3, 2>(s, g, dY, w, out, Yp, *bn, stats, stat_rows);
  if (g.k == 5 && g.s == 1) return dgrad_ks<T, 5, 1>(s, g, dY, w, out, Yp, *bn, stats, stat_rows);
  if (g.k == 5 && g.s == 2) return dgrad_ks<T, 5, 2>(s, g, dY, w, out, Yp, *bn, stats, stat_rows);
  set_error("dw: unsupported kernel/stride", __FILE__, __LINE__);
  return -1;
}

template int launch_dw_dgrad<float>(hipStream_t, const DwGeom&, const float*, const float*, float*, const float*,
                                    const BnBwdIn*, float*, int*);
template int launch_dw_dgrad<bf16>(hipStream_t, const DwGeom&, const bf16*, const float*, bf16*, const bf16*,
                                   const BnBwdIn*, float*, int*);
template int launch_dw_dgrad<f16>(hipStream_t, const DwGeom&, const f16*, const float*, f16*, const f16*,
                                   const BnBwdIn*, float*, int*);

}  // namespace dfd
