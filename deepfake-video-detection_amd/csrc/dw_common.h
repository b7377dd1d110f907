// Shared pieces of the depthwise-conv kernels (k_dw_fwd.hip, k_dw_dgrad.hip, k_dw_wgrad.hip).
//
// Design (HBM-bound op, AI 3-10 flop/B; the first profile showed the kernels VALU-bound, so the
// per-element instruction count is the second constraint):
//   * compile-time 2D tiles (TH x TW outputs) x 32 channels per workgroup; tile shapes are
//     chosen per layer from {16x16, 8x28, 14x14, 14x7, 8x8, 7x7} to divide the feature map exactly
//     (the EfficientNet-B0 maps are 112/56/28/14/7) and to fit LDS; all index math uses
//     compile-time divisors;
//   * the input tile (+halo) is staged ONCE into LDS as fp32, through the producer's
//     BatchNorm+SiLU, with every load of the tile issued before the first is used;
//   * the channel group is the fastest-varying workgroup index (gridDim.x % groups == 0), so
//     the groups of one pixel run together and their 64-B slices merge into full L2 lines;
//   * per-channel statistics accumulate in registers across all tiles of a workgroup and are
//     reduced once (wave shuffles + LDS) into one deterministic partial row.
#pragma once
#include <cstdio>
#include "kernels.h"

#include <cstdlib>

namespace dfd {

constexpr int DCG = 32;  // channels per workgroup (4 x 8-element vectors)

template <int TH, int TW, int K, int S>
struct DwT {
  static constexpr int NPX = TH * TW;                 // output (fwd/wgrad) or input (dgrad) pixels
  static constexpr int P = (NPX + 63) / 64;           // pixels per thread
  static constexpr int IH = (TH - 1) * S + K;         // fwd/wgrad input tile
  static constexpr int IW = (TW - 1) * S + K;
  static constexpr int NIN = IH * IW;
  static constexpr int GH = (TH - 1 + K - 1) / S + 2;  // dgrad dY tile (bound)
  static constexpr int GW = (TW - 1 + K - 1) / S + 2;
  static constexpr int NG = GH * GW;
  static constexpr int LDS_FWD = NIN * DCG * 4 + K * K * DCG * 4;
  static constexpr int LDS_DGRAD = NG * DCG * 4 + K * K * DCG * 4;
  static constexpr int LDS_WGRAD = (NIN + NPX) * DCG * 4;
  static constexpr int LDS_CAP = 60 * 1024;
  // k5 tiles keep <= 2 pixels per thread (P x 25 taps otherwise exceeds the register budget)
  static constexpr bool p_ok = K == 3 || P <= 2;
  static constexpr bool fwd_ok = p_ok && LDS_FWD <= LDS_CAP && (NIN + 63) / 64 <= 8;
  static constexpr bool dgrad_ok = p_ok && LDS_DGRAD <= LDS_CAP && (NG + 63) / 64 <= 8;
  static constexpr bool wgrad_ok = LDS_WGRAD <= LDS_CAP && (NIN + 63) / 64 <= 8;
};

__host__ __device__ __forceinline__ int floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// Stage an NR x NC pixel window (origin y0, x0; zero outside the map) of channel vector c of
// a [frames][H][W][C] tensor into fp32 LDS [NR*NC][32] (this thread's 8 channels), applying the
// producer's BN+SiLU when MODE != PRO_NONE.  All loads are issued before any is consumed.
// DI: columns stored de-interleaved (even columns, then odd: LDS column (rx&1)*ceil(NC/2) + rx/2),
// so the stride-2 forward's neighbouring output pixels read LDS pixels 128 B apart (the other half
// of the 64 banks) instead of 256 B apart (the same banks: 2-way conflicts on every tap read).
template <int NC, bool DI>
__device__ __forceinline__ int di_col(int rx) {
  return DI ? (rx & 1) * ((NC + 1) / 2) + (rx >> 1) : rx;
}
// The two halves of stage_tile: stage_issue puts the window's global loads in flight (registers),
// stage_commit converts, applies the producer and stores them to LDS.  Split so a kernel can
// issue the next tile's loads before it computes the current one.
template <typename T, int NR, int NC>
struct StageRegs {
  static constexpr int NLD = (NR * NC + 63) / 64;
  Raw8<T> raw[NLD];
  bool in[NLD];
};
template <typename T, int NR, int NC>
__device__ __forceinline__ void stage_issue(StageRegs<T, NR, NC>& r, const T* __restrict__ src, int f, int y0, int x0,
                                            int H, int W, int C, int c, bool cok, bool valid = true) {
  constexpr int N = NR * NC;
  const int tp = threadIdx.x >> 2;
#pragma unroll
  for (int i = 0; i < StageRegs<T, NR, NC>::NLD; ++i) {
    const int pix = tp + 64 * i;
    const int ry = pix / NC, rx = pix - (pix / NC) * NC;
    const int iy = y0 + ry, ix = x0 + rx;
    r.in[i] = valid && pix < N && cok && iy >= 0 && iy < H && ix >= 0 && ix < W;
    raw_ld(r.raw[i], src + (((int64_t)f * H + iy) * W + ix) * C + c, src, r.in[i]);
  }
}
template <typename T, int MODE, int NR, int NC, bool DI = false, typename LT = float>
__device__ __forceinline__ void stage_commit(LT* dst, const StageRegs<T, NR, NC>& r, const float (&sc)[8],
                                             const float (&sh)[8]) {
  constexpr int N = NR * NC;
  const int tp = threadIdx.x >> 2, vec = threadIdx.x & 3;
#pragma unroll
  for (int i = 0; i < StageRegs<T, NR, NC>::NLD; ++i) {
    const int pix = tp + 64 * i;
    if (pix < N) {
      float x[8];
      raw_to_f(r.raw[i], x);
      if (MODE != PRO_NONE) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = r.in[i] ? siluf_(x[j] * sc[j] + sh[j]) : 0.f;
      }
      if constexpr (DI) {
        const int ry = pix / NC, rx = pix - (pix / NC) * NC;
        st8(dst + (ry * NC + di_col<NC, true>(rx)) * DCG + vec * 8, x);
      } else {
        st8(dst + pix * DCG + vec * 8, x);
      }
    }
  }
}
template <typename T, int MODE, int NR, int NC, bool DI = false>
__device__ __forceinline__ void stage_tile(float* dst, const T* __restrict__ src, int f, int y0, int x0, int H, int W,
                                           int C, int c, bool cok, const float (&sc)[8], const float (&sh)[8]) {
  StageRegs<T, NR, NC> r;
  stage_issue<T, NR, NC>(r, src, f, y0, x0, H, W, C, c, cok);
  stage_commit<T, MODE, NR, NC, DI>(dst, r, sc, sh);
}

// Reduce per-thread 8-channel partials a (sum) and b over all threads with the same vec
// (wave shuffles, then 4 waves through LDS) and write out[0*C + c0 + ch], out[1*C + c0 + ch].
__device__ __forceinline__ void reduce_write_stats(float (&a)[8], float (&b)[8], float* red, float* out, int C,
                                                   int c0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, vec = tid & 3;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) {
      a[j] += __shfl_xor(a[j], o, 64);
      b[j] += __shfl_xor(b[j], o, 64);
    }
  }
  lds_barrier();
  if (lane < 4) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wave * 2 + 0) * DCG + vec * 8 + j] = a[j];
      red[(wave * 2 + 1) * DCG + vec * 8 + j] = b[j];
    }
  }
  lds_barrier();
  if (tid < 64) {
    const int ch = tid & 31, which = tid >> 5;
    const float s = red[(0 * 2 + which) * DCG + ch] + red[(1 * 2 + which) * DCG + ch] +
                    red[(2 * 2 + which) * DCG + ch] + red[(3 * 2 + which) * DCG + ch];
    if (c0 + ch < C) out[(int64_t)which * C + c0 + ch] = s;
  }
}

// Host: candidate tiles in preference order; pick the first that divides (rows, cols) and
// fits, else the first that fits (partial tiles are masked).
struct TileChoice {
  int th, tw;
};
constexpr int kNumDwTiles = 6;
constexpr TileChoice kDwTiles[kNumDwTiles] = {{16, 16}, {8, 28}, {14, 14}, {14, 7}, {8, 8}, {7, 7}};
constexpr int kDwFallback = 4;  // 8x8

// workgroups of KERN (NT threads, no dynamic LDS) co-resident on the whole device, measured once per kernel
template <auto KERN, int NT>
int resident_wgs() {
  static const int r = [] {
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, KERN, NT, 0) != hipSuccess || per_cu < 1) per_cu = 1;
#ifdef DFD_OCC_PRINT  // experiment builds (tools/r06): what the occupancy API and the kernel attributes say
    hipFuncAttributes fa{};
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(KERN));
    fprintf(stderr, "occupancy: %d per CU (regs %d, lds %zu, maxthreads %d)\n", per_cu, fa.numRegs,
            fa.sharedSizeBytes, fa.maxThreadsPerBlock);
#endif
#ifdef DFD_OCC_MULT
    per_cu *= DFD_OCC_MULT;
#endif
    return std::max(1, cus * per_cu);
  }();
  return r;
}

static inline int dw_grid(int64_t ntiles, int groups) {
  const int64_t per_group = std::min<int64_t>(ntiles, std::max<int64_t>(1, 1024 / groups));
  return (int)(per_group * groups);
}

// Register-blocked stride-1 forward (k_dw_strip.hip): 1 = launched, 0 = no config for this
// layer (use the tile kernel), -1 = launch error.  DFD_DW_STRIP=0 disables it (A/B runs).
template <typename T>
int try_dw_fwd_strip(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                     int* stat_rows);
static inline bool dw_strip_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("DFD_DW_STRIP");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace dfd
