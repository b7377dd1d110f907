// Depthwise k x k convolutions (k = 3, 5; stride 1, 2; timm symmetric padding k//2) on gfx950.
//
// Replaces aten conv2d(groups=C) of timm's conv_dw (reached from
// src/pretrained_detector.py:116) in forward, dgrad and wgrad.  HBM-bound (AI 3-10 flop/B):
// each workgroup owns an 8x8 output tile x 32 channels; the input tile (with halo) is
// staged ONCE into LDS through the producer's BatchNorm+SiLU (so the activation is never
// materialised), weights sit in LDS, and every global access is a 16-byte NHWC vector.
// The forward epilogue emits per-channel BN-stat partials for the following BatchNorm.
#include "kernels.h"

namespace dfd {

constexpr int DT = 8;     // output tile edge
constexpr int DCG = 32;   // channels per workgroup (4 x 8-element vectors)
constexpr int DNV = 4;

__host__ __device__ constexpr int dw_in_edge(int k, int s) { return (DT - 1) * s + k; }

// ------------------------------------------------------------------------------ forward
template <typename T, int K, int S, int MODE, bool STATS>
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwGeom g, const T* __restrict__ X, const float* __restrict__ w,
                                                     T* __restrict__ Y, Pro pro, float* __restrict__ stats,
                                                     int64_t ntiles) {
  constexpr int IE = dw_in_edge(K, S);
  __shared__ __attribute__((aligned(16))) T tin[IE * IE * DCG];
  __shared__ __attribute__((aligned(16))) float wts[K * K * DCG];
  __shared__ float st_sum[DCG], st_sq[DCG];
  const int tid = threadIdx.x, vec = tid & 3, pt = tid >> 2;
  const int c0 = blockIdx.y * DCG;
  const int C = g.C;
  const int tiles_x = (g.Wo + DT - 1) / DT, tiles_y = (g.Ho + DT - 1) / DT;
  // weights [c][kh][kw] -> LDS [tap][c_local]
  for (int i = tid; i < K * K * DCG; i += 256) {
    const int tap = i / DCG, cl = i - tap * DCG;
    wts[i] = (c0 + cl < C) ? w[(int64_t)(c0 + cl) * K * K + tap] : 0.f;
  }
  if constexpr (STATS) {
    if (tid < DCG) { st_sum[tid] = 0.f; st_sq[tid] = 0.f; }
  }
  const bool cvalid = c0 + vec * 8 < C;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int f = (int)(t / (tiles_x * tiles_y));
    const int rem = (int)(t - (int64_t)f * tiles_x * tiles_y);
    const int oy0 = (rem / tiles_x) * DT, ox0 = (rem % tiles_x) * DT;
    const int iy0 = oy0 * S - g.pad, ix0 = ox0 * S - g.pad;
    __syncthreads();
    for (int e = tid; e < IE * IE * DNV; e += 256) {
      const int pix = e >> 2, v = e & 3;
      const int iy = iy0 + pix / IE, ix = ix0 + pix % IE;
      const int c = c0 + v * 8;
      float x[8];
      if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W && c < C) {
        const int64_t row = ((int64_t)f * g.H + iy) * g.W + ix;
        ld8(X + row * C + c, x);
        apply_pro8<MODE>(pro, row, c, x);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = 0.f;
      }
      st8(tin + pix * DCG + v * 8, x);
    }
    __syncthreads();
    const int ly = pt >> 3, lx = pt & 7;
    const int oy = oy0 + ly, ox = ox0 + lx;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        float x[8], wv[8];
        ld8(tin + ((ly * S + kh) * IE + (lx * S + kw)) * DCG + vec * 8, x);
        ld8(wts + (kh * K + kw) * DCG + vec * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(x[j], wv[j], acc[j]);
      }
    const bool ovalid = oy < g.Ho && ox < g.Wo && cvalid;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = Tr<T>::round(acc[j]);
    if (ovalid) st8(Y + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * C + c0 + vec * 8, acc);
    if constexpr (STATS) {
      float s[8], q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] = ovalid ? acc[j] : 0.f;
        q[j] = s[j] * s[j];
      }
      // reduce over the 16 pixel-lanes of the wave that share `vec` (lane bits 2..5)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) {
          s[j] += __shfl_xor(s[j], o, 64);
          q[j] += __shfl_xor(q[j], o, 64);
        }
      }
      if ((tid & 63) < 4) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          atomicAdd(&st_sum[vec * 8 + j], s[j]);
          atomicAdd(&st_sq[vec * 8 + j], q[j]);
        }
      }
    }
  }
  if constexpr (STATS) {
    __syncthreads();
    if (tid < DCG && c0 + tid < C) {
      stats[((int64_t)blockIdx.x * 2 + 0) * C + c0 + tid] = st_sum[tid];
      stats[((int64_t)blockIdx.x * 2 + 1) * C + c0 + tid] = st_sq[tid];
    }
  }
}

static int dw_grid_x(const DwGeom& g, int64_t ntiles, int groups) {
  const int64_t cap = std::max<int64_t>(1, 2048 / groups);
  return (int)std::min<int64_t>(ntiles, cap);
}

template <typename T>
int launch_dw_fwd(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, int pro_mode,
                  float* stats, int* stat_rows) {
  if (g.C & 7) { set_error("dw: C must be a multiple of 8", __FILE__, __LINE__); return -1; }
  const int64_t ntiles = (int64_t)g.frames * cdiv(g.Ho, DT) * cdiv(g.Wo, DT);
  const int groups = cdiv(g.C, DCG);
  const int gx = dw_grid_x(g, ntiles, groups);
  dim3 grid(gx, groups), block(256);
  const bool st = stats != nullptr;
#define DW_F(KK, SS, MM, ST) hipLaunchKernelGGL((dw_fwd_kernel<T, KK, SS, MM, ST>), grid, block, 0, s, g, X, w, Y, pro, stats, ntiles)
#define DW_F2(KK, SS)                                                  \
  do {                                                                 \
    if (pro_mode == PRO_NONE) { if (st) DW_F(KK, SS, PRO_NONE, true); else DW_F(KK, SS, PRO_NONE, false); } \
    else { if (st) DW_F(KK, SS, PRO_BN_SILU, true); else DW_F(KK, SS, PRO_BN_SILU, false); }              \
  } while (0)
  if (g.k == 3 && g.s == 1) DW_F2(3, 1);
  else if (g.k == 3 && g.s == 2) DW_F2(3, 2);
  else if (g.k == 5 && g.s == 1) DW_F2(5, 1);
  else if (g.k == 5 && g.s == 2) DW_F2(5, 2);
  else { set_error("dw: unsupported kernel/stride", __FILE__, __LINE__); return -1; }
#undef DW_F2
#undef DW_F
  if (stat_rows) *stat_rows = gx;
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------ dgrad
// dX[f,iy,ix,c] = sum_{kh,kw : (iy+pad-kh) % S == 0} dY[f,(iy+pad-kh)/S,(ix+pad-kw)/S,c] * w[c][kh][kw]
__host__ __device__ constexpr int dw_gy_edge(int k, int s) { return (DT - 1 + k - 1) / s + 2; }

__device__ __forceinline__ int floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

template <typename T, int K, int S>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(DwGeom g, const T* __restrict__ dY, const float* __restrict__ w,
                                                       T* __restrict__ dX, int64_t ntiles) {
  constexpr int GE = dw_gy_edge(K, S);
  __shared__ __attribute__((aligned(16))) T tg[GE * GE * DCG];
  __shared__ __attribute__((aligned(16))) float wts[K * K * DCG];
  const int tid = threadIdx.x, vec = tid & 3, pt = tid >> 2;
  const int c0 = blockIdx.y * DCG;
  const int C = g.C;
  const int tiles_x = (g.W + DT - 1) / DT, tiles_y = (g.H + DT - 1) / DT;
  for (int i = tid; i < K * K * DCG; i += 256) {
    const int tap = i / DCG, cl = i - tap * DCG;
    wts[i] = (c0 + cl < C) ? w[(int64_t)(c0 + cl) * K * K + tap] : 0.f;
  }
  const bool cvalid = c0 + vec * 8 < C;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int f = (int)(t / (tiles_x * tiles_y));
    const int rem = (int)(t - (int64_t)f * tiles_x * tiles_y);
    const int iy0 = (rem / tiles_x) * DT, ix0 = (rem % tiles_x) * DT;
    const int gy0 = floordiv(iy0 + g.pad - (K - 1), S), gx0 = floordiv(ix0 + g.pad - (K - 1), S);
    __syncthreads();
    for (int e = tid; e < GE * GE * DNV; e += 256) {
      const int pix = e >> 2, v = e & 3;
      const int oy = gy0 + pix / GE, ox = gx0 + pix % GE;
      const int c = c0 + v * 8;
      float x[8];
      if (oy >= 0 && oy < g.Ho && ox >= 0 && ox < g.Wo && c < C) {
        ld8(dY + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * C + c, x);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = 0.f;
      }
      st8(tg + pix * DCG + v * 8, x);
    }
    __syncthreads();
    const int iy = iy0 + (pt >> 3), ix = ix0 + (pt & 7);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int ty = iy + g.pad - kh;
      if (S == 2 && (ty & 1)) continue;
      const int ly = floordiv(ty, S) - gy0;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int tx = ix + g.pad - kw;
        if (S == 2 && (tx & 1)) continue;
        const int lx = floordiv(tx, S) - gx0;
        float x[8], wv[8];
        ld8(tg + (ly * GE + lx) * DCG + vec * 8, x);
        ld8(wts + (kh * K + kw) * DCG + vec * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(x[j], wv[j], acc[j]);
      }
    }
    if (iy < g.H && ix < g.W && cvalid) st8(dX + (((int64_t)f * g.H + iy) * g.W + ix) * C + c0 + vec * 8, acc);
  }
}

template <typename T>
int launch_dw_dgrad(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* dX) {
  const int64_t ntiles = (int64_t)g.frames * cdiv(g.H, DT) * cdiv(g.W, DT);
  const int groups = cdiv(g.C, DCG);
  const int gx = dw_grid_x(g, ntiles, groups);
  dim3 grid(gx, groups), block(256);
#define DW_D(KK, SS) hipLaunchKernelGGL((dw_dgrad_kernel<T, KK, SS>), grid, block, 0, s, g, dY, w, dX, ntiles)
  if (g.k == 3 && g.s == 1) DW_D(3, 1);
  else if (g.k == 3 && g.s == 2) DW_D(3, 2);
  else if (g.k == 5 && g.s == 1) DW_D(5, 1);
  else if (g.k == 5 && g.s == 2) DW_D(5, 2);
  else { set_error("dw: unsupported kernel/stride", __FILE__, __LINE__); return -1; }
#undef DW_D
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------ wgrad
// dW[c][tap] = sum_{f,oy,ox} dY[f,oy,ox,c] * pro(X)[f, oy*S-pad+kh, ox*S-pad+kw, c]
// Thread (vec, tl): tap = tl % K^2, sub = tl / K^2 accumulates pixels p = sub (mod NSUB) of each tile.
template <typename T, int K, int S, int MODE>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(DwGeom g, const T* __restrict__ dY, const T* __restrict__ X,
                                                       Pro pro, float* __restrict__ slab, int64_t ntiles) {
  constexpr int IE = dw_in_edge(K, S);
  constexpr int KK = K * K;
  constexpr int NSUB = 64 / KK;
  __shared__ __attribute__((aligned(16))) T tin[IE * IE * DCG];
  __shared__ __attribute__((aligned(16))) T tg[DT * DT * DCG];
  __shared__ float red[NSUB * KK * DCG];
  const int tid = threadIdx.x, vec = tid & 3, tl = tid >> 2;
  const int tap = tl % KK, sub = tl / KK;
  const int kh = tap / K, kw = tap % K;
  const bool active = sub < NSUB;
  const int c0 = blockIdx.y * DCG;
  const int C = g.C;
  const int tiles_x = (g.Wo + DT - 1) / DT, tiles_y = (g.Ho + DT - 1) / DT;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int f = (int)(t / (tiles_x * tiles_y));
    const int rem = (int)(t - (int64_t)f * tiles_x * tiles_y);
    const int oy0 = (rem / tiles_x) * DT, ox0 = (rem % tiles_x) * DT;
    const int iy0 = oy0 * S - g.pad, ix0 = ox0 * S - g.pad;
    __syncthreads();
    for (int e = tid; e < IE * IE * DNV; e += 256) {
      const int pix = e >> 2, v = e & 3;
      const int iy = iy0 + pix / IE, ix = ix0 + pix % IE;
      const int c = c0 + v * 8;
      float x[8];
      if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W && c < C) {
        const int64_t row = ((int64_t)f * g.H + iy) * g.W + ix;
        ld8(X + row * C + c, x);
        apply_pro8<MODE>(pro, row, c, x);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = 0.f;
      }
      st8(tin + pix * DCG + v * 8, x);
    }
    for (int e = tid; e < DT * DT * DNV; e += 256) {
      const int pix = e >> 2, v = e & 3;
      const int oy = oy0 + pix / DT, ox = ox0 + pix % DT;
      const int c = c0 + v * 8;
      float x[8];
      if (oy < g.Ho && ox < g.Wo && c < C) {
        ld8(dY + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * C + c, x);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = 0.f;
      }
      st8(tg + pix * DCG + v * 8, x);
    }
    __syncthreads();
    if (active) {
      for (int p = sub; p < DT * DT; p += NSUB) {
        const int ly = p >> 3, lx = p & 7;
        float gy[8], xv[8];
        ld8(tg + p * DCG + vec * 8, gy);
        ld8(tin + ((ly * S + kh) * IE + (lx * S + kw)) * DCG + vec * 8, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(gy[j], xv[j], acc[j]);
      }
    }
  }
  __syncthreads();
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(sub * KK + tap) * DCG + vec * 8 + j] = acc[j];
  }
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * C * KK;
  for (int i = tid; i < KK * DCG; i += 256) {
    const int tp = i / DCG, cl = i - tp * DCG;
    float s = 0.f;
    for (int sb = 0; sb < NSUB; ++sb) s += red[(sb * KK + tp) * DCG + cl];
    if (c0 + cl < C) out[(int64_t)(c0 + cl) * KK + tp] = s;
  }
}

template <typename T>
int launch_dw_wgrad(hipStream_t s, const DwGeom& g, const T* dY, const T* X, const Pro& pro, int pro_mode, float* slab,
                    int64_t slab_cap, float* dW, bool accumulate) {
  const int64_t ntiles = (int64_t)g.frames * cdiv(g.Ho, DT) * cdiv(g.Wo, DT);
  const int groups = cdiv(g.C, DCG);
  const int64_t per = (int64_t)g.C * g.k * g.k;
  int gx = dw_grid_x(g, ntiles, groups);
  gx = (int)std::max<int64_t>(1, std::min<int64_t>(gx, slab_cap / per));
  dim3 grid(gx, groups), block(256);
#define DW_W(KK, SS, MM) hipLaunchKernelGGL((dw_wgrad_kernel<T, KK, SS, MM>), grid, block, 0, s, g, dY, X, pro, slab, ntiles)
#define DW_W2(KK, SS) do { if (pro_mode == PRO_NONE) DW_W(KK, SS, PRO_NONE); else DW_W(KK, SS, PRO_BN_SILU); } while (0)
  if (g.k == 3 && g.s == 1) DW_W2(3, 1);
  else if (g.k == 3 && g.s == 2) DW_W2(3, 2);
  else if (g.k == 5 && g.s == 1) DW_W2(5, 1);
  else if (g.k == 5 && g.s == 2) DW_W2(5, 2);
  else { set_error("dw: unsupported kernel/stride", __FILE__, __LINE__); return -1; }
#undef DW_W2
#undef DW_W
  DFD_HIP_CHECK(hipGetLastError());
  return launch_reduce_slabs(s, slab, gx, per, dW, accumulate);
}

#define DFD_DW_INST(T)                                                                                              \
  template int launch_dw_fwd<T>(hipStream_t, const DwGeom&, const T*, const float*, T*, const Pro&, int, float*,   \
                                int*);                                                                             \
  template int launch_dw_dgrad<T>(hipStream_t, const DwGeom&, const T*, const float*, T*);                         \
  template int launch_dw_wgrad<T>(hipStream_t, const DwGeom&, const T*, const T*, const Pro&, int, float*, int64_t, \
                                  float*, bool);
DFD_DW_INST(float)
DFD_DW_INST(bf16)
#undef DFD_DW_INST

}  // namespace dfd
