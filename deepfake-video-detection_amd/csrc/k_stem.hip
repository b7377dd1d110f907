// EfficientNet-B0 stem: conv2d 3->32, k3, s2, pad 1 (timm conv_stem), forward with BN-stat
// epilogue and weight gradient.  The fp32 input frames are read IN PLACE with arbitrary
// (frame, channel, row, col) strides -- the reference hands over channels-last-strided
// (B*T,3,H,W) tensors (app.py:2084-2086) -- so no transpose/copy precedes it.
#include "kernels.h"

namespace dfd {

constexpr int ST = 8;                 // output tile edge
constexpr int SIE = (ST - 1) * 2 + 3; // 17: input tile edge
constexpr int SCO = 32;               // output channels

template <typename T, bool STATS>
__global__ __launch_bounds__(256) void stem_fwd_kernel(StemGeom g, const float* __restrict__ x,
                                                       const float* __restrict__ w, T* __restrict__ Y,
                                                       float* __restrict__ stats, int64_t ntiles) {
  __shared__ float tin[3][SIE * SIE];
  __shared__ __attribute__((aligned(16))) float wts[27][SCO];  // [ci*9+tap][co]
  __shared__ float st_sum[SCO], st_sq[SCO];
  const int tid = threadIdx.x, vec = tid & 3, pt = tid >> 2;
  for (int i = tid; i < 27 * SCO; i += 256) {
    const int co = i / 27, r = i % 27;  // w[co][ci][kh][kw], r = ci*9 + kh*3 + kw
    wts[r][co] = w[i];
  }
  if (STATS && tid < SCO) { st_sum[tid] = 0.f; st_sq[tid] = 0.f; }
  const int tiles_x = (g.Wo + ST - 1) / ST, tiles_y = (g.Ho + ST - 1) / ST;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int f = (int)(t / (tiles_x * tiles_y));
    const int rem = (int)(t - (int64_t)f * tiles_x * tiles_y);
    const int oy0 = (rem / tiles_x) * ST, ox0 = (rem % tiles_x) * ST;
    const int iy0 = oy0 * 2 - 1, ix0 = ox0 * 2 - 1;
    __syncthreads();
    for (int e = tid; e < 3 * SIE * SIE; e += 256) {
      const int pix = e / 3, ci = e % 3;
      const int iy = iy0 + pix / SIE, ix = ix0 + pix % SIE;
      float v = 0.f;
      if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W) v = x[f * g.sf + ci * g.sc + iy * g.sh + ix * g.sw];
      tin[ci][pix] = v;
    }
    __syncthreads();
    const int ly = pt >> 3, lx = pt & 7;
    const int oy = oy0 + ly, ox = ox0 + lx;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const float xv = tin[ci][(ly * 2 + kh) * SIE + lx * 2 + kw];
          float wv[8];
          ld8(&wts[ci * 9 + kh * 3 + kw][vec * 8], wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv, wv[j], acc[j]);
        }
    const bool ovalid = oy < g.Ho && ox < g.Wo;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = Tr<T>::round(acc[j]);
    if (ovalid) st8(Y + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * SCO + vec * 8, acc);
    if constexpr (STATS) {
      float s[8], q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] = ovalid ? acc[j] : 0.f; q[j] = s[j] * s[j]; }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) {
          s[j] += __shfl_xor(s[j], o, 64);
          q[j] += __shfl_xor(q[j], o, 64);
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
    if (tid < SCO) {
      stats[((int64_t)blockIdx.x * 2 + 0) * SCO + tid] = st_sum[tid];
      stats[((int64_t)blockIdx.x * 2 + 1) * SCO + tid] = st_sq[tid];
    }
  }
}

template <typename T>
int launch_stem_fwd(hipStream_t s, const StemGeom& g, const float* x, const float* w, T* Y, float* stats,
                    int* stat_rows) {
  const int64_t ntiles = (int64_t)g.frames * cdiv(g.Ho, ST) * cdiv(g.Wo, ST);
  const int gx = (int)std::min<int64_t>(ntiles, 2048);
  if (stats)
    hipLaunchKernelGGL((stem_fwd_kernel<T, true>), dim3(gx), dim3(256), 0, s, g, x, w, Y, stats, ntiles);
  else
    hipLaunchKernelGGL((stem_fwd_kernel<T, false>), dim3(gx), dim3(256), 0, s, g, x, w, Y, stats, ntiles);
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = gx;
  return 0;
}

// dW[co][ci][kh][kw] = sum dY[f,oy,ox,co] * x[f,ci,2oy-1+kh,2ox-1+kw]
// thread (co = tid & 31, sub = tid >> 5) accumulates all 27 taps over pixels p = sub (mod 8)
template <typename T>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(StemGeom g, const float* __restrict__ x,
                                                         const T* __restrict__ dY, float* __restrict__ slab,
                                                         int64_t ntiles) {
  __shared__ float tin[3][SIE * SIE];
  __shared__ __attribute__((aligned(16))) float tg[ST * ST][SCO];
  __shared__ float red[8][27][SCO];
  const int tid = threadIdx.x, co = tid & 31, sub = tid >> 5;
  float acc[27];
#pragma unroll
  for (int r = 0; r < 27; ++r) acc[r] = 0.f;
  const int tiles_x = (g.Wo + ST - 1) / ST, tiles_y = (g.Ho + ST - 1) / ST;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int f = (int)(t / (tiles_x * tiles_y));
    const int rem = (int)(t - (int64_t)f * tiles_x * tiles_y);
    const int oy0 = (rem / tiles_x) * ST, ox0 = (rem % tiles_x) * ST;
    const int iy0 = oy0 * 2 - 1, ix0 = ox0 * 2 - 1;
    __syncthreads();
    for (int e = tid; e < 3 * SIE * SIE; e += 256) {
      const int pix = e / 3, ci = e % 3;
      const int iy = iy0 + pix / SIE, ix = ix0 + pix % SIE;
      float v = 0.f;
      if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W) v = x[f * g.sf + ci * g.sc + iy * g.sh + ix * g.sw];
      tin[ci][pix] = v;
    }
    for (int e = tid; e < ST * ST * 4; e += 256) {
      const int pix = e >> 2, v = e & 3;
      const int oy = oy0 + pix / ST, ox = ox0 + pix % ST;
      float d[8];
      if (oy < g.Ho && ox < g.Wo) {
        ld8(dY + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * SCO + v * 8, d);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = 0.f;
      }
      st8(&tg[pix][v * 8], d);
    }
    __syncthreads();
    for (int p = sub; p < ST * ST; p += 8) {
      const int ly = p >> 3, lx = p & 7;
      const float d = tg[p][co];
#pragma unroll
      for (int ci = 0; ci < 3; ++ci)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw)
            acc[ci * 9 + kh * 3 + kw] = fmaf(d, tin[ci][(ly * 2 + kh) * SIE + lx * 2 + kw], acc[ci * 9 + kh * 3 + kw]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 27; ++r) red[sub][r][co] = acc[r];
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * 27 * SCO;
  for (int i = tid; i < 27 * SCO; i += 256) {
    const int c = i / 27, r = i % 27;
    float a = 0.f;
    for (int sb = 0; sb < 8; ++sb) a += red[sb][r][c];
    out[i] = a;
  }
}

template <typename T>
int launch_stem_wgrad(hipStream_t s, const StemGeom& g, const float* x, const T* dY, float* slab, int64_t slab_cap,
                      float* dW, bool accumulate) {
  const int64_t ntiles = (int64_t)g.frames * cdiv(g.Ho, ST) * cdiv(g.Wo, ST);
  int gx = (int)std::min<int64_t>(ntiles, 1024);
  gx = (int)std::max<int64_t>(1, std::min<int64_t>(gx, slab_cap / (27 * SCO)));
  hipLaunchKernelGGL((stem_wgrad_kernel<T>), dim3(gx), dim3(256), 0, s, g, x, dY, slab, ntiles);
  DFD_HIP_CHECK(hipGetLastError());
  return launch_reduce_slabs(s, slab, gx, 27 * SCO, dW, accumulate);
}

template int launch_stem_fwd<float>(hipStream_t, const StemGeom&, const float*, const float*, float*, float*, int*);
template int launch_stem_fwd<bf16>(hipStream_t, const StemGeom&, const float*, const float*, bf16*, float*, int*);
template int launch_stem_wgrad<float>(hipStream_t, const StemGeom&, const float*, const float*, float*, int64_t,
                                      float*, bool);
template int launch_stem_wgrad<bf16>(hipStream_t, const StemGeom&, const float*, const bf16*, float*, int64_t, float*,
                                     bool);

}  // namespace dfd
