// ResNet-50 member of EnsembleDetector (src/pretrained_detector.py:37-40: torchvision resnet50
// minus fc, the app's default ensemble ENSEMBLE_BACKBONES, app.py:661,1597), inference path.
// Layout NHWC.  Every convolution is the implicit-GEMM MFMA kernel of k_rnconv.hip (dfd_rn_conv;
// conv1 on its im2col rows through dfd_rn_gemm, the same kernel as a 1x1 GEMM) with the eval-mode
// BatchNorm folded into its weights and bias, the ReLU and the bottleneck's identity add in its
// epilogue; no library GEMM.  What is not a convolution lives here:
//   im2col      NHWC T -> [N*Ho*Wo][Kp] T, column (ky*kw + kx)*C + c, zero padding (k > 1 or stride 2)
//   stem im2col the (N,3,H,W) frames (any strides; fp32, or uint8 normalised like the B0 stem) for
//               conv1 7x7/2 -> [N*112*112][152] (147 taps zero padded to 16-B rows)
//   maxpool     3x3/2 pad 1 (torchvision resnet.maxpool)
//   avgpool     global average -> (N, C) fp32 (AdaptiveAvgPool2d((1,1)), fixed-order sum)
#include "kernels.h"

namespace dfd {

template <typename T>
__global__ __launch_bounds__(256) void rn_im2col_vec_kernel(const T* __restrict__ x, int H, int W, int C, int kh,
                                                            int kw, int stride, int pad, int Ho, int Wo, int Kp,
                                                            int64_t rows, T* __restrict__ out) {
  // one lane = 8 channels of one tap of one output pixel
  const int cv = C / 8, per_row = kh * kw * cv;
  const int64_t total = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / per_row;
    const int r = (int)(i - m * per_row), tap = r / cv, c8 = (r - tap * cv) * 8;
    const int ky = tap / kw, kx = tap - ky * kw;
    const int64_t n = m / ((int64_t)Ho * Wo);
    const int rem = (int)(m - n * Ho * Wo), oy = rem / Wo, ox = rem - oy * Wo;
    const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) ld8(x + ((n * H + iy) * W + ix) * C + c8, v);
    st8(out + m * Kp + tap * C + c8, v);
  }
}

// conv1 rows: Kp = 152 columns = 147 taps (ky, kx, c) + 5 zeros.  One thread per output pixel: the
// 147 (ky, kx, c) column decompositions are compile-time constants, the pixel's index math is done
// once, uint8 values are normalised through a 3 x 256 LDS table built with the same operations in
// the same order (bit-identical values).  bf16 rows (304 B) are staged per wave in LDS and leave as
// contiguous 1-KB wave stores (a thread's own row as 19 16-B stores 304 B apart measured 871 us for
// 256 frames; an element per thread with two 64-bit and two fp32 divisions each, 1.35 ms).
template <typename T, bool U8>
__global__ __launch_bounds__(128) void rn_stem_rows_kernel(const void* __restrict__ x, int64_t sn, int64_t sc,
                                                           int64_t sh, int64_t sw, InputFmt in, int H, int W, int Ho,
                                                           int Wo, int64_t rows, T* __restrict__ out) {
  constexpr int KS = 7, KP = 152, NV = KP / 8;
  constexpr bool STG = sizeof(T) == 2;  // 16-B chunks of 8 bf16
  __shared__ float lut[U8 ? 3 * 256 : 1];
  __shared__ uint4 stg[STG ? 2 * 64 * NV : 1];
  if constexpr (U8) {
    for (int i = threadIdx.x; i < 3 * 256; i += 128) {
      const int c = i >> 8;
      lut[i] = ((float)(i & 255) / 255.0f - in.mean[c]) / in.stdv[c];
    }
    __syncthreads();
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t hw = (int64_t)Ho * Wo;
  for (int64_t m0 = ((int64_t)blockIdx.x * 2 + wave) * 64, step = (int64_t)gridDim.x * 128; m0 - wave * 64 < rows;
       m0 += step) {
    const int64_t m = m0 + lane;
    if (m < rows) {
      const int64_t n = m / hw;
      const int rem = (int)(m - n * hw), oy = rem / Wo, ox = rem - oy * Wo;
      const int iy0 = oy * 2 - 3, ix0 = ox * 2 - 3;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = 8 * v + j;
          o[j] = 0.f;
          if (col < KS * KS * 3) {
            const int tap = col / 3, c = col % 3, ky = tap / KS, kx = tap % KS;
            const int iy = iy0 + ky, ix = ix0 + kx;
            if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
              const int64_t e = n * sn + c * sc + iy * sh + ix * sw;
              if constexpr (U8) o[j] = lut[c * 256 + static_cast<const uint8_t*>(x)[e]];
              else o[j] = static_cast<const float*>(x)[e];
            }
          }
        }
        if constexpr (STG) {
          stg[(wave * 64 + lane) * NV + v] =
              make_uint4(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]), pack2bf(o[4], o[5]), pack2bf(o[6], o[7]));
        } else {
          st8(out + m * KP + 8 * v, o);
        }
      }
    }
    if constexpr (STG) {
      __syncthreads();
      // the wave's 64 rows are 64 x 19 contiguous 16-B chunks of the output
      uint4* dst = reinterpret_cast<uint4*>(out + m0 * KP);
#pragma unroll
      for (int it = 0; it < NV; ++it) {
        const int q = it * 64 + lane;
        if (m0 + q / NV < rows) dst[q] = stg[wave * 64 * NV + q];
      }
      __syncthreads();
    }
  }
}

// conv1 (7x7/2 pad 3, 3 -> 64, folded BN + ReLU) as an implicit GEMM, bf16: no im2col rows in HBM.
// Per 16 x 16 output tile: the 37 x 37 x 3 input window normalised into LDS (uint8 through the
// 3 x 256 table, the same operations as the im2col rows), then 5 k-steps of 32 taps (147 + zeros):
// each thread writes its pixel's 32 taps of the step (compile-time tap decomposition) into a
// wave-local im2col slice, and each wave runs D[co][pix] += W[co][k] . patch[pix][k] on
// v_mfma_f32_16x16x32_bf16 for its 64 pixels x 64 channels; bias + ReLU, one rounding, 16-B row
// stores through an LDS slab.  Replaces 976 MB of im2col writes + reads per 256 frames.
constexpr int RST = 16, RIE = (RST - 1) * 2 + 7, RNIN = RIE * RIE * 3;  // 37 x 37 x 3 window
constexpr int RKS = 160, RXS = 40, RCS = 72;  // padded K; im2col / output slab row strides (bf16)
constexpr int RTINB = (RNIN * 4 + 15) / 16 * 16, RXSB = 256 * RXS * 2, RCSB = 256 * RCS * 2;
constexpr int RUNI = RTINB + RXSB > RCSB ? RTINB + RXSB : RCSB;  // tin + im2col, later the output slab
typedef short rs_bf16x8 __attribute__((ext_vector_type(8)));
#ifndef DFD_RSTEM_PF  // 1: the next tile's window loads fly during this tile's MFMAs (A/B build switch;
                      // measured neutral, ab_rstem_pf_r04t.jsonl, at 256 instead of 244 VGPRs: off)
#define DFD_RSTEM_PF 0
#endif
typedef float rs_f32x4 __attribute__((ext_vector_type(4)));

template <bool U8>
__global__ __launch_bounds__(256, 2) void rn_stem_conv_kernel(const void* __restrict__ x, int64_t sn, int64_t sc,
                                                              int64_t sh, int64_t sw, InputFmt in, int H, int W, int Ho,
                                                              int Wo, const bf16* __restrict__ Wt,
                                                              const float* __restrict__ bias, bf16* __restrict__ out,
                                                              int64_t ntiles) {
  __shared__ __attribute__((aligned(16))) char uni[RUNI];
  __shared__ float lut[U8 ? 3 * 256 : 1];
  __shared__ __attribute__((aligned(16))) bf16 wsb[64 * RKS];
  float* tin = reinterpret_cast<float*>(uni);
  bf16* xs = reinterpret_cast<bf16*>(uni + RTINB);
  bf16* ct = reinterpret_cast<bf16*>(uni);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if constexpr (U8) {
    for (int i = tid; i < 3 * 256; i += 256) {
      const int c = i >> 8;
      lut[i] = ((float)(i & 255) / 255.0f - in.mean[c]) / in.stdv[c];
    }
  }
  for (int i = tid; i < 64 * RKS; i += 256) {  // W [64][152] -> [64][160], zero pad
    const int co = i / RKS, k = i - co * RKS;
    wsb[i] = k < 152 ? Wt[co * 152 + k] : bf16{0};
  }
  const int tpf = (Ho / RST) * (Wo / RST), tx = Wo / RST;
  float bsv[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) bsv[a][r] = bias[16 * a + 4 * (lane >> 4) + r];
  const int ly = tid / RST, lx = tid % RST;
  // the next tile's window in registers while this tile computes: raw bytes (U8) or fp32 bits, and a
  // bit per load for the positions inside the map
  constexpr int NLD = (RNIN + 255) / 256;
  static_assert(NLD <= 32, "validity mask");
  uint32_t raw[NLD], okm = 0u;
  auto load = [&](int64_t t) {
    okm = 0u;
    const int64_t n = t / tpf;
    const int r = (int)(t - n * tpf), iy0 = (r / tx) * RST * 2 - 3, ix0 = (r % tx) * RST * 2 - 3;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = tid + 256 * i;
      const int pix = e / 3, c = e - pix * 3, ry = pix / RIE, rx = pix - ry * RIE;
      const int iy = iy0 + ry, ix = ix0 + rx;
      uint32_t v = 0u;
      if (e < RNIN && iy >= 0 && iy < H && ix >= 0 && ix < W) {
        const int64_t o = n * sn + c * sc + iy * sh + ix * sw;
        if constexpr (U8) v = static_cast<const uint8_t*>(x)[o];
        else v = __float_as_uint(static_cast<const float*>(x)[o]);
        okm |= 1u << i;
      }
      raw[i] = v;
    }
  };
  if (DFD_RSTEM_PF && blockIdx.x < ntiles) load(blockIdx.x);
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t n = t / tpf;
    const int r = (int)(t - n * tpf), oy0 = (r / tx) * RST, ox0 = (r % tx) * RST;
    if (!DFD_RSTEM_PF) load(t);
    __syncthreads();  // the previous tile's output slab (aliases tin / xs) has been stored
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = tid + 256 * i;
      if (e < RNIN) {
        const int c = e % 3;
        float v = 0.f;  // zero padding after normalisation, as conv2d pads
        if ((okm >> i) & 1u) {
          if constexpr (U8) v = lut[c * 256 + raw[i]];
          else v = __uint_as_float(raw[i]);
        }
        tin[e] = v;
      }
    }
    __syncthreads();
    if (DFD_RSTEM_PF && t + gridDim.x < ntiles) load(t + gridDim.x);
    rs_f32x4 acc[4][4];
#pragma unroll
    for (int pb = 0; pb < 4; ++pb)
#pragma unroll
      for (int a = 0; a < 4; ++a) acc[pb][a] = rs_f32x4{0.f, 0.f, 0.f, 0.f};
    const float* tp = tin + (ly * 2 * RIE + lx * 2) * 3;  // this thread's pixel window origin
#pragma unroll
    for (int s = 0; s < RKS / 32; ++s) {
      // this pixel's 32 taps of k-step s into its im2col row (rows of this wave only: wave-local)
#pragma unroll
      for (int c8 = 0; c8 < 4; ++c8) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * s + 8 * c8 + j;
          if (k < 147) {
            const int tap = k / 3, c = k % 3, ky = tap / 7, kx = tap % 7;
            v[j] = tp[(ky * RIE + kx) * 3 + c];
          } else {
            v[j] = 0.f;
          }
        }
        st8(xs + tid * RXS + 8 * c8, v);
      }
      rs_bf16x8 wf[4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
        wf[a] = *reinterpret_cast<const rs_bf16x8*>(wsb + (16 * a + (lane & 15)) * RKS + 32 * s + 8 * (lane >> 4));
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        const int p0 = wave * 64 + 16 * pb;
        const rs_bf16x8 pf = *reinterpret_cast<const rs_bf16x8*>(xs + (p0 + (lane & 15)) * RXS + 8 * (lane >> 4));
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[pb][a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[a], pf, acc[pb][a], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done with tin (the slab overwrites it)
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      const int pix = wave * 64 + 16 * pb + (lane & 15);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = fmaxf(Tr<bf16>::round(acc[pb][a][q] + bsv[a][q]), 0.f);
        *reinterpret_cast<uint2*>(ct + pix * RCS + 16 * a + 4 * (lane >> 4)) =
            make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // 256 pixels x 8 vectors of 8 channels
      const int e = tid + 256 * i, pix = e >> 3, v = e & 7;
      const int oy = oy0 + pix / RST, ox = ox0 + pix % RST;
      *reinterpret_cast<uint4*>(out + (((int64_t)n * Ho + oy) * Wo + ox) * 64 + 8 * v) =
          *reinterpret_cast<const uint4*>(ct + pix * RCS + 8 * v);
    }
  }
}

int launch_rn_stem_conv(hipStream_t s, const void* x, const InputFmt& in, const int64_t* strides, int N, int H, int W,
                        const bf16* Wt, const float* bias, bf16* out) {
  const int Ho = (H + 6 - 7) / 2 + 1, Wo = (W + 6 - 7) / 2 + 1;
  if (Ho % RST || Wo % RST) { set_error("resnet stem conv: output map not a multiple of 16", __FILE__, __LINE__); return -1; }
  const int64_t ntiles = (int64_t)N * (Ho / RST) * (Wo / RST);
  const int gx = (int)std::min<int64_t>(ntiles, 1024);
  if (in.u8)
    hipLaunchKernelGGL(rn_stem_conv_kernel<true>, dim3(gx), dim3(256), 0, s, x, strides[0], strides[1], strides[2],
                       strides[3], in, H, W, Ho, Wo, Wt, bias, out, ntiles);
  else
    hipLaunchKernelGGL(rn_stem_conv_kernel<false>, dim3(gx), dim3(256), 0, s, x, strides[0], strides[1], strides[2],
                       strides[3], in, H, W, Ho, Wo, Wt, bias, out, ntiles);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

template <typename T>
__global__ __launch_bounds__(256) void rn_maxpool_kernel(const T* __restrict__ x, int N, int H, int W, int C, int Ho,
                                                         int Wo, T* __restrict__ out) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * Ho * Wo * cv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(i % cv) * 8;
    const int64_t p = i / cv;
    const int64_t n = p / ((int64_t)Ho * Wo);
    const int rem = (int)(p - n * Ho * Wo), oy = rem / Wo, ox = rem - oy * Wo;
    float mx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) mx[j] = -INFINITY;
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * 2 - 1 + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * 2 - 1 + kx;
        if (ix < 0 || ix >= W) continue;
        float v[8];
        ld8(x + ((n * H + iy) * W + ix) * C + c8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) mx[j] = fmaxf(mx[j], v[j]);
      }
    }
    st8(out + p * C + c8, mx);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void rn_avgpool_kernel(const T* __restrict__ x, int HW, int C, float inv,
                                                         float* __restrict__ out) {
  const int n = blockIdx.y;
  for (int c = blockIdx.x * 256 + threadIdx.x; c < C; c += gridDim.x * 256) {
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += Tr<T>::to_f(x[((int64_t)n * HW + p) * C + c]);
    out[(int64_t)n * C + c] = s * inv;
  }
}

static int ew_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 8192)); }

template <typename T>
int launch_rn_im2col(hipStream_t s, const T* x, int N, int H, int W, int C, int kh, int kw, int stride, int pad,
                     int Kp, T* out) {
  if (C % 8 || Kp < kh * kw * C) { set_error("resnet im2col: C % 8 != 0 or Kp too small", __FILE__, __LINE__); return -1; }
  const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  const int64_t rows = (int64_t)N * Ho * Wo;
  hipLaunchKernelGGL(rn_im2col_vec_kernel<T>, dim3(ew_grid(rows * kh * kw * (C / 8))), dim3(256), 0, s, x, H, W, C, kh,
                     kw, stride, pad, Ho, Wo, Kp, rows, out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

template <typename T>
int launch_rn_stem_im2col(hipStream_t s, const void* x, const InputFmt& in, const int64_t* strides, int N, int H,
                          int W, T* out) {
  const int Ho = (H + 6 - 7) / 2 + 1, Wo = (W + 6 - 7) / 2 + 1;
  const int64_t rows = (int64_t)N * Ho * Wo;
  const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(rows, 128), 8192));
  if (in.u8)
    hipLaunchKernelGGL((rn_stem_rows_kernel<T, true>), dim3(gx), dim3(128), 0, s, x, strides[0], strides[1],
                       strides[2], strides[3], in, H, W, Ho, Wo, rows, out);
  else
    hipLaunchKernelGGL((rn_stem_rows_kernel<T, false>), dim3(gx), dim3(128), 0, s, x, strides[0],
                       strides[1], strides[2], strides[3], in, H, W, Ho, Wo, rows, out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

template <typename T>
int launch_rn_maxpool(hipStream_t s, const T* x, int N, int H, int W, int C, T* out) {
  if (C % 8) { set_error("resnet maxpool: C % 8 != 0", __FILE__, __LINE__); return -1; }
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(rn_maxpool_kernel<T>, dim3(ew_grid((int64_t)N * Ho * Wo * (C / 8))), dim3(256), 0, s, x, N, H, W,
                     C, Ho, Wo, out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

template <typename T>
int launch_rn_avgpool(hipStream_t s, const T* x, int N, int HW, int C, float* out) {
  if (N > 65535) { set_error("resnet avgpool: at most 65535 frames", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL(rn_avgpool_kernel<T>, dim3(cdiv(C, 256), N), dim3(256), 0, s, x, HW, C, 1.0f / (float)HW, out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

#define DFD_RN_INST(T)                                                                                           \
  template int launch_rn_im2col<T>(hipStream_t, const T*, int, int, int, int, int, int, int, int, int, T*);       \
  template int launch_rn_stem_im2col<T>(hipStream_t, const void*, const InputFmt&, const int64_t*, int, int, int, \
                                        T*);                                                                    \
  template int launch_rn_maxpool<T>(hipStream_t, const T*, int, int, int, int, T*);                                \
  template int launch_rn_avgpool<T>(hipStream_t, const T*, int, int, int, float*);
DFD_RN_INST(float)
DFD_RN_INST(bf16)

}  // namespace dfd
