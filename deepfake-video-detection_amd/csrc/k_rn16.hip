// ResNet-50 ensemble member, TRAINING in bf16 (EnsembleTrainer.train_epoch over the app's default
// EnsembleDetector(['efficientnet_b0', 'resnet50']), src/ensemble_trainer.py:158-229,
// src/pretrained_detector.py:146-218; the member is torchvision resnet50 minus fc, :37-40).
//
// The fp32 training path (k_conv.hip / k_rntrain.hip) runs every convolution on exact fp32 MFMA; here
// the bottleneck convolutions (every conv after the stem) run on v_mfma_f32_16x16x32_bf16 with bf16
// activations and fp32 accumulation, master weights fp32 (packed to bf16 once per step):
//   forward  y[m][co]      = sum_(ky,kx,ci) x(m; ky,kx,ci) wf[co][ky][kx][ci]    + BN-stat partials
//   dgrad    dx[p][ci]     = sum_(ky,kx,co) dy(p; ky,kx,co) wd[ci][ky][kx][co]   (+ the other path's dx)
//   wgrad    dw[co][(ky,kx,ci)] = sum_m dy[m][co] x(m; ky,kx,ci)                (split over m, slabs)
// The tile loops are the EfficientNet-B0 1x1 GEMMs' (gemm_body.h: pw_gemm_body, pw_wgrad_body) reading
// their A / X operand through ConvGather -- the implicit-GEMM gather, one tap per k-step (C % 64 == 0),
// whole 16-B channel vectors (a stride-2 data gradient's taps are integral or not per pixel, never per
// channel).  Train-mode BatchNorm (batch statistics, running buffers like torch) in fp32 / fp64 around
// them, in torch's centred order: out = relu?((y - mean) * scale + beta (+ res)),
// dy = k1*g + k2*(y - mean) + k3.  conv1 (Cin = 3) + its BN + ReLU + max-pool stay on the fp32 kernels.
#include "gemm_body.h"
#include "rn16.h"

namespace dfd {

// ------------------------------------------------------------------ convolutions
template <int BM, int BN, int WN, int D, int BK, int OCC>
__global__ __launch_bounds__(256, OCC) void rn16_conv_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                              bf16* __restrict__ y, int64_t M, int N, int K,
                                                              float* __restrict__ stats, int64_t tiles_m, int ntn,
                                                              ConvGather cg) {
  using G = GemmCfg<bf16, BM, BN, WN, D, BK>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  __shared__ float st_sum[BN];
  __shared__ float st_sq[BN];
  __shared__ float st_part[G::WM][2][BN];
  pw_gemm_body<bf16, PRO_NONE, true, 0, BM, BN, WN, D, BK, 1>(x, wf, y, nullptr, nullptr, nullptr, M, N, K, Pro{}, stats,
                                                             tiles_m, ntn, (int)blockIdx.x, (int)gridDim.x, smem,
                                                             st_sum, st_sq, &st_part[0][0][0], nullptr, cg);
}

template <int EPI, int BM, int BN, int WN, int D, int BK, int OCC>
__global__ __launch_bounds__(256, OCC) void rn16_conv_dgrad_kernel(const bf16* __restrict__ dy,
                                                                const bf16* __restrict__ wd, bf16* __restrict__ dx,
                                                                const bf16* __restrict__ res, int64_t M, int N, int K,
                                                                int64_t tiles_m, int ntn, ConvGather cg) {
  using G = GemmCfg<bf16, BM, BN, WN, D, BK>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  pw_gemm_body<bf16, PRO_NONE, false, EPI, BM, BN, WN, D, BK, 1>(dy, wd, dx, res, nullptr, nullptr, M, N, K, Pro{},
                                                                nullptr, tiles_m, ntn, (int)blockIdx.x, (int)gridDim.x,
                                                                smem, nullptr, nullptr, nullptr, nullptr, cg);
}

__global__ __launch_bounds__(256, 3) void rn16_conv_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                              int64_t M, int N, int K, float* __restrict__ slab, int tnk,
                                                              int64_t m_per_split, ConvGather cg) {
  __shared__ __attribute__((aligned(16))) char smem[WgCfg<bf16>::SMEM];
  pw_wgrad_body<bf16, PRO_NONE, 1, 1>(dy, x, M, N, K, Pro{}, slab, tnk, m_per_split,
                                      (int)(blockIdx.y * gridDim.x + blockIdx.x), (int)(gridDim.x * gridDim.y),
                                      (int)gridDim.x, smem, cg);
}

static ConvGather make_gather(int C, int H, int W, int Ho, int Wo, int kw, int s, int p, int dgrad) {
  ConvGather g{};
  g.C = C; g.H = H; g.W = W; g.Ho = Ho; g.Wo = Wo; g.KW = kw; g.S = s; g.P = p; g.dgrad = dgrad;
  conv_gather_fdiv((uint32_t)(Ho * Wo), g.mhw, g.lhw);
  conv_gather_fdiv((uint32_t)Wo, g.mw, g.lw);
  return g;
}

static bool rn16_shape_ok(int N, int H, int W, int Cin, int Cout, int kh, int kw, int s, int p) {
  if (N <= 0 || H <= 0 || W <= 0 || kh != kw || (kh != 1 && kh != 3) || (s != 1 && s != 2) || p != (kh - 1) / 2)
    return false;
  if (Cin % 64 || Cout % 64) return false;  // one tap per 64-deep k-step / K tile
  const int Ho = (H + 2 * p - kh) / s + 1, Wo = (W + 2 * p - kw) / s + 1;
  return (int64_t)N * H * W <= (int64_t)INT32_MAX / 2 && (int64_t)N * Ho * Wo * Cout < (1ll << 40);
}

// the tile of a (rows, N) product: these convolutions have long K (576..4608) and are MFMA-bound, so the
// largest tile that still gives the 256 CUs enough workgroups -- 128x128 (16 MFMAs per wave per 32-deep
// k-slice) from 384 tiles, 128x64 from 256, else 32x64 (64-deep k-steps) on the 7x7 map
static int rn16_cfg(int64_t M, int N) {
  const int64_t t128 = cdiv64(M, 128);
  if (N > 64 && t128 * cdiv(N, 128) >= 384) return 0;
  if (t128 * cdiv(N, 64) >= 256) return 1;
  return 3;
}

#ifndef DFD_RN16_BK  // k-step depth of the 128-row tiles (A/B build switch: 32 or 64)
#define DFD_RN16_BK 64
#endif
#define DFD_RN16_CFGS(GO)                                                  \
  if (cfg == 0) GO(128, 128, 1, DFD_RN16_BK == 64 ? 1 : 2, DFD_RN16_BK, 2); \
  else if (cfg == 1) GO(128, 64, 1, DFD_RN16_BK == 64 ? 2 : 3, DFD_RN16_BK, 2); \
  else GO(32, 64, 2, 2, 64, 3);

static int rn16_grid(int64_t M, int N, int cfg, int64_t* tiles_m, int* ntn) {
  const int bm = cfg == 0 || cfg == 1 ? 128 : 32, bn = cfg == 0 ? 128 : 64;
  *ntn = cdiv(N, bn);
  *tiles_m = cdiv64(M, bm);
  return (int)std::min<int64_t>(*tiles_m, std::max<int64_t>(1, 1024 / *ntn));
}

int rn16_conv_fwd(hipStream_t s, const bf16* x, int N, int H, int W, int Cin, const bf16* wf, int Cout, int k, int stride,
                  int pad, bf16* y, float* stats, int* stat_rows) {
  if (!rn16_shape_ok(N, H, W, Cin, Cout, k, k, stride, pad)) {
    set_error("rn16 conv: shape outside the bf16 training kernels (1x1 / 3x3, stride 1 / 2, C % 64)", __FILE__,
              __LINE__);
    return -1;
  }
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t M = (int64_t)N * Ho * Wo;
  const int K = k * k * Cin;
  const ConvGather cg = make_gather(Cin, H, W, Ho, Wo, k, stride, pad, 0);
  const int cfg = rn16_cfg(M, Cout);
  int64_t tiles_m;
  int ntn;
  const int gx = rn16_grid(M, Cout, cfg, &tiles_m, &ntn);
#define DFD_GO(BM_, BN_, WN_, D_, BK_, OCC_)                                                                          \
  hipLaunchKernelGGL((rn16_conv_fwd_kernel<BM_, BN_, WN_, D_, BK_, OCC_>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, \
                     x, wf, y, M, Cout, K, stats, tiles_m, ntn, cg)
  DFD_RN16_CFGS(DFD_GO)
#undef DFD_GO
  DFD_HIP_CHECK(hipGetLastError());
  *stat_rows = gx;
  return 0;
}

int rn16_conv_dgrad(hipStream_t s, const bf16* dy, int N, int H, int W, int Cin, const bf16* wd, int Cout, int k,
                    int stride, int pad, const bf16* res, bf16* dx) {
  if (!rn16_shape_ok(N, H, W, Cin, Cout, k, k, stride, pad)) {
    set_error("rn16 dgrad: shape outside the bf16 training kernels", __FILE__, __LINE__);
    return -1;
  }
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t M = (int64_t)N * H * W;  // rows: input pixels
  const int K = k * k * Cout;
  // source: dy [N][Ho][Wo][Cout]; rows map: the input map (H, W)
  const ConvGather cg = make_gather(Cout, Ho, Wo, H, W, k, stride, pad, 1);
  const int cfg = rn16_cfg(M, Cin);
  int64_t tiles_m;
  int ntn;
  const int gx = rn16_grid(M, Cin, cfg, &tiles_m, &ntn);
#define DFD_GO(BM_, BN_, WN_, D_, BK_, OCC_)                                                                        \
  do {                                                                                                              \
    if (res)                                                                                                        \
      hipLaunchKernelGGL((rn16_conv_dgrad_kernel<EPI_RESID, BM_, BN_, WN_, D_, BK_, OCC_>), dim3((unsigned)(gx * ntn)), \
                         dim3(256), 0, s, dy, wd, dx, res, M, Cin, K, tiles_m, ntn, cg);                            \
    else                                                                                                            \
      hipLaunchKernelGGL((rn16_conv_dgrad_kernel<0, BM_, BN_, WN_, D_, BK_, OCC_>), dim3((unsigned)(gx * ntn)),      \
                         dim3(256), 0, s, dy, wd, dx, res, M, Cin, K, tiles_m, ntn, cg);                            \
  } while (0)
  DFD_RN16_CFGS(DFD_GO)
#undef DFD_GO
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// the weight gradient's M-split: ~512 workgroups, 128-row multiples (pw_wgrad_body's m-steps)
static void rn16_wgrad_split(int64_t M, int N, int K, int64_t slab_floats, int* tnk, int* tiles, int64_t* splits,
                             int64_t* mps) {
  *tnk = cdiv(K, 64);
  *tiles = cdiv(N, 64) * *tnk;
  int64_t sp = std::max<int64_t>(1, 512 / *tiles);
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, cdiv64(M, 128)));
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, slab_floats / ((int64_t)N * K) - 1));  // + the packed sum
  *mps = cdiv64(cdiv64(std::max<int64_t>(M, 1), sp), 128) * 128;
  *splits = cdiv64(std::max<int64_t>(M, 1), *mps);
}

int64_t rn16_conv_wgrad_slab_floats(int N, int H, int W, int Cin, int Cout, int k, int stride, int pad) {
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t M = (int64_t)N * Ho * Wo;
  const int K = k * k * Cin;
  int tnk, tiles;
  int64_t splits, mps;
  rn16_wgrad_split(M, Cout, K, INT64_MAX / 4, &tnk, &tiles, &splits, &mps);
  return (splits + 1) * (int64_t)Cout * K;
}

__global__ void rn16_unpack_grad_kernel(const float* __restrict__ packed, int Co, int Ci, int KK, float* __restrict__ dw) {
  // packed [Co][KK][Ci] -> dw [Co][Ci][KK] (torch's conv weight layout)
  const int64_t n = (int64_t)Co * Ci * KK;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int t = (int)(i % KK);
    const int64_t r = i / KK;
    const int ci = (int)(r % Ci), co = (int)(r / Ci);
    dw[i] = packed[((int64_t)co * KK + t) * Ci + ci];
  }
}

static int ew_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 8192)); }

int rn16_conv_wgrad(hipStream_t s, const bf16* x, int N, int H, int W, int Cin, const bf16* dy, int Cout, int k,
                    int stride, int pad, float* slab, int64_t slab_floats, float* dw) {
  if (!rn16_shape_ok(N, H, W, Cin, Cout, k, k, stride, pad)) {
    set_error("rn16 wgrad: shape outside the bf16 training kernels", __FILE__, __LINE__);
    return -1;
  }
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t M = (int64_t)N * Ho * Wo;
  const int K = k * k * Cin;
  const int64_t nk = (int64_t)Cout * K;
  if (slab_floats < 2 * nk) { set_error("rn16 wgrad: slab too small", __FILE__, __LINE__); return -1; }
  int tnk, tiles;
  int64_t splits, mps;
  rn16_wgrad_split(M, Cout, K, slab_floats, &tnk, &tiles, &splits, &mps);
  const ConvGather cg = make_gather(Cin, H, W, Ho, Wo, k, stride, pad, 0);
  hipLaunchKernelGGL(rn16_conv_wgrad_kernel, dim3((unsigned)tiles, (unsigned)splits), dim3(256), 0, s, dy, x, M, Cout, K,
                     slab, tnk, mps, cg);
  DFD_HIP_CHECK(hipGetLastError());
  if (k == 1) return launch_reduce_slabs(s, slab, (int)splits, nk, dw, false);  // [Co][Ci] either way
  float* packed = slab + splits * nk;
  DFD_TRY(launch_reduce_slabs(s, slab, (int)splits, nk, packed, false));
  hipLaunchKernelGGL(rn16_unpack_grad_kernel, dim3(ew_blocks(nk)), dim3(256), 0, s, packed, Cout, Cin, k * k, dw);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// fp32 w [Co][Ci][KK] -> bf16 wf [Co][KK][Ci] (forward) and wd [Ci][KK][Co] (data gradient)
__global__ void rn16_pack_kernel(const float* __restrict__ w, int Co, int Ci, int KK, bf16* __restrict__ wf,
                                 bf16* __restrict__ wd) {
  const int64_t n = (int64_t)Co * Ci * KK;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int t = (int)(i % KK);
    const int64_t r = i / KK;
    const int ci = (int)(r % Ci), co = (int)(r / Ci);
    const bf16 v = Tr<bf16>::from_f(w[i]);
    wf[((int64_t)co * KK + t) * Ci + ci] = v;
    if (wd) wd[((int64_t)ci * KK + t) * Co + co] = v;
  }
}

// every convolution of the step in ONE launch: table row i = {fp32 weight pointer, Co, Ci, KK, wf offset,
// wd offset (elements of out, -1: none)}; blockIdx.y = row
__global__ void rn16_pack_all_kernel(const int64_t* __restrict__ table, bf16* __restrict__ out) {
  const int64_t* t = table + 6 * blockIdx.y;
  const float* w = reinterpret_cast<const float*>(t[0]);
  const int Co = (int)t[1], Ci = (int)t[2], KK = (int)t[3];
  bf16* wf = out + t[4];
  bf16* wd = t[5] >= 0 ? out + t[5] : nullptr;
  const int64_t n = (int64_t)Co * Ci * KK;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int tp = (int)(i % KK);
    const int64_t r = i / KK;
    const int ci = (int)(r % Ci), co = (int)(r / Ci);
    const bf16 v = Tr<bf16>::from_f(w[i]);
    wf[((int64_t)co * KK + tp) * Ci + ci] = v;
    if (wd) wd[((int64_t)ci * KK + tp) * Co + co] = v;
  }
}

int rn16_pack_all(hipStream_t s, const int64_t* table, int n, int64_t max_elems, bf16* out) {
  if (n <= 0) return 0;
  const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(max_elems, 256), 256));
  hipLaunchKernelGGL(rn16_pack_all_kernel, dim3((unsigned)gx, (unsigned)n), dim3(256), 0, s, table, out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int rn16_pack_weights(hipStream_t s, const float* w, int Co, int Ci, int KK, bf16* wf, bf16* wd) {
  hipLaunchKernelGGL(rn16_pack_kernel, dim3(ew_blocks((int64_t)Co * Ci * KK)), dim3(256), 0, s, w, Co, Ci, KK, wf, wd);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ BatchNorm / ReLU / pool pieces (8 channels per thread)
__global__ __launch_bounds__(256) void rn16_bn_act_kernel(const bf16* __restrict__ y, const float* __restrict__ mu,
                                                          const float* __restrict__ sc, const float* __restrict__ be,
                                                          const bf16* __restrict__ r, int relu, int64_t nvec, int cv,
                                                          bf16* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    float v[8], m8[8], s8[8], b8[8];
    ld8(y + i * 8, v);
    ld8f(mu + c, m8);
    ld8f(sc + c, s8);
    ld8f(be + c, b8);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (v[j] - m8[j]) * s8[j] + b8[j];
    if (r) {
      float q[8];
      ld8(r + i * 8, q);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += q[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    st8(out + i * 8, v);
  }
}

__global__ __launch_bounds__(256) void rn16_relu_bwd_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ out,
                                                            int64_t nvec, bf16* __restrict__ g) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float d[8], a[8];
    ld8(dout + i * 8, d);
    ld8(out + i * 8, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = a[j] > 0.f ? d[j] : 0.f;
    st8(g + i * 8, d);
  }
}

__global__ __launch_bounds__(256) void rn16_bn_bwd_apply_kernel(const bf16* __restrict__ g, const bf16* __restrict__ y,
                                                                const float* __restrict__ mu,
                                                                const float* __restrict__ coef, int64_t nvec, int C,
                                                                bf16* __restrict__ dy) {
  const int cv = C / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    float ga[8], ya[8], m8[8], k1[8], k2[8], k3[8];
    ld8(g + i * 8, ga);
    ld8(y + i * 8, ya);
    ld8f(mu + c, m8);
    ld8f(coef + c, k1);
    ld8f(coef + C + c, k2);
    ld8f(coef + 2 * C + c, k3);
#pragma unroll
    for (int j = 0; j < 8; ++j) ga[j] = k1[j] * ga[j] + k2[j] * (ya[j] - m8[j]) + k3[j];
    st8(dy + i * 8, ga);
  }
}

__global__ __launch_bounds__(256) void rn16_gap_bwd_kernel(const float* __restrict__ dfeat, const bf16* __restrict__ out,
                                                           int HW, int C, int64_t nvec, float inv_hw,
                                                           bf16* __restrict__ g) {
  const int cv = C / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t f = i / cv / HW;
    float a[8], d[8];
    ld8(out + i * 8, a);
    ld8f(dfeat + f * C + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = a[j] > 0.f ? d[j] * inv_hw : 0.f;
    st8(g + i * 8, d);
  }
}

__global__ void rn16_cast_kernel(const void* __restrict__ src, int to_bf16, int64_t nvec, void* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float v[8];
    if (to_bf16) {
      ld8f(reinterpret_cast<const float*>(src) + i * 8, v);
      st8(reinterpret_cast<bf16*>(dst) + i * 8, v);
    } else {
      ld8(reinterpret_cast<const bf16*>(src) + i * 8, v);
      st8(reinterpret_cast<float*>(dst) + i * 8, v);
    }
  }
}

int rn16_bn_act(hipStream_t s, const bf16* y, const float* mean, const float* sc, const float* beta, const bf16* r,
                int relu, int64_t M, int C, bf16* out) {
  if (C % 8) { set_error("rn16_bn_act: C % 8", __FILE__, __LINE__); return -1; }
  const int64_t nvec = M * C / 8;
  hipLaunchKernelGGL(rn16_bn_act_kernel, dim3(ew_blocks(nvec)), dim3(256), 0, s, y, mean, sc, beta, r, relu, nvec, C / 8,
                     out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int rn16_relu_bwd(hipStream_t s, const bf16* dout, const bf16* out, int64_t n, bf16* g) {
  if (n % 8) { set_error("rn16_relu_bwd: n % 8", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL(rn16_relu_bwd_kernel, dim3(ew_blocks(n / 8)), dim3(256), 0, s, dout, out, n / 8, g);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int rn16_gap_bwd(hipStream_t s, const float* dfeat, const bf16* out, int N, int HW, int C, bf16* g) {
  if (C % 8) { set_error("rn16_gap_bwd: C % 8", __FILE__, __LINE__); return -1; }
  const int64_t nvec = (int64_t)N * HW * C / 8;
  hipLaunchKernelGGL(rn16_gap_bwd_kernel, dim3(ew_blocks(nvec)), dim3(256), 0, s, dfeat, out, HW, C, nvec,
                     1.0f / (float)HW, g);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int rn16_cast(hipStream_t s, const void* src, int to_bf16, int64_t n, void* dst) {
  if (n % 8) { set_error("rn16_cast: n % 8", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL(rn16_cast_kernel, dim3(ew_blocks(n / 8)), dim3(256), 0, s, src, to_bf16, n / 8, dst);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// The ReLU between a BN and the next convolution folded into the BN backward: g = (a > 0) * da is never
// materialised.  Partial rows (sum g, sum g * (y - mean) * invstd) per row chunk x 64-channel group
// (8 channel vectors x 32 row lanes, two rows' loads in flight, lanes added in order through LDS:
// deterministic), in launch_bn_bwd_finalize's [rows][2][C] layout.
template <typename T>  // bf16 (this file's training path) or float (the fp32 training path, k_rntrain.hip)
__global__ __launch_bounds__(256) void rn16_bn_bwd_reduce_relu_kernel(const T* __restrict__ da,
                                                                      const T* __restrict__ a,
                                                                      const T* __restrict__ y,
                                                                      const float* __restrict__ mean,
                                                                      const float* __restrict__ invstd, int64_t M, int C,
                                                                      int64_t rows_per_wg, float* __restrict__ stats) {
  __shared__ float sh[2][32][65];
  const int tid = threadIdx.x, v = tid & 7, rl = tid >> 3;
  const int c = blockIdx.y * 64 + v * 8;
  float mu[8], is[8], s8[8], q8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s8[j] = 0.f; q8[j] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg, r1 = min(M, r0 + rows_per_wg);
  if (c < C) {
    ld8f(mean + c, mu);
    ld8f(invstd + c, is);
    auto one = [&](const float (&d)[8], const float (&av)[8], const float (&yv)[8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = av[j] > 0.f ? d[j] : 0.f;
        s8[j] += g;
        q8[j] += g * ((yv[j] - mu[j]) * is[j]);
      }
    };
    int64_t r = r0 + rl;
    for (; r + 32 < r1; r += 64) {
      float d0[8], a0[8], y0[8], d1[8], a1[8], y1[8];
      ld8(da + r * C + c, d0); ld8(a + r * C + c, a0); ld8(y + r * C + c, y0);
      ld8(da + (r + 32) * C + c, d1); ld8(a + (r + 32) * C + c, a1); ld8(y + (r + 32) * C + c, y1);
      one(d0, a0, y0);
      one(d1, a1, y1);
    }
    if (r < r1) {
      float d0[8], a0[8], y0[8];
      ld8(da + r * C + c, d0); ld8(a + r * C + c, a0); ld8(y + r * C + c, y0);
      one(d0, a0, y0);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { sh[0][rl][v * 8 + j] = s8[j]; sh[1][rl][v * 8 + j] = q8[j]; }
  __syncthreads();
  if (tid < 128) {
    const int which = tid >> 6, cl = tid & 63;
    float acc = 0.f;
    for (int l = 0; l < 32; ++l) acc += sh[which][l][cl];
    if (blockIdx.y * 64 + cl < C) stats[((int64_t)blockIdx.x * 2 + which) * C + blockIdx.y * 64 + cl] = acc;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void rn16_bn_bwd_apply_relu_kernel(const T* __restrict__ da,
                                                                     const T* __restrict__ a,
                                                                     const T* __restrict__ y,
                                                                     const float* __restrict__ mu,
                                                                     const float* __restrict__ coef, int64_t nvec, int C,
                                                                     T* __restrict__ dy) {
  const int cv = C / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    float ga[8], av[8], ya[8], m8[8], k1[8], k2[8], k3[8];
    ld8(da + i * 8, ga);
    ld8(a + i * 8, av);
    ld8(y + i * 8, ya);
    ld8f(mu + c, m8);
    ld8f(coef + c, k1);
    ld8f(coef + C + c, k2);
    ld8f(coef + 2 * C + c, k3);
#pragma unroll
    for (int j = 0; j < 8; ++j) ga[j] = k1[j] * (av[j] > 0.f ? ga[j] : 0.f) + k2[j] * (ya[j] - m8[j]) + k3[j];
    st8(dy + i * 8, ga);
  }
}

// the masked form for either storage type: reduce, finalize (centred), apply
template <typename T>
static int bn_train_bwd_relu(hipStream_t s, const T* g, const T* relu_out, const T* y, int64_t M, int C,
                             const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                             float* stats, float* coef, T* dy) {
  if (C % 64) { set_error("bn_train_bwd: C % 64 with the ReLU mask", __FILE__, __LINE__); return -1; }
  const int groups = C / 64;
  const int64_t nx = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(512, cdiv64(M, 64)),
                                                            std::max(1, 1024 / groups)));
  const int64_t rpw = cdiv64(M, nx);
  const int rows = (int)cdiv64(M, rpw);
  hipLaunchKernelGGL(rn16_bn_bwd_reduce_relu_kernel<T>, dim3((unsigned)rows, (unsigned)groups), dim3(256), 0, s, g,
                     relu_out, y, mean, invstd, M, C, rpw, stats);
  DFD_HIP_CHECK(hipGetLastError());
  DFD_TRY(launch_bn_bwd_finalize(s, stats, rows, M, C, gamma, mean, invstd, true, dgamma, dbeta, false, coef, true));
  const int64_t nvec = M * C / 8;
  hipLaunchKernelGGL(rn16_bn_bwd_apply_relu_kernel<T>, dim3(ew_blocks(nvec)), dim3(256), 0, s, g, relu_out, y, mean,
                     coef, nvec, C, dy);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// fp32 training path: g = (relu_out > 0) * da folded into the BN backward (k_rntrain.hip's unmasked form
// otherwise)
int rn_bn_train_bwd_relu(hipStream_t s, const float* da, const float* relu_out, const float* y, int64_t M, int C,
                         const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                         float* stats, float* coef, float* dy) {
  return bn_train_bwd_relu<float>(s, da, relu_out, y, M, C, mean, invstd, gamma, dgamma, dbeta, stats, coef, dy);
}

// the BN backward of a train-mode BatchNorm2d from its output gradient g (identity activation), centred;
// relu_out != null: g = (relu_out > 0) * g, the ReLU that followed this BN's output (its saved output)
int rn16_bn_train_bwd(hipStream_t s, const bf16* g, const bf16* relu_out, const bf16* y, int64_t M, int C,
                      const float* mean, const float* invstd, const float* scale, const float* shift,
                      const float* gamma, float* dgamma, float* dbeta, float* stats, float* coef, bf16* dy) {
  if (C % 8) { set_error("rn16_bn_train_bwd: C % 8", __FILE__, __LINE__); return -1; }
  if (relu_out)
    return bn_train_bwd_relu<bf16>(s, g, relu_out, y, M, C, mean, invstd, gamma, dgamma, dbeta, stats, coef, dy);
  BnBwdIn in{};
  in.dZ = g;
  in.silu = false;
  in.mean = mean;
  in.invstd = invstd;
  in.scale = scale;
  in.shift = shift;
  int rows = 0;
  DFD_TRY(launch_bn_bwd_reduce<bf16>(s, in, y, M, C, stats, &rows));
  DFD_TRY(launch_bn_bwd_finalize(s, stats, rows, M, C, gamma, mean, invstd, true, dgamma, dbeta, false, coef, true));
  const int64_t nvec = M * C / 8;
  hipLaunchKernelGGL(rn16_bn_bwd_apply_kernel, dim3(ew_blocks(nvec)), dim3(256), 0, s, g, y, mean, coef, nvec, C, dy);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
