// CNNLSTMHybrid (src/models.py:20-85) forward/backward orchestration on HIP, fp32.
//
//   x (B,T,3,H,W) -> frames (B*T, 3, H, W) [strided, channels-last allowed]
//   -> conv7x7/2 (3->64) +BN+ReLU -> maxpool3/2 -> conv5x5 (64->128) +BN+ReLU -> maxpool
//   -> conv3x3 (128->256) +BN+ReLU -> maxpool -> conv3x3 (256->512) +BN+ReLU -> GAP  (B*T, 512)
//   -> nn.LSTM(512, hidden, layers, dropout between layers, batch_first) -> (B, T, hidden)
//   -> attention softmax_t(Linear->tanh->Linear) -> context -> Linear->ReLU->Dropout->Linear (logits)
// BatchNorm uses batch statistics in training (running stats updated, momentum 0.1, eps 1e-5) and
// running statistics in eval; its backward reuses the EfficientNet BN kernels (k_bn.hip).
#include "../../include/dfd_hip.h"
#include "cnnlstm.h"
#include "kernels.h"
#include "rnn.h"

namespace dfd {

// ------------------------------------------------------------------ small kernels
__device__ __forceinline__ float cl_keep(uint64_t seed, uint32_t st, int64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  uint64_t z = seed ^ ((uint64_t)st << 56) ^ (uint64_t)idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}
__global__ void cl_dropout_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, float p, uint64_t seed,
                                  uint32_t st) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = x[i] * cl_keep(seed, st, i, p);
}
// h = relu(h) in place, hd = dropout(h)
__global__ void cl_relu_drop_kernel(float* __restrict__ h, float* __restrict__ hd, int64_t n, float p, uint64_t seed,
                                    uint32_t st) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = fmaxf(h[i], 0.f);
    h[i] = v;
    hd[i] = v * cl_keep(seed, st, i, p);
  }
}
__global__ void cl_relu_drop_bwd_kernel(const float* __restrict__ dhd, const float* __restrict__ h,
                                        float* __restrict__ dh, int64_t n, float p, uint64_t seed, uint32_t st) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dh[i] = h[i] > 0.f ? dhd[i] * cl_keep(seed, st, i, p) : 0.f;
}
// conv bias gradient = sum_m dY = k1 * sum g + k2 * sum y + k3 * M  (BN-backward identities)
__global__ void cl_bias_grad_kernel(const float* __restrict__ coef, const float* __restrict__ sum_g,
                                    const float* __restrict__ mean_y, int64_t M, int C, float* __restrict__ gb) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const double m = (double)M;
  gb[c] = (float)((double)coef[c] * sum_g[c] + (double)coef[C + c] * mean_y[c] * m + (double)coef[2 * C + c] * m);
}

int dropout_apply(hipStream_t s, const float* x, float* y, int64_t n, float p, uint64_t seed, uint32_t stream) {
  hipLaunchKernelGGL(cl_dropout_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 2048))),
                     dim3(256), 0, s, x, y, n, p, seed, stream);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
static dim3 ew1(int64_t n) { return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 2048))); }

// ------------------------------------------------------------------ geometry / workspace
struct ClDims {
  int B, T, H, W, Hid, L, NC;
};
static int conv_out(int h, int k, int s, int p) { return (h + 2 * p - k) / s + 1; }
constexpr int kConvCo[4] = {64, 128, 256, 512};
constexpr int kConvK[4] = {7, 5, 3, 3};
constexpr int kConvS[4] = {2, 1, 1, 1};
constexpr int kClsHidden = 128;

struct ClLayout {
  ConvGeom g[4];
  int Hp[3], Wp[3];  // pooled maps after conv 0..2
  int64_t N;
  // work (floats unless noted): Y[4], P[3], arg[3] (bytes, rounded to floats), BN mean/invstd/scale/shift [4][512 each],
  // F [N][512], per-layer LSTM input/outputs and work, E, att, ctx, h1, hd, wf (packed weights)
  int64_t oY[4], oP[3], oArg[3], oBN[4], oF, oH[8], oHd[8], oLw[8], oE, oAtt, oCtx, oH1, oHd1, oWf, oStats, total;
  // scratch
  int64_t sG, sD, sdP, sWd, sSlab, sLstm, sdH[2], sdF, sAttn, sCls, sStat, sCoef, stotal;
  int64_t stats_cap, slab_cap;
};

static ClLayout cl_layout(const ClDims& d) {
  ClLayout L{};
  L.N = (int64_t)d.B * d.T;
  int h = d.H, w = d.W, ci = 3;
  for (int i = 0; i < 4; ++i) {
    const int k = kConvK[i], s = kConvS[i], p = k / 2;
    const int ho = conv_out(h, k, s, p), wo = conv_out(w, k, s, p);
    L.g[i] = ConvGeom{(int)L.N, h, w, ci, kConvCo[i], k, k, s, p, ho, wo};
    if (i < 3) {
      L.Hp[i] = conv_out(ho, 3, 2, 1);
      L.Wp[i] = conv_out(wo, 3, 2, 1);
      h = L.Hp[i];
      w = L.Wp[i];
    }
    ci = kConvCo[i];
  }
  int64_t cur = 0;
  auto take = [&](int64_t n) { const int64_t o = cur; cur += (n + 63) & ~int64_t(63); return o; };
  const int64_t BT = L.N;
  for (int i = 0; i < 4; ++i) L.oY[i] = take(L.N * L.g[i].Ho * L.g[i].Wo * L.g[i].Co);
  for (int i = 0; i < 3; ++i) {
    L.oP[i] = take(L.N * L.Hp[i] * L.Wp[i] * L.g[i].Co);
    L.oArg[i] = take((L.N * L.Hp[i] * L.Wp[i] * L.g[i].Co + 3) / 4);
  }
  for (int i = 0; i < 4; ++i) L.oBN[i] = take(4 * 512);
  L.oF = take(BT * 512);
  for (int l = 0; l < d.L; ++l) {
    const int in = l == 0 ? 512 : d.Hid;
    L.oH[l] = take(BT * d.Hid);
    L.oHd[l] = take(BT * d.Hid);
    L.oLw[l] = take(lstm_layer_work_floats(d.B, d.T, in, d.Hid));
  }
  L.oE = take(BT * d.Hid);
  L.oAtt = take(BT);
  L.oCtx = take((int64_t)d.B * d.Hid);
  L.oH1 = take((int64_t)d.B * kClsHidden);
  L.oHd1 = take((int64_t)d.B * kClsHidden);
  int64_t wmax = 0;
  for (int i = 0; i < 4; ++i) wmax = std::max<int64_t>(wmax, (int64_t)L.g[i].Co * L.g[i].Ci * L.g[i].KH * L.g[i].KW);
  L.oWf = take(wmax);
  int64_t st = 0;
  for (int i = 0; i < 4; ++i) st = std::max<int64_t>(st, cdiv64(L.N * L.g[i].Ho * L.g[i].Wo, 64) * 2 * L.g[i].Co);
  L.stats_cap = st;
  L.oStats = take(st);
  L.total = cur;
  // scratch
  cur = 0;
  int64_t ymax = 0, pmax = 0;
  for (int i = 0; i < 4; ++i) ymax = std::max<int64_t>(ymax, L.N * L.g[i].Ho * L.g[i].Wo * L.g[i].Co);
  for (int i = 0; i < 3; ++i) pmax = std::max<int64_t>(pmax, L.N * L.Hp[i] * L.Wp[i] * L.g[i].Co);
  L.sG = take(ymax);
  L.sD = take(ymax);
  L.sdP = take(pmax);
  L.sWd = take(wmax);
  L.slab_cap = std::max<int64_t>(wmax * 8, (int64_t)4 << 20);
  L.sSlab = take(L.slab_cap);
  int64_t lmax = 0;
  for (int l = 0; l < d.L; ++l) lmax = std::max(lmax, lstm_layer_scratch_floats(d.B, d.T, l == 0 ? 512 : d.Hid, d.Hid));
  L.sLstm = take(lmax);
  L.sdH[0] = take(BT * std::max(512, d.Hid));
  L.sdH[1] = take(BT * std::max(512, d.Hid));
  L.sdF = take(BT * 512);
  L.sAttn = take(2 * BT * d.Hid + BT);
  L.sCls = take((int64_t)d.B * (d.NC + 2 * kClsHidden + d.Hid));
  L.sStat = take((int64_t)1024 * 2 * 512);
  L.sCoef = take(3 * 512 + 2 * 512);
  L.stotal = cur;
  return L;
}

// parameter table (named_parameters order): cnn.{0,1,4,5,8,9,12,13}.{weight,bias} (16),
// lstm.{weight_ih,weight_hh,bias_ih,bias_hh}_l{k} (4 per layer), attention.{0,2}.{weight,bias},
// classifier.{0,3}.{weight,bias}.  BN buffers: cnn.{1,5,9,13}.{running_mean,running_var} (8).
struct ClParams {
  float *conv_w[4], *conv_b[4], *bn_g[4], *bn_b[4];
  LstmLayerW lstm[8];
  float *aw1, *ab1, *aw2, *ab2, *cw1, *cb1, *cw2, *cb2;
};
static ClParams cl_params(float* const* t, int L) {
  ClParams P{};
  for (int i = 0; i < 4; ++i) {
    P.conv_w[i] = t[4 * i];
    P.conv_b[i] = t[4 * i + 1];
    P.bn_g[i] = t[4 * i + 2];
    P.bn_b[i] = t[4 * i + 3];
  }
  for (int l = 0; l < L; ++l) P.lstm[l] = LstmLayerW{t[16 + 4 * l], t[17 + 4 * l], t[18 + 4 * l], t[19 + 4 * l]};
  float* const* q = t + 16 + 4 * L;
  P.aw1 = q[0]; P.ab1 = q[1]; P.aw2 = q[2]; P.ab2 = q[3];
  P.cw1 = q[4]; P.cb1 = q[5]; P.cw2 = q[6]; P.cb2 = q[7];
  return P;
}

static int bad_dims(const ClDims& d) {
  if (d.B <= 0 || d.T <= 0 || d.H < 16 || d.W < 16 || d.Hid <= 0 || d.Hid % 8 || d.L < 1 || d.L > 8 || d.NC <= 0) {
    set_error("cnnlstm: bad dimensions", __FILE__, __LINE__);
    return -1;
  }
  return 0;
}

// ------------------------------------------------------------------ forward
static int cl_forward(hipStream_t s, const ClDims& d, const ClParams& P, float* const* bn_run, const float* x,
                      const int64_t* xs4, float* work, int training, float momentum, uint64_t seed, float p,
                      float* logits) {
  const ClLayout L = cl_layout(d);
  float* W = work;
  const int64_t BT = L.N;
  // frame CNN
  const float* src = x;
  int64_t ss[4] = {xs4[0], xs4[2], xs4[3], xs4[1]};  // (n, c, h, w) strides -> (n, y, x, c)
  for (int i = 0; i < 4; ++i) {
    const ConvGeom& g = L.g[i];
    float* Y = W + L.oY[i];
    int rows = 0;
    DFD_TRY(conv_forward(s, g, src, ss, P.conv_w[i], P.conv_b[i], W + L.oWf, Y, W + L.oStats, &rows));
    float* bn = W + L.oBN[i];  // mean, invstd, scale, shift
    DFD_TRY(launch_bn_finalize(s, W + L.oStats, rows, BT * g.Ho * g.Wo, g.Co, P.bn_g[i], P.bn_b[i], bn_run[2 * i],
                               bn_run[2 * i + 1], momentum, 1e-5f, training != 0, bn, bn + 512, bn + 1024, bn + 1536,
                               kConvStatRows));
    if (i < 3) {
      float* Pout = W + L.oP[i];
      DFD_TRY(bn_relu_pool_fwd(s, Y, nullptr, bn + 1024, bn + 1536, (int)BT, g.Ho, g.Wo, g.Co, L.Hp[i], L.Wp[i], Pout,
                               reinterpret_cast<uint8_t*>(W + L.oArg[i])));
      src = Pout;
      const int64_t C = g.Co;
      ss[0] = (int64_t)L.Hp[i] * L.Wp[i] * C; ss[1] = (int64_t)L.Wp[i] * C; ss[2] = C; ss[3] = 1;
    } else {
      DFD_TRY(bn_relu_gap_fwd(s, Y, bn + 1024, bn + 1536, (int)BT, g.Ho * g.Wo, g.Co, W + L.oF));
    }
  }
  // LSTM stack
  const float* in = W + L.oF;
  for (int l = 0; l < d.L; ++l) {
    const int IN = l == 0 ? 512 : d.Hid;
    DFD_TRY(lstm_layer_forward(s, d.B, d.T, IN, d.Hid, P.lstm[l], in, W + L.oLw[l], W + L.oH[l]));
    if (l < d.L - 1) {
      DFD_TRY(dropout_apply(s, W + L.oH[l], W + L.oHd[l], BT * d.Hid, p, seed, 20u + l));
      in = W + L.oHd[l];
    }
  }
  const float* O = W + L.oH[d.L - 1];
  DFD_TRY(attn_forward(s, O, d.B, d.T, d.Hid, P.aw1, P.ab1, P.aw2, P.ab2, W + L.oE, W + L.oAtt, W + L.oCtx));
  DFD_TRY(launch_sgemm(s, false, false, W + L.oCtx, d.Hid, P.cw1, d.Hid, W + L.oH1, kClsHidden, d.B, kClsHidden, d.Hid,
                       0.f, P.cb1));
  hipLaunchKernelGGL(cl_relu_drop_kernel, ew1((int64_t)d.B * kClsHidden), dim3(256), 0, s, W + L.oH1, W + L.oHd1,
                     (int64_t)d.B * kClsHidden, p, seed, 30u);
  DFD_HIP_CHECK(hipGetLastError());
  DFD_TRY(launch_sgemm(s, false, false, W + L.oHd1, kClsHidden, P.cw2, kClsHidden, logits, d.NC, d.B, d.NC,
                       kClsHidden, 0.f, P.cb2));
  return 0;
}

// ------------------------------------------------------------------ backward
static int cl_backward(hipStream_t s, const ClDims& d, const ClParams& P, const ClParams& G, const float* x,
                       const int64_t* xs4, float* work, float* scratch, int training, uint64_t seed, float p,
                       const float* dlogits) {
  const ClLayout L = cl_layout(d);
  float* W = work;
  float* S = scratch;
  const int64_t BT = L.N;
  // classifier
  float* dhd = S + L.sCls;
  float* dh = dhd + (int64_t)d.B * kClsHidden;
  float* dctx = dh + (int64_t)d.B * kClsHidden;
  DFD_TRY(launch_sgemm(s, true, true, dlogits, d.NC, W + L.oHd1, kClsHidden, G.cw2, kClsHidden, d.NC, kClsHidden, d.B,
                       0.f, nullptr));
  DFD_TRY(colsum(s, dlogits, d.B, d.NC, d.NC, G.cb2));
  DFD_TRY(launch_sgemm(s, false, true, dlogits, d.NC, P.cw2, kClsHidden, dhd, kClsHidden, d.B, kClsHidden, d.NC, 0.f,
                       nullptr));
  hipLaunchKernelGGL(cl_relu_drop_bwd_kernel, ew1((int64_t)d.B * kClsHidden), dim3(256), 0, s, dhd, W + L.oH1, dh,
                     (int64_t)d.B * kClsHidden, p, seed, 30u);
  DFD_TRY(launch_sgemm(s, true, true, dh, kClsHidden, W + L.oCtx, d.Hid, G.cw1, d.Hid, kClsHidden, d.Hid, d.B, 0.f,
                       nullptr));
  DFD_TRY(colsum(s, dh, d.B, kClsHidden, kClsHidden, G.cb1));
  DFD_TRY(launch_sgemm(s, false, true, dh, kClsHidden, P.cw1, d.Hid, dctx, d.Hid, d.B, d.Hid, kClsHidden, 0.f,
                       nullptr));
  // attention -> gradient of the last LSTM layer's outputs
  float* dO = S + L.sdH[0];
  DFD_TRY(attn_backward(s, W + L.oH[d.L - 1], W + L.oE, W + L.oAtt, dctx, P.aw1, P.aw2, d.B, d.T, d.Hid, S + L.sAttn,
                        dO, G.aw1, G.ab1, G.aw2, G.ab2));
  // LSTM layers, top down
  float* dcur = dO;
  for (int l = d.L - 1; l >= 0; --l) {
    const int IN = l == 0 ? 512 : d.Hid;
    const float* Xin = l == 0 ? W + L.oF : W + L.oHd[l - 1];
    float* dX = l == 0 ? S + L.sdF : S + L.sdH[(d.L - l) & 1];
    LstmLayerG gl{G.lstm[l].w_ih ? const_cast<float*>(G.lstm[l].w_ih) : nullptr, const_cast<float*>(G.lstm[l].w_hh),
                  const_cast<float*>(G.lstm[l].b_ih), const_cast<float*>(G.lstm[l].b_hh)};
    DFD_TRY(lstm_layer_backward(s, d.B, d.T, IN, d.Hid, P.lstm[l], Xin, W + L.oLw[l], dcur, S + L.sLstm, gl, dX));
    if (l > 0) {  // through the inter-layer dropout of layer l-1's output
      DFD_TRY(dropout_apply(s, dX, dX, BT * d.Hid, p, seed, 20u + (l - 1)));
      dcur = dX;
    }
  }
  // frame CNN, top down
  float* g = S + L.sG;   // gradient w.r.t. the BN output (post-ReLU mask applied)
  float* dY = S + L.sD;  // gradient w.r.t. the conv output (pre-BN)
  float* dP = S + L.sdP;
  for (int i = 3; i >= 0; --i) {
    const ConvGeom& cg = L.g[i];
    const int64_t M = BT * cg.Ho * cg.Wo;
    float* Y = W + L.oY[i];
    float* bn = W + L.oBN[i];
    if (i == 3) DFD_TRY(bn_relu_gap_bwd(s, S + L.sdF, Y, bn + 1024, bn + 1536, (int)BT, cg.Ho * cg.Wo, cg.Co, g));
    else
      DFD_TRY(bn_relu_pool_bwd(s, dP, reinterpret_cast<const uint8_t*>(W + L.oArg[i]), Y, nullptr, bn + 1024, bn + 1536, (int)BT,
                               cg.Ho, cg.Wo, cg.Co, L.Hp[i], L.Wp[i], g));
    BnBwdIn in{};
    in.dZ = g;
    in.silu = false;
    in.mean = bn;
    in.invstd = bn + 512;
    in.scale = bn + 1024;
    in.shift = bn + 1536;
    int rows = 0;
    DFD_TRY(launch_bn_bwd_reduce<float>(s, in, Y, M, cg.Co, S + L.sStat, &rows));
    float* coef = S + L.sCoef;
    DFD_TRY(launch_bn_bwd_finalize(s, S + L.sStat, rows, M, cg.Co, P.bn_g[i], bn, bn + 512, training != 0, G.bn_g[i],
                                   G.bn_b[i], false, coef));
    DFD_TRY(launch_bn_bwd_apply<float>(s, in, Y, coef, dY, M, cg.Co));
    hipLaunchKernelGGL(cl_bias_grad_kernel, dim3((unsigned)cdiv(cg.Co, 256)), dim3(256), 0, s, coef, G.bn_b[i], bn, M,
                       cg.Co, G.conv_b[i]);
    DFD_HIP_CHECK(hipGetLastError());
    // conv input of layer i
    const float* src;
    int64_t ss[4];
    if (i == 0) {
      src = x;
      ss[0] = xs4[0]; ss[1] = xs4[2]; ss[2] = xs4[3]; ss[3] = xs4[1];
    } else {
      src = W + L.oP[i - 1];
      const int64_t C = cg.Ci;
      ss[0] = (int64_t)cg.H * cg.W * C; ss[1] = (int64_t)cg.W * C; ss[2] = C; ss[3] = 1;
    }
    DFD_TRY(conv_wgrad(s, cg, src, ss, dY, S + L.sSlab, L.slab_cap, G.conv_w[i]));
    if (i > 0) DFD_TRY(conv_dgrad(s, cg, dY, P.conv_w[i], W + L.oWf, S + L.sWd, dP));
  }
  return 0;
}

}  // namespace dfd

// ------------------------------------------------------------------ C ABI
using dfd::ClDims;

static int cl_check(const ClDims& d) { return dfd::bad_dims(d); }

int64_t dfd_cnnlstm_work_floats(int B, int T, int H, int W, int hidden, int layers, int num_classes) {
  const ClDims d{B, T, H, W, hidden, layers, num_classes};
  if (cl_check(d)) return -1;
  return dfd::cl_layout(d).total;
}
int64_t dfd_cnnlstm_scratch_floats(int B, int T, int H, int W, int hidden, int layers, int num_classes) {
  const ClDims d{B, T, H, W, hidden, layers, num_classes};
  if (cl_check(d)) return -1;
  return dfd::cl_layout(d).stotal;
}
int dfd_cnnlstm_forward(void* stream, int B, int T, int H, int W, int hidden, int layers, int num_classes,
                        const float* x, const int64_t* x_strides4, float* const* params, float* const* bn_running,
                        float* work, int training, float momentum, uint64_t seed, float p, float* logits) {
  try {
    const ClDims d{B, T, H, W, hidden, layers, num_classes};
    if (cl_check(d)) return -1;
    if (!x || !x_strides4 || !params || !bn_running || !work || !logits) {
      dfd::set_error("null argument", __FILE__, __LINE__);
      return -1;
    }
    const dfd::ClParams P = dfd::cl_params(params, layers);
    return dfd::cl_forward((hipStream_t)stream, d, P, bn_running, x, x_strides4, work, training, momentum, seed, p,
                           logits);
  } catch (const std::exception& e) {
    dfd::set_error(e.what(), __FILE__, __LINE__);
    return -1;
  }
}
int dfd_cnnlstm_backward(void* stream, int B, int T, int H, int W, int hidden, int layers, int num_classes,
                         const float* x, const int64_t* x_strides4, float* const* params, float* work, float* scratch,
                         int training, uint64_t seed, float p, const float* dlogits, float* const* grads) {
  try {
    const ClDims d{B, T, H, W, hidden, layers, num_classes};
    if (cl_check(d)) return -1;
    if (!x || !x_strides4 || !params || !work || !scratch || !dlogits || !grads) {
      dfd::set_error("null argument", __FILE__, __LINE__);
      return -1;
    }
    const dfd::ClParams P = dfd::cl_params(params, layers);
    const dfd::ClParams G = dfd::cl_params(grads, layers);
    return dfd::cl_backward((hipStream_t)stream, d, P, G, x, x_strides4, work, scratch, training, seed, p, dlogits);
  } catch (const std::exception& e) {
    dfd::set_error(e.what(), __FILE__, __LINE__);
    return -1;
  }
}
