// ResNet-50 ensemble member, TRAINING step pieces (fp32), for EnsembleTrainer.train_epoch training
// every member of the app's default ensemble (src/ensemble_trainer.py:158-229 over
// EnsembleDetector(['efficientnet_b0', 'resnet50']), src/pretrained_detector.py:146-218; the member
// is torchvision resnet50 minus fc, :37-40).  Train-mode BatchNorm uses the batch statistics and
// updates the running buffers like torch (biased variance normalises, unbiased updates).
//
// The convolutions are the implicit-GEMM kernels of k_conv.hip (exact fp32 MFMA, gathers in the
// LDS staging, no im2col buffer): forward with the BN-stat partials in its epilogue, data gradient
// (stride 1 and 2: the gather visits only the taps whose output position is integral) and weight
// gradient (split over pixels, ordered slab sum).  The BN backward is k_bn.hip's reduce / finalize /
// apply with the identity activation; here live the elementwise pieces around them:
//   bn_act    out = relu?((y - mean) * scale + beta (+ res))  (BN apply, bottleneck add, ReLU)
//   bn_bwd    dy = k1*g + k2*(y - mean) + k3                   (BN backward apply)
// Both in torch's centred form: the folded y * scale + (beta - mean * scale) loses
// eps * |mean| / std of the normalised value where |mean| >> std (VERDICT r3 item 1;
// tools/rn_bn_numerics.py emulates both forms against fp64).
//   relu_bwd  g = out > 0 ? dout : 0                          (through a saved ReLU output)
//   gap_bwd   g = out > 0 ? dfeat[n][c] / HW : 0              (AdaptiveAvgPool2d + the last ReLU)
#include "cnnlstm.h"
#include "kernels.h"

namespace dfd {

__global__ __launch_bounds__(256) void rn_bn_act_kernel(const float* __restrict__ y, const float* __restrict__ mu,
                                                        const float* __restrict__ sc, const float* __restrict__ be,
                                                        const float* __restrict__ r, int relu, int64_t nvec, int cv,
                                                        float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 4;
    const float4 v = reinterpret_cast<const float4*>(y)[i];
    float o[4] = {(v.x - mu[c]) * sc[c] + be[c], (v.y - mu[c + 1]) * sc[c + 1] + be[c + 1],
                  (v.z - mu[c + 2]) * sc[c + 2] + be[c + 2], (v.w - mu[c + 3]) * sc[c + 3] + be[c + 3]};
    if (r) {
      const float4 q = reinterpret_cast<const float4*>(r)[i];
      o[0] += q.x; o[1] += q.y; o[2] += q.z; o[3] += q.w;
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    reinterpret_cast<float4*>(out)[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

__global__ __launch_bounds__(256) void rn_relu_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ out,
                                                          int64_t nvec, float* __restrict__ g) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const float4 d = reinterpret_cast<const float4*>(dout)[i], a = reinterpret_cast<const float4*>(out)[i];
    reinterpret_cast<float4*>(g)[i] =
        make_float4(a.x > 0.f ? d.x : 0.f, a.y > 0.f ? d.y : 0.f, a.z > 0.f ? d.z : 0.f, a.w > 0.f ? d.w : 0.f);
  }
}

__global__ __launch_bounds__(256) void rn_gap_bwd_kernel(const float* __restrict__ dfeat, const float* __restrict__ out,
                                                         int HW, int C, int64_t n, float inv_hw,
                                                         float* __restrict__ g) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int64_t f = i / C / HW;
    g[i] = out[i] > 0.f ? dfeat[f * C + c] * inv_hw : 0.f;
  }
}

// dy = k1*g + k2*(y - mean) + k3 (coef rows k1, k2, k3 of the centred finalize)
__global__ __launch_bounds__(256) void rn_bn_bwd_apply_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                              const float* __restrict__ mu,
                                                              const float* __restrict__ coef, int64_t nvec, int C,
                                                              float* __restrict__ dy) {
  const int cv = C / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 4;
    const float4 a = reinterpret_cast<const float4*>(g)[i], v = reinterpret_cast<const float4*>(y)[i];
    const float ga[4] = {a.x, a.y, a.z, a.w}, ya[4] = {v.x, v.y, v.z, v.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = coef[c + j] * ga[j] + coef[C + c + j] * (ya[j] - mu[c + j]) + coef[2 * C + c + j];
    reinterpret_cast<float4*>(dy)[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

static int rn_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 4096)); }

int rn_bn_act(hipStream_t s, const float* y, const float* mean, const float* sc, const float* beta, const float* r,
              int relu, int64_t M, int C, float* out) {
  if (C % 4) { set_error("rn_bn_act: C % 4", __FILE__, __LINE__); return -1; }
  const int64_t nvec = M * C / 4;
  hipLaunchKernelGGL(rn_bn_act_kernel, dim3(rn_grid(nvec)), dim3(256), 0, s, y, mean, sc, beta, r, relu, nvec, C / 4,
                     out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int rn_relu_bwd(hipStream_t s, const float* dout, const float* out, int64_t n, float* g) {
  if (n % 4) { set_error("rn_relu_bwd: n % 4", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL(rn_relu_bwd_kernel, dim3(rn_grid(n / 4)), dim3(256), 0, s, dout, out, n / 4, g);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int rn_gap_bwd(hipStream_t s, const float* dfeat, const float* out, int N, int HW, int C, float* g) {
  const int64_t n = (int64_t)N * HW * C;
  hipLaunchKernelGGL(rn_gap_bwd_kernel, dim3(rn_grid(n)), dim3(256), 0, s, dfeat, out, HW, C, n, 1.0f / (float)HW, g);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// the BN backward of a train-mode BatchNorm2d whose output gradient is g (identity activation):
// dgamma, dbeta (written) and dy = k1*g + k2*(y - mean) + k3
int rn_bn_train_bwd(hipStream_t s, const float* g, const float* y, int64_t M, int C, const float* mean,
                    const float* invstd, const float* scale, const float* shift, const float* gamma, float* dgamma,
                    float* dbeta, float* stats, float* coef, float* dy) {
  BnBwdIn in{};
  in.dZ = g;
  in.silu = false;
  in.mean = mean;
  in.invstd = invstd;
  in.scale = scale;
  in.shift = shift;
  int rows = 0;
  DFD_TRY(launch_bn_bwd_reduce<float>(s, in, y, M, C, stats, &rows));
  DFD_TRY(launch_bn_bwd_finalize(s, stats, rows, M, C, gamma, mean, invstd, true, dgamma, dbeta, false, coef, true));
  if (C % 4) { set_error("rn_bn_train_bwd: C % 4", __FILE__, __LINE__); return -1; }
  const int64_t nvec = M * C / 4;
  hipLaunchKernelGGL(rn_bn_bwd_apply_kernel, dim3(rn_grid(nvec)), dim3(256), 0, s, g, y, mean, coef, nvec, C, dy);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
