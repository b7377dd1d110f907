// ResNet-50 ensemble member, bf16 training pieces (k_rn16.hip); C entry points dfd_rn16_* (capi.cpp).
// Shapes: every bottleneck convolution (1x1 / 3x3, stride 1 / 2, pad (k - 1) / 2, Cin % 64, Cout % 64);
// activations NHWC bf16, weights packed bf16 per step from the fp32 masters, BN statistics fp32 / fp64.
#pragma once
#include "kernels.h"

namespace dfd {

// fp32 w [Co][Ci][k*k] -> bf16 wf [Co][k*k][Ci] (forward) and, if wd, wd [Ci][k*k][Co] (data gradient)
int rn16_pack_weights(hipStream_t s, const float* w, int Co, int Ci, int KK, bf16* wf, bf16* wd);
// the same for n convolutions in one launch: table (device) rows {w, Co, Ci, KK, wf offset, wd offset or -1}
// into out (bf16 elements); max_elems the largest Co*Ci*KK
int rn16_pack_all(hipStream_t s, const int64_t* table, int n, int64_t max_elems, bf16* out);
// y = conv(x) (no bias), per-workgroup BN partial rows (sum, sum of squares) of y into stats (<= 2048 x Cout
// floats; *stat_rows rows written), for launch_bn_finalize
int rn16_conv_fwd(hipStream_t s, const bf16* x, int N, int H, int W, int Cin, const bf16* wf, int Cout, int k, int stride,
                  int pad, bf16* y, float* stats, int* stat_rows);
// dx = conv^T(dy) (+ res): dx, res [N][H][W][Cin]
int rn16_conv_dgrad(hipStream_t s, const bf16* dy, int N, int H, int W, int Cin, const bf16* wd, int Cout, int k,
                    int stride, int pad, const bf16* res, bf16* dx);
int64_t rn16_conv_wgrad_slab_floats(int N, int H, int W, int Cin, int Cout, int k, int stride, int pad);
// dw [Cout][Cin][k][k] fp32 (written) from x and dy
int rn16_conv_wgrad(hipStream_t s, const bf16* x, int N, int H, int W, int Cin, const bf16* dy, int Cout, int k,
                    int stride, int pad, float* slab, int64_t slab_floats, float* dw);
int rn16_bn_act(hipStream_t s, const bf16* y, const float* mean, const float* sc, const float* beta, const bf16* r,
                int relu, int64_t M, int C, bf16* out);
int rn16_relu_bwd(hipStream_t s, const bf16* dout, const bf16* out, int64_t n, bf16* g);
int rn16_gap_bwd(hipStream_t s, const float* dfeat, const bf16* out, int N, int HW, int C, bf16* g);
int rn16_cast(hipStream_t s, const void* src, int to_bf16, int64_t n, void* dst);
// relu_out (or null): the saved output of the ReLU that followed this BN -- g is masked by it inline
int rn_bn_train_bwd_relu(hipStream_t s, const float* da, const float* relu_out, const float* y, int64_t M, int C,
                         const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                         float* stats, float* coef, float* dy);
int rn16_bn_train_bwd(hipStream_t s, const bf16* g, const bf16* relu_out, const bf16* y, int64_t M, int C,
                      const float* mean, const float* invstd, const float* scale, const float* shift,
                      const float* gamma, float* dgamma, float* dbeta, float* stats, float* coef, bf16* dy);

}  // namespace dfd
