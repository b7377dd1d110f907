// CNNLSTMHybrid (src/models.py:20-85) launchers: dense conv passes (k_conv.hip), nn.LSTM
// (k_lstm.hip) and the model orchestration (cnnlstm.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfd {

struct ConvGeom {
  int N, H, W, Ci, Co, KH, KW, S, P, Ho, Wo;
  bool fold = false;  // two-level K summation (k_conv.hip): the ResNet-50 training convolutions
};

int conv_forward(hipStream_t s, const ConvGeom& g, const float* x, const int64_t (&xs)[4], const float* w,
                 const float* bias, float* wf, float* Y, float* stats, int* stat_rows);
// res (optional): dX = data gradient + res (the bottleneck's other path, same layout as dX)
int conv_dgrad(hipStream_t s, const ConvGeom& g, const float* dY, const float* w, float* wf, float* wd, float* dX,
               const float* res = nullptr);
int64_t conv_wgrad_slab_floats(const ConvGeom& g);  // the slab conv_wgrad uses in full
int conv_wgrad(hipStream_t s, const ConvGeom& g, const float* x, const int64_t (&xs)[4], const float* dY, float* slab,
               int64_t slab_cap, float* gw);
// z = mu ? (Y - mu) * sc + sh : Y * sc + sh  (the centred form with sh = beta when mu is given)
int bn_relu_pool_fwd(hipStream_t s, const float* Y, const float* mu, const float* sc, const float* sh, int N, int H,
                     int W, int C, int Ho, int Wo, float* P, uint8_t* arg);
int bn_relu_pool_bwd(hipStream_t s, const float* dP, const uint8_t* arg, const float* Y, const float* mu,
                     const float* sc, const float* sh, int N, int H, int W, int C, int Ho, int Wo, float* g);
int bn_relu_gap_fwd(hipStream_t s, const float* Y, const float* sc, const float* sh, int N, int HW, int C,
                    float* feat);
int bn_relu_gap_bwd(hipStream_t s, const float* dfeat, const float* Y, const float* sc, const float* sh, int N,
                    int HW, int C, float* g);

// nn.LSTM (batch_first, gate order i, f, g, o), one layer over all T steps
struct LstmLayerW {
  const float *w_ih, *w_hh, *b_ih, *b_hh;  // [4H][IN], [4H][H], [4H], [4H]
};
struct LstmLayerG {
  float *w_ih, *w_hh, *b_ih, *b_hh;
};
int64_t lstm_layer_work_floats(int B, int T, int IN, int H);
// X [B][T][IN] -> Hout [B][T][H]; work keeps the activations for backward
int lstm_layer_forward(hipStream_t s, int B, int T, int IN, int H, const LstmLayerW& w, const float* X, float* work,
                       float* Hout);
// dH [B][T][H] (gradient of Hout) -> grads (overwritten) and dX [B][T][IN] (if not null)
int lstm_layer_backward(hipStream_t s, int B, int T, int IN, int H, const LstmLayerW& w, const float* X, float* work,
                        const float* dH, float* scratch, LstmLayerG& g, float* dX);
int64_t lstm_layer_scratch_floats(int B, int T, int IN, int H);

// dropout with the library's counter hash (y = x * keep / (1 - p)), and its backward
int dropout_apply(hipStream_t s, const float* x, float* y, int64_t n, float p, uint64_t seed, uint32_t stream);

}  // namespace dfd
