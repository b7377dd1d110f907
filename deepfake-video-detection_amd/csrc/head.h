// Host-side interfaces of the detector head, loss and optimizer kernels (k_head.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfd {

struct HeadDims {
  int B, T, D, H, F1, NC;  // clips, frames/clip, feature dim 1280, attn hidden 64, fc1 256, classes
  int use_attn;
};
struct HeadParams {  // device pointers (fp32)
  const float *ta_w1, *ta_b1, *ta_w2, *ta_b2, *fc1_w, *fc1_b, *fc2_w, *fc2_b;
};
struct HeadWork {  // device scratch (fp32)
  float* hid;   // [B*T][H]   relu(W1 f + b1)
  float* e;     // [B*T]      sigmoid scores
  float* g;     // [B][D]     attention-pooled feature
  float* h1;    // [B][F1]    relu(fc1)
  float* dh1;   // [B][F1]
  float* dg;    // [B][D]
  float* dpe;   // [B*T]
  float* dhid;  // [B*T][H]
};
struct AdamHyper {
  float omb1, beta2, omb2, eps, weight_decay;
  float decay;      // 1 - lr*weight_decay (AdamW)
  float step_size;  // lr / (1 - beta1^step)
  float bc2_sqrt;   // sqrt(1 - beta2^step)
  float grad_scale; // multiplies the gradient first (e.g. 1/world_size)
  int decoupled;    // 1 = AdamW, 0 = Adam (L2 folded into the gradient)
  // dynamic loss scaling (fp16 training): null, or the scaler state [scale, growth tracker, found_inf,
  // applied steps].  With it the gradient is unscaled by 1/scale, a step whose gradient norm was
  // non-finite is skipped, and the bias corrections use the applied-step count (lr, beta1, beta2).
  const float* scaler;
  double lr, beta1d, beta2d;
};

int head_forward(hipStream_t s, const HeadDims& d, const HeadParams& P, const float* F, HeadWork& w, uint64_t seed,
                 float p, float* logits, float* scores);
int head_backward(hipStream_t s, const HeadDims& d, const HeadParams& P, const float* F, HeadWork& w, uint64_t seed,
                  float p, const float* scores, const float* dlogits, const float* dscores, float* dF,
                  HeadParams& G);
int ce_forward(hipStream_t s, const float* z, const int64_t* y, const float* w, int B, int NC, int64_t ignore,
               float* loss, float* wsum);
int ce_backward(hipStream_t s, const float* z, const int64_t* y, const float* w, int B, int NC, int64_t ignore,
                const float* wsum, const float* gout, float* dz);
int grad_norm(hipStream_t s, const float* g, int64_t n, float max_norm, double* part, int nparts, float* out,
              float* scaler = nullptr);
int loss_scale_update(hipStream_t s, float* scaler, float growth, float backoff, int interval);
int adam_step(hipStream_t s, float* p, float* g, float* m, float* v, int64_t n, const AdamHyper& h, const float* coef);

}  // namespace dfd
