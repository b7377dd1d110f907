// LogicRNNLSTM launchers (k_rnn.hip); see the header comment there for the algorithm.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfd {

// one LogicCell's parameters (src/RNNModel.py:9-19): the six gates on u = [x, h] in the order
// and, or, forget, input, cell, output (each weight [H][in+H], bias [H]) and the not-gate on h.
struct RnnLayerW {
  float* wu[6];
  float* bu[6];
  float* wn;
  float* bn;
};
struct RnnParams {
  RnnLayerW layer[8];
  float *att_w1, *att_b1, *att_w2, *att_b2;  // attention.0 (H->H), attention.2 (H->1)
  float *cls_w1, *cls_b1, *cls_w2, *cls_b2;  // classifier.0 (H->H), classifier.3 (H->1)
};
struct RnnDims {
  int B, T, IN, H, L;
};

int launch_sgemm(hipStream_t s, bool ta, bool tb, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
                 int M, int N, int K, float beta, const float* bias);
// K-sliced form for products with few output tiles: sgemm_splits picks the slice count and
// length (kc); launch_sgemm_part writes part[z][M][N], the consumer sums z = 0.. in order
int sgemm_splits(int M, int N, int K, int* kc);
// K slices of the large weight-gradient products (split-K partials for the big-tile kernel)
int sgemm_wsplits(int M, int N, int K, int* kc);
int launch_sgemm_part(hipStream_t s, bool ta, bool tb, const float* A, int lda, const float* B, int ldb, float* part,
                      int M, int N, int K, int splits, int kc);
int64_t rnn_work_floats(const RnnDims& d);
int64_t rnn_scratch_floats(const RnnDims& d);
int rnn_forward(hipStream_t s, const RnnDims& d, const RnnParams& P, const float* x, const int64_t* order,
                const int64_t* lens, float* work, float* y, uint64_t seed, float p);
int rnn_backward(hipStream_t s, const RnnDims& d, const RnnParams& P, const float* x, const int64_t* order,
                 const int64_t* lens, float* work, float* scratch, const float* dy, RnnParams& Gr, uint64_t seed,
                 float p);
int attn_forward(hipStream_t s, const float* O, int B, int T, int H, const float* w1, const float* b1, const float* w2,
                 const float* b2, float* E, float* att, float* ctx);
int attn_backward(hipStream_t s, const float* O, const float* E, const float* att, const float* dctx, const float* w1,
                  const float* w2, int B, int T, int H, float* scratch, float* dO, float* gw1, float* gb1, float* gw2,
                  float* gb2);
int colsum(hipStream_t s, const float* X, int M, int N, int ld, float* out);
// one launch per recurrent cell (k_rnn_step.hip): the forward cell with its own gate products, and
// the backward's product into the next cell's hidden gradient as KSL = rnn_step_slices() K slices
struct RnnStep {
  int B, T, H, L;
  const float* P[8];      // packed recurrent weights [7H][H]
  const float* bias7[8];  // [7H]
  const float* X0;        // layer-0 x projection [B*T][6H]
  float* UH[8];           // hidden inputs (rows b*T + t, ld T*H)
  float* CI[8];           // cell inputs
  float* ACT[8];          // saved activated gates [B*T][7H]
  float* CN[8];
  float* CL[8];
  float* O;               // last layer's h' [B*T][H]
  float p;
  uint64_t seed;
  unsigned long long* ts;  // development timing: per-workgroup phase stamps [grid][8] (nullptr: off)
};
bool rnn_step_supported(const RnnDims& d);
int rnn_step_slices();
int launch_rnn_step_fwd(hipStream_t s, const RnnStep& a, int t, int l);
int launch_rnn_dh(hipStream_t s, const float* DZ, int64_t ldz, const float* P, int B, int H, float* part);
int64_t set_rnn_step(int64_t v);  // 1 on (default), 0 = K-sliced products + cell kernels; returns the previous value
// table of 14*L + 8 pointers in the reference's named_parameters() order -> RnnParams
int rnn_params_from_table(float* const* t, int L, RnnParams& P);

}  // namespace dfd
