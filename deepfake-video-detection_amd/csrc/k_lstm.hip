// nn.LSTM layer (batch_first; gate order i, f, g, o) for CNNLSTMHybrid (src/models.py:49-55), fp32:
//   z_t = x_t W_ih^T + b_ih + h_{t-1} W_hh^T + b_hh ; i,f,o = sigmoid, g = tanh
//   c_t = f c_{t-1} + i g ; h_t = o tanh(c_t)
// The input projection of all T steps is one MFMA GEMM; each step runs the recurrent GEMM
// (h @ W_hh^T) and one fused cell kernel.  Backward: BPTT over the saved gate activations, then
// one GEMM per weight over all B*T rows.
#include "kernels.h"
#include "rnn.h"
#include "cnnlstm.h"

namespace dfd {

__device__ __forceinline__ float lsig(float x) { return 1.f / (1.f + __expf(-x)); }

// The per-step recurrent products have only B = 64 rows: they run K-sliced (rnn.h
// sgemm_splits / launch_sgemm_part) and the cell kernels add the slices in order.
// work layout (floats): XP [BT][4H] | ACT [BT][4H] | CT [BT][H] | CP [BT][H] | HP [BT][H] | G [sf][B][4H] | h, c [B][H]
int64_t lstm_layer_work_floats(int B, int T, int IN, int H) {
  const int64_t BT = (int64_t)B * T;
  int kc;
  const int64_t sf = sgemm_splits(B, 4 * H, H, &kc);
  return BT * 4 * H * 2 + BT * H * 3 + sf * B * 4 * H + 2LL * B * H + 64;
}
// scratch: DZ [BT][4H] | dh slices [sb][B][H] | dc [B][H]
int64_t lstm_layer_scratch_floats(int B, int T, int IN, int H) {
  const int64_t BT = (int64_t)B * T;
  int kc;
  const int64_t sb = sgemm_splits(B, H, 4 * H, &kc);
  return BT * 4 * H + (sb + 1) * B * H + 4 * H + 64;
}

__global__ void lstm_cell_fwd_kernel(const float* __restrict__ XP, const float* __restrict__ G, int gsplit,
                                     const float* __restrict__ b_hh, int B, int T, int t, int H,
                                     float* __restrict__ ACT, float* __restrict__ CT, float* __restrict__ CP,
                                     float* __restrict__ HP, float* __restrict__ h, float* __restrict__ c,
                                     float* __restrict__ Hout) {
  const int n = B * H;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int b = e / H, j = e - b * H;
    const int64_t row = (int64_t)b * T + t;
    float z[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) z[q] = G[(int64_t)b * 4 * H + q * H + j];
    for (int sp = 1; sp < gsplit; ++sp)
#pragma unroll
      for (int q = 0; q < 4; ++q) z[q] += G[((int64_t)sp * B + b) * 4 * H + q * H + j];
#pragma unroll
    for (int q = 0; q < 4; ++q) z[q] = XP[row * 4 * H + q * H + j] + z[q] + b_hh[q * H + j];
    const float i = lsig(z[0]), f = lsig(z[1]), g = tanhf(z[2]), o = lsig(z[3]);
    const float cp = c[e], hp = h[e];
    const float cn = f * cp + i * g;
    const float hn = o * tanhf(cn);
    float* act = ACT + row * 4 * H;
    act[j] = i; act[H + j] = f; act[2 * H + j] = g; act[3 * H + j] = o;
    CT[row * H + j] = cn;
    CP[row * H + j] = cp;
    HP[row * H + j] = hp;
    c[e] = cn;
    h[e] = hn;
    Hout[row * H + j] = hn;
  }
}

__global__ void lstm_cell_bwd_kernel(const float* __restrict__ dH, const float* __restrict__ ACT,
                                     const float* __restrict__ CT, const float* __restrict__ CP, int B, int T, int t,
                                     int H, const float* __restrict__ dh, int bsplit, float* __restrict__ dc,
                                     float* __restrict__ DZ) {
  const int n = B * H;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int b = e / H, j = e - b * H;
    const int64_t row = (int64_t)b * T + t;
    const float* act = ACT + row * 4 * H;
    const float i = act[j], f = act[H + j], g = act[2 * H + j], o = act[3 * H + j];
    const float tc = tanhf(CT[row * H + j]);
    float rec = 0.f;  // dh_t from step t+1: K slices of dz_{t+1} W_hh (none at t = T-1)
    if (dh) {
      rec = dh[e];
      int sp = 1;  // slices added in order, four loads in flight
      for (; sp + 4 <= bsplit; sp += 4) {
        const float a0 = dh[(int64_t)sp * n + e], a1 = dh[(int64_t)(sp + 1) * n + e];
        const float a2 = dh[(int64_t)(sp + 2) * n + e], a3 = dh[(int64_t)(sp + 3) * n + e];
        rec += a0; rec += a1; rec += a2; rec += a3;
      }
      for (; sp < bsplit; ++sp) rec += dh[(int64_t)sp * n + e];
    }
    const float gh = dH[row * H + j] + rec;
    const float dcc = gh * o * (1.f - tc * tc) + dc[e];
    float* dz = DZ + row * 4 * H;
    dz[j] = dcc * g * i * (1.f - i);
    dz[H + j] = dcc * CP[row * H + j] * f * (1.f - f);
    dz[2 * H + j] = dcc * i * (1.f - g * g);
    dz[3 * H + j] = gh * tc * o * (1.f - o);
    dc[e] = dcc * f;
  }
}

static int lew(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 2048)); }

int lstm_layer_forward(hipStream_t s, int B, int T, int IN, int H, const LstmLayerW& w, const float* X, float* work,
                       float* Hout) {
  const int64_t BT = (int64_t)B * T;
  float* XP = work;
  float* ACT = XP + BT * 4 * H;
  float* CT = ACT + BT * 4 * H;
  float* CP = CT + BT * H;
  float* HP = CP + BT * H;
  float* G = HP + BT * H;
  DFD_TRY(launch_sgemm(s, false, false, X, IN, w.w_ih, IN, XP, 4 * H, (int)BT, 4 * H, IN, 0.f, w.b_ih));
  int kc;
  const int sf = sgemm_splits(B, 4 * H, H, &kc);
  float* h = G + (int64_t)sf * B * 4 * H;
  float* c = h + (int64_t)B * H;
  DFD_HIP_CHECK(hipMemsetAsync(h, 0, sizeof(float) * 2 * B * H, s));
  for (int t = 0; t < T; ++t) {
    DFD_TRY(launch_sgemm_part(s, false, false, h, H, w.w_hh, H, G, B, 4 * H, H, sf, kc));
    hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3(lew((int64_t)B * H)), dim3(256), 0, s, XP, G, sf, w.b_hh, B, T, t, H,
                       ACT, CT, CP, HP, h, c, Hout);
    DFD_HIP_CHECK(hipGetLastError());
  }
  return 0;
}

int lstm_layer_backward(hipStream_t s, int B, int T, int IN, int H, const LstmLayerW& w, const float* X, float* work,
                        const float* dH, float* scratch, LstmLayerG& g, float* dX) {
  const int64_t BT = (int64_t)B * T;
  float* ACT = work + BT * 4 * H;
  float* CT = ACT + BT * 4 * H;
  float* CP = CT + BT * H;
  float* HP = CP + BT * H;
  float* DZ = scratch;
  int kc;
  const int sb = sgemm_splits(B, H, 4 * H, &kc);
  float* dh = DZ + BT * 4 * H;
  float* dc = dh + (int64_t)sb * B * H;
  DFD_HIP_CHECK(hipMemsetAsync(dc, 0, sizeof(float) * B * H, s));
  for (int t = T - 1; t >= 0; --t) {
    hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(lew((int64_t)B * H)), dim3(256), 0, s, dH, ACT, CT, CP, B, T, t, H,
                       t == T - 1 ? nullptr : dh, sb, dc, DZ);
    DFD_HIP_CHECK(hipGetLastError());
    // dh_{t-1} = dz_t W_hh   (rows b*T + t of DZ), K slices; none needed into h_{-1} = 0
    if (t > 0)
      DFD_TRY(launch_sgemm_part(s, false, true, DZ + (int64_t)t * 4 * H, T * 4 * H, w.w_hh, H, dh, B, H, 4 * H, sb, kc));
  }
  DFD_TRY(launch_sgemm(s, true, true, DZ, 4 * H, HP, H, g.w_hh, H, 4 * H, H, (int)BT, 0.f, nullptr));
  DFD_TRY(launch_sgemm(s, true, true, DZ, 4 * H, X, IN, g.w_ih, IN, 4 * H, IN, (int)BT, 0.f, nullptr));
  DFD_TRY(launch_reduce_slabs(s, DZ, (int)BT, 4 * H, g.b_ih, false));
  DFD_TRY(launch_reduce_slabs(s, DZ, (int)BT, 4 * H, g.b_hh, false));
  if (dX) DFD_TRY(launch_sgemm(s, false, true, DZ, 4 * H, w.w_ih, IN, dX, IN, (int)BT, IN, 4 * H, 0.f, nullptr));
  return 0;
}

}  // namespace dfd
