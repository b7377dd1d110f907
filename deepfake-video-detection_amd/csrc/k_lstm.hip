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

// work layout (floats): XP [BT][4H] | ACT [BT][4H] | CT [BT][H] | CP [BT][H] | HP [BT][H] | G [B][4H] | h, c [B][H]
int64_t lstm_layer_work_floats(int B, int T, int IN, int H) {
  const int64_t BT = (int64_t)B * T;
  return BT * 4 * H * 2 + BT * H * 3 + (int64_t)B * 4 * H + 2LL * B * H + 64;
}
int64_t lstm_layer_scratch_floats(int B, int T, int IN, int H) {
  const int64_t BT = (int64_t)B * T;
  return BT * 4 * H + 4LL * B * H + 4 * H + 64;
}

__global__ void lstm_cell_fwd_kernel(const float* __restrict__ XP, const float* __restrict__ G,
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
    for (int q = 0; q < 4; ++q) z[q] = XP[row * 4 * H + q * H + j] + G[(int64_t)b * 4 * H + q * H + j] + b_hh[q * H + j];
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
                                     int H, float* __restrict__ dh, float* __restrict__ dc, float* __restrict__ DZ) {
  const int n = B * H;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int b = e / H, j = e - b * H;
    const int64_t row = (int64_t)b * T + t;
    const float* act = ACT + row * 4 * H;
    const float i = act[j], f = act[H + j], g = act[2 * H + j], o = act[3 * H + j];
    const float tc = tanhf(CT[row * H + j]);
    const float gh = dH[row * H + j] + dh[e];
    const float dcc = gh * o * (1.f - tc * tc) + dc[e];
    float* dz = DZ + row * 4 * H;
    dz[j] = dcc * g * i * (1.f - i);
    dz[H + j] = dcc * CP[row * H + j] * f * (1.f - f);
    dz[2 * H + j] = dcc * i * (1.f - g * g);
    dz[3 * H + j] = gh * tc * o * (1.f - o);
    dc[e] = dcc * f;
  }
}

__global__ void lstm_colsum2_kernel(const float* __restrict__ X, int M, int N, float* __restrict__ a,
                                    float* __restrict__ b) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int m = 0; m < M; ++m) s += X[(int64_t)m * N + n];
  a[n] = s;
  b[n] = s;
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
  float* h = G + (int64_t)B * 4 * H;
  float* c = h + (int64_t)B * H;
  DFD_TRY(launch_sgemm(s, false, false, X, IN, w.w_ih, IN, XP, 4 * H, (int)BT, 4 * H, IN, 0.f, w.b_ih));
  DFD_HIP_CHECK(hipMemsetAsync(h, 0, sizeof(float) * 2 * B * H, s));
  for (int t = 0; t < T; ++t) {
    DFD_TRY(launch_sgemm(s, false, false, h, H, w.w_hh, H, G, 4 * H, B, 4 * H, H, 0.f, nullptr));
    hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3(lew((int64_t)B * H)), dim3(256), 0, s, XP, G, w.b_hh, B, T, t, H, ACT,
                       CT, CP, HP, h, c, Hout);
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
  float* dh = DZ + BT * 4 * H;
  float* dc = dh + (int64_t)B * H;
  DFD_HIP_CHECK(hipMemsetAsync(dh, 0, sizeof(float) * 2 * B * H, s));
  for (int t = T - 1; t >= 0; --t) {
    hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(lew((int64_t)B * H)), dim3(256), 0, s, dH, ACT, CT, CP, B, T, t, H,
                       dh, dc, DZ);
    DFD_HIP_CHECK(hipGetLastError());
    // dh_{t-1} = dz_t W_hh   (rows b*T + t of DZ)
    DFD_TRY(launch_sgemm(s, false, true, DZ + (int64_t)t * 4 * H, T * 4 * H, w.w_hh, H, dh, H, B, H, 4 * H, 0.f,
                         nullptr));
  }
  DFD_TRY(launch_sgemm(s, true, true, DZ, 4 * H, HP, H, g.w_hh, H, 4 * H, H, (int)BT, 0.f, nullptr));
  DFD_TRY(launch_sgemm(s, true, true, DZ, 4 * H, X, IN, g.w_ih, IN, 4 * H, IN, (int)BT, 0.f, nullptr));
  hipLaunchKernelGGL(lstm_colsum2_kernel, dim3((unsigned)cdiv(4 * H, 256)), dim3(256), 0, s, DZ, (int)BT, 4 * H, g.b_ih,
                     g.b_hh);
  DFD_HIP_CHECK(hipGetLastError());
  if (dX) DFD_TRY(launch_sgemm(s, false, true, DZ, 4 * H, w.w_ih, IN, dX, IN, (int)BT, IN, 4 * H, 0.f, nullptr));
  return 0;
}

}  // namespace dfd
