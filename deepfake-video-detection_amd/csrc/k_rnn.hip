// LogicRNNLSTM (src/RNNModel.py:5-147) on gfx950, fp32 throughout (the reference is fp32).
//
// Forward per timestep t, layer l (RNNModel.py:103-115; all layers share one (h, c) per step):
//   u = [x_l, h_l];  a = sig(Wa u), o_ = sig(Wo u), n = tanh(Wn h_l), f = sig(Wf u), i = sig(Wi u),
//   g = tanh(Wg u);  cn = f*c + i*g;  cl = a*cn + o_*n;  out = sig(Wout u);  h' = out * tanh(cl)
// with x_0 = x_t, h_0 = h_{t-1}, c_0 = c_{t-1} (the LAST layer's state of step t-1), and for
// l >= 1: x_l = h_l = dropout(h'_{l-1}) (the reference passes h_temp as both arguments), c_l = cl_{l-1}.
// Hence layer 0 = precomputed x-projection (one GEMM over all B*T rows) + h @ P0^T with
// P0 = [Wa..Wout h-columns ; Wn] (7H x H), and layer l >= 1 = h @ Pl^T with Pl = [(Wx + Wh) ; Wn].
//
// Kernels: sgemm_kernel<TA,TB> (fp32 v_mfma_f32_16x16x4f32, exact fp32 products, 64x64 tiles,
// LDS-staged with coalesced loads along the contiguous dimension of either operand layout),
// rnn_cell_fwd/bwd (fused gate nonlinearities + cell algebra + saved activations),
// rnn_attn_* (attention pooling over T), weight pack/scatter, column sums.
#include <atomic>
#include "kernels.h"
#include "rnn.h"

namespace dfd {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ fp32 MFMA GEMM
// C[m][n] = beta*C[m][n] + sum_k A(m,k) B(n,k) (+ bias[n]),  A(m,k) = TA ? A[k*lda+m] : A[m*lda+k],
// B(n,k) = TB ? B[k*ldb+n] : B[n*ldb+k].  64x64 tile per 256-thread block, BK = 16; wave w owns
// rows 32*(w>>1).. and cols 32*(w&1).. (2x2 MFMA 16x16 blocks).
constexpr int SG_T = 64, SG_K = 16;

template <bool T_>
__device__ __forceinline__ void sg_load(const float* __restrict__ P, int ld, int r0, int k0, int R, int K, float (&v)[4],
                                        bool (&ok)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    int r, k;
    if (T_) { k = e / SG_T; r = e % SG_T; }   // contiguous along r
    else { r = e / SG_K; k = e % SG_K; }      // contiguous along k
    const int gr = r0 + r, gk = k0 + k;
    ok[i] = gr < R && gk < K;
    const float* q = T_ ? P + (int64_t)gk * ld + gr : P + (int64_t)gr * ld + gk;
    v[i] = *(ok[i] ? q : P);
  }
}
template <bool T_>
__device__ __forceinline__ void sg_store(float (*S)[SG_K + 1], const float (&v)[4], const bool (&ok)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    int r, k;
    if (T_) { k = e / SG_T; r = e % SG_T; }
    else { r = e / SG_K; k = e % SG_K; }
    S[r][k] = ok[i] ? v[i] : 0.f;
  }
}

// K is split over blockIdx.z: slice z covers k in [z*kc, min(K, z*kc + kc)) and writes its
// partial product to C + z*zstride (beta = 0, no bias when split).  The recurrent steps have
// M = B = 64 rows, so without the split a (64 x 512, K = 3584) product is 8 workgroups that walk
// 224 K-steps each; with it every step fills the chip (consumers add the slices in order).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void sgemm_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                    int ldb, float* __restrict__ C, int ldc, int M, int N, int K,
                                                    float beta, const float* __restrict__ bias, int kc,
                                                    int64_t zstride) {
  __shared__ float As[SG_T][SG_K + 1], Bs[SG_T][SG_K + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * SG_T, n0 = blockIdx.x * SG_T;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int kb = blockIdx.z * kc, ke = min(K, kb + kc);
  C += (int64_t)blockIdx.z * zstride;
  f32x4_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float va[4], vb[4];
  bool oa[4], ob[4];
  sg_load<TA>(A, lda, m0, kb, M, ke, va, oa);
  sg_load<TB>(B, ldb, n0, kb, N, ke, vb, ob);
  for (int k0 = kb; k0 < ke; k0 += SG_K) {
    lds_barrier();
    sg_store<TA>(As, va, oa);
    sg_store<TB>(Bs, vb, ob);
    lds_barrier();
    if (k0 + SG_K < ke) {
      sg_load<TA>(A, lda, m0, k0 + SG_K, M, ke, va, oa);
      sg_load<TB>(B, ldb, n0, k0 + SG_K, N, ke, vb, ob);
    }
#pragma unroll
    for (int s = 0; s < SG_K / 4; ++s) {
      const int kk = 4 * s + (lane >> 4);
      const float a0 = As[wm + (lane & 15)][kk], a1 = As[wm + 16 + (lane & 15)][kk];
      const float b0 = Bs[wn + (lane & 15)][kk], b1 = Bs[wn + 16 + (lane & 15)][kk];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + a * 16 + 4 * (lane >> 4) + r, n = n0 + wn + b * 16 + (lane & 15);
        if (m < M && n < N) {
          float v = acc[a][b][r];
          if (bias) v += bias[n];
          float* c = C + (int64_t)m * ldc + n;
          *c = beta != 0.f ? beta * *c + v : v;
        }
      }
}

// Large-tile form for the big products (weight gradients over all B*T rows, input projections):
// 128 x 64 tile per 256-thread block, BK = 32, LDS double-buffered (one barrier per k-step), k-major
// LDS rows padded by 16 floats (the four k rows of an MFMA operand read hit disjoint bank quarters);
// wave w owns a 64 x 32 quarter = 4 x 2 MFMA blocks.  Needs M % 128 == 0, N % 64 == 0, K % 16 == 0
// and 16-B aligned rows (sgemm_go checks; other shapes take sgemm_kernel).
constexpr int SB_M = 128, SB_N = 64, SB_K = 32, SB_PM = SB_M + 16, SB_PN = SB_N + 16;

template <int R> constexpr int sb_nv() { return R * SB_K / 4 / 256; }  // float4 per thread of an R x SB_K operand tile
template <bool T_, int R>  // R rows (m or n) x SB_K of one operand -> registers
__device__ __forceinline__ void sb_load(const float* __restrict__ P, int ld, int r0, int k0, float4 (&v)[sb_nv<R>()]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < sb_nv<R>(); ++i) {
    const int e = tid + 256 * i;
    if (T_) {  // contiguous along r: k row e / (R/4), r4 = (e % (R/4)) * 4
      const int k = e / (R / 4), r4 = (e % (R / 4)) * 4;
      v[i] = *reinterpret_cast<const float4*>(P + (int64_t)(k0 + k) * ld + r0 + r4);
    } else {   // contiguous along k: r = e / (SB_K/4), k4 = (e % (SB_K/4)) * 4
      const int r = e / (SB_K / 4), k4 = (e % (SB_K / 4)) * 4;
      v[i] = *reinterpret_cast<const float4*>(P + (int64_t)(r0 + r) * ld + k0 + k4);
    }
  }
}
// LDS image [SB_K][PR] k-major; element (k, r) sits at column r ^ sb_swz(k): the XOR permutes
// 4-column groups inside each 16-column block, so the MFMA reads (16 consecutive r of one k) stay
// conflict-free while the transposing scalar stores of a k-contiguous operand (8 k x 4 r per 32
// lanes) spread over 16 banks (2-way: free for ds_write_b32) instead of 4 (8-way)
__device__ __forceinline__ int sb_swz(int k) { return ((k >> 2) & 3) << 2; }
template <bool T_, int R, int PR>
__device__ __forceinline__ void sb_store(float* S, const float4 (&v)[sb_nv<R>()]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < sb_nv<R>(); ++i) {
    const int e = tid + 256 * i;
    if (T_) {
      const int k = e / (R / 4), r4 = (e % (R / 4)) * 4;
      *reinterpret_cast<float4*>(S + k * PR + (r4 ^ sb_swz(k))) = v[i];
    } else {
      const int r = e / (SB_K / 4), k4 = (e % (SB_K / 4)) * 4, rs = r ^ sb_swz(k4);  // k4..k4+3 share sb_swz
      S[(k4 + 0) * PR + rs] = v[i].x;
      S[(k4 + 1) * PR + rs] = v[i].y;
      S[(k4 + 2) * PR + rs] = v[i].z;
      S[(k4 + 3) * PR + rs] = v[i].w;
    }
  }
}

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void sgemm_big_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                        int ldb, float* __restrict__ C, int ldc, int K, float beta,
                                                        const float* __restrict__ bias, int kc, int64_t zstride) {
  __shared__ __attribute__((aligned(16))) float As[2][SB_K * SB_PM];
  __shared__ __attribute__((aligned(16))) float Bs[2][SB_K * SB_PN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * SB_M, n0 = blockIdx.x * SB_N;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 32;
  f32x4_t acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // K slice of this z (split-K partials: slice z writes C + z * zstride; kc % SB_K == 0)
  const int kb = blockIdx.z * kc, nk = (min(K, kb + kc) - kb) / SB_K;
  C += (int64_t)blockIdx.z * zstride;
  float4 va[sb_nv<SB_M>()], vb[sb_nv<SB_N>()];
  sb_load<TA, SB_M>(A, lda, m0, kb, va);
  sb_load<TB, SB_N>(B, ldb, n0, kb, vb);
  sb_store<TA, SB_M, SB_PM>(As[0], va);
  sb_store<TB, SB_N, SB_PN>(Bs[0], vb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      sb_load<TA, SB_M>(A, lda, m0, kb + (kt + 1) * SB_K, va);
      sb_load<TB, SB_N>(B, ldb, n0, kb + (kt + 1) * SB_K, vb);
    }
#pragma unroll
    for (int s4 = 0; s4 < SB_K / 4; ++s4) {
      // k = 4*s4 + (lane >> 4): sb_swz(k) = (s4 & 3) << 2 for every lane
      const int rl = (lane & 15) ^ ((s4 & 3) << 2);
      const float* as = As[cur] + (lane >> 4) * SB_PM + wm + rl;
      const float* bs = Bs[cur] + (lane >> 4) * SB_PN + wn + rl;
      float af[4], bf[2];
#pragma unroll
      for (int a = 0; a < 4; ++a) af[a] = as[s4 * 4 * SB_PM + a * 16];
#pragma unroll
      for (int b = 0; b < 2; ++b) bf[b] = bs[s4 * 4 * SB_PN + b * 16];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      sb_store<TA, SB_M, SB_PM>(As[cur ^ 1], va);
      sb_store<TB, SB_N, SB_PN>(Bs[cur ^ 1], vb);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + a * 16 + 4 * (lane >> 4) + r, n = n0 + wn + b * 16 + (lane & 15);
        float v = acc[a][b][r];
        if (bias) v += bias[n];
        float* c = C + (int64_t)m * ldc + n;
        *c = beta != 0.f ? beta * *c + v : v;
      }
}

static bool sgemm_big_ok(const float* A, int lda, const float* B, int ldb, int M, int N, int K, int kc) {
  return M % SB_M == 0 && N % SB_N == 0 && K % SB_K == 0 && kc % SB_K == 0 && K > 0 && lda % 4 == 0 &&
         ldb % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(B) & 15) == 0;
}

static int sgemm_go(hipStream_t s, bool ta, bool tb, const float* A, int lda, const float* B, int ldb, float* C,
                    int ldc, int M, int N, int K, float beta, const float* bias, int splits, int kc, int64_t zs) {
  if (sgemm_big_ok(A, lda, B, ldb, M, N, K, splits == 1 ? K : kc)) {
    const dim3 g((unsigned)(N / SB_N), (unsigned)(M / SB_M), (unsigned)splits);
    const int kcb = splits == 1 ? K : kc;
#define DFD_SB(a_, b_)                                                                                           \
  hipLaunchKernelGGL((sgemm_big_kernel<a_, b_>), g, dim3(256), 0, s, A, lda, B, ldb, C, ldc, K, beta, bias, kcb, \
                     zs)
    if (!ta && !tb) DFD_SB(false, false);
    else if (!ta && tb) DFD_SB(false, true);
    else if (ta && !tb) DFD_SB(true, false);
    else DFD_SB(true, true);
#undef DFD_SB
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
  const dim3 grid((unsigned)cdiv(N, SG_T), (unsigned)cdiv(M, SG_T), (unsigned)splits);
#define DFD_SG(a_, b_) \
  hipLaunchKernelGGL((sgemm_kernel<a_, b_>), grid, dim3(256), 0, s, A, lda, B, ldb, C, ldc, M, N, K, beta, bias, kc, zs)
  if (!ta && !tb) DFD_SG(false, false);
  else if (!ta && tb) DFD_SG(false, true);
  else if (ta && !tb) DFD_SG(true, false);
  else DFD_SG(true, true);
#undef DFD_SG
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int launch_sgemm(hipStream_t s, bool ta, bool tb, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
                 int M, int N, int K, float beta, const float* bias) {
  if (M <= 0 || N <= 0) return 0;
  return sgemm_go(s, ta, tb, A, lda, B, ldb, C, ldc, M, N, K, beta, bias, 1, std::max(K, 1), 0);
}

// K slices of the big-tile weight-gradient products (M x N outputs over K = B*T rows): enough
// 128 x 64 tiles x slices for ~2 workgroups per CU, slices of >= 256 k, at most 8
int sgemm_wsplits(int M, int N, int K, int* kc) {
  const int tiles = std::max(1, (M / SB_M) * (N / SB_N));
  int sp = std::min(std::min(8, std::max(1, K / 256)), std::max(1, (512 + tiles - 1) / tiles));
  *kc = cdiv(cdiv(std::max(K, 1), sp), SB_K) * SB_K;
  return cdiv(std::max(K, 1), *kc);
}

// K slices for a product of few output tiles: aim at ~256 workgroups, at least 64 k per slice;
// returns the slice count and (kc) the slice length, a multiple of the 16-deep K step
int sgemm_splits(int M, int N, int K, int* kc) {
  const int tiles = cdiv(N, SG_T) * cdiv(M, SG_T);
  int sp = std::max(1, 256 / std::max(tiles, 1));
  sp = std::min(std::min(sp, std::max(1, K / 64)), 64);
  *kc = cdiv(cdiv(std::max(K, 1), sp), SG_K) * SG_K;
  return cdiv(std::max(K, 1), *kc);
}

// part[z][M][N] = the K-slice z (k in [z*kc, z*kc + kc)) of A.B^T: fixed slice boundaries, so the
// consumer's in-order sum over z is deterministic
int launch_sgemm_part(hipStream_t s, bool ta, bool tb, const float* A, int lda, const float* B, int ldb, float* part,
                      int M, int N, int K, int splits, int kc) {
  if (M <= 0 || N <= 0) return 0;
  if (kc <= 0 || kc % SG_K || cdiv(std::max(K, 1), kc) != splits) {
    set_error("sgemm_part: slice length/count mismatch", __FILE__, __LINE__);
    return -1;
  }
  return sgemm_go(s, ta, tb, A, lda, B, ldb, part, N, M, N, K, 0.f, nullptr, splits, kc, (int64_t)M * N);
}

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ float sig_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_(float x) { return tanhf(x); }

// dropout keep-scale for element idx of stream `st` (same counter hash as the detector head)
__device__ __forceinline__ float rnn_drop(uint64_t seed, uint32_t st, int64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  uint64_t z = seed ^ ((uint64_t)st << 56) ^ (uint64_t)idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// xs[b][t][:] = x[order[b]][t][:]   (the reference's x[sort_idx], RNNModel.py:92-95)
__global__ void rnn_gather_kernel(const float* __restrict__ x, const int64_t* __restrict__ order, float* __restrict__ xs,
                                  int B, int64_t row) {
  const int64_t n = (int64_t)B * row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / row);
    xs[i] = x[order[b] * row + (i - (int64_t)b * row)];
  }
}

// pack the recurrent weights of layer l (rows: a, o_, f, i, g, out gates then not; cols H):
//   l == 0 : h-columns [in, in+H) of the six u-gates, then Wn
//   l >= 1 : x-columns + h-columns (x = h = dropout(h_{l-1})), then Wn
// and (l == 0) the x-columns of the six u-gates into WX0 [6H][in]; biases into bias7 [7H].
__global__ void rnn_pack_kernel(RnnLayerW w, int in, int H, int layer, float* __restrict__ P, float* __restrict__ WX0,
                                float* __restrict__ bias7) {
  const int ld = in + H;
  const int64_t nP = (int64_t)7 * H * H;
  const int64_t nX = layer == 0 ? (int64_t)6 * H * in : 0;
  const int64_t n = nP + nX + 7 * H;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (i < nP) {
      const int row = (int)(i / H), k = (int)(i - (int64_t)row * H);
      const int g = row / H, r = row - g * H;
      float v;
      if (g == 6) v = w.wn[(int64_t)r * H + k];
      else {
        const float* W = w.wu[g] + (int64_t)r * ld;
        v = layer == 0 ? W[in + k] : W[k] + W[in + k];
      }
      P[i] = v;
    } else if (i < nP + nX) {
      const int64_t j = i - nP;
      const int row = (int)(j / in), k = (int)(j - (int64_t)row * in);
      const int g = row / H, r = row - g * H;
      WX0[j] = w.wu[g][(int64_t)r * ld + k];
    } else {
      const int j = (int)(i - nP - nX), g = j / H, r = j - g * H;
      bias7[j] = g == 6 ? w.bn[r] : w.bu[g][r];
    }
  }
}

// sum_{s < n} p[s * st], added in slice order; four slices' loads are issued before their adds
__device__ __forceinline__ float slice_sum(const float* __restrict__ p, int n, int64_t st) {
  float v = p[0];
  int sp = 1;
  for (; sp + 4 <= n; sp += 4) {
    const float a0 = p[sp * st], a1 = p[(sp + 1) * st], a2 = p[(sp + 2) * st], a3 = p[(sp + 3) * st];
    v += a0; v += a1; v += a2; v += a3;
  }
  for (; sp < n; ++sp) v += p[sp * st];
  return v;
}

// forward cell of one (step, layer) for all B rows:
//   z[b][:] = sum_s G[s][b][:] (recurrent product, K-sliced, 7H) + bias7 (+ X0[b*T+t][:6H], layer 0)
// saved (row = b*T + t): ACT[row][7H] activated gates, CN, CL.  Outputs (each optional): h' to
// h_out, h' (times the layer's dropout keep-scale if h2_drop) to h2_out, c' to c_out -- the
// caller points them straight at the next consumer's rows (O, UH, CI), so no state copies.
__global__ void rnn_cell_fwd_kernel(const float* __restrict__ G, int gsplit, int64_t gstride,
                                    const float* __restrict__ X0, const float* __restrict__ bias7,
                                    const float* __restrict__ c_in, int c_in_ld, int B, int T, int t, int H,
                                    float* __restrict__ ACT, float* __restrict__ CN, float* __restrict__ CL,
                                    float* __restrict__ h_out, int h_ld, float* __restrict__ h2_out, int h2_ld,
                                    int h2_drop, float* __restrict__ c_out, int c_ld, float p, uint64_t seed,
                                    uint32_t stream) {
  const int n = B * H;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int b = i / H, j = i - b * H;
    const int64_t row = (int64_t)b * T + t;
    float z[7];
#pragma unroll
    for (int g = 0; g < 7; ++g) z[g] = slice_sum(G + (int64_t)b * 7 * H + g * H + j, gsplit, gstride);
#pragma unroll
    for (int g = 0; g < 7; ++g) {
      float v = z[g] + bias7[g * H + j];
      if (X0 && g < 6) v += X0[row * 6 * H + g * H + j];
      z[g] = v;
    }
    const float a = sig_(z[0]), o_ = sig_(z[1]), f = sig_(z[2]), ii = sig_(z[3]), gg = tanh_(z[4]), ou = sig_(z[5]);
    const float nn = tanh_(z[6]);
    const float c = c_in[(int64_t)b * c_in_ld + j];
    const float cn = f * c + ii * gg;
    const float cl = a * cn + o_ * nn;
    const float h = ou * tanh_(cl);
    float* act = ACT + row * 7 * H;
    act[0 * H + j] = a; act[1 * H + j] = o_; act[2 * H + j] = f; act[3 * H + j] = ii;
    act[4 * H + j] = gg; act[5 * H + j] = ou; act[6 * H + j] = nn;
    CN[row * H + j] = cn;
    CL[row * H + j] = cl;
    if (h_out) h_out[(int64_t)b * h_ld + j] = h;
    if (h2_out) h2_out[(int64_t)b * h2_ld + j] = h2_drop ? h * rnn_drop(seed, stream, row * H + j, p) : h;
    if (c_out) c_out[(int64_t)b * c_ld + j] = cl;
  }
}

// backward cell: from dh (gradient of h') and dc (gradient of c' = cl) -> dz (7H pre-activation
// grads, row b*T+t) and dc_in.  dh = dh_a[b] (+ sum_s dh_b[s][b], times the layer's dropout
// keep-scale if b_drop: the K-sliced product from the layer above), dc = dc_a[b].  dc_a and
// dc_out may alias (each element is read, then written, by the same thread).
__global__ void rnn_cell_bwd_kernel(const float* __restrict__ dh_a, int dh_a_ld, const float* __restrict__ dh_b,
                                    int bsplit, int64_t bstride, int b_drop, float p, uint64_t seed, uint32_t stream,
                                    const float* dc_a, const float* __restrict__ ACT, const float* __restrict__ CN,
                                    const float* __restrict__ CL, const float* __restrict__ c_in, int c_in_ld, int B,
                                    int T, int t, int H, float* __restrict__ DZ, float* dc_out) {
  const int n = B * H;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int b = i / H, j = i - b * H;
    const int64_t row = (int64_t)b * T + t;
    float dh = dh_a ? dh_a[(int64_t)b * dh_a_ld + j] : 0.f;
    if (dh_b) {
      float v = slice_sum(dh_b + i, bsplit, bstride);
      if (b_drop) v *= rnn_drop(seed, stream, row * H + j, p);
      dh += v;
    }
    const float dcl0 = dc_a ? dc_a[(int64_t)b * H + j] : 0.f;
    const float* act = ACT + row * 7 * H;
    const float a = act[0 * H + j], o_ = act[1 * H + j], f = act[2 * H + j], ii = act[3 * H + j];
    const float gg = act[4 * H + j], ou = act[5 * H + j], nn = act[6 * H + j];
    const float cn = CN[row * H + j], cl = CL[row * H + j];
    const float c = c_in[(int64_t)b * c_in_ld + j];
    const float tc = tanh_(cl);
    const float dou = dh * tc;
    const float dcl = dh * ou * (1.f - tc * tc) + dcl0;
    const float da = dcl * cn, dcn = dcl * a, do_ = dcl * nn, dnn = dcl * o_;
    const float df = dcn * c, di = dcn * gg, dg = dcn * ii;
    float* dz = DZ + row * 7 * H;
    dz[0 * H + j] = da * a * (1.f - a);
    dz[1 * H + j] = do_ * o_ * (1.f - o_);
    dz[2 * H + j] = df * f * (1.f - f);
    dz[3 * H + j] = di * ii * (1.f - ii);
    dz[4 * H + j] = dg * (1.f - gg * gg);
    dz[5 * H + j] = dou * ou * (1.f - ou);
    dz[6 * H + j] = dnn * (1.f - nn * nn);
    dc_out[(int64_t)b * H + j] = dcn * f;
  }
}

// scatter packed gradients back into the per-gate weight gradients of layer l (accumulating)
// dP / dWX0 arrive as np / nx K slices (split-K partials, slice stride = the matrix size), added in order
__global__ void rnn_scatter_kernel(RnnLayerW gw, int in, int H, int layer, const float* __restrict__ dP, int np,
                                   const float* __restrict__ dWX0, int nx, const float* __restrict__ dbias7) {
  const int64_t pst = (int64_t)7 * H * H, xst = (int64_t)6 * H * in;
  const int ld = in + H;
  const int64_t nU = (int64_t)6 * H * ld, nN = (int64_t)H * H;
  const int64_t n = nU + nN + 7 * H;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (i < nU) {
      const int grow = (int)(i / ld), k = (int)(i - (int64_t)grow * ld);
      const int g = grow / H, r = grow - g * H;
      float v;
      if (layer == 0) v = k < in ? slice_sum(dWX0 + (int64_t)(g * H + r) * in + k, nx, xst)
                                 : slice_sum(dP + (int64_t)(g * H + r) * H + (k - in), np, pst);
      else v = slice_sum(dP + (int64_t)(g * H + r) * H + (k < in ? k : k - in), np, pst);
      gw.wu[g][(int64_t)r * ld + k] = v;
    } else if (i < nU + nN) {
      const int64_t j = i - nU;
      gw.wn[j] = slice_sum(dP + (int64_t)6 * H * H + j, np, pst);
    } else {
      const int j = (int)(i - nU - nN), g = j / H, r = j - g * H;
      if (g == 6) gw.bn[r] = dbias7[j];
      else gw.bu[g][r] = dbias7[j];
    }
  }
}

// ------------------------------------------------------------------ attention + classifier
// Om[b][t][:] = O * (t < len[b]);  E = tanh(Om W1^T + b1) (GEMM + tanh in place);
// s[b][t] = E . w2 + b2 ; a = softmax_t(s) ; ctx[b] = sum_t a * Om
__global__ void rnn_mask_kernel(const float* __restrict__ O, const int64_t* __restrict__ len, float* __restrict__ Om,
                                int B, int T, int H) {
  const int64_t n = (int64_t)B * T * H;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / H;
    const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
    Om[i] = (len == nullptr || t < len[b]) ? O[i] : 0.f;
  }
}
__global__ void rnn_tanh_kernel(float* __restrict__ X, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) X[i] = tanh_(X[i]);
}
// one block per clip: scores, softmax over T, context
__global__ void rnn_attn_fwd_kernel(const float* __restrict__ Om, const float* __restrict__ E,
                                    const float* __restrict__ w2, const float* __restrict__ b2, int T, int H,
                                    float* __restrict__ att, float* __restrict__ ctx) {
  extern __shared__ float sh[];  // [T]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int t = wave; t < T; t += 4) {
    const float* e = E + ((int64_t)b * T + t) * H;
    float a = 0.f;
    for (int j = lane; j < H; j += 64) a += e[j] * w2[j];
    a = wave_sum(a);
    if (lane == 0) sh[t] = a + b2[0];
  }
  __syncthreads();
  if (tid == 0) {
    float mx = -INFINITY;
    for (int t = 0; t < T; ++t) mx = fmaxf(mx, sh[t]);
    float s = 0.f;
    for (int t = 0; t < T; ++t) { sh[t] = __expf(sh[t] - mx); s += sh[t]; }
    for (int t = 0; t < T; ++t) { sh[t] /= s; att[(int64_t)b * T + t] = sh[t]; }
  }
  __syncthreads();
  for (int j = tid; j < H; j += 256) {
    float a = 0.f;
    for (int t = 0; t < T; ++t) a += sh[t] * Om[((int64_t)b * T + t) * H + j];
    ctx[(int64_t)b * H + j] = a;
  }
}
// classifier tail: h1 = relu(ctx W1^T + b1) (GEMM, then this kernel), dropout, z = h1d . w2 + b2, y = sigmoid(z)
__global__ void rnn_cls_fwd_kernel(float* __restrict__ h1, const float* __restrict__ w2, const float* __restrict__ b2,
                                   int H, float p, uint64_t seed, float* __restrict__ y) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float red[4];
  float a = 0.f;
  for (int j = tid; j < H; j += 256) {
    float v = fmaxf(h1[(int64_t)b * H + j], 0.f);
    h1[(int64_t)b * H + j] = v;  // relu in place (saved for backward)
    a += v * rnn_drop(seed, 9u, (int64_t)b * H + j, p) * w2[j];
  }
  a = wave_sum(a);
  if (lane == 0) red[wave] = a;
  __syncthreads();
  if (tid == 0) {
    const float z = red[0] + red[1] + red[2] + red[3] + b2[0];
    y[b] = sig_(z);
  }
}

// backward of the tail: dy -> dz = dy*y*(1-y) ; dw2 = sum_b dz*h1d ; db2 ; dh1 = dz*w2*drop*relu'
// 1024 threads = 64 hidden units x 16 clip lanes; lane bl takes clips bl, bl+16, ... in order and
// the 16 partial sums of dw2 are added in lane order (deterministic)
__global__ __launch_bounds__(1024) void rnn_cls_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                           const float* __restrict__ h1, const float* __restrict__ w2,
                                                           int B, int H, float p, uint64_t seed,
                                                           float* __restrict__ dh1, float* __restrict__ gw2,
                                                           float* __restrict__ gb2) {
  __shared__ float sh[16][64];
  const int cl = threadIdx.x & 63, bl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  float a = 0.f;
  if (j < H) {
    for (int b = bl; b < B; b += 16) {
      const float dz = dy[b] * y[b] * (1.f - y[b]);
      const float d = rnn_drop(seed, 9u, (int64_t)b * H + j, p);
      const float hv = h1[(int64_t)b * H + j];
      a += dz * hv * d;
      dh1[(int64_t)b * H + j] = hv > 0.f ? dz * w2[j] * d : 0.f;
    }
  }
  sh[bl][cl] = a;
  __syncthreads();
  if (bl == 0 && j < H) {
    float v = 0.f;
    for (int l = 0; l < 16; ++l) v += sh[l][cl];
    gw2[j] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float v = 0.f;
    for (int b = 0; b < B; ++b) v += dy[b] * y[b] * (1.f - y[b]);
    gb2[0] = v;
  }
}

// attention backward, one block per clip:
//   dctx[b] -> dOm += a_t * dctx ; da_t = dctx . Om_t ; ds = a*(da - sum a*da) ;
//   dE[b][t][:] = ds_t * w2 * (1 - E^2)  ; gw2 += ds_t * E ; gb2 += ds_t
__global__ void rnn_attn_bwd_kernel(const float* __restrict__ Om, const float* __restrict__ E,
                                    const float* __restrict__ att, const float* __restrict__ dctx,
                                    const float* __restrict__ w2, int T, int H, float* __restrict__ dOm,
                                    float* __restrict__ dE, float* __restrict__ ds_out) {
  extern __shared__ float sh[];  // [2T]
  float* da = sh;
  float* ds = sh + T;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int t = wave; t < T; t += 4) {
    const float* o = Om + ((int64_t)b * T + t) * H;
    float a = 0.f;
    for (int j = lane; j < H; j += 64) a += dctx[(int64_t)b * H + j] * o[j];
    a = wave_sum(a);
    if (lane == 0) da[t] = a;
  }
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += att[(int64_t)b * T + t] * da[t];
    for (int t = 0; t < T; ++t) {
      const float a = att[(int64_t)b * T + t];
      ds[t] = a * (da[t] - s);
      ds_out[(int64_t)b * T + t] = ds[t];
    }
  }
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const float a = att[(int64_t)b * T + t];
    for (int j = tid; j < H; j += 256) {
      const int64_t idx = ((int64_t)b * T + t) * H + j;
      dOm[idx] = a * dctx[(int64_t)b * H + j];
      const float e = E[idx];
      dE[idx] = ds[t] * w2[j] * (1.f - e * e);
    }
  }
}
// gw2[j] = sum_{b,t} ds[b][t] * E[b][t][j] ; gb2 = sum ds.  1024 threads = 64 columns x 16 row
// lanes (lane rl takes rows rl, rl+16, ... in order; lanes added in order: deterministic)
__global__ __launch_bounds__(1024) void rnn_attn_w2_kernel(const float* __restrict__ E, const float* __restrict__ ds,
                                                           int BT, int H, float* __restrict__ gw2,
                                                           float* __restrict__ gb2) {
  __shared__ float sh[16][64];
  __shared__ float sb[1024];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  float a = 0.f;
  if (j < H)
    for (int r = rl; r < BT; r += 16) a += ds[r] * E[(int64_t)r * H + j];
  sh[rl][cl] = a;
  __syncthreads();
  if (rl == 0 && j < H) {
    float v = 0.f;
    for (int l = 0; l < 16; ++l) v += sh[l][cl];
    gw2[j] = v;
  }
  if (blockIdx.x == 0) {  // uniform per block
    float v = 0.f;
    for (int r = threadIdx.x; r < BT; r += 1024) v += ds[r];
    sb[threadIdx.x] = v;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) sb[threadIdx.x] += sb[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) gb2[0] = sb[0];
  }
}
// dO = (dOm_ctx + dOm_att) * mask   (in place into dOm)
__global__ void rnn_mask_bwd_kernel(float* __restrict__ dOm, const float* __restrict__ dOm2, const int64_t* __restrict__ len,
                                    int B, int T, int H) {
  const int64_t n = (int64_t)B * T * H;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / H;
    const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
    const float v = dOm[i] + dOm2[i];
    dOm[i] = (len == nullptr || t < len[b]) ? v : 0.f;
  }
}

static int ew_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 2048)); }

// ------------------------------------------------------------------ host orchestration
// one launch per cell (k_rnn_step.hip) where its shape rules hold: 1 on (default), 0 off
static std::atomic<int64_t> g_rnn_step{1};
int64_t set_rnn_step(int64_t v) { return g_rnn_step.exchange(v); }
static bool rnn_use_step(const RnnDims& d) {
  return g_rnn_step.load(std::memory_order_relaxed) != 0 && rnn_step_supported(d);
}

// K slices of the per-step recurrent products (fixed per shape; the workspace holds them)
static int fwd_splits(const RnnDims& d, int* kc) { return sgemm_splits(d.B, 7 * d.H, d.H, kc); }
static int bwd_splits(const RnnDims& d, int* kc) { return sgemm_splits(d.B, d.H, 7 * d.H, kc); }

struct RnnWs {
  float *xs, *X0, *G, *P[8], *bias7[8], *WX0, *ACT[8], *CN[8], *CL[8], *UH[8], *CI[8], *O, *Om, *E, *att, *ctx, *h1,
      *y;
  int64_t floats;  // extent of the layout (rnn_work_floats)
};
// one layout function for both the size query (w = nullptr) and the pointers
static RnnWs rnn_ws(const RnnDims& d, float* w) {
  RnnWs s{};
  const int64_t BT = (int64_t)d.B * d.T, H = d.H;
  int64_t off = 0;
  auto take = [&](int64_t n) { float* r = w ? w + off : nullptr; off += (n + 63) & ~int64_t(63); return r; };
  int kc;
  s.xs = take(BT * d.IN);                        // sorted input
  s.X0 = take(BT * 6 * H);                       // layer-0 x projection, all rows
  s.G = take((int64_t)fwd_splits(d, &kc) * d.B * 7 * H);  // one step's recurrent product, K slices
  for (int l = 0; l < d.L; ++l) { s.P[l] = take(7 * H * H); s.bias7[l] = take(7 * H); }
  s.WX0 = take(6 * H * d.IN);
  for (int l = 0; l < d.L; ++l) {  // saved: gates, c', cl, hidden input, c input (rows b*T+t)
    s.ACT[l] = take(BT * 7 * H); s.CN[l] = take(BT * H); s.CL[l] = take(BT * H); s.UH[l] = take(BT * H);
    s.CI[l] = take(BT * H);
  }
  s.O = take(BT * H); s.Om = take(BT * H); s.E = take(BT * H);
  s.att = take(BT);
  s.ctx = take((int64_t)d.B * H); s.h1 = take((int64_t)d.B * H);
  s.y = take(d.B);
  s.floats = off;
  return s;
}
int64_t rnn_work_floats(const RnnDims& d) { return rnn_ws(d, nullptr).floats; }

int rnn_forward(hipStream_t s, const RnnDims& d, const RnnParams& P, const float* x, const int64_t* order,
                const int64_t* lens, float* work, float* y, uint64_t seed, float p) {
  if (d.L < 1 || d.L > 8) { set_error("rnn: 1..8 layers supported", __FILE__, __LINE__); return -1; }
  const int B = d.B, T = d.T, H = d.H, IN = d.IN;
  const int64_t BT = (int64_t)B * T;
  RnnWs w = rnn_ws(d, work);
  // (sorted) input
  const float* xs = x;
  if (order) {
    hipLaunchKernelGGL(rnn_gather_kernel, dim3(ew_blocks(BT * IN)), dim3(256), 0, s, x, order, w.xs, B, (int64_t)T * IN);
    xs = w.xs;
  }
  for (int l = 0; l < d.L; ++l)
    hipLaunchKernelGGL(rnn_pack_kernel, dim3(ew_blocks((int64_t)7 * H * H + (l == 0 ? 6LL * H * IN : 0) + 7 * H)),
                       dim3(256), 0, s, P.layer[l], l == 0 ? IN : H, H, l, w.P[l], w.WX0, w.bias7[l]);
  DFD_HIP_CHECK(hipGetLastError());
  // layer-0 x projection for all rows (b*T + t)
  DFD_TRY(launch_sgemm(s, false, false, xs, IN, w.WX0, IN, w.X0, 6 * H, (int)BT, 6 * H, IN, 0.f, nullptr));
  // Every step's hidden/cell inputs live in the saved UH/CI rows (row b*T+t, ld T*H): the cell
  // kernels write their outputs there directly.  Step 0 of layer 0 starts from h = c = 0.
  const int64_t ldr = (int64_t)T * H;
  DFD_HIP_CHECK(hipMemset2DAsync(w.UH[0], (size_t)ldr * 4, 0, (size_t)H * 4, B, s));
  DFD_HIP_CHECK(hipMemset2DAsync(w.CI[0], (size_t)ldr * 4, 0, (size_t)H * 4, B, s));
  int kc;
  const int sf = fwd_splits(d, &kc);
  const int eb = ew_blocks((int64_t)B * H);
  const bool step = rnn_use_step(d);
  if (step) {  // one launch per cell (k_rnn_step.hip)
    RnnStep a{};
    a.B = B; a.T = T; a.H = H; a.L = d.L;
    for (int l = 0; l < d.L; ++l) {
      a.P[l] = w.P[l]; a.bias7[l] = w.bias7[l]; a.UH[l] = w.UH[l]; a.CI[l] = w.CI[l];
      a.ACT[l] = w.ACT[l]; a.CN[l] = w.CN[l]; a.CL[l] = w.CL[l];
    }
    a.X0 = w.X0; a.O = w.O; a.p = p; a.seed = seed;
    for (int t = 0; t < T; ++t)
      for (int l = 0; l < d.L; ++l) DFD_TRY(launch_rnn_step_fwd(s, a, t, l));
  }
  for (int t = 0; t < T && !step; ++t) {
    for (int l = 0; l < d.L; ++l) {
      // recurrent product h_in @ P_l^T in K slices (summed by the cell kernel)
      DFD_TRY(launch_sgemm_part(s, false, false, w.UH[l] + (int64_t)t * H, (int)ldr, w.P[l], H, w.G, B, 7 * H, H, sf,
                                kc));
      const bool last = l == d.L - 1;
      const float* cin = w.CI[l] + (int64_t)t * H;
      if (last) {
        // h' -> O[b][t] and the next step's layer-0 hidden input; c' -> its cell input
        const bool more = t + 1 < T;
        hipLaunchKernelGGL(rnn_cell_fwd_kernel, dim3(eb), dim3(256), 0, s, w.G, sf, (int64_t)B * 7 * H,
                           l == 0 ? w.X0 : nullptr, w.bias7[l], cin, (int)ldr, B, T, t, H, w.ACT[l], w.CN[l], w.CL[l],
                           w.O + (int64_t)t * H, (int)ldr, more ? w.UH[0] + (int64_t)(t + 1) * H : nullptr, (int)ldr,
                           0, more ? w.CI[0] + (int64_t)(t + 1) * H : nullptr, (int)ldr, p, seed, (uint32_t)l);
      } else {
        // dropout(h') is both x and h of layer l+1 (RNNModel.py:113-114); c' its cell input
        hipLaunchKernelGGL(rnn_cell_fwd_kernel, dim3(eb), dim3(256), 0, s, w.G, sf, (int64_t)B * 7 * H,
                           l == 0 ? w.X0 : nullptr, w.bias7[l], cin, (int)ldr, B, T, t, H, w.ACT[l], w.CN[l], w.CL[l],
                           nullptr, 0, w.UH[l + 1] + (int64_t)t * H, (int)ldr, 1, w.CI[l + 1] + (int64_t)t * H,
                           (int)ldr, p, seed, (uint32_t)l);
      }
      DFD_HIP_CHECK(hipGetLastError());
    }
  }
  // mask, attention, classifier
  hipLaunchKernelGGL(rnn_mask_kernel, dim3(ew_blocks(BT * H)), dim3(256), 0, s, w.O, lens, w.Om, B, T, H);
  DFD_TRY(launch_sgemm(s, false, false, w.Om, H, P.att_w1, H, w.E, H, (int)BT, H, H, 0.f, P.att_b1));
  hipLaunchKernelGGL(rnn_tanh_kernel, dim3(ew_blocks(BT * H)), dim3(256), 0, s, w.E, BT * H);
  hipLaunchKernelGGL(rnn_attn_fwd_kernel, dim3(B), dim3(256), T * sizeof(float), s, w.Om, w.E, P.att_w2, P.att_b2, T, H,
                     w.att, w.ctx);
  DFD_TRY(launch_sgemm(s, false, false, w.ctx, H, P.cls_w1, H, w.h1, H, B, H, H, 0.f, P.cls_b1));
  hipLaunchKernelGGL(rnn_cls_fwd_kernel, dim3(B), dim3(256), 0, s, w.h1, P.cls_w2, P.cls_b2, H, p, seed, w.y);
  DFD_HIP_CHECK(hipGetLastError());
  DFD_HIP_CHECK(hipMemcpyAsync(y, w.y, sizeof(float) * B, hipMemcpyDeviceToDevice, s));
  return 0;
}

int rnn_backward(hipStream_t s, const RnnDims& d, const RnnParams& P, const float* x, const int64_t* order,
                 const int64_t* lens, float* work, float* scratch, const float* dy, RnnParams& Gr, uint64_t seed,
                 float p) {
  const int B = d.B, T = d.T, H = d.H, IN = d.IN;
  const int64_t BT = (int64_t)B * T;
  RnnWs w = rnn_ws(d, work);
  // scratch layout: dh1 [B][H], dctx [B][H], dE [BT][H], dOm [BT][H], dOm2 [BT][H], ds [BT],
  //                 DZ per layer [BT][7H], dP [7H][H], dWX0 [6H][IN], dbias [7H], dh/dc state
  float* q = scratch;
  auto take = [&](int64_t n) { float* r = q; q += (n + 63) & ~int64_t(63); return r; };
  int kc;
  const int sb = bwd_splits(d, &kc);
  float* dh1 = take((int64_t)B * H);
  float* dctx = take((int64_t)B * H);
  float* dE = take(BT * H);
  float* dOm = take(BT * H);
  float* dOm2 = take(BT * H);
  float* ds = take(BT);
  float* DZ[8];
  for (int l = 0; l < d.L; ++l) DZ[l] = take(BT * 7 * H);
  int kq;
  float* dP = take((int64_t)sgemm_wsplits(7 * H, H, (int)BT, &kq) * 7 * H * H);      // split-K partials
  float* dWX0 = take((int64_t)sgemm_wsplits(6 * H, IN, (int)BT, &kq) * 6 * H * IN);  // split-K partials
  float* dbias = take(7 * H);
  float* dhs = take((int64_t)sb * B * H);   // K slices: gradient into the last layer's h' of step t-1
  float* dhls = take((int64_t)sb * B * H);  // K slices: gradient into an inner layer's output
  float* dc = take((int64_t)B * H);         // gradient into the last layer's c'
  float* dcl = take((int64_t)B * H);        // gradient into an inner layer's c'
  float* spart = take((int64_t)rnn_step_slices() * B * H);  // per-cell path: product slices
  // classifier tail
  const dim3 gH((unsigned)cdiv(H, 256)), gH64((unsigned)cdiv(H, 64));
  hipLaunchKernelGGL(rnn_cls_bwd_kernel, gH64, dim3(1024), 0, s, dy, w.y, w.h1, P.cls_w2, B, H, p, seed, dh1,
                     Gr.cls_w2, Gr.cls_b2);
  DFD_TRY(launch_sgemm(s, true, true, dh1, H, w.ctx, H, Gr.cls_w1, H, H, H, B, 0.f, nullptr));   // dW1 = dh1^T ctx
  DFD_TRY(launch_reduce_slabs(s, dh1, B, H, Gr.cls_b1, false));
  DFD_TRY(launch_sgemm(s, false, true, dh1, H, P.cls_w1, H, dctx, H, B, H, H, 0.f, nullptr));     // dctx = dh1 W1
  // attention
  hipLaunchKernelGGL(rnn_attn_bwd_kernel, dim3(B), dim3(256), 2 * T * sizeof(float), s, w.Om, w.E, w.att, dctx,
                     P.att_w2, T, H, dOm, dE, ds);
  hipLaunchKernelGGL(rnn_attn_w2_kernel, gH64, dim3(1024), 0, s, w.E, ds, (int)BT, H, Gr.att_w2, Gr.att_b2);
  DFD_TRY(launch_sgemm(s, true, true, dE, H, w.Om, H, Gr.att_w1, H, H, H, (int)BT, 0.f, nullptr));  // dWa1 = dE^T Om
  DFD_TRY(launch_reduce_slabs(s, dE, (int)BT, H, Gr.att_b1, false));
  DFD_TRY(launch_sgemm(s, false, true, dE, H, P.att_w1, H, dOm2, H, (int)BT, H, H, 0.f, nullptr));  // dOm2 = dE Wa1
  hipLaunchKernelGGL(rnn_mask_bwd_kernel, dim3(ew_blocks(BT * H)), dim3(256), 0, s, dOm, dOm2, lens, B, T, H);
  DFD_HIP_CHECK(hipGetLastError());
  // BPTT.  The recurrent products into h are K-sliced (dhs/dhls) and summed by the consuming
  // cell kernel; the c gradients are updated in place (dc for the last layer, dcl inside).
  const int64_t ldr = (int64_t)T * H, slab = (int64_t)B * H;
  const int eb = ew_blocks((int64_t)B * H);
  const bool step = rnn_use_step(d);
  for (int t = T - 1; t >= 0 && step; --t) {  // k_rnn_step.hip's product, 8 slices
    for (int l = d.L - 1; l >= 0; --l) {
      const bool last = l == d.L - 1;
      const bool first = t == T - 1;
      hipLaunchKernelGGL(rnn_cell_bwd_kernel, dim3(eb), dim3(256), 0, s, last ? dOm + (int64_t)t * H : nullptr,
                         (int)ldr, (last && first) ? nullptr : spart, rnn_step_slices(), slab, last ? 0 : 1, p, seed,
                         (uint32_t)l, last ? (first ? nullptr : dc) : dcl, w.ACT[l], w.CN[l], w.CL[l],
                         w.CI[l] + (int64_t)t * H, (int)ldr, B, T, t, H, DZ[l], l > 0 ? dcl : dc);
      DFD_HIP_CHECK(hipGetLastError());
      if (l > 0 || t > 0)
        DFD_TRY(launch_rnn_dh(s, DZ[l] + (int64_t)t * 7 * H, (int64_t)T * 7 * H, w.P[l], B, H, spart));
    }
  }
  for (int t = T - 1; t >= 0 && !step; --t) {
    for (int l = d.L - 1; l >= 0; --l) {
      const bool last = l == d.L - 1;
      const bool first = t == T - 1;  // nothing flows back from step T yet
      const float* gh_a = last ? dOm + (int64_t)t * H : nullptr;
      const float* gh_b = last ? (first ? nullptr : dhs) : dhls;
      const float* gc = last ? (first ? nullptr : dc) : dcl;
      hipLaunchKernelGGL(rnn_cell_bwd_kernel, dim3(eb), dim3(256), 0, s, gh_a, (int)ldr, gh_b, sb, slab, last ? 0 : 1,
                         p, seed, (uint32_t)l, gc, w.ACT[l], w.CN[l], w.CL[l], w.CI[l] + (int64_t)t * H, (int)ldr, B,
                         T, t, H, DZ[l], l > 0 ? dcl : dc);
      DFD_HIP_CHECK(hipGetLastError());
      // gradient into the layer's hidden input: dz (rows b*T+t) @ P_l (none needed into step 0's h = 0)
      if (l > 0 || t > 0)
        DFD_TRY(launch_sgemm_part(s, false, true, DZ[l] + (int64_t)t * 7 * H, T * 7 * H, w.P[l], H, l == 0 ? dhs : dhls,
                                  B, H, 7 * H, sb, kc));
    }
  }
  // weight gradients, one GEMM per layer over all B*T rows
  for (int l = 0; l < d.L; ++l) {
    // dP[7H][H] = DZ^T UH ; dWX0[6H][IN] = DZ[:, :6H]^T X   (sums over all B*T rows)
    // as split-K partials (sgemm_wsplits slices, added in order by the scatter)
    int kp, kx = 0;
    const int np = sgemm_wsplits(7 * H, H, (int)BT, &kp);
    DFD_TRY(launch_sgemm_part(s, true, true, DZ[l], 7 * H, w.UH[l], H, dP, 7 * H, H, (int)BT, np, kp));
    int nx = 1;
    if (l == 0) {
      nx = sgemm_wsplits(6 * H, IN, (int)BT, &kx);
      DFD_TRY(launch_sgemm_part(s, true, true, DZ[0], 7 * H, order ? w.xs : x, IN, dWX0, 6 * H, IN, (int)BT, nx, kx));
    }
    DFD_TRY(launch_reduce_slabs(s, DZ[l], (int)BT, 7 * H, dbias, false));
    hipLaunchKernelGGL(rnn_scatter_kernel, dim3(ew_blocks((int64_t)6 * H * (IN + H) + (int64_t)H * H + 7 * H)),
                       dim3(256), 0, s, Gr.layer[l], l == 0 ? IN : H, H, l, dP, np, dWX0, nx, dbias);
    DFD_HIP_CHECK(hipGetLastError());
  }
  return 0;
}

int rnn_params_from_table(float* const* t, int L, RnnParams& P) {
  if (L < 1 || L > 8) { set_error("rnn: 1..8 layers supported", __FILE__, __LINE__); return -1; }
  // named_parameters() order of LogicCell: and, or, not, forget, input, cell, output (weight, bias)
  for (int l = 0; l < L; ++l) {
    float* const* q = t + 14 * l;
    RnnLayerW& w = P.layer[l];
    w.wu[0] = q[0]; w.bu[0] = q[1];    // and
    w.wu[1] = q[2]; w.bu[1] = q[3];    // or
    w.wn = q[4]; w.bn = q[5];          // not
    w.wu[2] = q[6]; w.bu[2] = q[7];    // forget
    w.wu[3] = q[8]; w.bu[3] = q[9];    // input
    w.wu[4] = q[10]; w.bu[4] = q[11];  // cell
    w.wu[5] = q[12]; w.bu[5] = q[13];  // output
  }
  float* const* q = t + 14 * L;
  P.att_w1 = q[0]; P.att_b1 = q[1]; P.att_w2 = q[2]; P.att_b2 = q[3];
  P.cls_w1 = q[4]; P.cls_b1 = q[5]; P.cls_w2 = q[6]; P.cls_b2 = q[7];
  for (int i = 0; i < 14 * L + 8; ++i)
    if (!t[i]) { set_error("rnn: null parameter pointer", __FILE__, __LINE__); return -1; }
  return 0;
}

// attention pooling used by CNNLSTMHybrid too (models.py:60-64, no mask):
//   E = tanh(O W1^T + b1) ; att = softmax_t(E w2 + b2) ; ctx = sum_t att * O
int attn_forward(hipStream_t s, const float* O, int B, int T, int H, const float* w1, const float* b1, const float* w2,
                 const float* b2, float* E, float* att, float* ctx) {
  const int64_t BT = (int64_t)B * T;
  DFD_TRY(launch_sgemm(s, false, false, O, H, w1, H, E, H, (int)BT, H, H, 0.f, b1));
  hipLaunchKernelGGL(rnn_tanh_kernel, dim3(ew_blocks(BT * H)), dim3(256), 0, s, E, BT * H);
  hipLaunchKernelGGL(rnn_attn_fwd_kernel, dim3(B), dim3(256), T * sizeof(float), s, O, E, w2, b2, T, H, att, ctx);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
// scratch: 2*BT*H + BT floats
int attn_backward(hipStream_t s, const float* O, const float* E, const float* att, const float* dctx, const float* w1,
                  const float* w2, int B, int T, int H, float* scratch, float* dO, float* gw1, float* gb1, float* gw2,
                  float* gb2) {
  const int64_t BT = (int64_t)B * T;
  float* dE = scratch;
  float* dO2 = dE + BT * H;
  float* ds = dO2 + BT * H;
  const dim3 gH((unsigned)cdiv(H, 256));
  hipLaunchKernelGGL(rnn_attn_bwd_kernel, dim3(B), dim3(256), 2 * T * sizeof(float), s, O, E, att, dctx, w2, T, H, dO,
                     dE, ds);
  hipLaunchKernelGGL(rnn_attn_w2_kernel, dim3((unsigned)cdiv(H, 64)), dim3(1024), 0, s, E, ds, (int)BT, H, gw2, gb2);
  DFD_TRY(launch_sgemm(s, true, true, dE, H, O, H, gw1, H, H, H, (int)BT, 0.f, nullptr));
  DFD_TRY(launch_reduce_slabs(s, dE, (int)BT, H, gb1, false));
  DFD_TRY(launch_sgemm(s, false, true, dE, H, w1, H, dO2, H, (int)BT, H, H, 0.f, nullptr));
  hipLaunchKernelGGL(rnn_mask_bwd_kernel, dim3(ew_blocks(BT * H)), dim3(256), 0, s, dO, dO2, (const int64_t*)nullptr,
                     B, T, H);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int colsum(hipStream_t s, const float* X, int M, int N, int ld, float* out) {
  return launch_reduce_slabs_strided(s, X, M, N, ld, out, false);
}

int64_t rnn_scratch_floats(const RnnDims& d) {  // the takes of rnn_backward, padded the same way
  const int64_t BT = (int64_t)d.B * d.T, H = d.H;
  int kc;
  const int64_t sb = bwd_splits(d, &kc);
  int kq;
  const int64_t np = sgemm_wsplits(7 * (int)H, (int)H, (int)BT, &kq), nx = sgemm_wsplits(6 * (int)H, d.IN, (int)BT, &kq);
  const int64_t sizes[] = {d.B * H, d.B * H, BT * H, BT * H, BT * H, BT, np * 7 * H * H, nx * 6 * H * d.IN, 7 * H,
                           sb * d.B * H, sb * d.B * H, d.B * H, d.B * H, (int64_t)rnn_step_slices() * d.B * H};
  int64_t n = d.L * ((BT * 7 * H + 63) & ~int64_t(63));
  for (int64_t v : sizes) n += (v + 63) & ~int64_t(63);
  return n;
}

}  // namespace dfd
