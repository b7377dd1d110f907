// Dense convolutions of CNNLSTMHybrid's frame CNN (src/models.py:26-45) on gfx950, fp32.
//
// All three passes are one implicit-GEMM kernel on v_mfma_f32_16x16x4f32 (exact fp32 products),
// 64x64 output tile per 256-thread block, BK = 16, operands staged through LDS by "operand
// policies" that gather on the fly (no im2col buffer):
//   forward  Y[m][co]  = b[co] + sum_{ky,kx,ci} X[n, oy*s-p+ky, ox*s-p+kx, ci] * W[co][ky][kx][ci]
//   dgrad    dX[m][ci] = sum_{ky,kx,co} dY[n, (iy+p-ky)/s, (ix+p-kx)/s, co] * W[co][ci][ky][kx]
//            over the taps whose output position is integral (s = 1 or 2)
//   wgrad    dW[co][(ky,kx,ci)] = sum_m dY[m][co] * X(m, ky, kx, ci)     (split over m, slabs)
// NHWC activations (the input frames are read through their strides, channels-last per
// SURVEY F10); the forward epilogue writes per-tile BatchNorm partial rows (sum, sum of squares).
// BatchNorm+ReLU+MaxPool(3, 2, 1) is one fused kernel (argmax kept for backward, first maximum
// in scan order like PyTorch's max_pool2d), BatchNorm+ReLU+global-average-pool another.
#include "cnnlstm.h"
#include "gemm_body.h"
#include "kernels.h"

namespace dfd {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int CG_T = 64, CG_K = 16;
static_assert(CG_T == kConvStatRows, "BN partial rows of conv_forward");

// Division by a launch-invariant divisor without the ~30-instruction integer division: q = x / d
// for every 32-bit x as (mulhi(x, m) + x) >> l with l = ceil(log2 d), m = 2^32 (2^l - d) / d + 1
// (round-up multiplier, 33-bit intermediate).  The gathers below divide pixel and k indices by map
// sizes and channel counts on every element of every k-step (the wgrad B gather: two per element).
struct FDiv {
  uint32_t m, l;
};
static FDiv fdiv_make(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  return FDiv{(uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d + 1) & 0xffffffffu), l};
}
__device__ __forceinline__ int fdiv(int x, FDiv f) {
  return (int)((((uint64_t)__umulhi((uint32_t)x, f.m)) + (uint32_t)x) >> f.l);
}

// ------------------------------------------------------------------ operand policies
// load(): the thread's 4 elements of the (64 rows x 16 k) tile at (r0, k0) into v / ok.
// kR == false: element e = tid + 256 i -> (r = e / 16, k = e % 16)   (contiguous along k)
// kR == true : element e -> (r = e % 64, k = e / 64)                  (contiguous along r)
struct OpRows {  // a(r, k) = p[r * ld + k]
  const float* p;
  int ld, R, K;
  static constexpr bool kR = false;
  __device__ void prep(int) {}
  __device__ void load(int r0, int k0, float (&v)[4], bool (&ok)[4]) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, r = r0 + e / CG_K, k = k0 + e % CG_K;
      ok[i] = r < R && k < K;
      v[i] = *(ok[i] ? p + (int64_t)r * ld + k : p);
    }
  }
};
struct OpCols {  // a(r, k) = p[k * ld + r]
  const float* p;
  int ld, R, K;
  static constexpr bool kR = true;
  __device__ void prep(int) {}
  __device__ void load(int r0, int k0, float (&v)[4], bool (&ok)[4]) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, r = r0 + e % CG_T, k = k0 + e / CG_T;
      ok[i] = r < R && k < K;
      v[i] = *(ok[i] ? p + (int64_t)k * ld + r : p);
    }
  }
};
// forward gather: rows = output pixels m = (n, oy, ox); k = (ky, kx, ci), ci fastest
struct OpConvA {
  const float* x;
  int64_t sn, sy, sx, sc;  // element strides of the source (n, y, x, c)
  int H, W, C, KW, S, P, Ho, Wo, R, K;
  FDiv fC, fKW, fHW, fWo;  // set by the launcher (fdiv_make)
  int iy0[4], ix0[4];
  int64_t base[4];
  static constexpr bool kR = false;
  __device__ void prep(int r0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = min(r0 + (tid + 256 * i) / CG_K, R - 1);
      const int hw = Ho * Wo, n = fdiv(r, fHW), q = r - n * hw, oy = fdiv(q, fWo), ox = q - oy * Wo;
      iy0[i] = oy * S - P;
      ix0[i] = ox * S - P;
      base[i] = (int64_t)n * sn;
    }
  }
  __device__ void load(int r0, int k0, float (&v)[4], bool (&ok)[4]) const {
    const int tid = threadIdx.x;
    const int k = k0 + (tid & 15);
    const int tap = fdiv(k, fC), ci = k - tap * C, ky = fdiv(tap, fKW), kx = tap - ky * KW;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + (tid + 256 * i) / CG_K;
      const int iy = iy0[i] + ky, ix = ix0[i] + kx;
      ok[i] = r < R && k < K && iy >= 0 && iy < H && ix >= 0 && ix < W;
      v[i] = *(ok[i] ? x + base[i] + iy * sy + ix * sx + ci * sc : x);
    }
  }
};
// dgrad gather: rows = input pixels (n, iy, ix); k = (ky, kx, co), co fastest; source dY
// [N][Ho][Wo][Co] at ((iy + p - ky) / S, (ix + p - kx) / S) where both divide (S = 1 or 2; the
// other taps of a stride-2 conv never touched this pixel and read as zero).  S is a template
// parameter: the runtime stride test in the gather's inner loop cost the stride-1 CNN-LSTM data
// gradients ~16 % (149.2 -> 154.8 ms/step after the stride-2 support went in)
template <int S>
struct OpConvDgradA {
  const float* dy;
  int Ho, Wo, Co, KW, P, H, W, R, K;
  FDiv fCo, fKW, fHW, fW;  // set by the launcher (fdiv_make)
  int iy[4], ix[4];
  int64_t base[4];
  static constexpr bool kR = false;
  __device__ void prep(int r0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = min(r0 + (tid + 256 * i) / CG_K, R - 1);
      const int hw = H * W, n = fdiv(r, fHW), q = r - n * hw;
      iy[i] = fdiv(q, fW) + P;
      ix[i] = q - fdiv(q, fW) * W + P;
      base[i] = (int64_t)n * Ho * Wo * Co;
    }
  }
  __device__ void load(int r0, int k0, float (&v)[4], bool (&ok)[4]) const {
    const int tid = threadIdx.x;
    const int k = k0 + (tid & 15);
    const int tap = fdiv(k, fCo), co = k - tap * Co, ky = fdiv(tap, fKW), kx = tap - ky * KW;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + (tid + 256 * i) / CG_K;
      const int ty = iy[i] - ky, tx = ix[i] - kx;  // = oy * S, ox * S
      int oy, ox;
      if constexpr (S == 1) {
        oy = ty; ox = tx;
        ok[i] = r < R && k < K && ty >= 0 && tx >= 0 && oy < Ho && ox < Wo;
      } else {
        oy = ty >> 1; ox = tx >> 1;
        ok[i] = r < R && k < K && ty >= 0 && tx >= 0 && ((ty | tx) & 1) == 0 && oy < Ho && ox < Wo;
      }
      v[i] = *(ok[i] ? dy + base[i] + ((int64_t)oy * Wo + ox) * Co + co : dy);
    }
  }
};
// wgrad B operand: b(j, m) = X(m, j) with j = (ky, kx, ci) (contiguous along j), m = output pixel
struct OpConvBT {
  const float* x;
  int64_t sn, sy, sx, sc;
  int H, W, C, KW, S, P, Ho, Wo, R /* = KH*KW*C */, K /* = M */;
  FDiv fHW, fWo;  // set by the launcher (fdiv_make)
  int ky, kx, ci;
  bool jok;
  static constexpr bool kR = true;
  __device__ void prep(int j0) {
    const int j = j0 + (threadIdx.x & 63);
    jok = j < R;
    const int jj = jok ? j : 0;
    const int tap = jj / C;
    ci = jj - tap * C;
    ky = tap / KW;
    kx = tap - ky * KW;
  }
  __device__ void load(int j0, int m0, float (&v)[4], bool (&ok)[4]) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + (tid >> 6) + 4 * i;
      const int hw = Ho * Wo, n = fdiv(m, fHW), q = m - n * hw, oy = fdiv(q, fWo), ox = q - oy * Wo;
      const int iy = oy * S - P + ky, ix = ox * S - P + kx;
      ok[i] = jok && m < K && iy >= 0 && iy < H && ix >= 0 && ix < W;
      v[i] = *(ok[i] ? x + (int64_t)n * sn + iy * sy + ix * sx + ci * sc : x);
    }
  }
};

template <bool kR>
__device__ __forceinline__ void cg_store(float (*S)[CG_K + 1], const float (&v)[4], const bool (&ok)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    const int r = kR ? e % CG_T : e / CG_K, k = kR ? e / CG_T : e % CG_K;
    S[r][k] = ok[i] ? v[i] : 0.f;
  }
}

enum { CEPI_STORE = 0, CEPI_STATS = 1, CEPI_SLAB = 2 };

// C[m][n] = sum_k A(m,k) B(n,k) (+ bias[n]); grid.x = n-tiles * m-tiles (n fastest), grid.y = k splits.
// Main loop: 32-deep k-steps (two 16-deep halves per operand policy load) through two LDS stages --
// the next step's gathers are in flight while this step's MFMAs run, and one barrier per step
// (four per 32 k in the single-buffered form) hands the stages over.  The MFMA sequence over k is
// unchanged (exact fp32 products); with FOLD each step's 32 products are summed into a fresh tile first.
template <class PA, class PB, int EPI, bool FOLD>
__global__ __launch_bounds__(256) void conv_gemm_kernel(PA pa, PB pb, float* __restrict__ C, int ldc, int M, int N,
                                                        int K, int ksplit, const float* __restrict__ bias,
                                                        float* __restrict__ stats) {
  __shared__ float As[2][2][CG_T][CG_K + 1], Bs[2][2][CG_T][CG_K + 1];  // [stage][half]
  __shared__ float red[2][2][CG_T];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (N + CG_T - 1) / CG_T;
  const int nt = blockIdx.x % ntn, mt = blockIdx.x / ntn;
  const int m0 = mt * CG_T, n0 = nt * CG_T;
  const int kb = blockIdx.y * ksplit, ke = min(K, kb + ksplit);
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  pa.prep(m0);
  pb.prep(n0);
  f32x4_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float va[2][4], vb[2][4];
  bool oa[2][4], ob[2][4];
  // gathers of the 32-deep step at k0 (a half past ke loads nothing)
  auto fetch = [&](int k0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kh = k0 + h * CG_K;
      if (kh < ke) {
        pa.load(m0, kh, va[h], oa[h]);
        pb.load(n0, kh, vb[h], ob[h]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) { oa[h][i] = false; ob[h][i] = false; }
      }
    }
  };
  // registers -> LDS stage st; elements past ke belong to the next split: zero
  auto commit = [&](int st, int k0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kh = k0 + h * CG_K;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = tid + 256 * i;
        const int ka = kh + (PA::kR ? e / CG_T : e % CG_K), kbb = kh + (PB::kR ? e / CG_T : e % CG_K);
        oa[h][i] = oa[h][i] && ka < ke;
        ob[h][i] = ob[h][i] && kbb < ke;
      }
      cg_store<PA::kR>(As[st][h], va[h], oa[h]);
      cg_store<PB::kR>(Bs[st][h], vb[h], ob[h]);
    }
  };
  if (kb < ke) {
    fetch(kb);
    commit(0, kb);
  }
  lds_barrier();
  int cur = 0;
  // FOLD (the ResNet-50 training convolutions): two-level summation -- each 32-deep step accumulates
  // into a fresh tile that is then added to the running sum, so the fp32 rounding error grows with
  // ~32 + K/32 terms instead of K (the train-mode BatchNorm chain amplifies conv rounding into the
  // gradients; folding only every 4th step measured 4x torch fp32's error on a BN gradient again).
  // It costs 2-5 % (the VALU reads drain the MFMA chain each step), so the CNN-LSTM convolutions,
  // whose parity bounds the plain K-order sum meets, keep FOLD = false
  auto mma = [&](f32x4_t (&d)[2][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int s = 0; s < CG_K / 4; ++s) {
        const int kk = 4 * s + (lane >> 4);
        const float a0 = As[cur][h][wm + (lane & 15)][kk], a1 = As[cur][h][wm + 16 + (lane & 15)][kk];
        const float b0 = Bs[cur][h][wn + (lane & 15)][kk], b1 = Bs[cur][h][wn + 16 + (lane & 15)][kk];
        d[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, d[0][0], 0, 0, 0);
        d[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, d[0][1], 0, 0, 0);
        d[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, d[1][0], 0, 0, 0);
        d[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, d[1][1], 0, 0, 0);
      }
  };
  for (int k0 = kb; k0 < ke; k0 += 2 * CG_K) {
    const bool more = k0 + 2 * CG_K < ke;
    if (more) fetch(k0 + 2 * CG_K);
    if constexpr (FOLD) {
      f32x4_t part[2][2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) part[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      mma(part);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] += part[a][b];
    } else {
      mma(acc);
    }
    if (more) commit(cur ^ 1, k0 + 2 * CG_K);
    lds_barrier();
    cur ^= 1;
  }
  float* Cz = EPI == CEPI_SLAB ? C + (int64_t)blockIdx.y * M * N : C;
  float cs[2] = {0.f, 0.f}, cq[2] = {0.f, 0.f};
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
          acc[a][b][r] = v;
          Cz[(int64_t)m * ldc + n] = v;
          if (EPI == CEPI_STATS) cs[b] += v;
        }
      }
  if constexpr (EPI == CEPI_STATS) {
    // BatchNorm partials of the 64-row tile, centred: (sum, M2 = sum (v - tile mean)^2) per column,
    // merged over tiles in fp64 by the finalize (Chan) -- the one-pass sum of squares cancels when
    // |mean| >> std.  Per column: lanes with equal (lane & 15) hold its 4-row groups -> xor 16, 32;
    // then the two row-halves of the tile (waves 0/1 and 2/3) in a fixed order through LDS
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      cs[b] += __shfl_xor(cs[b], 16, 64); cs[b] += __shfl_xor(cs[b], 32, 64);
      if (lane < 16) red[wave >> 1][0][wn + b * 16 + lane] = cs[b];
    }
    lds_barrier();
    const float inv_n = 1.0f / (float)min(CG_T, M - m0);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int cl = wn + b * 16 + (lane & 15);
      const float tmean = (red[0][0][cl] + red[1][0][cl]) * inv_n;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm + a * 16 + 4 * (lane >> 4) + r, n = n0 + cl;
          if (m < M && n < N) {
            const float d = acc[a][b][r] - tmean;
            cq[b] += d * d;
          }
        }
      cq[b] += __shfl_xor(cq[b], 16, 64); cq[b] += __shfl_xor(cq[b], 32, 64);
      if (lane < 16) red[wave >> 1][1][wn + b * 16 + lane] = cq[b];
    }
    lds_barrier();
    if (tid < 2 * CG_T) {
      const int which = tid / CG_T, c = tid % CG_T;
      if (n0 + c < N) stats[((int64_t)mt * 2 + which) * N + n0 + c] = red[0][which][c] + red[1][which][c];
    }
  }
}

template <class PA, class PB, int EPI>
static int conv_gemm(hipStream_t s, const PA& pa, const PB& pb, float* C, int ldc, int M, int N, int K, int splits,
                     const float* bias, float* stats, bool fold) {
  const int64_t tiles = (int64_t)cdiv(N, CG_T) * cdiv(M, CG_T);
  if (tiles > 0x7fffffff) { set_error("conv: too many tiles", __FILE__, __LINE__); return -1; }
  const int ksplit = cdiv(cdiv(K, splits), CG_K) * CG_K;
  splits = cdiv(K, ksplit);
  if (fold)
    hipLaunchKernelGGL((conv_gemm_kernel<PA, PB, EPI, true>), dim3((unsigned)tiles, (unsigned)splits), dim3(256), 0, s,
                       pa, pb, C, ldc, M, N, K, ksplit, bias, stats);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<PA, PB, EPI, false>), dim3((unsigned)tiles, (unsigned)splits), dim3(256), 0, s,
                       pa, pb, C, ldc, M, N, K, ksplit, bias, stats);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ weight layouts
// W [Co][Ci][KH][KW] -> Wf [Co][KH][KW][Ci] (forward) and Wd [Ci][KH][KW][Co] (dgrad)
__global__ void conv_pack_kernel(const float* __restrict__ w, int Co, int Ci, int KK, float* __restrict__ wf,
                                 float* __restrict__ wd) {
  const int64_t n = (int64_t)Co * Ci * KK;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int co = (int)(i / ((int64_t)Ci * KK));
    const int rem = (int)(i - (int64_t)co * Ci * KK), ci = rem / KK, t = rem - ci * KK;
    const float v = w[i];
    wf[((int64_t)co * KK + t) * Ci + ci] = v;
    if (wd) wd[((int64_t)ci * KK + t) * Co + co] = v;
  }
}
// gw [Co][Ci][KH][KW] = sum_s slab[s][co][(t, ci)]
__global__ void conv_unpack_grad_kernel(const float* __restrict__ slab, int splits, int Co, int Ci, int KK,
                                        float* __restrict__ gw) {
  const int64_t n = (int64_t)Co * Ci * KK;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int co = (int)(i / ((int64_t)Ci * KK));
    const int rem = (int)(i - (int64_t)co * Ci * KK), ci = rem / KK, t = rem - ci * KK;
    const int64_t j = ((int64_t)co * KK + t) * Ci + ci;
    float a = 0.f;
    for (int sp = 0; sp < splits; ++sp) a += slab[(int64_t)sp * n + j];
    gw[i] = a;
  }
}

// ------------------------------------------------------------------ BN + ReLU + MaxPool(3,2,1)
// mu given: the centred form (Y - mu) * sc + sh (sh = beta), as torch's (y - mean) * invstd * gamma + beta
// (the ResNet-50 training member: y * sc + (beta - mu * sc) cancels where |mean| >> std)
__device__ __forceinline__ float bn_z(float y, const float* mu, float sc, float sh, int c) {
  return mu ? (y - mu[c]) * sc + sh : y * sc + sh;
}
__global__ void bn_relu_pool_fwd_kernel(const float* __restrict__ Y, const float* __restrict__ mu,
                                        const float* __restrict__ sc, const float* __restrict__ sh, int N, int H,
                                        int W, int C, int Ho, int Wo, float* __restrict__ P,
                                        uint8_t* __restrict__ arg) {
  const int64_t n = (int64_t)N * Ho * Wo * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int64_t pix = i / C;
    const int ox = (int)(pix % Wo);
    const int64_t t = pix / Wo;
    const int oy = (int)(t % Ho);
    const int f = (int)(t / Ho);
    float best = -INFINITY;
    int bi = 0;
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * 2 - 1 + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * 2 - 1 + kx;
        if (ix < 0 || ix >= W) continue;
        const float z = fmaxf(bn_z(Y[(((int64_t)f * H + iy) * W + ix) * C + c], mu, sc[c], sh[c], c), 0.f);
        if (z > best) { best = z; bi = ky * 3 + kx; }
      }
    }
    P[i] = best;
    arg[i] = (uint8_t)bi;
  }
}
// g[n][iy][ix][c] = relu'(z) * sum of dP over the windows whose argmax is (iy, ix)
__global__ void bn_relu_pool_bwd_kernel(const float* __restrict__ dP, const uint8_t* __restrict__ arg,
                                        const float* __restrict__ Y, const float* __restrict__ mu,
                                        const float* __restrict__ sc,
                                        const float* __restrict__ sh, int N, int H, int W, int C, int Ho, int Wo,
                                        float* __restrict__ g) {
  const int64_t n = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int64_t pix = i / C;
    const int ix = (int)(pix % W);
    const int64_t t = pix / W;
    const int iy = (int)(t % H);
    const int f = (int)(t / H);
    float a = 0.f;
    const int oy_lo = max(0, (iy) / 2 - 0), oy_hi = min(Ho - 1, (iy + 1) / 2);
    const int ox_lo = max(0, (ix) / 2 - 0), ox_hi = min(Wo - 1, (ix + 1) / 2);
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      const int ky = iy - (oy * 2 - 1);
      if (ky < 0 || ky > 2) continue;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const int kx = ix - (ox * 2 - 1);
        if (kx < 0 || kx > 2) continue;
        const int64_t o = (((int64_t)f * Ho + oy) * Wo + ox) * C + c;
        if (arg[o] == ky * 3 + kx) a += dP[o];
      }
    }
    const float z = bn_z(Y[i], mu, sc[c], sh[c], c);
    g[i] = z > 0.f ? a : 0.f;
  }
}

// ------------------------------------------------------------------ BN + ReLU + global average pool
// feat[f][c] = mean_hw relu(Y*sc+sh); one block per (frame, 64-channel group), fixed-order sums
__global__ void bn_relu_gap_fwd_kernel(const float* __restrict__ Y, const float* __restrict__ sc,
                                       const float* __restrict__ sh, int HW, int C, float* __restrict__ feat) {
  __shared__ float red[4][64];
  const int f = blockIdx.x, c = blockIdx.y * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  float a = 0.f;
  if (c < C)
    for (int p = q; p < HW; p += 4) a += fmaxf(Y[((int64_t)f * HW + p) * C + c] * sc[c] + sh[c], 0.f);
  red[q][threadIdx.x & 63] = a;
  __syncthreads();
  if (q == 0 && c < C)
    feat[(int64_t)f * C + c] = (((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                                red[3][threadIdx.x]) / (float)HW;
}
__global__ void bn_relu_gap_bwd_kernel(const float* __restrict__ dfeat, const float* __restrict__ Y,
                                       const float* __restrict__ sc, const float* __restrict__ sh, int64_t M, int HW,
                                       int C, float* __restrict__ g) {
  const int64_t n = M * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int64_t row = i / C;
    const float z = Y[i] * sc[c] + sh[c];
    g[i] = z > 0.f ? dfeat[(row / HW) * C + c] / (float)HW : 0.f;
  }
}

static int ew(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 4096)); }

// ------------------------------------------------------------------ wide-vector tile loops
// The stride-1 KxK layers with Cin, Cout % 64 (CNNLSTMHybrid's conv 2..4: 5x5 64->128, 3x3 128->256,
// 3x3 256->512 over dense NHWC maps) run the EfficientNet-B0 tile loops of gemm_body.h in their fp32
// form (v_mfma_f32_16x16x4f32, exact fp32 products) with the implicit-GEMM gather ConvGather: one tap
// per 32-deep k-step, whole 32-B channel vectors per load instead of the per-element gathers above,
// 128 x 128 / 128 x 64 tiles of two wave rows.  The forward's BN partials are centred per wave row
// (STATS = 2: 64 consecutive rows each, the same (sum, M2) rows conv_gemm's epilogue writes).
constexpr int CG32_BK = 32;
template <int EPI, int BM, int BN, int WN, int OCC, bool FOLD = false>
__global__ __launch_bounds__(256, OCC) void cg32_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wf,
                                                          const float* __restrict__ bias, float* __restrict__ y,
                                                          int64_t M, int N, int K, float* __restrict__ stats,
                                                          int64_t tiles_m, int ntn, ConvGather cg) {
  using G = GemmCfg<float, BM, BN, WN, 2, CG32_BK>;
  static_assert(BM / G::WM == kConvStatRows, "BN partial rows of conv_forward");
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  __shared__ float st_part[G::WM][2][BN];
  pw_gemm_body<float, PRO_NONE, 2, EPI, BM, BN, WN, 2, CG32_BK, 1, FOLD>(
      x, wf, y, nullptr, bias, nullptr, M, N, K, Pro{}, stats, tiles_m, ntn, (int)blockIdx.x, (int)gridDim.x, smem,
      nullptr, nullptr, &st_part[0][0][0], nullptr, cg);
}
template <int BM, int BN, int WN, int OCC, bool FOLD = false, int EPI = 0>
__global__ __launch_bounds__(256, OCC) void cg32_dgrad_kernel(const float* __restrict__ dy, const float* __restrict__ wd,
                                                            float* __restrict__ dx, const float* __restrict__ res,
                                                            int64_t M, int N, int K, int64_t tiles_m, int ntn,
                                                            ConvGather cg) {
  using G = GemmCfg<float, BM, BN, WN, 2, CG32_BK>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  pw_gemm_body<float, PRO_NONE, 0, EPI, BM, BN, WN, 2, CG32_BK, 1, FOLD>(dy, wd, dx, res, nullptr, nullptr, M, N, K, Pro{},
                                                                 nullptr, tiles_m, ntn, (int)blockIdx.x,
                                                                 (int)gridDim.x, smem, nullptr, nullptr, nullptr,
                                                                 nullptr, cg);
}
#ifndef DFD_CG32_WPF  // m-steps of loads in flight in the weight gradient (2: +0.2 ms, ab_cg32_r06ah.txt)
#define DFD_CG32_WPF 1
#endif
#ifndef DFD_CG32_N64  // 64-wide data gradients: 1 = 256 x 64 tiles of 4 x 1 waves (CNN-LSTM step -0.25..-0.9 ms, ab_cg32_r06ah.txt), 0 = 128 x 64 of 2 x 2
#define DFD_CG32_N64 1
#endif
template <bool FOLD>
__global__ __launch_bounds__(256, 2) void cg32_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           int64_t M, int N, int K, float* __restrict__ slab, int tnk,
                                                           int64_t m_per_split, ConvGather cg) {
  __shared__ __attribute__((aligned(16))) char smem[WgCfg<float>::SMEM];
  pw_wgrad_body<float, PRO_NONE, DFD_CG32_WPF, 1, FOLD>(dy, x, M, N, K, Pro{}, slab, tnk, m_per_split,
                                       (int)(blockIdx.y * gridDim.x + blockIdx.x), (int)(gridDim.x * gridDim.y),
                                       (int)gridDim.x, smem, cg);
}

static bool dense_nhwc(const int64_t (&xs)[4], int H, int W, int C) {
  return xs[3] == 1 && xs[2] == C && xs[1] == (int64_t)W * C && xs[0] == (int64_t)H * W * C;
}
// the wide-vector path's shapes (above); DFD_CG32 = 0 keeps every layer on conv_gemm (A/B builds)
#ifndef DFD_CG32
#define DFD_CG32 1
#endif
// The ResNet-50 training convolutions (g.fold) take the two-level K / M sum (FOLD): their train-mode BN
// amplifies conv rounding, and the plain K-order sum measured 3-5x torch fp32's error on the layer4.2
// gradients.  Stride 2 through the gather's parity test.
#ifndef DFD_CG32_FOLD  // 1: the fold convolutions (ResNet-50 fp32 training) on these loops too (A/B build switch)
#define DFD_CG32_FOLD 1
#endif
static bool cg32_ok(const ConvGeom& g) {
  return DFD_CG32 && (!g.fold || DFD_CG32_FOLD) && (g.S == 1 || g.S == 2) && g.KH == g.KW && (g.KH & 1) &&
         g.P == g.KH / 2 && g.Ci % 64 == 0 && g.Co % 64 == 0 && (int64_t)g.N * g.H * g.W < (1ll << 31);
}
static ConvGather cg32_gather(int C, int H, int W, int Ho, int Wo, int kw, int s, int p, int dgrad) {
  ConvGather c{};
  c.C = C; c.H = H; c.W = W; c.Ho = Ho; c.Wo = Wo; c.KW = kw; c.S = s; c.P = p; c.dgrad = dgrad;
  conv_gather_fdiv((uint32_t)(Ho * Wo), c.mhw, c.lhw);
  conv_gather_fdiv((uint32_t)Wo, c.mw, c.lw);
  return c;
}
// 128 x 128 tiles where N > 64, else 128 x 64; a persistent grid of <= 1024 workgroups
template <bool FWD>
static int cg32_launch(hipStream_t s, const float* a, const float* b, const float* bias, float* c, int64_t M, int N,
                       int K, float* stats, const ConvGather& cg, int* stat_rows, bool fold,
                       const float* res = nullptr) {
  if (fold) {  // 128 x 64 tiles (the fresh per-step tile doubles the accumulators)
    const int ntn = cdiv(N, 64);
    const int64_t tiles_m = cdiv64(M, 128);
    const int gx = (int)std::min<int64_t>(tiles_m, std::max<int64_t>(1, 1024 / ntn));
    if (FWD) {
      if (stat_rows) *stat_rows = (int)cdiv64(M, kConvStatRows);
      if (bias)
        hipLaunchKernelGGL((cg32_fwd_kernel<EPI_BIAS, 128, 64, 2, 2, true>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, a,
                           b, bias, c, M, N, K, stats, tiles_m, ntn, cg);
      else
        hipLaunchKernelGGL((cg32_fwd_kernel<0, 128, 64, 2, 2, true>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, a, b,
                           bias, c, M, N, K, stats, tiles_m, ntn, cg);
    } else {
      if (res)  // the bottleneck's residual path added in the epilogue
        hipLaunchKernelGGL((cg32_dgrad_kernel<128, 64, 2, 2, true, EPI_RESID>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s,
                           a, b, c, res, M, N, K, tiles_m, ntn, cg);
      else
        hipLaunchKernelGGL((cg32_dgrad_kernel<128, 64, 2, 2, true>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, a, b, c,
                           res, M, N, K, tiles_m, ntn, cg);
    }
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
  const int bn = N > 64 ? 128 : 64;
  const int ntn = cdiv(N, bn);
  const int64_t tiles_m = cdiv64(M, 128);
  const int gx = (int)std::min<int64_t>(tiles_m, std::max<int64_t>(1, 1024 / ntn));
  if (stat_rows) *stat_rows = (int)cdiv64(M, kConvStatRows);
  if (FWD) {  // the conv bias (CNNLSTMHybrid) is optional (ResNet-50: none)
#define DFD_CG32F(E)                                                                                                 \
  if (bn == 128)                                                                                                     \
    hipLaunchKernelGGL((cg32_fwd_kernel<E, 128, 128, 2, 2>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, a, b, bias, \
                       c, M, N, K, stats, tiles_m, ntn, cg);                                                         \
  else                                                                                                               \
    hipLaunchKernelGGL((cg32_fwd_kernel<E, 128, 64, 2, 3>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, a, b, bias,  \
                       c, M, N, K, stats, tiles_m, ntn, cg);
    if (bias) { DFD_CG32F(EPI_BIAS) } else { DFD_CG32F(0) }
#undef DFD_CG32F
  } else {
    if (bn == 128) {
      hipLaunchKernelGGL((cg32_dgrad_kernel<128, 128, 2, 2>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, a, b, c, res, M,
                         N, K, tiles_m, ntn, cg);
    } else if (DFD_CG32_N64) {
      const int64_t t256 = cdiv64(M, 256);
      const int g2 = (int)std::min<int64_t>(t256, std::max<int64_t>(1, 1024 / ntn));
      hipLaunchKernelGGL((cg32_dgrad_kernel<256, 64, 1, 2>), dim3((unsigned)(g2 * ntn)), dim3(256), 0, s, a, b, c, res, M,
                         N, K, t256, ntn, cg);
    } else {
      hipLaunchKernelGGL((cg32_dgrad_kernel<128, 64, 2, 3>), dim3((unsigned)(gx * ntn)), dim3(256), 0, s, a, b, c, res, M,
                         N, K, tiles_m, ntn, cg);
    }
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
// the weight gradient's M-split: ~512 workgroups of 64 x 64 tiles, 128-row multiples
static void cg32_wgrad_split(int64_t M, int N, int K, int64_t slab_floats, int* tnk, int* tiles, int64_t* splits,
                             int64_t* mps) {
  *tnk = cdiv(K, 64);
  *tiles = cdiv(N, 64) * *tnk;
  int64_t sp = std::max<int64_t>(1, 512 / *tiles);
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, cdiv64(M, 128)));
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, slab_floats / ((int64_t)N * K)));
  *mps = cdiv64(cdiv64(std::max<int64_t>(M, 1), sp), 128) * 128;
  *splits = cdiv64(std::max<int64_t>(M, 1), *mps);
}

// ------------------------------------------------------------------ layer launchers
// a 1x1 stride-1 unpadded convolution over a dense NHWC input is a plain GEMM on the activation rows
static bool plain_1x1(const ConvGeom& g, const int64_t (&xs)[4]) {
  return g.KH == 1 && g.KW == 1 && g.S == 1 && g.P == 0 && xs[3] == 1 && xs[2] == g.Ci &&
         xs[1] == (int64_t)g.W * g.Ci && xs[0] == (int64_t)g.H * g.W * g.Ci;
}

int conv_forward(hipStream_t s, const ConvGeom& g, const float* x, const int64_t (&xs)[4], const float* w,
                 const float* bias, float* wf, float* Y, float* stats, int* stat_rows) {
  const int KK = g.KH * g.KW;
  hipLaunchKernelGGL(conv_pack_kernel, dim3(ew((int64_t)g.Co * g.Ci * KK)), dim3(256), 0, s, w, g.Co, g.Ci, KK, wf,
                     (float*)nullptr);
  const int M = g.N * g.Ho * g.Wo, K = KK * g.Ci;
  if (cg32_ok(g) && dense_nhwc(xs, g.H, g.W, g.Ci) && stats) {
    const ConvGather cg = cg32_gather(g.Ci, g.H, g.W, g.Ho, g.Wo, g.KW, g.S, g.P, 0);
    DFD_TRY(cg32_launch<true>(s, x, wf, bias, Y, M, g.Co, K, stats, cg, stat_rows, g.fold));
    return 0;
  }
  OpRows pb{wf, K, g.Co, K};
  if (stat_rows) *stat_rows = cdiv(M, CG_T);
  if (plain_1x1(g, xs))  // the activation rows themselves are the A operand (no gather index math)
    return conv_gemm<OpRows, OpRows, CEPI_STATS>(s, OpRows{x, g.Ci, M, K}, pb, Y, g.Co, M, g.Co, K, 1, bias, stats,
                                                 g.fold);
  OpConvA pa{x, xs[0], xs[1], xs[2], xs[3], g.H, g.W, g.Ci, g.KW, g.S, g.P, g.Ho, g.Wo, M, K};
  pa.fC = fdiv_make(g.Ci); pa.fKW = fdiv_make(g.KW); pa.fHW = fdiv_make(g.Ho * g.Wo); pa.fWo = fdiv_make(g.Wo);
  return conv_gemm<OpConvA, OpRows, CEPI_STATS>(s, pa, pb, Y, g.Co, M, g.Co, K, 1, bias, stats, g.fold);
}

int conv_dgrad(hipStream_t s, const ConvGeom& g, const float* dY, const float* w, float* wf, float* wd, float* dX,
               const float* res) {
  if (g.S != 1 && g.S != 2) { set_error("conv dgrad: stride 1 or 2", __FILE__, __LINE__); return -1; }
  const int KK = g.KH * g.KW;
  hipLaunchKernelGGL(conv_pack_kernel, dim3(ew((int64_t)g.Co * g.Ci * KK)), dim3(256), 0, s, w, g.Co, g.Ci, KK, wf,
                     wd);
  const int M = g.N * g.H * g.W, K = KK * g.Co;
  if (cg32_ok(g)) {  // rows: input pixels; source: dY [N][Ho][Wo][Co]
    const ConvGather cg = cg32_gather(g.Co, g.Ho, g.Wo, g.H, g.W, g.KW, g.S, g.P, 1);
    if (res && !g.fold) { set_error("conv dgrad: residual form is the fold (ResNet-50) path's", __FILE__, __LINE__); return -1; }
    return cg32_launch<false>(s, dY, wd, nullptr, dX, M, g.Ci, K, nullptr, cg, nullptr, g.fold, res);
  }
  if (res) { set_error("conv dgrad: residual form needs Cin, Cout % 64", __FILE__, __LINE__); return -1; }
  OpRows pb{wd, K, g.Ci, K};
  if (g.KH == 1 && g.KW == 1 && g.S == 1 && g.P == 0)  // dY rows are the A operand
    return conv_gemm<OpRows, OpRows, CEPI_STORE>(s, OpRows{dY, g.Co, M, K}, pb, dX, g.Ci, M, g.Ci, K, 1, nullptr,
                                                 nullptr, g.fold);
  auto run = [&](auto pa) {
    pa.dy = dY; pa.Ho = g.Ho; pa.Wo = g.Wo; pa.Co = g.Co; pa.KW = g.KW; pa.P = g.P; pa.H = g.H; pa.W = g.W;
    pa.R = M; pa.K = K;
    pa.fCo = fdiv_make(g.Co); pa.fKW = fdiv_make(g.KW); pa.fHW = fdiv_make(g.H * g.W); pa.fW = fdiv_make(g.W);
    return conv_gemm<decltype(pa), OpRows, CEPI_STORE>(s, pa, pb, dX, g.Ci, M, g.Ci, K, 1, nullptr, nullptr, g.fold);
  };
  return g.S == 1 ? run(OpConvDgradA<1>{}) : run(OpConvDgradA<2>{});
}

// pixel splits of the weight gradient (each its own slab of Co x Kp partial sums)
static int conv_wgrad_splits(const ConvGeom& g) {
  const int M = g.N * g.Ho * g.Wo, Kp = g.KH * g.KW * g.Ci;
  const int tiles = cdiv(g.Co, CG_T) * cdiv(Kp, CG_T);
  return std::max(1, std::min(cdiv(M, 256), 2048 / std::max(tiles, 1)));
}
int64_t conv_wgrad_slab_floats(const ConvGeom& g) {
  return (int64_t)conv_wgrad_splits(g) * g.Co * g.KH * g.KW * g.Ci;
}

int conv_wgrad(hipStream_t s, const ConvGeom& g, const float* x, const int64_t (&xs)[4], const float* dY, float* slab,
               int64_t slab_cap, float* gw) {
  const int KK = g.KH * g.KW;
  const int M = g.N * g.Ho * g.Wo, Kp = KK * g.Ci;  // GEMM: C[Co][Kp] = sum_m dY[m][co] X(m, kp)
  const int64_t per = (int64_t)g.Co * Kp;
  if (cg32_ok(g) && dense_nhwc(xs, g.H, g.W, g.Ci)) {
    int tnk, tiles;
    int64_t sp, mps;
    cg32_wgrad_split(M, g.Co, Kp, slab_cap, &tnk, &tiles, &sp, &mps);
    const ConvGather cg = cg32_gather(g.Ci, g.H, g.W, g.Ho, g.Wo, g.KW, g.S, g.P, 0);
    if (g.fold)
      hipLaunchKernelGGL(cg32_wgrad_kernel<true>, dim3((unsigned)tiles, (unsigned)sp), dim3(256), 0, s, dY, x,
                         (int64_t)M, g.Co, Kp, slab, tnk, mps, cg);
    else
      hipLaunchKernelGGL(cg32_wgrad_kernel<false>, dim3((unsigned)tiles, (unsigned)sp), dim3(256), 0, s, dY, x,
                         (int64_t)M, g.Co, Kp, slab, tnk, mps, cg);
    DFD_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(conv_unpack_grad_kernel, dim3(ew(per)), dim3(256), 0, s, slab, (int)sp, g.Co, g.Ci, KK, gw);
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
  int splits = conv_wgrad_splits(g);
  splits = (int)std::max<int64_t>(1, std::min<int64_t>(splits, slab_cap / per));
  OpCols pa{dY, g.Co, g.Co, M};
  const int ksplit = cdiv(cdiv(M, splits), CG_K) * CG_K;
  const int used = cdiv(M, ksplit);
  if (plain_1x1(g, xs)) {  // b(j, m) = x[m][j]: the activation rows, read column-wise
    DFD_TRY((conv_gemm<OpCols, OpCols, CEPI_SLAB>(s, pa, OpCols{x, g.Ci, Kp, M}, slab, Kp, g.Co, Kp, M, splits, nullptr,
                                                  nullptr, g.fold)));
  } else {
    OpConvBT pb{x, xs[0], xs[1], xs[2], xs[3], g.H, g.W, g.Ci, g.KW, g.S, g.P, g.Ho, g.Wo, Kp, M};
    pb.fHW = fdiv_make(g.Ho * g.Wo); pb.fWo = fdiv_make(g.Wo);
    DFD_TRY((conv_gemm<OpCols, OpConvBT, CEPI_SLAB>(s, pa, pb, slab, Kp, g.Co, Kp, M, splits, nullptr, nullptr,
                                                    g.fold)));
  }
  hipLaunchKernelGGL(conv_unpack_grad_kernel, dim3(ew(per)), dim3(256), 0, s, slab, used, g.Co, g.Ci, KK, gw);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// The same two passes on 4-channel vectors: one row of the output (forward) / input (backward) map
// (a run of workgroups per row), 32-bit index math (the element-wise forms above divide 64-bit indices six times
// per element).  Same window scan order, same first-maximum rule, same summation order: identical
// results.  C % 4 == 0.
__global__ __launch_bounds__(256) void bn_relu_pool_fwd4_kernel(const float* __restrict__ Y, const float* __restrict__ mu,
                                                                const float* __restrict__ sc, const float* __restrict__ sh,
                                                                int H, int W, int C, int Ho, int Wo,
                                                                float* __restrict__ P, uint8_t* __restrict__ arg) {
  const int C4 = C >> 2, xb = (Wo * C4 + 255) >> 8;  // blocks per output row
  const int row = blockIdx.x / xb, e = (blockIdx.x - row * xb) * 256 + threadIdx.x;
  if (e >= Wo * C4) return;
  const int f = row / Ho, oy = row - f * Ho;
  const int ox = e / C4, c = (e - ox * C4) * 4;
  float scv[4], shv[4], best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int bi[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 4; ++j) { scv[j] = sc[c + j]; shv[j] = sh[c + j]; }
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * 2 - 1 + ky;
    if (iy < 0 || iy >= H) continue;
    const float* yr = Y + ((int64_t)f * H + iy) * W * C + c;
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * 2 - 1 + kx;
      if (ix < 0 || ix >= W) continue;
      const float4 y4 = *reinterpret_cast<const float4*>(yr + (int64_t)ix * C);
      const float yv[4] = {y4.x, y4.y, y4.z, y4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float z = fmaxf(bn_z(yv[j], mu, scv[j], shv[j], c + j), 0.f);
        if (z > best[j]) { best[j] = z; bi[j] = ky * 3 + kx; }
      }
    }
  }
  const int64_t o = ((int64_t)row * Wo + ox) * C + c;
  *reinterpret_cast<float4*>(P + o) = make_float4(best[0], best[1], best[2], best[3]);
  *reinterpret_cast<uchar4*>(arg + o) = make_uchar4((unsigned char)bi[0], (unsigned char)bi[1], (unsigned char)bi[2],
                                                    (unsigned char)bi[3]);
}

__global__ __launch_bounds__(256) void bn_relu_pool_bwd4_kernel(const float* __restrict__ dP, const uint8_t* __restrict__ arg,
                                                                const float* __restrict__ Y, const float* __restrict__ mu,
                                                                const float* __restrict__ sc, const float* __restrict__ sh,
                                                                int H, int W, int C, int Ho, int Wo, float* __restrict__ g) {
  const int C4 = C >> 2, xb = (W * C4 + 255) >> 8;  // blocks per input row
  const int row = blockIdx.x / xb, e = (blockIdx.x - row * xb) * 256 + threadIdx.x;
  if (e >= W * C4) return;
  const int f = row / H, iy = row - f * H;
  const int ix = e / C4, c = (e - ix * C4) * 4;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  const int oy_lo = max(0, iy / 2), oy_hi = min(Ho - 1, (iy + 1) / 2);
  const int ox_lo = max(0, ix / 2), ox_hi = min(Wo - 1, (ix + 1) / 2);
  for (int oy = oy_lo; oy <= oy_hi; ++oy) {
    const int ky = iy - (oy * 2 - 1);
    if (ky < 0 || ky > 2) continue;
    for (int ox = ox_lo; ox <= ox_hi; ++ox) {
      const int kx = ix - (ox * 2 - 1);
      if (kx < 0 || kx > 2) continue;
      const int64_t o = (((int64_t)f * Ho + oy) * Wo + ox) * C + c;
      const uchar4 a4 = *reinterpret_cast<const uchar4*>(arg + o);
      const float4 d4 = *reinterpret_cast<const float4*>(dP + o);
      const int tap = ky * 3 + kx;
      if (a4.x == tap) a[0] += d4.x;
      if (a4.y == tap) a[1] += d4.y;
      if (a4.z == tap) a[2] += d4.z;
      if (a4.w == tap) a[3] += d4.w;
    }
  }
  const int64_t i = ((int64_t)row * W + ix) * C + c;
  const float4 y4 = *reinterpret_cast<const float4*>(Y + i);
  const float yv[4] = {y4.x, y4.y, y4.z, y4.w};
  float out[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) out[j] = bn_z(yv[j], mu, sc[c + j], sh[c + j], c + j) > 0.f ? a[j] : 0.f;
  *reinterpret_cast<float4*>(g + i) = make_float4(out[0], out[1], out[2], out[3]);
}

int bn_relu_pool_fwd(hipStream_t s, const float* Y, const float* mu, const float* sc, const float* sh, int N, int H,
                     int W, int C, int Ho, int Wo, float* P, uint8_t* arg) {
  if (C % 4 == 0 && (int64_t)N * Ho * cdiv(Wo * (C / 4), 256) < (1ll << 31)) {
    hipLaunchKernelGGL(bn_relu_pool_fwd4_kernel, dim3((unsigned)((int64_t)N * Ho * cdiv(Wo * (C / 4), 256))), dim3(256), 0,
                       s, Y, mu, sc, sh, H, W, C, Ho, Wo, P, arg);
  } else {
    hipLaunchKernelGGL(bn_relu_pool_fwd_kernel, dim3(ew((int64_t)N * Ho * Wo * C)), dim3(256), 0, s, Y, mu, sc, sh, N, H,
                       W, C, Ho, Wo, P, arg);
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int bn_relu_pool_bwd(hipStream_t s, const float* dP, const uint8_t* arg, const float* Y, const float* mu,
                     const float* sc, const float* sh, int N, int H, int W, int C, int Ho, int Wo, float* g) {
  if (C % 4 == 0 && (int64_t)N * H * cdiv(W * (C / 4), 256) < (1ll << 31)) {
    hipLaunchKernelGGL(bn_relu_pool_bwd4_kernel, dim3((unsigned)((int64_t)N * H * cdiv(W * (C / 4), 256))), dim3(256), 0,
                       s, dP, arg, Y, mu, sc, sh, H, W, C, Ho, Wo, g);
  } else {
    hipLaunchKernelGGL(bn_relu_pool_bwd_kernel, dim3(ew((int64_t)N * H * W * C)), dim3(256), 0, s, dP, arg, Y, mu, sc,
                       sh, N, H, W, C, Ho, Wo, g);
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int bn_relu_gap_fwd(hipStream_t s, const float* Y, const float* sc, const float* sh, int N, int HW, int C,
                    float* feat) {
  hipLaunchKernelGGL(bn_relu_gap_fwd_kernel, dim3(N, cdiv(C, 64)), dim3(256), 0, s, Y, sc, sh, HW, C, feat);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int bn_relu_gap_bwd(hipStream_t s, const float* dfeat, const float* Y, const float* sc, const float* sh, int N,
                    int HW, int C, float* g) {
  hipLaunchKernelGGL(bn_relu_gap_bwd_kernel, dim3(ew((int64_t)N * HW * C)), dim3(256), 0, s, dfeat, Y, sc, sh,
                     (int64_t)N * HW, HW, C, g);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
