// ViT-B/16 + SimpleGCN kernels (DeepfakeModel, src/models.py:88-107, 199-291; timm
// vit_base_patch16_224 restated in oracle/vit_cpu.py).  The linear layers run on the pointwise
// MFMA GEMM (k_gemm.hip: launch_tf_gemm / launch_pw_wgrad); this file holds everything else:
//
//   bgemm_kernel      batched strided GEMM for the attention products (QK^T, PV and their
//                     backward), operands addressed as base + (b / inner)*s_outer + (b % inner)*s_inner
//   softmax fwd/bwd   one wave per score row
//   layernorm fwd/bwd one wave per token row; gamma/beta gradients as fixed-order partial rows
//   patch gather, token assembly (+cls, +pos) and its backward
//   weight cast (+ LDS-tiled transpose) into the GEMM operand layouts
//   GCN head: A_norm mixing, bias/ReLU/dropout, node mean (fp32)
#include "kernels.h"
#include "vit.h"

namespace dfd {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// batched GEMM: C[b] (M x N, ldc) = alpha * opA(A[b]) (M x K) * opB(B[b]) (K x N)
//   TA = false: A stored [m][k] (k contiguous, lda);  TA = true: stored [k][m] (m contiguous)
//   TB = true : B stored [n][k] (k contiguous, ldb);  TB = false: stored [k][n] (n contiguous)
// 64 x 64 output tile, 4 waves (2 x 2 of 32 x 32), K step 32; LDS holds both tiles K-contiguous.
// Every operand row must stay inside its allocation for the 8-wide vector reads: callers pad
// the contiguous dimension to a multiple of 8 (score rows are 200 wide for 197 tokens).
constexpr int BG_T = 64, BG_K = 32;

template <typename T>
struct BgCfg {
  static constexpr int LS = BG_K + (sizeof(T) == 2 ? 8 : 4);
};

// load 8 contiguous elements (masked per element against `lim`) into registers as floats
template <typename T>
__device__ __forceinline__ void bg_ld(const T* p, int first, int lim, bool rowok, float (&v)[8]) {
  if (rowok && first + 8 <= lim) {
    ld8(p, v);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (rowok && first + j < lim) ? Tr<T>::to_f(p[j]) : 0.f;
  }
}

template <typename T, bool TA, bool TB>
__global__ __launch_bounds__(256) void bgemm_kernel(BgOp a, BgOp b, BgOp c, int M, int N, int K, float alpha,
                                                    const T* __restrict__ A, const T* __restrict__ B,
                                                    T* __restrict__ C) {
  using G = BgCfg<T>;
  __shared__ __attribute__((aligned(16))) T As[BG_T * G::LS];
  __shared__ __attribute__((aligned(16))) T Bs[BG_T * G::LS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz = blockIdx.z;
  const T* Ab = A + a.off(bz);
  const T* Bb = B + b.off(bz);
  T* Cb = C + c.off(bz);
  const int m0 = blockIdx.y * BG_T, n0 = blockIdx.x * BG_T;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += BG_K) {
    // ---- stage A (64 x 32) and B (64 x 32) K-contiguous; 256 threads x 8 elements each ----
    {
      float v[8];
      if constexpr (!TA) {
        const int r = tid >> 2, kc = (tid & 3) * 8;
        bg_ld<T>(Ab + (int64_t)(m0 + r) * a.ld + k0 + kc, k0 + kc, K, m0 + r < M, v);
        lds_st8v(As + r * G::LS + kc, v);
      } else {
        const int kr = tid >> 3, mc = (tid & 7) * 8;  // row k0+kr, columns m0+mc..+7
        bg_ld<T>(Ab + (int64_t)(k0 + kr) * a.ld + m0 + mc, m0 + mc, M, k0 + kr < K, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) As[(mc + j) * G::LS + kr] = Tr<T>::from_f(v[j]);
      }
      if constexpr (TB) {
        const int r = tid >> 2, kc = (tid & 3) * 8;
        bg_ld<T>(Bb + (int64_t)(n0 + r) * b.ld + k0 + kc, k0 + kc, K, n0 + r < N, v);
        lds_st8v(Bs + r * G::LS + kc, v);
      } else {
        const int kr = tid >> 3, nc = (tid & 7) * 8;
        bg_ld<T>(Bb + (int64_t)(k0 + kr) * b.ld + n0 + nc, n0 + nc, N, k0 + kr < K, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) Bs[(nc + j) * G::LS + kr] = Tr<T>::from_f(v[j]);
      }
    }
    lds_barrier();
    if constexpr (sizeof(T) == 2) {
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = *reinterpret_cast<const bf16x8_t*>(As + (wm + i * 16 + (lane & 15)) * G::LS + 8 * (lane >> 4));
        bfr[i] = *reinterpret_cast<const bf16x8_t*>(Bs + (wn + i * 16 + (lane & 15)) * G::LS + 8 * (lane >> 4));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
      const float* Af = reinterpret_cast<const float*>(As);
      const float* Bf = reinterpret_cast<const float*>(Bs);
#pragma unroll
      for (int s = 0; s < BG_K / 4; ++s) {
        const int kk = 4 * s + (lane >> 4);
        float av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          av[i] = Af[(wm + i * 16 + (lane & 15)) * G::LS + kk];
          bv[i] = Bf[(wn + i * 16 + (lane & 15)) * G::LS + kk];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    lds_barrier();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + 4 * (lane >> 4) + r, n = n0 + wn + j * 16 + (lane & 15);
        if (m < M && n < N) Cb[(int64_t)m * c.ld + n] = Tr<T>::from_f(alpha * acc[i][j][r]);
      }
}

template <typename T>
int launch_bgemm(hipStream_t s, bool ta, bool tb, int batch, int M, int N, int K, float alpha, const T* A,
                 const BgOp& a, const T* B, const BgOp& b, T* C, const BgOp& c) {
  if (batch <= 0 || M <= 0 || N <= 0) return 0;
  if ((a.ld & 7) || (b.ld & 7)) { set_error("bgemm: operand strides must be multiples of 8", __FILE__, __LINE__); return -1; }
  const dim3 grid((unsigned)cdiv(N, BG_T), (unsigned)cdiv(M, BG_T), (unsigned)batch);
#define BG_L(TA_, TB_) \
  hipLaunchKernelGGL((bgemm_kernel<T, TA_, TB_>), grid, dim3(256), 0, s, a, b, c, M, N, K, alpha, A, B, C)
  if (!ta && tb) BG_L(false, true);
  else if (!ta && !tb) BG_L(false, false);
  else if (ta && !tb) BG_L(true, false);
  else BG_L(true, true);
#undef BG_L
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------
// softmax over score rows: P[r][j] = exp(S - max) / sum, j < n; pad columns [n, ld) set to 0
template <typename T>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ S, T* __restrict__ P, int64_t rows,
                                                          int n, int ld) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const T* s = S + r * ld;
  float v[VIT_SM_PER_LANE];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < VIT_SM_PER_LANE; ++i) {
    const int j = lane + 64 * i;
    v[i] = j < n ? Tr<T>::to_f(s[j]) : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < VIT_SM_PER_LANE; ++i) {
    v[i] = lane + 64 * i < n ? __expf(v[i] - mx) : 0.f;
    sum += v[i];
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  T* p = P + r * ld;
#pragma unroll
  for (int i = 0; i < VIT_SM_PER_LANE; ++i) {
    const int j = lane + 64 * i;
    if (j < ld) p[j] = Tr<T>::from_f(v[i] * inv);
  }
}

// dS = scale * P * (dP - sum_j P dP)   (in place over dP allowed)
template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ P, const T* dP, T* dS, int64_t rows,
                                                          int n, int ld, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float p[VIT_SM_PER_LANE], g[VIT_SM_PER_LANE];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < VIT_SM_PER_LANE; ++i) {
    const int j = lane + 64 * i;
    p[i] = j < n ? Tr<T>::to_f(P[r * ld + j]) : 0.f;
    g[i] = j < n ? Tr<T>::to_f(dP[r * ld + j]) : 0.f;
    dot += p[i] * g[i];
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int i = 0; i < VIT_SM_PER_LANE; ++i) {
    const int j = lane + 64 * i;
    if (j < ld) dS[r * ld + j] = Tr<T>::from_f(j < n ? scale * p[i] * (g[i] - dot) : 0.f);
  }
}

// ------------------------------------------------------------------------------------------
// LayerNorm over C (multiple of 8, <= 64 * 8 * VIT_LN_VEC) per row; rows addressed with a stride
// (the final norm reads only the CLS rows).  One wave per row; fp32 statistics.
template <typename T, typename O>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ X, int64_t ldx, const float* __restrict__ g,
                                                     const float* __restrict__ bta, O* __restrict__ Y, int64_t ldy,
                                                     float* __restrict__ mean, float* __restrict__ rstd, int64_t rows,
                                                     int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int nv = C >> 3;
  float x[VIT_LN_VEC][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VIT_LN_VEC; ++i) {
    const int v = lane + 64 * i;
    if (v < nv) {
      ld8(X + r * ldx + v * 8, x[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[i][j];
    }
  }
  const float mu = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VIT_LN_VEC; ++i)
    if (lane + 64 * i < nv)
#pragma unroll
      for (int j = 0; j < 8; ++j) q += (x[i][j] - mu) * (x[i][j] - mu);
  const float rs = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int i = 0; i < VIT_LN_VEC; ++i) {
    const int v = lane + 64 * i;
    if (v < nv) {
      float gg[8], bb[8], y[8];
      ld8(g + v * 8, gg);
      ld8(bta + v * 8, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = (x[i][j] - mu) * rs * gg[j] + bb[j];
      st8(Y + r * ldy + v * 8, y);
    }
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

// rows of loads in flight per wave in the LayerNorm backward, and its grid (0: one round of co-resident
// workgroups) -- A/B build switches
#ifndef DFD_LN_PF
#define DFD_LN_PF 2
#endif
#ifndef DFD_LN_GRID
#define DFD_LN_GRID 0
#endif
// dX = dres + rstd * (dxh - mean(dxh) - xhat * mean(dxh * xhat)),  dxh = dY * gamma.
// Workgroup w handles rows [w*rpb, (w+1)*rpb): per-column partials of dY*xhat (dgamma) and dY
// (dbeta) go to part[w][2][C] in a fixed order (waves summed in order through LDS).
template <typename T, typename D>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ X, int64_t ldx, const D* __restrict__ dY,
                                                     int64_t ldd, const float* __restrict__ g,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const T* __restrict__ dres, T* __restrict__ dX, int64_t rows,
                                                     int C, int rpb, float* __restrict__ part) {
  __shared__ float red[4][2][VIT_LN_MAXC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = C >> 3;
  float pg[VIT_LN_VEC][8], pb[VIT_LN_VEC][8];
#pragma unroll
  for (int i = 0; i < VIT_LN_VEC; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { pg[i][j] = 0.f; pb[i][j] = 0.f; }
  const int64_t rbeg = (int64_t)blockIdx.x * rpb, rend = min(rows, rbeg + rpb);
  // a row's x, dY and residual gradient are loaded together into raw registers, DFD_LN_PF rows ahead
  // (ring of register sets), so the wave's loads of the next rows are in flight while row r is reduced
  // and written
  struct RowRaw {
    Raw8<T> x[VIT_LN_VEC], r[VIT_LN_VEC];
    Raw8<D> d[VIT_LN_VEC];
  };
  auto row_ld = [&](RowRaw& w, int64_t r) {
    const bool live = r < rend;
#pragma unroll
    for (int i = 0; i < VIT_LN_VEC; ++i) {
      const int v = lane + 64 * i;
      const bool ok = live && v < nv;
      raw_ld(w.x[i], X + r * ldx + v * 8, X, ok);
      raw_ld(w.d[i], dY + r * ldd + v * 8, dY, ok);
      raw_ld(w.r[i], dres ? dres + r * ldx + v * 8 : X, X, ok && dres != nullptr);
    }
  };
  float gv[VIT_LN_VEC][8];
#pragma unroll
  for (int i = 0; i < VIT_LN_VEC; ++i) {
    const int v = lane + 64 * i;
    if (v < nv) ld8(g + v * 8, gv[i]);
  }
  // row r from its raw registers; the set is refilled with row r + 4 * DFD_LN_PF before the reductions
  auto row_do = [&](RowRaw& w, int64_t r) {
    const float mu = mean[r], rs = rstd[r];
    float xh[VIT_LN_VEC][8], dxh[VIT_LN_VEC][8], res[VIT_LN_VEC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VIT_LN_VEC; ++i) {
      const int v = lane + 64 * i;
      if (v < nv) {
        float x[8], dy[8];
        raw_to_f(w.x[i], x);
        raw_to_f(w.d[i], dy);
        raw_to_f(w.r[i], res[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = (x[j] - mu) * rs;
          dxh[i][j] = dy[j] * gv[i][j];
          s1 += dxh[i][j];
          s2 += dxh[i][j] * xh[i][j];
          pg[i][j] += dy[j] * xh[i][j];
          pb[i][j] += dy[j];
        }
      }
    }
    row_ld(w, r + 4 * DFD_LN_PF);
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < VIT_LN_VEC; ++i) {
      const int v = lane + 64 * i;
      if (v < nv) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (dres ? res[i][j] : 0.f) + rs * (dxh[i][j] - s1 - xh[i][j] * s2);
        st8(dX + r * ldx + v * 8, o);
      }
    }
  };
  RowRaw ring[DFD_LN_PF];
#pragma unroll
  for (int k = 0; k < DFD_LN_PF; ++k) row_ld(ring[k], rbeg + wave + 4 * k);
  for (int64_t r = rbeg + wave; r < rend; r += 4 * DFD_LN_PF) {
#pragma unroll
    for (int k = 0; k < DFD_LN_PF; ++k)
      if (r + 4 * k < rend) row_do(ring[k], r + 4 * k);
  }
#pragma unroll
  for (int i = 0; i < VIT_LN_VEC; ++i) {
    const int v = lane + 64 * i;
    if (v < nv)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[wave][0][v * 8 + j] = pg[i][j];
        red[wave][1][v * 8 + j] = pb[i][j];
      }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int w = i / C, cc = i - w * C;
    part[((int64_t)blockIdx.x * 2 + w) * C + cc] =
        ((red[0][w][cc] + red[1][w][cc]) + red[2][w][cc]) + red[3][w][cc];
  }
}

// ------------------------------------------------------------------------------------------
// patch gather: A[(i*P + p)][k], k = c*256 + ky*16 + kx (Conv2d weight flattening), from the
// fp32 image batch with element strides (image i = (b, n) -> b*sb + n*sn).
template <typename T>
__global__ __launch_bounds__(256) void patch_gather_kernel(const float* __restrict__ x, VitImg im, int images,
                                                           T* __restrict__ A) {
  const int gp = im.W / VIT_PATCH, np = (im.H / VIT_PATCH) * gp;
  const int64_t nvec = (int64_t)images * np * (3 * VIT_PATCH * VIT_PATCH / 8);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nvec; e += (int64_t)gridDim.x * 256) {
    const int kv = (int)(e % (3 * VIT_PATCH * VIT_PATCH / 8));
    const int64_t rowi = e / (3 * VIT_PATCH * VIT_PATCH / 8);
    const int p = (int)(rowi % np), i = (int)(rowi / np);
    const int k = kv * 8, c = k / (VIT_PATCH * VIT_PATCH), ky = (k / VIT_PATCH) % VIT_PATCH, kx = k % VIT_PATCH;
    const int py = p / gp, px = p - (p / gp) * gp;
    const float* src = x + (int64_t)(i / im.nodes) * im.sb + (int64_t)(i % im.nodes) * im.sn + (int64_t)c * im.sc +
                       (int64_t)(py * VIT_PATCH + ky) * im.sh + (int64_t)(px * VIT_PATCH + kx) * im.sw;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = src[(int64_t)j * im.sw];
    st8(A + rowi * (3 * VIT_PATCH * VIT_PATCH) + k, v);
  }
}

// X0[i][t][:] = (t == 0 ? cls : PE[i*P + t-1]) + pos[t]
template <typename T>
__global__ __launch_bounds__(256) void tokens_fwd_kernel(const T* __restrict__ PE, const float* __restrict__ cls,
                                                         const float* __restrict__ pos, int images, int ntok, int D,
                                                         T* __restrict__ X0) {
  const int64_t nvec = (int64_t)images * ntok * (D / 8);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nvec; e += (int64_t)gridDim.x * 256) {
    const int dv = (int)(e % (D / 8)) * 8;
    const int64_t rt = e / (D / 8);
    const int t = (int)(rt % ntok), i = (int)(rt / ntok);
    float a[8], p[8];
    if (t == 0) ld8(cls + dv, a);
    else ld8(PE + ((int64_t)i * (ntok - 1) + t - 1) * D + dv, a);
    ld8(pos + (int64_t)t * D + dv, p);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += p[j];
    st8(X0 + rt * D + dv, a);
  }
}

// backward of the token assembly: dPE rows = dX0 rows t >= 1; dpos[t][d] = sum_i dX0[i][t][d];
// dcls[d] = dpos[0][d] (the CLS row of every image)
template <typename T>
__global__ __launch_bounds__(256) void tokens_bwd_kernel(const T* __restrict__ dX0, int images, int ntok, int D,
                                                         T* __restrict__ dPE, float* __restrict__ dpos,
                                                         float* __restrict__ dcls) {
  const int64_t n = (int64_t)ntok * D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e / D), d = (int)(e - (e / D) * D);
    float s = 0.f;
    int i = 0;
    for (; i + 8 <= images; i += 8) {  // 8 images' loads in flight, added in image order
      T v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = dX0[((int64_t)(i + u) * ntok + t) * D + d];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s += Tr<T>::to_f(v[u]);
        if (t > 0) dPE[((int64_t)(i + u) * (ntok - 1) + t - 1) * D + d] = v[u];
      }
    }
    for (; i < images; ++i) {
      const T v = dX0[((int64_t)i * ntok + t) * D + d];
      s += Tr<T>::to_f(v);
      if (t > 0) dPE[((int64_t)i * (ntok - 1) + t - 1) * D + d] = v;
    }
    dpos[e] = s;
    if (t == 0) dcls[d] = s;
  }
}

// ------------------------------------------------------------------------------------------
// weight casts: cast(W) ([rows][cols]) and / or its transpose ([cols][rows]) from ONE read of the fp32
// source, 32x32 LDS tiles; blockIdx.x = the segment's tile (the grid spans the largest segment)
template <typename T>
__global__ __launch_bounds__(256) void wcast_kernel(VitCast cs) {
  const VitCastSeg sg = cs.seg[blockIdx.z];
  const int tr = (sg.cols + 31) / 32;
  if ((int)blockIdx.x >= tr * ((sg.rows + 31) / 32)) return;
  const int ty = blockIdx.x / tr, tx = blockIdx.x - (blockIdx.x / tr) * tr;
  __shared__ float tile[32][33];
  const int lx = threadIdx.x & 31, ly = threadIdx.x >> 5;
  T* out = reinterpret_cast<T*>(sg.dst);
  T* out_t = reinterpret_cast<T*>(sg.dst_t);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = ty * 32 + ly + 8 * i, c = tx * 32 + lx;
    const float v = (r < sg.rows && c < sg.cols) ? sg.src[(int64_t)r * sg.cols + c] : 0.f;
    if (out && r < sg.rows && c < sg.cols) out[(int64_t)r * sg.cols + c] = Tr<T>::from_f(v);
    tile[ly + 8 * i][lx] = v;
  }
  if (!out_t) return;  // uniform per segment
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tx * 32 + ly + 8 * i, r = ty * 32 + lx;  // out_t[c][r]
    if (r < sg.rows && c < sg.cols) out_t[(int64_t)c * sg.rows + r] = Tr<T>::from_f(tile[lx][ly + 8 * i]);
  }
}

// the same on 64 x 64 tiles with 16-B source loads and 8-B stores in both layouts (16-bit T; rows,
// cols % 64: every ViT-B weight): a thread moves 4 consecutive elements per access
template <typename T>
__global__ __launch_bounds__(256) void wcast64_kernel(VitCast cs) {
  const VitCastSeg sg = cs.seg[blockIdx.z];
  const int tr = sg.cols / 64;
  if ((int)blockIdx.x >= tr * (sg.rows / 64)) return;
  const int ty = blockIdx.x / tr, tx = blockIdx.x - (blockIdx.x / tr) * tr;
  __shared__ float tile[64][65];
  const int l4 = threadIdx.x & 15, ly = threadIdx.x >> 4;
  T* out = reinterpret_cast<T*>(sg.dst);
  T* out_t = reinterpret_cast<T*>(sg.dst_t);
  float4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // all four loads in flight first
    const int r = ty * 64 + ly + 16 * i, c = tx * 64 + 4 * l4;
    v[i] = *reinterpret_cast<const float4*>(sg.src + (int64_t)r * sg.cols + c);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = ly + 16 * i, r = ty * 64 + rl, c = tx * 64 + 4 * l4;
    if (out)
      *reinterpret_cast<uint2*>(out + (int64_t)r * sg.cols + c) =
          make_uint2(Tr<T>::pack2(v[i].x, v[i].y), Tr<T>::pack2(v[i].z, v[i].w));
    tile[rl][4 * l4] = v[i].x;
    tile[rl][4 * l4 + 1] = v[i].y;
    tile[rl][4 * l4 + 2] = v[i].z;
    tile[rl][4 * l4 + 3] = v[i].w;
  }
  if (!out_t) return;  // uniform per segment
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // out_t[c][r .. r + 3]
    const int cl = ly + 16 * i, c = tx * 64 + cl, r = ty * 64 + 4 * l4;
    *reinterpret_cast<uint2*>(out_t + (int64_t)c * sg.rows + r) =
        make_uint2(Tr<T>::pack2(tile[4 * l4][cl], tile[4 * l4 + 1][cl]), Tr<T>::pack2(tile[4 * l4 + 2][cl], tile[4 * l4 + 3][cl]));
  }
}

template <typename T>
int launch_wcast(hipStream_t s, const VitCast& cs, int nseg) {
  if (nseg <= 0) return 0;
  bool t64 = true;
  int tiles64 = 0;
  for (int i = 0; i < nseg; ++i) {
    t64 = t64 && cs.seg[i].rows % 64 == 0 && cs.seg[i].cols % 64 == 0;
    tiles64 = std::max(tiles64, (cs.seg[i].rows / 64) * (cs.seg[i].cols / 64));
  }
  if constexpr (sizeof(T) == 2) {  // 16-bit storage (the fp32 parity mode keeps the 32 x 32 form)
    if (t64) {
      hipLaunchKernelGGL((wcast64_kernel<T>), dim3((unsigned)tiles64, 1, (unsigned)nseg), dim3(256), 0, s, cs);
      DFD_HIP_CHECK(hipGetLastError());
      return 0;
    }
  }
  int tiles = 0;
  for (int i = 0; i < nseg; ++i) tiles = std::max(tiles, cdiv(cs.seg[i].rows, 32) * cdiv(cs.seg[i].cols, 32));
  const dim3 grid((unsigned)tiles, 1, (unsigned)nseg);
  hipLaunchKernelGGL((wcast_kernel<T>), grid, dim3(256), 0, s, cs);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------
// GCN head (fp32).  H1[b][i][:] = sum_j A[b][i][j] F[b][j][:]   (transpose: sum_j A[b][j][i] ...)
__global__ void gcn_mix_kernel(const float* __restrict__ A, const float* __restrict__ F, int B, int N, int D,
                               bool transpose, float* __restrict__ H) {
  const int64_t n = (int64_t)B * N * D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int d = (int)(e % D);
    const int64_t bi = e / D;
    const int i = (int)(bi % N), b = (int)(bi / N);
    const float* a = A + (int64_t)b * N * N;
    float s = 0.f;
    for (int j = 0; j < N; ++j) s += (transpose ? a[j * N + i] : a[i * N + j]) * F[((int64_t)b * N + j) * D + d];
    H[e] = s;
  }
}

// dropout keep-scale: the counter hash shared with the detector head and the RNN
__device__ __forceinline__ float vit_drop(uint64_t seed, uint32_t st, int64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  uint64_t z = seed ^ ((uint64_t)st << 56) ^ (uint64_t)idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// Y = relu(Y) in place; D (optional) = dropout(relu(Y)) with stream st
__global__ void relu_drop_kernel(float* __restrict__ Y, float* __restrict__ D, int64_t n, uint64_t seed, uint32_t st,
                                 float p) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const float v = fmaxf(Y[e], 0.f);
    Y[e] = v;
    if (D) D[e] = v * vit_drop(seed, st, e, p);
  }
}

// dY = dD * keep(e) * (Y > 0)   (Y = the saved post-ReLU value; dD may alias dY)
__global__ void relu_drop_bwd_kernel(const float* __restrict__ Y, const float* dD, float* dY, int64_t n, uint64_t seed,
                                     uint32_t st, float p) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    dY[e] = Y[e] > 0.f ? dD[e] * vit_drop(seed, st, e, p) : 0.f;
}

// G[b][:] = mean_i H[b][i][:]   / backward: dH[b][i][:] = dG[b][:] / N
__global__ void node_mean_kernel(const float* __restrict__ H, int B, int N, int D, float* __restrict__ G) {
  const int n = B * D;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int b = e / D, d = e - (e / D) * D;
    float s = 0.f;
    for (int i = 0; i < N; ++i) s += H[((int64_t)b * N + i) * D + d];
    G[e] = s / N;
  }
}
__global__ void node_mean_bwd_kernel(const float* __restrict__ dG, int B, int N, int D, float* __restrict__ dH) {
  const int64_t n = (int64_t)B * N * D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int d = (int)(e % D);
    const int b = (int)(e / ((int64_t)N * D));
    dH[e] = dG[(int64_t)b * D + d] / N;
  }
}

// column sums of a [M][N] T matrix: part[split][N] (fixed order) -> reduce_slabs
template <typename T>
__global__ __launch_bounds__(256) void colsum_part_kernel(const T* __restrict__ X, int64_t M, int N, int64_t mps,
                                                          float* __restrict__ part) {
  const int nv = N >> 3;
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= nv) return;
  const int64_t mb = (int64_t)blockIdx.y * mps, me = min(M, mb + mps);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t m = mb; m < me; ++m) {
    float x[8];
    ld8(X + m * N + v * 8, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += x[j];
  }
  st8(part + (int64_t)blockIdx.y * N + v * 8, s);
}

// ------------------------------------------------------------------------------------------
static int ew(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(n, 256), 8192)); }

template <typename T>
int launch_softmax_fwd(hipStream_t s, const T* S, T* P, int64_t rows, int n, int ld) {
  if (n > 64 * VIT_SM_PER_LANE || ld > 64 * VIT_SM_PER_LANE) { set_error("softmax: row too long", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL((softmax_fwd_kernel<T>), dim3((unsigned)cdiv64(rows, 4)), dim3(256), 0, s, S, P, rows, n, ld);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template <typename T>
int launch_softmax_bwd(hipStream_t s, const T* P, const T* dP, T* dS, int64_t rows, int n, int ld, float scale) {
  hipLaunchKernelGGL((softmax_bwd_kernel<T>), dim3((unsigned)cdiv64(rows, 4)), dim3(256), 0, s, P, dP, dS, rows, n, ld,
                     scale);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template <typename T, typename O>
int launch_ln_fwd(hipStream_t s, const T* X, int64_t ldx, const float* g, const float* b, O* Y, int64_t ldy, float* mean,
                  float* rstd, int64_t rows, int C, float eps) {
  if ((C & 7) || C > VIT_LN_MAXC) { set_error("layernorm: unsupported width", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL((ln_fwd_kernel<T, O>), dim3((unsigned)cdiv64(rows, 4)), dim3(256), 0, s, X, ldx, g, b, Y, ldy, mean,
                     rstd, rows, C, eps);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template <typename T, typename D>
int launch_ln_bwd(hipStream_t s, const T* X, int64_t ldx, const D* dY, int64_t ldd, const float* g, const float* mean,
                  const float* rstd, const T* dres, T* dX, int64_t rows, int C, float* part, int64_t part_cap,
                  float* dgamma, float* dbeta, bool accumulate) {
  if ((C & 7) || C > VIT_LN_MAXC) { set_error("layernorm: unsupported width", __FILE__, __LINE__); return -1; }
  // one round of co-resident workgroups (the rows of a wave then pipeline DFD_LN_PF deep)
  static const int resident = [] {
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ln_bwd_kernel<T, D>, 256, 0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    return std::max(1, cus * per_cu);
  }();
  int blocks = (int)std::min<int64_t>(DFD_LN_GRID ? DFD_LN_GRID : resident, cdiv64(rows, 16));
  blocks = (int)std::min<int64_t>(blocks, std::max<int64_t>(1, part_cap / (2LL * C)));
  const int rpb = (int)cdiv64(rows, blocks);
  blocks = (int)cdiv64(rows, rpb);
  hipLaunchKernelGGL((ln_bwd_kernel<T, D>), dim3((unsigned)blocks), dim3(256), 0, s, X, ldx, dY, ldd, g, mean, rstd,
                     dres, dX, rows, C, rpb, part);
  DFD_HIP_CHECK(hipGetLastError());
  // part rows alternate [dgamma; dbeta]: where the two gradients are adjacent (timm's weight, bias
  // order in one flat gradient buffer) the whole rows reduce in one launch, else each column set
  // with a stride-2C view
  if (dbeta == dgamma + C) return launch_reduce_slabs(s, part, blocks, 2LL * C, dgamma, accumulate);
  DFD_TRY(launch_reduce_slabs_strided(s, part, blocks, C, 2LL * C, dgamma, accumulate));
  DFD_TRY(launch_reduce_slabs_strided(s, part + C, blocks, C, 2LL * C, dbeta, accumulate));
  return 0;
}
template <typename T>
int launch_patch_gather(hipStream_t s, const float* x, const VitImg& im, int images, T* A) {
  if (im.H % VIT_PATCH || im.W % VIT_PATCH) { set_error("vit: image size must be a multiple of 16", __FILE__, __LINE__); return -1; }
  const int64_t n = (int64_t)images * (im.H / VIT_PATCH) * (im.W / VIT_PATCH) * (3 * VIT_PATCH * VIT_PATCH / 8);
  hipLaunchKernelGGL((patch_gather_kernel<T>), dim3(ew(n)), dim3(256), 0, s, x, im, images, A);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template <typename T>
int launch_tokens_fwd(hipStream_t s, const T* PE, const float* cls, const float* pos, int images, int ntok, int D, T* X0) {
  hipLaunchKernelGGL((tokens_fwd_kernel<T>), dim3(ew((int64_t)images * ntok * D / 8)), dim3(256), 0, s, PE, cls, pos,
                     images, ntok, D, X0);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template <typename T>
int launch_tokens_bwd(hipStream_t s, const T* dX0, int images, int ntok, int D, T* dPE, float* dpos, float* dcls) {
  hipLaunchKernelGGL((tokens_bwd_kernel<T>), dim3(ew((int64_t)ntok * D)), dim3(256), 0, s, dX0, images, ntok, D, dPE,
                     dpos, dcls);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template <typename T>
int launch_colsum(hipStream_t s, const T* X, int64_t M, int N, float* part, int64_t part_cap, float* out,
                  bool accumulate) {
  if (N & 7) { set_error("colsum: N must be a multiple of 8", __FILE__, __LINE__); return -1; }
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(cdiv64(M, 64), 256));
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, part_cap / N));
  const int64_t mps = cdiv64(M, splits);
  splits = cdiv64(M, mps);
  hipLaunchKernelGGL((colsum_part_kernel<T>), dim3((unsigned)cdiv(N / 8, 256), (unsigned)splits), dim3(256), 0, s, X, M,
                     N, mps, part);
  DFD_HIP_CHECK(hipGetLastError());
  return launch_reduce_slabs(s, part, (int)splits, N, out, accumulate);
}
int launch_gcn_mix(hipStream_t s, const float* A, const float* F, int B, int N, int D, bool transpose, float* H) {
  hipLaunchKernelGGL(gcn_mix_kernel, dim3(ew((int64_t)B * N * D)), dim3(256), 0, s, A, F, B, N, D, transpose, H);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int launch_relu_drop(hipStream_t s, float* Y, float* D, int64_t n, uint64_t seed, uint32_t st, float p) {
  hipLaunchKernelGGL(relu_drop_kernel, dim3(ew(n)), dim3(256), 0, s, Y, D, n, seed, st, p);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int launch_relu_drop_bwd(hipStream_t s, const float* Y, const float* dD, float* dY, int64_t n, uint64_t seed,
                         uint32_t st, float p) {
  hipLaunchKernelGGL(relu_drop_bwd_kernel, dim3(ew(n)), dim3(256), 0, s, Y, dD, dY, n, seed, st, p);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int launch_node_mean(hipStream_t s, const float* H, int B, int N, int D, float* G) {
  hipLaunchKernelGGL(node_mean_kernel, dim3(ew((int64_t)B * D)), dim3(256), 0, s, H, B, N, D, G);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
int launch_node_mean_bwd(hipStream_t s, const float* dG, int B, int N, int D, float* dH) {
  hipLaunchKernelGGL(node_mean_bwd_kernel, dim3(ew((int64_t)B * N * D)), dim3(256), 0, s, dG, B, N, D, dH);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ---- exact-erf GELU passes of the bf16 MLP for shapes the vgemm kernels do not cover (k_vgemm.hip
// applies the same in its epilogues), 8 elements per lane:
//   GELU_PAIR  G = gelu(Z) and, in place, Z := gelu'(Z)  (the forward keeps the derivative, not Z)
//   GELU_MULD  dZ *= D  (D = the derivative kept by the forward)
__global__ __launch_bounds__(256) void gelu_pair_kernel(bf16* __restrict__ Z, bf16* __restrict__ G, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float z[8], g[8];
    ld8(Z + i * 8, z);
#pragma unroll
    for (int j = 0; j < 8; ++j) gelu_pair_(z[j], g[j], z[j]);
    st8(G + i * 8, g);
    st8(Z + i * 8, z);
  }
}
__global__ __launch_bounds__(256) void gelu_muld_kernel(const bf16* __restrict__ D, bf16* __restrict__ dZ, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float dd[8], d[8];
    ld8(D + i * 8, dd);
    ld8(dZ + i * 8, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= dd[j];
    st8(dZ + i * 8, d);
  }
}
int launch_gelu(hipStream_t s, bf16* Z, bf16* out, int64_t n, int mode) {
  if (n <= 0) return 0;
  if (n % 8) { set_error("gelu: element count must be a multiple of 8", __FILE__, __LINE__); return -1; }
  const int64_t n8 = n / 8;
  const int g = (int)std::min<int64_t>(cdiv64(n8, 256), 4096);
  if (mode == GELU_PAIR) hipLaunchKernelGGL(gelu_pair_kernel, dim3(g), dim3(256), 0, s, Z, out, n8);
  else if (mode == GELU_MULD) hipLaunchKernelGGL(gelu_muld_kernel, dim3(g), dim3(256), 0, s, Z, out, n8);
  else { set_error("gelu: mode", __FILE__, __LINE__); return -1; }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

#define DFD_VIT_INST(T)                                                                                              \
  template int launch_bgemm<T>(hipStream_t, bool, bool, int, int, int, int, float, const T*, const BgOp&, const T*,   \
                               const BgOp&, T*, const BgOp&);                                                        \
  template int launch_softmax_fwd<T>(hipStream_t, const T*, T*, int64_t, int, int);                                  \
  template int launch_softmax_bwd<T>(hipStream_t, const T*, const T*, T*, int64_t, int, int, float);                 \
  template int launch_ln_fwd<T, T>(hipStream_t, const T*, int64_t, const float*, const float*, T*, int64_t, float*,   \
                                   float*, int64_t, int, float);                                                     \
  template int launch_ln_bwd<T, T>(hipStream_t, const T*, int64_t, const T*, int64_t, const float*, const float*,     \
                                   const float*, const T*, T*, int64_t, int, float*, int64_t, float*, float*, bool); \
  template int launch_patch_gather<T>(hipStream_t, const float*, const VitImg&, int, T*);                            \
  template int launch_tokens_fwd<T>(hipStream_t, const T*, const float*, const float*, int, int, int, T*);           \
  template int launch_tokens_bwd<T>(hipStream_t, const T*, int, int, int, T*, float*, float*);                       \
  template int launch_colsum<T>(hipStream_t, const T*, int64_t, int, float*, int64_t, float*, bool);                 \
  template int launch_wcast<T>(hipStream_t, const VitCast&, int);
DFD_VIT_INST(float)
DFD_VIT_INST(bf16)
template int launch_ln_fwd<bf16, float>(hipStream_t, const bf16*, int64_t, const float*, const float*, float*, int64_t,
                                        float*, float*, int64_t, int, float);
template int launch_ln_bwd<bf16, float>(hipStream_t, const bf16*, int64_t, const float*, int64_t, const float*,
                                        const float*, const float*, const bf16*, bf16*, int64_t, int, float*, int64_t,
                                        float*, float*, bool);

}  // namespace dfd
