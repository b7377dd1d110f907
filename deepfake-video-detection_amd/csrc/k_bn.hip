// BatchNorm (training batch statistics / eval running statistics), SiLU, squeeze-excite and
// global-average-pool kernels for the EfficientNet-B0 hot path on gfx950.
//
// Replaces aten batch_norm + silu (timm BatchNormAct2d), the SE module (mean(2,3), two
// biased 1x1 convs, silu, sigmoid, mul) and adaptive_avg_pool2d+flatten reached from
// src/pretrained_detector.py:116, forward and backward.  Every BN statistic is a
// deterministic two-level reduction: producers write per-workgroup partial rows
// [rows][2][C] and bn_finalize sums them in a fixed order (fp64) -- no float atomics in HBM.
#include "kernels.h"

#include <mutex>
#include <utility>
#include <vector>
#include "tail.h"

namespace dfd {

// ------------------------------------------------------------------ partial-row reduction
// Sums rows of a [rows][2][C] slab for channels [blockIdx.x*CH, +CH) in fp64: 1024 threads = CH
// channels x (1024 / CH) row lanes; the row lanes of a wave are added by shuffles, the 16 waves by
// threads 0..CH-1 in wave order (deterministic; one barrier instead of a 6-level LDS tree).  Valid
// in threads 0..CH-1 (channel tid).  CH (16, 8 or 4) is chosen per launch so that each row lane
// reads at most 8 rows (one batch of loads in flight): the producers of the high-resolution maps
// write up to 1,024 partial rows of few channels, where 16 channels per workgroup left one or two
// workgroups walking 16 rows per lane in two dependent batches (10-12 us finalizes).
template <int CH>
__device__ void reduce_stat_rows(const float* __restrict__ stats, int rows, int C, double& s, double& q,
                                 double* sh_s, double* sh_q) {
  constexpr int FIN_CH = CH, FIN_RL = 1024 / CH;
  const int tid = threadIdx.x, cl = tid % FIN_CH, rl = tid / FIN_CH;
  const int c = blockIdx.x * FIN_CH + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    // loads of 8 rows issued before their adds (same summation order as one row at a time)
    int r = rl;
    for (; r + 7 * FIN_RL < rows; r += 8 * FIN_RL) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        va[u] = stats[((int64_t)(r + u * FIN_RL) * 2 + 0) * C + c];
        vb[u] = stats[((int64_t)(r + u * FIN_RL) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { a += va[u]; b += vb[u]; }
    }
    for (; r < rows; r += FIN_RL) {
      a += stats[((int64_t)r * 2 + 0) * C + c];
      b += stats[((int64_t)r * 2 + 1) * C + c];
    }
  }
  // lanes l, l^CH, l^2CH, ... of a wave hold the same channel
#pragma unroll
  for (int o = CH; o < 64; o <<= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  const int wave = tid >> 6;
  if ((tid & 63) < FIN_CH) {
    sh_s[wave * FIN_CH + cl] = a;
    sh_q[wave * FIN_CH + cl] = b;
  }
  __syncthreads();
  s = 0.0;
  q = 0.0;
  if (tid < FIN_CH) {
    for (int w = 0; w < 1024 / 64; ++w) {
      s += sh_s[w * FIN_CH + tid];
      q += sh_q[w * FIN_CH + tid];
    }
  }
}

// channels per finalize workgroup: at most 8 rows per row lane (reduce_stat_rows)
static int fin_ch(int rows) { return rows <= 8 * 64 ? 16 : (rows <= 8 * 128 ? 8 : 4); }

// chan_rows > 0: the rows are centred tile partials (sum, M2 about the tile's own mean) of
// consecutive chan_rows-row tiles (the conv epilogue, k_conv.hip): var = (sum M2 + sum_t n_t
// (mean_t - mean)^2) / n, the second term from a pass over the tile sums once the mean is known
template <int CH>
__device__ void chan_between(const float* __restrict__ stats, int rows, int C, int64_t count, int chan_rows,
                             double* sh_m, double& out, double* sh) {
  constexpr int FIN_RL = 1024 / CH;
  const int tid = threadIdx.x, cl = tid % CH, rl = tid / CH;
  const int c = blockIdx.x * CH + cl;
  double a = 0.0;
  if (c < C) {
    const double m = sh_m[cl];
    for (int r = rl; r < rows; r += FIN_RL) {
      const int64_t left = count - (int64_t)r * chan_rows, nt = left < chan_rows ? left : chan_rows;
      const double d = (double)stats[((int64_t)r * 2 + 0) * C + c] / (double)nt - m;
      a += (double)nt * d * d;
    }
  }
#pragma unroll
  for (int o = CH; o < 64; o <<= 1) a += __shfl_xor(a, o, 64);
  const int wave = tid >> 6;
  if ((tid & 63) < CH) sh[wave * CH + cl] = a;
  __syncthreads();
  out = 0.0;
  if (tid < CH)
    for (int w = 0; w < 1024 / 64; ++w) out += sh[w * CH + tid];
}

template <int FIN_CH>
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float* __restrict__ stats, int rows, int64_t count,
                                                           int C, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* run_mean,
                                                           float* run_var, float momentum, float eps, int training,
                                                           float* mean, float* invstd, float* scale, float* shift,
                                                           int chan_rows) {
  __shared__ double sh_s[1024 / 64 * FIN_CH], sh_q[1024 / 64 * FIN_CH], sh_m[FIN_CH];
  const int tid = threadIdx.x;
  const int c = blockIdx.x * FIN_CH + tid;
  // the channel's parameters and running buffers, loaded before the reduction (their latency under
  // the stat-row loads instead of after them: the kernel is a chain of dependent memory round trips)
  float p_g = 0.f, p_b = 0.f, p_rm = 0.f, p_rv = 0.f;
  if (tid < FIN_CH && c < C) {
    p_g = gamma[c];
    p_b = beta[c];
    if (run_mean) { p_rm = run_mean[c]; p_rv = run_var[c]; }
  }
  double s = 0.0, q = 0.0, between = 0.0;
  if (training) reduce_stat_rows<FIN_CH>(stats, rows, C, s, q, sh_s, sh_q);
  if (training && chan_rows > 0) {
    if (tid < FIN_CH) sh_m[tid] = s / (double)count;
    __syncthreads();
    chan_between<FIN_CH>(stats, rows, C, count, chan_rows, sh_m, between, sh_s);
  }
  if (tid < FIN_CH && c < C) {
    float mu, is;
    if (training) {
      const double m = s / (double)count;
      double var = chan_rows > 0 ? (q + between) / (double)count : q / (double)count - m * m;
      if (var < 0.0) var = 0.0;
      mu = (float)m;
      is = (float)(1.0 / sqrt(var + (double)eps));
      if (run_mean) {
        const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
        run_mean[c] = (float)((1.0 - momentum) * p_rm + momentum * m);
        run_var[c] = (float)((1.0 - momentum) * p_rv + momentum * unb);
      }
    } else {
      mu = p_rm;
      is = 1.0f / sqrtf(p_rv + eps);
    }
    const float sc = p_g * is;
    mean[c] = mu;
    invstd[c] = is;
    scale[c] = sc;
    shift[c] = p_b - mu * sc;
  }
}

// Many centred partial rows (the CNN-LSTM's early convolutions: up to 200k rows of 64-row tiles): the
// single-pass form over row chunks.  With S = sum_t s_t, Q = sum_t M2_t and P = sum_t s_t^2 / n_t,
// sum_t n_t (mean_t - mean)^2 = P - S^2 / count, so one pass gives every term: chunk partials (S, Q, P)
// in fp64 over CHUNK rows per workgroup (4 row lanes x 64 channels, lanes added in order), then one
// thread per channel adds the chunks in order (deterministic) and finalizes as bn_finalize_kernel.
constexpr int BNF_CHUNK = 512;
// the chunk partials' scratch (< 1 MB at 200k rows): one buffer per stream, kept and grown on demand
// (a stream's finalize calls are ordered on it; hipMallocAsync / hipFreeAsync per call measured ~2 ms
// per step of allocator traffic in the bf16 ensemble step)
static double* bn_chunk_scratch(hipStream_t s, size_t bytes) {
  static std::mutex mu;
  static std::vector<std::pair<hipStream_t, std::pair<void*, size_t>>> bufs;
  const std::lock_guard<std::mutex> lk(mu);
  for (auto& b : bufs)
    if (b.first == s) {
      if (b.second.second >= bytes) return static_cast<double*>(b.second.first);
      if (hipStreamSynchronize(s) != hipSuccess || hipFree(b.second.first) != hipSuccess) {
        set_error("bn finalize: scratch release failed", __FILE__, __LINE__);
        return nullptr;
      }
      b.second = {nullptr, 0};
      if (hipMalloc(&b.second.first, bytes) != hipSuccess) {
        set_error("bn finalize: scratch allocation failed", __FILE__, __LINE__);
        return nullptr;
      }
      b.second.second = bytes;
      return static_cast<double*>(b.second.first);
    }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    set_error("bn finalize: scratch allocation failed", __FILE__, __LINE__);
    return nullptr;
  }
  bufs.push_back({s, {p, bytes}});
  return static_cast<double*>(p);
}
__global__ __launch_bounds__(256) void bn_chan_chunks_kernel(const float* __restrict__ stats, int rows, int64_t count,
                                                             int C, int chan_rows, double* __restrict__ part) {
  __shared__ double sh[3][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const int r0 = blockIdx.x * BNF_CHUNK, r1 = min(rows, r0 + BNF_CHUNK);
  double S = 0.0, Q = 0.0, P = 0.0;
  if (c < C)
    for (int r = r0 + rl; r < r1; r += 4) {
      const int64_t left = count - (int64_t)r * chan_rows, nt = left < chan_rows ? left : chan_rows;
      const double st = stats[((int64_t)r * 2 + 0) * C + c];
      S += st;
      Q += (double)stats[((int64_t)r * 2 + 1) * C + c];
      P += st * st / (double)nt;
    }
  sh[0][rl][cl] = S;
  sh[1][rl][cl] = Q;
  sh[2][rl][cl] = P;
  __syncthreads();
  if (rl == 0 && c < C) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double v = ((sh[k][0][cl] + sh[k][1][cl]) + sh[k][2][cl]) + sh[k][3][cl];
      part[((int64_t)blockIdx.x * 3 + k) * C + c] = v;
    }
  }
}
__global__ void bn_chan_final_kernel(const double* __restrict__ part, int nchunks, int64_t count, int C,
                                     const float* __restrict__ gamma, const float* __restrict__ beta, float* run_mean,
                                     float* run_var, float momentum, float eps, float* mean, float* invstd,
                                     float* scale, float* shift) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double S = 0.0, Q = 0.0, P = 0.0;
  for (int k = 0; k < nchunks; ++k) {
    S += part[((int64_t)k * 3 + 0) * C + c];
    Q += part[((int64_t)k * 3 + 1) * C + c];
    P += part[((int64_t)k * 3 + 2) * C + c];
  }
  const double m = S / (double)count;
  double between = P - S * m;
  if (between < 0.0) between = 0.0;
  double var = (Q + between) / (double)count;
  if (var < 0.0) var = 0.0;
  const float mu = (float)m, is = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
    run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * m);
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
  }
  const float sc = gamma[c] * is;
  mean[c] = mu;
  invstd[c] = is;
  scale[c] = sc;
  shift[c] = beta[c] - mu * sc;
}

int launch_bn_finalize(hipStream_t s, const float* stats, int rows, int64_t count, int C, const float* gamma,
                       const float* beta, float* run_mean, float* run_var, float momentum, float eps, bool training,
                       float* mean, float* invstd, float* scale, float* shift, int chan_rows) {
  if (training && chan_rows > 0 && rows > 4 * BNF_CHUNK) {
    const int nch = cdiv(rows, BNF_CHUNK);
    double* part = bn_chunk_scratch(s, sizeof(double) * (size_t)nch * 3 * C);
    if (!part) return -1;
    hipLaunchKernelGGL(bn_chan_chunks_kernel, dim3((unsigned)nch, (unsigned)cdiv(C, 64)), dim3(256), 0, s, stats, rows,
                       count, C, chan_rows, part);
    DFD_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(bn_chan_final_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0, s, part, nch, count, C, gamma,
                       beta, run_mean, run_var, momentum, eps, mean, invstd, scale, shift);
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
  const int ch = training ? fin_ch(rows) : 16;
#define DFD_FIN(CH)                                                                                                 \
  hipLaunchKernelGGL((bn_finalize_kernel<CH>), dim3(cdiv(C, CH)), dim3(1024), 0, s, stats, rows, count, C, gamma, beta, \
                     run_mean, run_var, momentum, eps, training ? 1 : 0, mean, invstd, scale, shift, chan_rows)
  if (ch == 16) DFD_FIN(16);
  else if (ch == 8) DFD_FIN(8);
  else DFD_FIN(4);
#undef DFD_FIN
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int launch_bn_finalize_fin(hipStream_t s, const BnFwdFin& f, int C) {
  return launch_bn_finalize(s, f.stats, f.rows, f.count, C, f.gamma, f.beta, f.run_mean, f.run_var, f.momentum, f.eps,
                            true, f.mean, f.invstd, f.scale, f.shift);
}

// Eval mode: every BatchNorm of a plan from its running statistics in ONE launch (workgroup = layer):
// the same operations as bn_finalize_kernel's eval branch; one ~5 us launch instead of 49 per forward
__global__ __launch_bounds__(256) void bn_eval_all_kernel(const float* __restrict__ P, const float* __restrict__ bnb,
                                                          float* __restrict__ wsf, EvalBnTable t, float eps) {
  const EvalBnEntry e = t.e[blockIdx.x];
  for (int c = threadIdx.x; c < e.C; c += 256) {
    const float mu = bnb[e.rm + c];
    const float is = 1.0f / sqrtf(bnb[e.rv + c] + eps);
    const float sc = P[e.w + c] * is;
    wsf[e.mean + c] = mu;
    wsf[e.invstd + c] = is;
    wsf[e.scale + c] = sc;
    wsf[e.shift + c] = P[e.b + c] - mu * sc;
  }
}

int launch_bn_eval_all(hipStream_t s, const float* P, const float* bnb, float* wsf, const EvalBnTable& t, float eps) {
  if (t.n <= 0 || t.n > kEvalBnMax) { set_error("bn eval: table size", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL(bn_eval_all_kernel, dim3(t.n), dim3(256), 0, s, P, bnb, wsf, t, eps);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ elementwise grid
// "Channel-stationary" grid-stride: the launch uses a block count whose thread total is a
// multiple of the row width cv (in 8-vectors), so a thread's channel vector -- and every
// per-channel coefficient it needs -- is loop-invariant and the loop has no division.
static int ew_grid(int64_t nvec) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(nvec, 256), 4096)); }
static int gcd_int(int a, int b) { while (b) { const int t = a % b; a = b; b = t; } return a; }
static int cs_grid(int64_t nvec, int cv) {
  const int unit = cv / gcd_int(cv, 256);
  const int64_t want = std::max<int64_t>(1, std::min<int64_t>(cdiv64(nvec, 256), 4096));
  return (int)std::max<int64_t>(unit, (want / unit) * unit);
}

// ------------------------------------------------------------------ BN apply (+ residual)
template <typename T, bool RES>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ Y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const T* __restrict__ R,
                                                       T* __restrict__ X, int64_t nvec, int cv) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  const int64_t step = (int64_t)gridDim.x * 256;  // multiple of cv (cs_grid)
  const int c = (int)(i % cv) * 8;
  float sc[8], sh[8];
  ld8f(scale + c, sc);
  ld8f(shift + c, sh);
  for (; i < nvec; i += step) {
    float y[8];
    ld8(Y + i * 8, y);
    if constexpr (RES) {
      float r[8];
      ld8(R + i * 8, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = y[j] * sc[j] + sh[j] + r[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = y[j] * sc[j] + sh[j];
    }
    st8(X + i * 8, y);
  }
}

template <typename T>
int launch_bn_apply(hipStream_t s, const T* Y, const float* scale, const float* shift, const T* R, T* X, int64_t M,
                    int C) {
  const int64_t nvec = M * C / 8;
  const int gx = cs_grid(nvec, C / 8);
  if (R)
    hipLaunchKernelGGL((bn_apply_kernel<T, true>), dim3(gx), dim3(256), 0, s, Y, scale, shift, R, X, nvec, C / 8);
  else
    hipLaunchKernelGGL((bn_apply_kernel<T, false>), dim3(gx), dim3(256), 0, s, Y, scale, shift, R, X, nvec, C / 8);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ BN backward
// g = dA * act'(z),  z = y*scale + shift,  dA = dZ*gate + bc*bc_scale
// FL: compile-time presence flags of the optional inputs (one kernel instance per combination)
enum { BF_DZ = 1, BF_GATE = 2, BF_BC = 4, BF_SILU = 8 };
static int bn_flags(const BnBwdIn& in) {
  return (in.dZ ? BF_DZ : 0) | (in.gate ? BF_GATE : 0) | (in.bc ? BF_BC : 0) | (in.silu ? BF_SILU : 0);
}

// per-thread channel constants of the backward
struct BnBwdCh {
  float sc[8], sh[8];
};

template <typename T, int FL>
__device__ __forceinline__ void bn_bwd_g8(const BnBwdIn& in, const T* __restrict__ Y, int64_t row, uint32_t frame,
                                          int c, int C, const BnBwdCh& ch, float (&g)[8], float (&y)[8]) {
  ld8(Y + row * C + c, y);
  float da[8];
  if constexpr ((FL & BF_DZ) != 0) {
    ld8(reinterpret_cast<const T*>(in.dZ) + row * C + c, da);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) da[j] = 0.f;
  }
  if constexpr ((FL & BF_GATE) != 0) {
    float gt[8];
    ld8f(in.gate + (int64_t)frame * C + c, gt);
#pragma unroll
    for (int j = 0; j < 8; ++j) da[j] *= gt[j];
  }
  if constexpr ((FL & BF_BC) != 0) {
    float b[8];
    ld8f(in.bc + (int64_t)frame * C + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) da[j] += b[j] * in.bc_scale;
  }
  if constexpr ((FL & BF_SILU) != 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = da[j] * dsiluf_(y[j] * ch.sc[j] + ch.sh[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = da[j];
  }
}

template <int FL>
__device__ __forceinline__ void bn_bwd_ch(const BnBwdIn& in, int c, BnBwdCh& ch) {
  if constexpr ((FL & BF_SILU) != 0) {
    ld8f(in.scale + c, ch.sc);
    ld8f(in.shift + c, ch.sh);
  }
}

template <int FL>
__device__ __forceinline__ uint32_t bn_frame(const BnBwdIn& in, int64_t row) {
  if constexpr ((FL & (BF_GATE | BF_BC)) != 0) return (uint32_t)row / (uint32_t)in.rows_per_frame;
  return 0u;
}

// grid (gx, cdiv(C/8, VPG)); threads: vec = tid % vpg, rl = tid / vpg
template <typename T, int FL>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnBwdIn in, const T* __restrict__ Y, int64_t M, int C,
                                                            float* __restrict__ stats, int vpg) {
  __shared__ float sh[2][256][8];
  const int tid = threadIdx.x;
  const int vec = tid % vpg, rl = tid / vpg, nrl = 256 / vpg;
  const int c = (blockIdx.y * vpg + vec) * 8;
  float as[8], aq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { as[j] = 0.f; aq[j] = 0.f; }
  if (rl < nrl && c < C) {
    float mu[8], is[8];
    BnBwdCh ch;
    bn_bwd_ch<FL>(in, c, ch);
    ld8f(in.mean + c, mu);
    ld8f(in.invstd + c, is);
    // rows in pairs (both rows' loads issued before either is summed; same summation order)
    const int64_t rs = (int64_t)gridDim.x * nrl;
    int64_t r = (int64_t)blockIdx.x * nrl + rl;
    for (; r < M; r += 2 * rs) {
      float g[2][8], y[2][8];
      const bool two = r + rs < M;
      bn_bwd_g8<T, FL>(in, Y, r, bn_frame<FL>(in, r), c, C, ch, g[0], y[0]);
      if (two) bn_bwd_g8<T, FL>(in, Y, r + rs, bn_frame<FL>(in, r + rs), c, C, ch, g[1], y[1]);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          as[j] += g[u][j];
          aq[j] += g[u][j] * (y[u][j] - mu[j]) * is[j];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { sh[0][tid][j] = as[j]; sh[1][tid][j] = aq[j]; }
  __syncthreads();
  if (tid < vpg && c < C) {
    for (int r = 1; r < nrl; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        as[j] += sh[0][r * vpg + tid][j];
        aq[j] += sh[1][r * vpg + tid][j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      stats[((int64_t)blockIdx.x * 2 + 0) * C + c + j] = as[j];
      stats[((int64_t)blockIdx.x * 2 + 1) * C + c + j] = aq[j];
    }
  }
}

// channel groups of <= 16 eight-channel vectors, as EVEN as possible: C = 144 (18 vectors) is two
// groups of 9, not 16 + 2 (whose second group's workgroups ran a full-length loop with 2 of 16
// vectors busy: 2x the time of the layer's data on blocks.2.x)
static void bn_vpg_groups(int C, int& vpg, int& groups) {
  const int nv = C / 8;
  groups = cdiv(nv, 16);
  vpg = cdiv(nv, groups);
}

template <typename T>
int launch_bn_bwd_reduce(hipStream_t s, const BnBwdIn& in, const T* Y, int64_t M, int C, float* stats, int* stat_rows,
                         int max_rows) {
  if (M > (int64_t)UINT32_MAX) { set_error("bn: more than 2^32 rows", __FILE__, __LINE__); return -1; }
  int vpg, groups;
  bn_vpg_groups(C, vpg, groups);
  const int nrl = 256 / vpg;
  const int64_t rows_needed = cdiv64(M, nrl * 4);
  int gx = (int)std::max<int64_t>(1, std::min<int64_t>(rows_needed, std::max(1, 1024 / groups)));
  if (max_rows > 0) gx = std::min(gx, max_rows);
  switch (bn_flags(in)) {
#define DFD_BNR(F) case F: hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, F>), dim3(gx, groups), dim3(256), 0, s, in, Y, M, C, stats, vpg); break;
    DFD_BNR(0) DFD_BNR(1) DFD_BNR(2) DFD_BNR(3) DFD_BNR(4) DFD_BNR(5) DFD_BNR(6) DFD_BNR(7)
    DFD_BNR(8) DFD_BNR(9) DFD_BNR(10) DFD_BNR(11) DFD_BNR(12) DFD_BNR(13) DFD_BNR(14) DFD_BNR(15)
#undef DFD_BNR
  }
  DFD_HIP_CHECK(hipGetLastError());
  *stat_rows = gx;
  return 0;
}

template <int FIN_CH>
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(const float* __restrict__ stats, int rows, int64_t count,
                                                              int C, const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, int training,
                                                              float* dgamma, float* dbeta, int accumulate,
                                                              float* coef, int centred) {
  __shared__ double sh_s[1024 / 64 * FIN_CH], sh_q[1024 / 64 * FIN_CH];
  const int tid = threadIdx.x;
  const int c = blockIdx.x * FIN_CH + tid;
  // per-channel operands loaded before the reduction (see bn_finalize_kernel)
  float p_g = 0.f, p_is = 0.f, p_mu = 0.f, p_db = 0.f, p_dg = 0.f;
  if (tid < FIN_CH && c < C) {
    p_g = gamma[c];
    p_is = invstd[c];
    if (!centred) p_mu = mean[c];
    if (accumulate) { p_db = dbeta[c]; p_dg = dgamma[c]; }
  }
  double s = 0.0, q = 0.0;
  reduce_stat_rows<FIN_CH>(stats, rows, C, s, q, sh_s, sh_q);
  if (tid < FIN_CH && c < C) {
    const float db = (float)s, dg = (float)q;
    if (accumulate) { dbeta[c] = p_db + db; dgamma[c] = p_dg + dg; }
    else { dbeta[c] = db; dgamma[c] = dg; }
    const double gm = p_g, is = p_is;
    const double k1 = gm * is;
    double k2 = 0.0, k3 = 0.0;
    if (training) {
      const double n = (double)count;
      k2 = -gm * is * is * q / n;
      k3 = -gm * is * s / n;
      if (!centred) k3 += gm * is * is * (double)p_mu * q / n;
    }
    coef[c] = (float)k1;
    coef[C + c] = (float)k2;
    coef[2 * C + c] = (float)k3;
  }
}

int launch_bn_bwd_finalize(hipStream_t s, const float* stats, int rows, int64_t count, int C, const float* gamma,
                           const float* mean, const float* invstd, bool training, float* dgamma, float* dbeta,
                           bool accumulate, float* coef, bool centred) {
#define DFD_FIN(CH)                                                                                                \
  hipLaunchKernelGGL((bn_bwd_finalize_kernel<CH>), dim3(cdiv(C, CH)), dim3(1024), 0, s, stats, rows, count, C, gamma, \
                     mean, invstd, training ? 1 : 0, dgamma, dbeta, accumulate ? 1 : 0, coef, centred ? 1 : 0)
  const int ch = fin_ch(rows);
  if (ch == 16) DFD_FIN(16);
  else if (ch == 8) DFD_FIN(8);
  else DFD_FIN(4);
#undef DFD_FIN
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

template <typename T, int FL>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdIn in, const T* __restrict__ Y,
                                                           const float* __restrict__ coef, T* dY, int64_t nvec, int C) {
  const int cv = C / 8;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  const int64_t step = (int64_t)gridDim.x * 256;  // multiple of cv (cs_grid)
  const int64_t rstep = step / cv;
  int64_t row = i / cv;
  const int c = (int)(i - row * cv) * 8;
  float k1[8], k2[8], k3[8];
  BnBwdCh ch;
  bn_bwd_ch<FL>(in, c, ch);
  ld8f(coef + c, k1);
  ld8f(coef + C + c, k2);
  ld8f(coef + 2 * C + c, k3);
  for (; i < nvec; i += step, row += rstep) {
    float g[8], y[8];
    bn_bwd_g8<T, FL>(in, Y, row, bn_frame<FL>(in, row), c, C, ch, g, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = k1[j] * g[j] + k2[j] * y[j] + k3[j];
    st8(dY + i * 8, g);
  }
}

template <typename T>
int launch_bn_bwd_apply(hipStream_t s, const BnBwdIn& in, const T* Y, const float* coef, T* dY, int64_t M, int C) {
  if (M > (int64_t)UINT32_MAX) { set_error("bn: more than 2^32 rows", __FILE__, __LINE__); return -1; }
  const int64_t nvec = M * C / 8;
  const int gx = cs_grid(nvec, C / 8);
  switch (bn_flags(in)) {
#define DFD_BNA(F) case F: hipLaunchKernelGGL((bn_bwd_apply_kernel<T, F>), dim3(gx), dim3(256), 0, s, in, Y, coef, dY, nvec, C); break;
    DFD_BNA(0) DFD_BNA(1) DFD_BNA(2) DFD_BNA(3) DFD_BNA(4) DFD_BNA(5) DFD_BNA(6) DFD_BNA(7)
    DFD_BNA(8) DFD_BNA(9) DFD_BNA(10) DFD_BNA(11) DFD_BNA(12) DFD_BNA(13) DFD_BNA(14) DFD_BNA(15)
#undef DFD_BNA
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ BN backward finalize + apply
// The finalize (bn_bwd_finalize_kernel) and the apply pass in ONE launch where the producer wrote few
// stat rows: every workgroup owns 64 channels and a chunk of rows; it first reduces the stat rows of
// its channels (16 row lanes x 16 float4 columns, fp64, lanes added in a fixed order -- the same k1..k3
// in every workgroup of the channel group), the row-chunk-0 workgroup also stores dbeta / dgamma /
// coef, then it applies dY = k1*g + k2*y + k3 over its rows.  Saves the ~5 us finalize launch per BN
// backward; the reduction costs each workgroup rows / 16 x 2 loads per thread (used for rows <= 256).
constexpr int BAF_CH = 64, BAF_RL = 16, BAF_ROWS_MAX = 256;
constexpr int64_t BAF_M_MAX = 16384;
struct BnFinArgs {
  int64_t count;
  const float *gamma, *mean, *invstd;
  int training, accumulate;
  float *dgamma, *dbeta, *coef;
};

template <typename T, int FL>
__global__ __launch_bounds__(256) void bn_bwd_apply_fin_kernel(BnBwdIn in, const T* __restrict__ Y, int64_t M, int C,
                                                               const float* __restrict__ stats, int rows, BnFinArgs fa,
                                                               T* dY, int64_t rows_per_wg) {
  __shared__ double sh[2][BAF_RL][BAF_CH];
  __shared__ float kc[3][BAF_CH];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.y * BAF_CH;
  const int nch = min(BAF_CH, C - c0);
  {
    const int c4 = tid & 15, rl = tid >> 4;
    const int c = c0 + 4 * c4;
    double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
    if (4 * c4 < nch) {
      int r = rl;
      for (; r + 7 * BAF_RL < rows; r += 8 * BAF_RL) {  // 16 loads in flight, added in row order
        float4 vs[8], vq[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          vs[u] = *reinterpret_cast<const float4*>(stats + ((int64_t)(r + u * BAF_RL) * 2 + 0) * C + c);
          vq[u] = *reinterpret_cast<const float4*>(stats + ((int64_t)(r + u * BAF_RL) * 2 + 1) * C + c);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          s[0] += vs[u].x; s[1] += vs[u].y; s[2] += vs[u].z; s[3] += vs[u].w;
          q[0] += vq[u].x; q[1] += vq[u].y; q[2] += vq[u].z; q[3] += vq[u].w;
        }
      }
      for (; r < rows; r += BAF_RL) {
        const float4 vs = *reinterpret_cast<const float4*>(stats + ((int64_t)r * 2 + 0) * C + c);
        const float4 vq = *reinterpret_cast<const float4*>(stats + ((int64_t)r * 2 + 1) * C + c);
        s[0] += vs.x; s[1] += vs.y; s[2] += vs.z; s[3] += vs.w;
        q[0] += vq.x; q[1] += vq.y; q[2] += vq.z; q[3] += vq.w;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sh[0][rl][4 * c4 + j] = s[j];
      sh[1][rl][4 * c4 + j] = q[j];
    }
  }
  __syncthreads();
  if (tid < nch) {
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int l = 0; l < BAF_RL; ++l) { s += sh[0][l][tid]; q += sh[1][l][tid]; }
    const int c = c0 + tid;
    const double gm = fa.gamma[c], is = fa.invstd[c];
    const double k1 = gm * is;
    double k2 = 0.0, k3 = 0.0;
    if (fa.training) {
      const double n = (double)fa.count;
      k2 = -gm * is * is * q / n;
      k3 = -gm * is * s / n + gm * is * is * (double)fa.mean[c] * q / n;
    }
    kc[0][tid] = (float)k1;
    kc[1][tid] = (float)k2;
    kc[2][tid] = (float)k3;
    if (blockIdx.x == 0) {
      const float db = (float)s, dg = (float)q;
      fa.dbeta[c] = fa.accumulate ? fa.dbeta[c] + db : db;
      fa.dgamma[c] = fa.accumulate ? fa.dgamma[c] + dg : dg;
      if (fa.coef) {
        fa.coef[c] = (float)k1;
        fa.coef[C + c] = (float)k2;
        fa.coef[2 * C + c] = (float)k3;
      }
    }
  }
  __syncthreads();
  // apply: 8 channel vectors x 32 row lanes, two rows' loads in flight
  const int v = tid & 7, rl = tid >> 3;
  const int cl = 8 * v, c = c0 + cl;
  if (cl >= nch) return;
  float k1[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { k1[j] = kc[0][cl + j]; k2[j] = kc[1][cl + j]; k3[j] = kc[2][cl + j]; }
  BnBwdCh ch;
  bn_bwd_ch<FL>(in, c, ch);
  const int64_t rb = (int64_t)blockIdx.x * rows_per_wg, re = min(M, rb + rows_per_wg);
  int64_t row = rb + rl;
  for (; row + 32 < re; row += 64) {
    float g[2][8], y[2][8];
    bn_bwd_g8<T, FL>(in, Y, row, bn_frame<FL>(in, row), c, C, ch, g[0], y[0]);
    bn_bwd_g8<T, FL>(in, Y, row + 32, bn_frame<FL>(in, row + 32), c, C, ch, g[1], y[1]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[u][j] = k1[j] * g[u][j] + k2[j] * y[u][j] + k3[j];
      st8(dY + (row + 32 * u) * C + c, g[u]);
    }
  }
  if (row < re) {
    float g[8], y[8];
    bn_bwd_g8<T, FL>(in, Y, row, bn_frame<FL>(in, row), c, C, ch, g, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = k1[j] * g[j] + k2[j] * y[j] + k3[j];
    st8(dY + row * C + c, g);
  }
}

// 1: launched; 0: not covered (too many stat rows, or C % 8): the caller runs finalize + apply
template <typename T>
int launch_bn_bwd_apply_fin(hipStream_t s, const BnBwdIn& in, const T* Y, int64_t M, int C, const float* stats, int rows,
                            int64_t count, const float* gamma, const float* mean, const float* invstd, bool training,
                            float* dgamma, float* dbeta, bool accumulate, float* coef, T* dY) {
  // the small late-stage tensors only: at 50,176 rows x 480-672 channels the fused pass measured
  // 45 us against 30 + 5 us for apply + finalize (trace r05 C) -- its channel-group-major grid streams
  // worse than the channel-stationary apply, which the saved launch repays only on short passes
  if (rows < 1 || rows > BAF_ROWS_MAX || (C & 7) || M <= 0 || M > BAF_M_MAX) return 0;
  if (M > (int64_t)UINT32_MAX) { set_error("bn: more than 2^32 rows", __FILE__, __LINE__); return -1; }
  const int G = cdiv(C, BAF_CH);
  // >= 128 rows per workgroup (4 per row lane), <= ~2048 workgroups
  const int64_t rc = std::max<int64_t>(1, std::min<int64_t>(cdiv64(M, 128), std::max(1, 2048 / G)));
  const int64_t rpw = cdiv64(M, rc);
  const BnFinArgs fa{count, gamma, mean, invstd, training ? 1 : 0, accumulate ? 1 : 0, dgamma, dbeta, coef};
  const dim3 grid((unsigned)cdiv64(M, rpw), (unsigned)G);
  switch (bn_flags(in)) {
#define DFD_BAF(F) case F: hipLaunchKernelGGL((bn_bwd_apply_fin_kernel<T, F>), grid, dim3(256), 0, s, in, Y, M, C, stats, rows, fa, dY, rpw); break;
    DFD_BAF(0) DFD_BAF(1) DFD_BAF(2) DFD_BAF(3) DFD_BAF(4) DFD_BAF(5) DFD_BAF(6) DFD_BAF(7)
    DFD_BAF(8) DFD_BAF(9) DFD_BAF(10) DFD_BAF(11) DFD_BAF(12) DFD_BAF(13) DFD_BAF(14) DFD_BAF(15)
#undef DFD_BAF
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 1;
}

// ------------------------------------------------------------------ per-frame channel sums
// part[q][h][f][c] = sum over pixel chunk h of frame f of val_q(p, c), for the per-frame reductions
// of the SE module (one kernel, OP selects the values):
//   FR_SQUEEZE (Q = 1): silu(y*scale+shift); with s_out the activation is also stored (rounded to
//                       T): the late-stage conv_pwl forward and weight gradient read it instead of
//                       recomputing it per N tile
//   FR_SEBWD   (Q = 1): dZ * silu(y*scale+shift)
//   FR_SEBN    (Q = 5): the one-pass SE + BN backward sums D, P1..P4 (below)
// Work split: vpg 8-channel vectors x npl = 256/vpg pixel lanes per workgroup, the lanes being fpb
// frames x pl lanes per frame.  Small maps (7x7: 49 pixels) put several frames in one workgroup so a
// lane still walks ~8 pixels (one frame per workgroup left 3 pixels per lane and a workgroup's
// launch and reduction dominated); large maps split a frame into hsplit chunks.  A lane's pixels go
// in groups of FR_U (4; 2 for the register-heavy FR_SEBN) with every load of a group issued first; the pl lanes of a frame are added in
// lane order through LDS (fixed summation order: bit-reproducible).
enum { FR_SQUEEZE = 0, FR_SEBWD = 1, FR_SEBN = 2 };
struct FrGeom {
  int frames, HW, C, hsplit, vpg, pl, fpb;
};
struct FrCoef {
  const float *scale, *shift, *mean, *invstd;
};

// FIN (squeeze only): the BN's train-mode finalize from its producer's stat rows inside the launch
// (bnfin.h): every workgroup reduces the rows of its channel slice; blockIdx.x == 0 stores the
// constants and the running statistics
template <typename T, int OP, bool FIN = false>
__global__ __launch_bounds__(256) void frame_reduce_kernel(const T* __restrict__ dZ, const T* __restrict__ Y, FrCoef cf,
                                                           FrGeom g, float* __restrict__ part, T* __restrict__ s_out,
                                                           BnFwdFin fin) {
  constexpr int Q = OP == FR_SEBN ? 5 : 1;
  constexpr int FR_U = OP == FR_SEBN ? 2 : 4;  // the five FR_SEBN sums: 2 pixels in flight (occupancy)
  __shared__ float sh[Q][256][8];
  __shared__ double fscr[FIN ? kBnFinScratch : 1];
  __shared__ float fss[2][FIN ? 128 : 1];
  const int tid = threadIdx.x;
  const int vec = tid % g.vpg, l = tid / g.vpg;
  const int fi = l / g.pl, li = l - fi * g.pl;
  const int f = (blockIdx.x / g.hsplit) * g.fpb + fi, h = blockIdx.x % g.hsplit;
  const int c = (blockIdx.y * g.vpg + vec) * 8;
  const int cw0 = blockIdx.y * g.vpg * 8;  // this workgroup's channel slice
  if constexpr (FIN) {
    const int ncw = g.C - cw0 < g.vpg * 8 ? g.C - cw0 : g.vpg * 8;
    bn_fin_wg(fin, g.C, cw0, ncw, blockIdx.x == 0, fss[0], fss[1], fscr);
  }
  const bool act = fi < g.fpb && f < g.frames && c < g.C;
  const int chunk = (g.HW + g.hsplit - 1) / g.hsplit;
  const int p0 = h * chunk, p1 = min(g.HW, p0 + chunk);
  float acc[Q][8];
#pragma unroll
  for (int q = 0; q < Q; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
  if (act) {
    float sc[8], shf[8], mu[8], is[8];
    if constexpr (FIN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { sc[j] = fss[0][c - cw0 + j]; shf[j] = fss[1][c - cw0 + j]; }
    } else {
      ld8f(cf.scale + c, sc);
      ld8f(cf.shift + c, shf);
    }
    if constexpr (OP == FR_SEBN) {
      ld8f(cf.mean + c, mu);
      ld8f(cf.invstd + c, is);
    }
    const int64_t fbase = (int64_t)f * g.HW;
    auto one = [&](int64_t row, float (&y)[8], const float (&d)[8]) {
      if constexpr (OP == FR_SEBN) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float z = y[j] * sc[j] + shf[j];
          const float sg = sigmoidf_(z);
          const float sp = sg * (1.0f + z * (1.0f - sg));
          const float xh = (y[j] - mu[j]) * is[j];
          const float dsp = d[j] * sp;
          acc[0][j] += d[j] * (z * sg);
          acc[1][j] += dsp;
          acc[2 % Q][j] += sp;
          acc[3 % Q][j] += dsp * xh;
          acc[4 % Q][j] += sp * xh;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = siluf_(y[j] * sc[j] + shf[j]);
        if (OP == FR_SQUEEZE && s_out) st8(s_out + row * g.C + c, y);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[0][j] += OP == FR_SEBWD ? y[j] * d[j] : y[j];
      }
    };
    int p = p0 + li;
    for (; p + (FR_U - 1) * g.pl < p1; p += FR_U * g.pl) {
      float y[FR_U][8], d[FR_U][8];
#pragma unroll
      for (int u = 0; u < FR_U; ++u) {
        const int64_t row = fbase + p + u * g.pl;
        ld8(Y + row * g.C + c, y[u]);
        if constexpr (OP != FR_SQUEEZE) ld8(dZ + row * g.C + c, d[u]);
      }
#pragma unroll
      for (int u = 0; u < FR_U; ++u) one(fbase + p + u * g.pl, y[u], d[u]);
    }
    for (; p < p1; p += g.pl) {
      const int64_t row = fbase + p;
      float y[8], d[8];
      ld8(Y + row * g.C + c, y);
      if constexpr (OP != FR_SQUEEZE) ld8(dZ + row * g.C + c, d);
      one(row, y, d);
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) sh[q][tid][j] = acc[q][j];
  __syncthreads();
  if (act && li == 0) {
    for (int r = 1; r < g.pl; ++r) {
      const int idx = (l + r) * g.vpg + vec;
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[q][j] += sh[q][idx][j];
    }
    const int64_t n = (int64_t)g.frames * g.C;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      float* o = part + ((int64_t)q * g.hsplit + h) * n + (int64_t)f * g.C + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = acc[q][j];
    }
  }
}

template <typename T, int OP>
static int launch_frame_reduce(hipStream_t s, const T* dZ, const T* Y, const FrCoef& cf, int frames, int HW, int C,
                               float* part, int64_t part_cap, int* hsplit_out, T* s_out = nullptr,
                               const BnFwdFin* fin = nullptr) {
  constexpr int Q = OP == FR_SEBN ? 5 : 1;
  if (frames <= 0 || HW <= 0) { set_error("frame reduce: empty input", __FILE__, __LINE__); return -1; }
  if ((int64_t)Q * frames * C > part_cap) { set_error("frame reduce: partial buffer too small", __FILE__, __LINE__); return -1; }
  FrGeom g{frames, HW, C, 1, 0, 0, 1};
  int groups;
  bn_vpg_groups(C, g.vpg, groups);
  const int npl = 256 / g.vpg;
  g.fpb = std::max(1, std::min(npl, npl * 8 / HW));  // frames per workgroup: >= ~8 pixels per lane
  g.pl = npl / g.fpb;
  const int fgroups = cdiv(frames, g.fpb);
  while ((int64_t)fgroups * groups * g.hsplit < 1024 && HW / (g.hsplit * 2) >= g.pl * 8 &&
         (int64_t)Q * (g.hsplit * 2) * frames * C <= part_cap)
    g.hsplit *= 2;
  // the input BN's finalize: inside the launch where its stat rows are few (squeeze; channel slices of
  // <= 128), else its own launch first (cf.scale / cf.shift are that launch's outputs)
  const bool embed = OP == FR_SQUEEZE && fin && fin->rows > 0 && fin->rows <= kBnFinRowsMax && g.vpg * 8 <= 128;
  if (fin && fin->rows > 0 && !embed) DFD_TRY(launch_bn_finalize_fin(s, *fin, C));
  if constexpr (OP == FR_SQUEEZE) {
    if (embed) {
      hipLaunchKernelGGL((frame_reduce_kernel<T, OP, true>), dim3(fgroups * g.hsplit, groups), dim3(256), 0, s, dZ, Y,
                         cf, g, part, s_out, *fin);
      DFD_HIP_CHECK(hipGetLastError());
      *hsplit_out = g.hsplit;
      return 0;
    }
  }
    hipLaunchKernelGGL((frame_reduce_kernel<T, OP>), dim3(fgroups * g.hsplit, groups), dim3(256), 0, s, dZ, Y, cf, g,
                       part, s_out, BnFwdFin{});
  DFD_HIP_CHECK(hipGetLastError());
  *hsplit_out = g.hsplit;
  return 0;
}

// sum hsplit partials: out[f][c] = scale * sum_h part[h][f][c]
__global__ void sum_parts_kernel(const float* __restrict__ part, int hsplit, int64_t n, float scale,
                                 float* __restrict__ out) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float a = 0.f;
    int h = 0;
    for (; h + 4 <= hsplit; h += 4) {  // 4 loads in flight, added in order
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = part[(h + u) * n + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) a += v[u];
    }
    for (; h < hsplit; ++h) a += part[h * n + i];
    out[i] = a * scale;
  }
}

// the squeeze's per-frame partial sums part[h][f][c] (h < *hsplit); the excitation (se_chain_kernel)
// adds the partials and scales by 1/HW while loading them
template <typename T>
int launch_se_squeeze(hipStream_t s, const T* Y, const Pro& pro, int frames, int HW, int C, float* part,
                      int64_t part_cap, int* hsplit, T* s_out, const BnFwdFin* fin) {
  const FrCoef cf{pro.scale, pro.shift, nullptr, nullptr};
  return launch_frame_reduce<T, FR_SQUEEZE>(s, nullptr, Y, cf, frames, HW, C, part, part_cap, hsplit, s_out, fin);
}

template <typename T>
int launch_se_bwd_reduce(hipStream_t s, const T* dZ, const T* Y, const Pro& pro, int frames, int HW, int C,
                         float* part, int64_t part_cap, float* dgate) {
  int hs;
  const FrCoef cf{pro.scale, pro.shift, nullptr, nullptr};
  if (launch_frame_reduce<T, FR_SEBWD>(s, dZ, Y, cf, frames, HW, C, part, part_cap, &hs)) return -1;
  const int64_t n = (int64_t)frames * C;
  hipLaunchKernelGGL(sum_parts_kernel, dim3(ew_grid(n)), dim3(256), 0, s, part, hs, n, 1.0f, dgate);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ SE + BN backward, one pass
// Backward of  out = silu(z) * gate[f][c] (feeding conv_pwl),  z = y*scale + shift (BN, batch
// stats), sq = mean_hw silu(z) (SE squeeze).  With ge = dL/dout and bc[f][c] = dL/dsq / HW the
// BN's input gradient is g = (ge*gate + bc) * silu'(z); since gate and bc are constant per
// (frame, channel), every reduction the backward needs decomposes into per-frame sums that one
// pass over (ge, y) produces before bc is known (frame_reduce_kernel<FR_SEBN>):
//   D  = sum ge*silu(z)      (-> dgate, the SE branch)
//   P1 = sum ge*silu'(z)     P2 = sum silu'(z)     P3 = sum ge*silu'(z)*xhat     P4 = sum silu'(z)*xhat
// so that  sum g = sum_f gate*P1 + bc*P2  and  sum g*xhat = sum_f gate*P3 + bc*P4.  This replaces
// the separate SE-backward reduction and BN-backward reduction (two full passes over ge and y).
template <typename T>
int launch_se_bn_bwd_reduce(hipStream_t s, const T* dZ, const T* Y, const float* scale, const float* shift,
                            const float* mean, const float* invstd, int frames, int HW, int C, float* part,
                            int64_t part_cap, int* hsplit_out) {
  const FrCoef cf{scale, shift, mean, invstd};
  return launch_frame_reduce<T, FR_SEBN>(s, dZ, Y, cf, frames, HW, C, part, part_cap, hsplit_out);
}

// BN backward finalize from the per-frame sums of frame_reduce_kernel<FR_SEBN> once bc is known:
// dbeta = sum g, dgamma = sum g*xhat, coefficients k1..k3 of dy = k1*g + k2*y + k3 (fp64).
// The sums P1..P4 are the partials part[1..4][h][f][c] of that kernel, added over h in order.
// Block = 64 channels x 16 frame slices (the slices' frames unrolled by 4, all loads issued
// up front); slices added in order.
constexpr int FF_SL = 16;
struct PartSum {  // P[q][i] = sum_h part[(q + 1) * hsplit + h][i]  (q = 0..3 -> P1..P4)
  const float* part;
  int hsplit;
  int64_t n;
  __device__ __forceinline__ float operator()(int q, int64_t i) const {
    const float* b = part + ((int64_t)(q + 1) * hsplit) * n + i;
    float a = b[0];
    for (int h = 1; h < hsplit; ++h) a += b[(int64_t)h * n];
    return a;
  }
};
// ONE: chunk 0 of each q already holds the sum (hsplit == 1, or added by sum_parts4_kernel) -- plain
// loads, all issued up front
template <bool ONE>
__device__ __forceinline__ float part_sum(const PartSum& ps, int q, int64_t i) {
  if constexpr (ONE) return ps.part[(int64_t)(q + 1) * ps.hsplit * ps.n + i];
  return ps(q, i);
}
// part[q][h][i] (q = 1..4) -> part[q][0][i] = sum over h in order (in place: element (q, i) is read
// and written by one thread only); the finalize then reads chunk 0 of each q
__global__ void sum_parts4_kernel(float* __restrict__ part, int hsplit, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < 4 * n; i += (int64_t)gridDim.x * 256) {
    const int64_t q = i / n + 1, k = i - (q - 1) * n;
    float a = 0.f;
    for (int h = 0; h < hsplit; ++h) a += part[(q * hsplit + h) * n + k];
    part[q * hsplit * n + k] = a;
  }
}

template <bool ONE>
__global__ __launch_bounds__(1024) void bn_bwd_finalize_frames_kernel(
    const float* __restrict__ part, int hsplit, const float* __restrict__ gate, const float* __restrict__ bc, int frames,
    int C, int64_t count, const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ invstd, int training, float* dgamma, float* dbeta, int accumulate, float* coef) {
  __shared__ double red[2][FF_SL][64];
  const int tid = threadIdx.x, cl = tid & 63, sl = tid >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int64_t n = (int64_t)frames * C;
  const PartSum pf{part, hsplit, n};
  // per-channel operands loaded before the reduction (see bn_finalize_kernel)
  float p_g = 0.f, p_is = 0.f, p_mu = 0.f, p_db = 0.f, p_dg = 0.f;
  if (sl == 0 && c < C) {
    p_g = gamma[c];
    p_is = invstd[c];
    p_mu = mean[c];
    if (accumulate) { p_db = dbeta[c]; p_dg = dgamma[c]; }
  }
  double s = 0.0, q = 0.0;
  if (c < C) {
    const int per = (frames + FF_SL - 1) / FF_SL;
    const int f0 = sl * per, f1 = min(frames, f0 + per);
    int f = f0;
    for (; f + 4 <= f1; f += 4) {
      float gt[4], b[4], p1[4], p2[4], p3[4], p4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = (int64_t)(f + u) * C + c;
        gt[u] = gate[i]; b[u] = bc[i];
        p1[u] = part_sum<ONE>(pf, 0, i); p2[u] = part_sum<ONE>(pf, 1, i);
        p3[u] = part_sum<ONE>(pf, 2, i); p4[u] = part_sum<ONE>(pf, 3, i);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += (double)gt[u] * (double)p1[u] + (double)b[u] * (double)p2[u];
        q += (double)gt[u] * (double)p3[u] + (double)b[u] * (double)p4[u];
      }
    }
    for (; f < f1; ++f) {
      const int64_t i = (int64_t)f * C + c;
      s += (double)gate[i] * (double)part_sum<ONE>(pf, 0, i) + (double)bc[i] * (double)part_sum<ONE>(pf, 1, i);
      q += (double)gate[i] * (double)part_sum<ONE>(pf, 2, i) + (double)bc[i] * (double)part_sum<ONE>(pf, 3, i);
    }
  }
  red[0][sl][cl] = s;
  red[1][sl][cl] = q;
  __syncthreads();
  if (sl == 0 && c < C) {
    s = 0.0;
    q = 0.0;
    for (int k = 0; k < FF_SL; ++k) { s += red[0][k][cl]; q += red[1][k][cl]; }
    const float db = (float)s, dg = (float)q;
    if (accumulate) { dbeta[c] = p_db + db; dgamma[c] = p_dg + dg; }
    else { dbeta[c] = db; dgamma[c] = dg; }
    const double gm = p_g, is = p_is;
    double k2 = 0.0, k3 = 0.0;
    if (training) {
      const double cnt = (double)count;
      k2 = -gm * is * is * q / cnt;
      k3 = -gm * is * s / cnt + gm * is * is * (double)p_mu * q / cnt;
    }
    coef[c] = (float)(gm * is);
    coef[C + c] = (float)k2;
    coef[2 * C + c] = (float)k3;
  }
}

int launch_bn_bwd_finalize_frames(hipStream_t s, float* part, int hsplit, const float* gate, const float* bc,
                                  int frames, int C, int64_t count, const float* gamma, const float* mean,
                                  const float* invstd, bool training, float* dgamma, float* dbeta, bool accumulate,
                                  float* coef) {
  if (hsplit > 1) {
    // the finalize has only C/64 workgroups: add the pixel-chunk partials of q = 1..4 in a parallel
    // pass first (in place into chunk 0, h ascending)
    const int64_t n = (int64_t)frames * C;
    hipLaunchKernelGGL(sum_parts4_kernel, dim3(ew_grid(4 * n)), dim3(256), 0, s, part, hsplit, n);
    DFD_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(bn_bwd_finalize_frames_kernel<true>, dim3(cdiv(C, 64)), dim3(1024), 0, s, part, hsplit, gate, bc,
                     frames, C, count, gamma, mean, invstd, training ? 1 : 0, dgamma, dbeta, accumulate ? 1 : 0, coef);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ conv_pw backward through its BN
// The BN after conv_pw (no activation) has the input gradient ge1 = k1*g + k2*y1 + k3 (per output
// channel k of the conv; bn_bwd_finalize), and y1 = x . W^T is itself a linear function of the
// block input x.  By linearity the conv's gradients need g and x only -- never y1, and no
// materialised ge1 (three full passes over the 6x-expanded tensor saved):
//   dX = g . (diag(k1) W) + x . (W^T diag(k2) W) + W^T k3
//   dW = diag(k1) (g^T x) + diag(k2) W (x^T x) + k3 (1^T x)
// bn_fold_pw: W1t[c][k] = W[k][c] k1[k] (dgrad operand), Q[c][c'] = sum_k W[k][c] k2[k] W[k][c'],
// bv[c] = sum_k k3[k] W[k][c]  (W: fp32 master weights [mid][cin]; sums in fp64, k ascending).
// One workgroup per input channel c (plus one more block per 256 W1t elements): row c of Q and
// bv[c] as k-sliced dot products (4 slices of k per output, fp64, slices added in order).
template <typename T>
__global__ __launch_bounds__(256) void bn_fold_pw_kernel(const float* __restrict__ W, const float* __restrict__ coef,
                                                         int mid, int cin, T* __restrict__ w1t, T* __restrict__ q,
                                                         float* __restrict__ bv) {
  __shared__ double red[4][64];
  if ((int)blockIdx.x >= cin) {  // W1t[c][k] = W[k][c] k1[k]
    const int64_t i = (int64_t)(blockIdx.x - cin) * 256 + threadIdx.x;
    if (i < (int64_t)cin * mid) {
      const int c = (int)(i / mid), k = (int)(i - (int64_t)c * mid);
      w1t[i] = Tr<T>::from_f(W[(int64_t)k * cin + c] * coef[k]);
    }
    return;
  }
  const int c = blockIdx.x, tid = threadIdx.x, cl = tid & 63, sl = tid >> 6;
  const int per = (mid + 3) / 4, k0 = sl * per, k1 = min(mid, k0 + per);
  for (int c2b = 0; c2b <= cin; c2b += 64) {  // column cin = bv
    const int c2 = c2b + cl;
    double a = 0.0;
    if (c2 < cin) {
      for (int k = k0; k < k1; ++k) a += (double)(W[(int64_t)k * cin + c] * coef[mid + k]) * W[(int64_t)k * cin + c2];
    } else if (c2 == cin) {
      for (int k = k0; k < k1; ++k) a += (double)coef[2 * mid + k] * W[(int64_t)k * cin + c];
    }
    red[sl][cl] = a;
    __syncthreads();
    if (sl == 0 && c2 <= cin) {
      const double v = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
      if (c2 < cin) q[(int64_t)c * cin + c2] = Tr<T>::from_f((float)v);
      else bv[c] = (float)v;
    }
    __syncthreads();
  }
}

template <typename T>
int launch_bn_fold_pw(hipStream_t s, const float* W, const float* coef, int mid, int cin, T* w1t, T* q, float* bv) {
  const int blocks = cin + (int)cdiv64((int64_t)cin * mid, 256);
  hipLaunchKernelGGL((bn_fold_pw_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, W, coef, mid, cin, w1t, q, bv);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// dW[k][c] (+)= k1[k] Tg[k][c] + k2[k] sum_c' W[k][c'] G[c'][c] + k3[k] cs[c]: one workgroup per k,
// W row in LDS, thread c sums c' in order (fp64)
__global__ __launch_bounds__(256) void pw_wgrad_bn_combine_kernel(const float* __restrict__ Tg,
                                                                  const float* __restrict__ G,
                                                                  const float* __restrict__ cs,
                                                                  const float* __restrict__ W,
                                                                  const float* __restrict__ coef, int mid, int cin,
                                                                  float* dW, int accumulate) {
  __shared__ float wr[256];
  const int k = blockIdx.x;
  for (int i = threadIdx.x; i < cin; i += 256) wr[i] = W[(int64_t)k * cin + i];
  __syncthreads();
  for (int c = threadIdx.x; c < cin; c += 256) {
    double t = 0.0;
    for (int c2 = 0; c2 < cin; ++c2) t += (double)wr[c2] * G[(int64_t)c2 * cin + c];
    const int64_t i = (int64_t)k * cin + c;
    const double a = (double)coef[k] * Tg[i] + (double)coef[mid + k] * t + (double)coef[2 * mid + k] * cs[c];
    dW[i] = accumulate ? dW[i] + (float)a : (float)a;
  }
}

int launch_pw_wgrad_bn_combine(hipStream_t s, const float* Tg, const float* G, const float* cs, const float* W,
                               const float* coef, int mid, int cin, float* dW, bool accumulate) {
  if (cin > 256) { set_error("pw bn combine: cin > 256", __FILE__, __LINE__); return -1; }
  hipLaunchKernelGGL(pw_wgrad_bn_combine_kernel, dim3((unsigned)mid), dim3(256), 0, s, Tg, G, cs, W, coef, mid, cin,
                     dW, accumulate ? 1 : 0);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// column sums of X [M][C]: part rows [gx][C] (vpg threads per row, rows strided, fixed-order
// tree over the block's row lanes), then the slab reducer
template <typename T>
__global__ __launch_bounds__(256) void col_sums_kernel(const T* __restrict__ X, int64_t M, int C, int vpg,
                                                       float* __restrict__ part) {
  __shared__ float sh[256][8];
  const int tid = threadIdx.x, vec = tid % vpg, rl = tid / vpg, nrl = 256 / vpg;
  const int c = (blockIdx.y * vpg + vec) * 8;
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  if (rl < nrl && c < C) {
    for (int64_t r = (int64_t)blockIdx.x * nrl + rl; r < M; r += (int64_t)gridDim.x * nrl) {
      float x[8];
      ld8(X + r * C + c, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += x[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[tid][j] = a[j];
  __syncthreads();
  if (tid < vpg && c < C) {
    for (int r = 1; r < nrl; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += sh[r * vpg + tid][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) part[(int64_t)blockIdx.x * C + c + j] = a[j];
  }
}

template <typename T>
int launch_col_sums(hipStream_t s, const T* X, int64_t M, int C, float* part, int64_t part_cap, float* out) {
  int vpg, groups;
  bn_vpg_groups(C, vpg, groups);
  const int nrl = 256 / vpg;
  int64_t gx = std::max<int64_t>(1, std::min<int64_t>(cdiv64(M, nrl * 8), std::max(1, 1024 / groups)));
  gx = std::max<int64_t>(1, std::min<int64_t>(gx, part_cap / C));
  hipLaunchKernelGGL((col_sums_kernel<T>), dim3((unsigned)gx, groups), dim3(256), 0, s, X, M, C, vpg, part);
  DFD_HIP_CHECK(hipGetLastError());
  return launch_reduce_slabs(s, part, (int)gx, C, out, false);
}

template <typename T>
int launch_gap(hipStream_t s, const T* Y, const Pro& pro, int frames, int HW, int C, float* feat, const BnFwdFin* fin) {
  // HW is tiny (7x7 at 224^2): one partial per frame (the partial buffer is feat itself, so
  // hsplit = 1), then the means in place
  const FrCoef cf{pro.scale, pro.shift, nullptr, nullptr};
  int hs = 1;
  if (launch_frame_reduce<T, FR_SQUEEZE>(s, nullptr, Y, cf, frames, HW, C, feat, (int64_t)frames * C, &hs, nullptr,
                                         fin))
    return -1;
  const int64_t n = (int64_t)frames * C;
  hipLaunchKernelGGL(sum_parts_kernel, dim3(ew_grid(n)), dim3(256), 0, s, feat, 1, n, 1.0f / (float)HW, feat);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ SE excitation (per frame)
// timm SqueezeExcite conv_reduce / act / conv_expand / sigmoid on the per-frame channel means,
// forward and input-gradient backward, as ONE launch each: two chained small GEMMs per tile of
// 16 frames on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact products, fixed summation order):
//   T[f][j]   = epi1( sum_c A[f][c] B1(c, j) )      j < rd  (the 16 waves split c; LDS sum in order)
//   out[f][c] = epi2( sum_j T[f][j] B2(j, c) )      c in this workgroup's channel slice
// forward  A = sq: B1(c,j) = Wr[j][c], T1 = rpre = . + br (saved), T = silu(rpre);
//          B2(j,c) = We[c][j], out = gate = sigmoid(. + be)
// backward A = de = dgate g (1-g): B1(c,j) = We[c][j], T = dz = . * silu'(rpre) (saved);
//          B2(j,c) = Wr[j][c], out = bc = inv_hw * .   (the squeeze path's input gradient)
// The channel slices (gridDim.y) recompute the small first product instead of a second launch.
constexpr int SE_RDMAX = 48, SE_TS = SE_RDMAX + 4, SE_CSL = 256, SE_W = 16;  // SE_W waves per workgroup
#ifndef DFD_SE_B2PF
#define DFD_SE_B2PF 1
#endif
typedef float se_f32x4 __attribute__((ext_vector_type(4)));

// A is read from the squeeze / SE-backward partials A[h][f][c] (h < hsplit, added in order):
// forward A = a_scale * sum (the squeeze mean), backward A = sum * g (1 - g) with g = a_gate[f][c]
// (de = dgate * sigmoid'); the workgroups of channel slice 0 store A to a_out (sq / de), which the
// backward's weight gradients read.
// FIN (backward only): the BN2 backward finalize of bn_bwd_finalize_frames_kernel folded into the
// same launch -- every workgroup adds its 16 frames' terms gate*P1 + bc*P2 / gate*P3 + bc*P4 (fp64)
// for its channel slice into a partial row, and the last-arriving workgroup of the slice (tail.h)
// sums the frame tiles' rows in order and writes dbeta, dgamma and the coefficients k1..k3.
struct SeFin {
  const float* part;  // frame_reduce<FR_SEBN> partials part[5][hsplit][frames][C] (q = 1..4 read)
  int hsplit;
  double* rows;       // [frame tiles][2][C] scratch
  unsigned* ctr;      // one zeroed counter per channel slice
  int64_t count;      // BN rows (frames x HW)
  const float *gamma, *mean, *invstd;
  int training, accumulate;
  float *dgamma, *dbeta, *coef;
};

// SPLIT (SeSplit.on): the first product is split over the channel slices too -- the workgroup of
// slice s sums only k in its own slice (one 16-deep k step per wave instead of C / 256), writes its
// partial T to scratch, the slices of a frame tile meet at a counter barrier (the grid is launched
// slice-fastest and only when every workgroup is co-resident, so the spin cannot starve a sibling)
// and each adds the slices' partials in slice order.  Used where C > 256 (several slices), whose
// first product was a chain of C / 256 dependent load round trips per wave.
struct SeSplit {
  float* tp;      // [frame tiles][slices][16][SE_TS] partial first products
  unsigned* bar;  // 2 zeroed counters (arrive, depart) per frame tile
  int on;
  SyncAbort ab;   // a timed-out slice barrier is reported here (the plan raises on its next call)
};

// the slice barrier: group_sync (tail.h); false when it timed out (the workgroup leaves)
__device__ __forceinline__ bool se_group_sync(unsigned* arrive, unsigned* depart, unsigned n, const SyncAbort& ab) {
  return group_sync(arrive, depart, n, ab);
}

// grid: x = channel slice (fastest), y = 16-frame tile
template <bool FWD, bool FIN = false>
__global__ __launch_bounds__(64 * SE_W) void se_chain_kernel(const float* __restrict__ A, int hsplit, float a_scale,
                                                       const float* __restrict__ a_gate, float* __restrict__ a_out,
                                                       int frames, int C, int rd,
                                                       const float* __restrict__ W1, const float* __restrict__ b1,
                                                       const float* __restrict__ rpre_in,
                                                       const float* __restrict__ W2, const float* __restrict__ b2,
                                                       float scale2, float* __restrict__ t1_out,
                                                       float* __restrict__ out, SeFin fin, SeSplit sp) {
  __shared__ float red[SE_W][3][4][64];
  __shared__ float Ts[16][SE_TS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int slc = blockIdx.x, nsl = gridDim.x, ftile = blockIdx.y, nft = gridDim.y;
  const int f0 = ftile * 16;
  const int nt1 = (rd + 15) / 16;
  const int cbeg = slc * SE_CSL, cend = min(C, cbeg + SE_CSL);
  // FIN: this lane's second-product outputs are column cbeg + 16 wave + li, frames f0 + 4 lk + r; their
  // gate and frame sums P1..P4 (added over the pixel chunks) are loaded up front, off the chain
  float fgt[4], fp[4][4];
  if constexpr (FIN) {
    const int n = cbeg + 16 * wave + li;
    const int64_t nfc = (int64_t)frames * C;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = f0 + 4 * lk + r;
      const bool ok = f < frames && n < C;
      const int64_t i = ok ? (int64_t)f * C + n : 0;
      fgt[r] = ok ? a_gate[i] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) fp[r][q] = ok ? fin.part[(int64_t)(q + 1) * fin.hsplit * nfc + i] : 0.f;
    }
    for (int h = 1; h < fin.hsplit; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = f0 + 4 * lk + r;
        const bool ok = f < frames && n < C;
        const int64_t i = ok ? (int64_t)f * C + n : 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) fp[r][q] += ok ? fin.part[((int64_t)(q + 1) * fin.hsplit + h) * nfc + i] : 0.f;
      }
  }
  // the second product's B2 column of this wave's first (usually only) 16-channel block, loaded up front:
  // independent of T, so its round trip overlaps the first product and the slice barrier instead of
  // following them (DFD_SE_B2PF, A/B build switch)
  float bw0[SE_RDMAX / 4];
  if constexpr (DFD_SE_B2PF) {
    const int n = cbeg + 16 * wave + li;
#pragma unroll
    for (int i = 0; i < SE_RDMAX / 4; ++i) {
      const int k = 4 * i + lk;
      const bool ok = n < cend && k < rd;
      bw0[i] = ok ? (FWD ? W2[(int64_t)n * rd + k] : W2[(int64_t)k * C + n]) : 0.f;
    }
  }
  // ---- T = A[16 frames][C] . B1[C][rd] ----
  se_f32x4 acc1[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc1[t] = se_f32x4{0.f, 0.f, 0.f, 0.f};
  const bool fok = f0 + li < frames;
  // k range of the first product: this slice's channels (split) or all of them
  const int kbeg = sp.on ? cbeg : 0, kend = sp.on ? cend : C;
  const bool store_a = sp.on || slc == 0;  // every A element stored once (sq / de for the weight gradients)
  // 16 k per iteration; lane group lk takes k = k0 + 4 lk + u in MFMA step u (the same
  // permutation on both operands), so the row-major operands load as 16-B vectors (C % 8 == 0)
  for (int k0 = kbeg + 16 * wave; k0 < kend; k0 += 16 * SE_W) {
    const int kq = k0 + 4 * lk;
    const bool kok = kq < kend;
    float av[4], bv[4][3];
    if (fok && kok) {
      const int64_t ai = (int64_t)(f0 + li) * C + kq, hn = (int64_t)frames * C;
      float4 a4 = *reinterpret_cast<const float4*>(A + ai);
      if (hsplit > 1)
      for (int h = 1; h < hsplit; ++h) {
        const float4 v = *reinterpret_cast<const float4*>(A + h * hn + ai);
        a4.x += v.x; a4.y += v.y; a4.z += v.z; a4.w += v.w;
      }
      if constexpr (FWD) {
        a4.x *= a_scale; a4.y *= a_scale; a4.z *= a_scale; a4.w *= a_scale;
      } else {
        const float4 g = *reinterpret_cast<const float4*>(a_gate + ai);
        a4.x = a4.x * g.x * (1.f - g.x); a4.y = a4.y * g.y * (1.f - g.y);
        a4.z = a4.z * g.z * (1.f - g.z); a4.w = a4.w * g.w * (1.f - g.w);
      }
      if (store_a) *reinterpret_cast<float4*>(a_out + ai) = a4;
      av[0] = a4.x; av[1] = a4.y; av[2] = a4.z; av[3] = a4.w;
    } else {
      av[0] = av[1] = av[2] = av[3] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int n = 16 * t + li;
      const bool ok = t < nt1 && n < rd && kok;
      if constexpr (FWD) {
        const float4 b4 = ok ? *reinterpret_cast<const float4*>(W1 + (int64_t)n * C + kq) : make_float4(0.f, 0.f, 0.f, 0.f);
        bv[0][t] = b4.x; bv[1][t] = b4.y; bv[2][t] = b4.z; bv[3][t] = b4.w;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) bv[u][t] = ok ? W1[(int64_t)(kq + u) * rd + n] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        if (t < nt1) acc1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u][t], acc1[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][t][r][lane] = acc1[t][r];
  __syncthreads();
  // element (fl, j): MFMA D layout lane = 16 * (fl / 4) + j % 16, register fl % 4, tile j / 16;
  // 16 x SE_TS < 64 SE_W: one element per thread
  static_assert(16 * SE_TS <= 64 * SE_W, "one first-product element per thread");
  const int fl = tid / SE_TS, j = tid - fl * SE_TS;
  const bool el = tid < 16 * SE_TS && j < rd;
  float v = 0.f;
  if (el) {
    const int t = j >> 4, ln = 16 * (fl >> 2) + (j & 15), r = fl & 3;
#pragma unroll
    for (int w = 0; w < SE_W; ++w) v += red[w][t][r][ln];
  }
  if (sp.on) {  // the slices' partials of this frame tile, added in slice order
    float* tp = sp.tp + (int64_t)ftile * nsl * 16 * SE_TS;
    if (el) tp[slc * 16 * SE_TS + tid] = v;
    if (!se_group_sync(sp.bar + 2 * ftile, sp.bar + 2 * ftile + 1, (unsigned)nsl, sp.ab)) return;
    if (el) {  // up to 8 slices' loads in flight, added in slice order
      float pv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) pv[q] = q < nsl ? tp[q * 16 * SE_TS + tid] : 0.f;
      v = pv[0];
#pragma unroll
      for (int q = 1; q < 8; ++q)
        if (q < nsl) v += pv[q];
      for (int q = 8; q < nsl; ++q) v += tp[q * 16 * SE_TS + tid];
    }
  }
  if (tid < 16 * SE_TS) {
    float tv = 0.f;
    const int f = f0 + fl;
    if (el && f < frames) {
      if constexpr (FWD) {
        v += b1[j];
        if (slc == 0) t1_out[(int64_t)f * rd + j] = v;
        tv = siluf_(v);
      } else {
        v *= dsiluf_(rpre_in[(int64_t)f * rd + j]);
        if (slc == 0) t1_out[(int64_t)f * rd + j] = v;
        tv = v;
      }
    }
    Ts[fl][j] = tv;  // zero for j >= rd and for frames past the end
  }
  __syncthreads();
  // ---- out = T[16][rd] . B2[rd][C slice] ----
  for (int n0 = cbeg + 16 * wave; n0 < cend; n0 += 16 * SE_W) {
    const int n = n0 + li;
    const bool nok = n < cend;
    // all of B2's column for this lane first (<= 12 independent loads in flight), then the MFMA
    // chain in the same k order (one serialized load per MFMA step was the kernel's latency chain)
    float bw[SE_RDMAX / 4];
    const bool pre = DFD_SE_B2PF && n0 == cbeg + 16 * wave;
#pragma unroll
    for (int i = 0; i < SE_RDMAX / 4; ++i) {
      const int k = 4 * i + lk;
      const bool ok = nok && k < rd;
      bw[i] = pre ? bw0[i] : ok ? (FWD ? W2[(int64_t)n * rd + k] : W2[(int64_t)k * C + n]) : 0.f;
    }
    se_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < SE_RDMAX / 4; ++i)
      if (4 * i < rd) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Ts[li][4 * i + lk], bw[i], acc, 0, 0, 0);
    double fs = 0.0, fq = 0.0;  // FIN: this lane's frames' BN2-backward terms
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = f0 + 4 * lk + r;
      if (f < frames && nok) {
        const float o = FWD ? sigmoidf_(acc[r] + b2[n]) : acc[r] * scale2;
        out[(int64_t)f * C + n] = o;
        if constexpr (FIN) {
          fs += (double)fgt[r] * (double)fp[r][0] + (double)o * (double)fp[r][1];
          fq += (double)fgt[r] * (double)fp[r][2] + (double)o * (double)fp[r][3];
        }
      }
    }
    if constexpr (FIN) {
      // the 4 frame groups of a column (lanes li, li+16, li+32, li+48) in a fixed order
      fs += __shfl_xor(fs, 16, 64);
      fq += __shfl_xor(fq, 16, 64);
      fs += __shfl_xor(fs, 32, 64);
      fq += __shfl_xor(fq, 32, 64);
      if (lk == 0 && nok) {
        tail_store(fin.rows + ((int64_t)ftile * 2 + 0) * C + n, fs);
        tail_store(fin.rows + ((int64_t)ftile * 2 + 1) * C + n, fq);
      }
    }
  }
  if constexpr (FIN) {
    if (!tail_arrive(fin.ctr + slc, nft)) return;
    // last workgroup of this channel slice: frame tiles in order, then bn_bwd_finalize_frames' arithmetic
    const int c = cbeg + tid;
    if (c < cend) {
      const float p_g = fin.gamma[c], p_is = fin.invstd[c], p_mu = fin.mean[c];
      const float p_db = fin.accumulate ? fin.dbeta[c] : 0.f, p_dg = fin.accumulate ? fin.dgamma[c] : 0.f;
      double s = 0.0, q = 0.0;
      int t = 0;
      for (; t + 8 <= nft; t += 8) {  // 16 loads in flight, added in tile order
        double vs[8], vq[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          vs[u] = tail_load(fin.rows + ((int64_t)(t + u) * 2 + 0) * C + c);
          vq[u] = tail_load(fin.rows + ((int64_t)(t + u) * 2 + 1) * C + c);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) { s += vs[u]; q += vq[u]; }
      }
      for (; t < nft; ++t) {
        s += tail_load(fin.rows + ((int64_t)t * 2 + 0) * C + c);
        q += tail_load(fin.rows + ((int64_t)t * 2 + 1) * C + c);
      }
      const float db = (float)s, dg = (float)q;
      fin.dbeta[c] = fin.accumulate ? p_db + db : db;
      fin.dgamma[c] = fin.accumulate ? p_dg + dg : dg;
      const double gm = p_g, is = p_is;
      double k2 = 0.0, k3 = 0.0;
      if (fin.training) {
        const double cnt = (double)fin.count;
        k2 = -gm * is * is * q / cnt;
        k3 = -gm * is * s / cnt + gm * is * is * (double)p_mu * q / cnt;
      }
      fin.coef[c] = (float)(gm * is);
      fin.coef[C + c] = (float)k2;
      fin.coef[2 * C + c] = (float)k3;
    }
  }
}

// CUs of the current device (co-residency bound of the split excitation's barrier)
static int se_device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cus[dev] = n;
  }
  return cus[dev];
}

// the split form where it applies: several slices, one 1024-thread workgroup per CU fits the whole grid
static SeSplit se_split(const SeScratch* sc, int frames, int C) {
  SeSplit sp{};
  if (!sc || !sc->bar || !sc->tp) return sp;
  const int64_t nsl = cdiv(C, SE_CSL), nft = cdiv(frames, 16);
  // >= 4 slices (C > 768): the slice barrier costs ~3-4 us, which the split repays only where the
  // unsplit first product walks >= 4 dependent k steps per wave (trace r05 C: 7x7 stage -2 us per
  // launch, 14x14 stage +0.5..2 us)
  if (nsl < 4 || nsl * nft > se_device_cus() || 2 * nft > sc->bar_slots || nft * nsl * 16 * SE_TS > sc->tp_cap)
    return sp;
  sp.tp = sc->tp;
  sp.bar = sc->bar;
  sp.on = 1;
  static const unsigned long long budget = sync_budget_ticks(2.0);
  sp.ab = SyncAbort{sc->abort_dev, sc->abort_host, budget};
  return sp;
}

int launch_se_fc_fwd(hipStream_t s, const float* part, int hsplit, float inv_hw, float* sq, const float* wr,
                     const float* br, const float* we, const float* be, int frames, int C, int rd, float* rpre,
                     float* gate, const SeScratch* sc) {
  if (rd < 1 || rd > SE_RDMAX) { set_error("se: reduce width out of range", __FILE__, __LINE__); return -1; }
  const dim3 grid((unsigned)cdiv(C, SE_CSL), (unsigned)cdiv(frames, 16));
  hipLaunchKernelGGL(se_chain_kernel<true>, grid, dim3(64 * SE_W), 0, s, part, hsplit, inv_hw, nullptr, sq, frames, C,
                     rd, wr, br, nullptr, we, be, 1.f, rpre, gate, SeFin{}, se_split(sc, frames, C));
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// SE excitation backward from de = dgate * sigmoid'(.) (launch_se_bn_bwd_reduce):
//   dz[f][j]  = silu'(rpre[f][j]) sum_c de[f][c] we[c][j],  bc[f][c] = inv_hw sum_j dz[f][j] wr[j][c]
//                                                          (se_chain_kernel, one launch)
//   gwe[c][j] = sum_f de[f][c] silu(rpre[f][j]),  gbe = sum_f de      (frames ascending)
//   gwr[j][c] = sum_f dz[f][j] sq[f][c],          gbr = sum_f dz      (one paired MFMA launch)
int launch_se_fc_bwd(hipStream_t s, const float* part, int hsplit, const float* gate, float* de, const float* sq,
                     const float* rpre, const float* wr, const float* we, int frames, int C, int rd, float inv_hw,
                     float* tmp_dz, float* bc_out, float* gwr, float* gbr, float* gwe, float* gbe, bool accumulate,
                     MfmaGemm* defer2, const BnFramesFin* bnf, const SeScratch* sc) {
  if (rd < 1 || rd > SE_RDMAX) { set_error("se: reduce width out of range", __FILE__, __LINE__); return -1; }
  const dim3 grid((unsigned)cdiv(C, SE_CSL), (unsigned)cdiv(frames, 16));
  const SeSplit sp = se_split(sc, frames, C);
  if (bnf) {
    if ((int)grid.x > bnf->ctr_slots || (int64_t)grid.y * 2 * C * 2 > bnf->rows_cap) {
      set_error("se: fused finalize scratch too small", __FILE__, __LINE__);
      return -1;
    }
    const SeFin f{part, hsplit, bnf->rows, bnf->ctr, bnf->count, bnf->gamma, bnf->mean, bnf->invstd,
                  bnf->training ? 1 : 0, bnf->accumulate ? 1 : 0, bnf->dgamma, bnf->dbeta, bnf->coef};
    hipLaunchKernelGGL((se_chain_kernel<false, true>), grid, dim3(64 * SE_W), 0, s, part, hsplit, 1.f, gate, de, frames,
                       C, rd, we, nullptr, rpre, wr, nullptr, inv_hw, tmp_dz, bc_out, f, sp);
  } else {
    hipLaunchKernelGGL((se_chain_kernel<false>), grid, dim3(64 * SE_W), 0, s, part, hsplit, 1.f, gate, de, frames, C,
                       rd, we, nullptr, rpre, wr, nullptr, inv_hw, tmp_dz, bc_out, SeFin{}, sp);
  }
  DFD_HIP_CHECK(hipGetLastError());
  MfmaGemm ge{}, gr{};
  ge.A = de; ge.sam = 1; ge.sak = C; ge.B = rpre; ge.sbk = rd; ge.sbn = 1; ge.b_silu = 1; ge.C = gwe; ge.ldc = rd;
  ge.M = C; ge.N = rd; ge.K = frames; ge.asum = gbe; ge.accumulate = accumulate;
  gr.A = tmp_dz; gr.sam = 1; gr.sak = rd; gr.B = sq; gr.sbk = C; gr.sbn = 1; gr.C = gwr; gr.ldc = C;
  gr.M = rd; gr.N = C; gr.K = frames; gr.asum = gbr; gr.accumulate = accumulate;
  if (defer2) {
    defer2[0] = ge;
    defer2[1] = gr;
    return 0;
  }
  return launch_mfma_small_gemm2(s, ge, gr);
}

// ------------------------------------------------------------------ slab reduce
// out[i] (+)= sum_s slab[s][i]: a workgroup owns 256 consecutive elements (64 lanes x 4, 16-B loads
// when the row stride allows) x SL split lanes; lane sl adds rows sl, sl+SL, ... in order, then
// the SL lanes are added in order through LDS (deterministic, fixed for a given SL).
constexpr int RS_MAXSL = 16;
__device__ __forceinline__ void reduce_cols(const float* __restrict__ slab, int splits, int64_t n, int64_t stride,
                                            float* out, int accumulate, int64_t blk, float (*sh)[64][4]) {
  const int tid = threadIdx.x, il = tid & 63, sl = tid >> 6, nsl = blockDim.x >> 6;
  const int64_t e = (blk * 64 + il) * 4;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (e < n) {
    if (e + 3 < n && ((stride | e) & 3) == 0) {
#pragma unroll 4
      for (int sp = sl; sp < splits; sp += nsl) {
        const float4 v = *reinterpret_cast<const float4*>(slab + (int64_t)sp * stride + e);
        a[0] += v.x; a[1] += v.y; a[2] += v.z; a[3] += v.w;
      }
    } else {
      for (int sp = sl; sp < splits; sp += nsl)
        for (int j = 0; j < 4; ++j)
          if (e + j < n) a[j] += slab[(int64_t)sp * stride + e + j];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) sh[sl][il][j] = a[j];
  __syncthreads();
  if (sl == 0 && e < n) {
    for (int l = 1; l < nsl; ++l)
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] += sh[l][il][j];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (e + j < n) out[e + j] = accumulate ? out[e + j] + a[j] : a[j];
  }
}

__global__ __launch_bounds__(1024) void reduce_slabs_kernel(const float* __restrict__ slab, int splits, int64_t n,
                                                            int64_t stride, float* out, int accumulate) {
  __shared__ float sh[RS_MAXSL][64][4];
  reduce_cols(slab, splits, n, stride, out, accumulate, blockIdx.x, sh);
}

static int rs_lanes(int splits) { return splits > 96 ? 16 : splits > 24 ? 8 : 4; }

int launch_reduce_slabs(hipStream_t s, const float* slab, int splits, int64_t n, float* out, bool accumulate) {
  return launch_reduce_slabs_strided(s, slab, splits, n, n, out, accumulate);
}

// ------------------------------------------------------------------ deferred slab reductions
// Every weight gradient ends in a slab reduce; queued while a SlabDefer is active, a backward
// segment's reductions run as ONE launch (workgroup ranges per job).
struct SlabBatchArgs {
  SlabJob j[SlabDefer::kMax];
  int start[SlabDefer::kMax + 1];
  int nj;
};

__global__ __launch_bounds__(1024) void reduce_slabs_batch_kernel(SlabBatchArgs a) {
  __shared__ float sh[RS_MAXSL][64][4];
  int k = 0;
  while (k + 1 < a.nj && (int)blockIdx.x >= a.start[k + 1]) ++k;
  const SlabJob& jb = a.j[k];
  reduce_cols(jb.slab, jb.splits, jb.n, jb.n, jb.out, jb.accumulate, (int)blockIdx.x - a.start[k], sh);
}

static thread_local SlabDefer* t_slab_defer = nullptr;
SlabDefer* set_slab_defer(SlabDefer* d) {
  SlabDefer* prev = t_slab_defer;
  t_slab_defer = d;
  return prev;
}

int SlabDefer::flush() {
  if (aux) {  // the aux stream's queued slabs (and direct gradient writes) complete first
    DFD_HIP_CHECK(hipEventRecord(ev_aux, aux));
    DFD_HIP_CHECK(hipStreamWaitEvent(stream, ev_aux, 0));
  }
  if (n == 0) return 0;
  SlabBatchArgs a{};
  int blocks = 0, lanes = 4;
  for (int k = 0; k < n; ++k) {
    a.j[k] = jobs[k];
    a.start[k] = blocks;
    blocks += (int)cdiv64(jobs[k].n, 256);
    lanes = std::max(lanes, rs_lanes(jobs[k].splits));
  }
  a.start[n] = blocks;
  a.nj = n;
  n = 0;
  hipLaunchKernelGGL(reduce_slabs_batch_kernel, dim3((unsigned)blocks), dim3(64 * lanes), 0, stream, a);
  DFD_HIP_CHECK(hipGetLastError());
  if (aux) {  // the regions just reduced may be handed to aux-stream kernels next
    DFD_HIP_CHECK(hipEventRecord(ev_main, stream));
    DFD_HIP_CHECK(hipStreamWaitEvent(aux, ev_main, 0));
  }
  return 0;
}

int launch_reduce_slabs_strided(hipStream_t s, const float* slab, int splits, int64_t n, int64_t stride, float* out,
                                bool accumulate) {
  SlabDefer* d = t_slab_defer;
  if (d && (d->stream == s || (d->aux && d->aux == s)) && stride == n && out >= d->lo && out + n <= d->hi && n <= ((int64_t)1 << 30)) {
    if (d->n == SlabDefer::kMax) DFD_TRY(d->flush());
    d->jobs[d->n++] = SlabJob{slab, n, out, splits, accumulate ? 1 : 0};
    return 0;
  }
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3((unsigned)cdiv64(n, 256)), dim3(64 * rs_lanes(splits)), 0, s, slab,
                     splits, n, stride, out, accumulate ? 1 : 0);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

#define DFD_BN_INST(T)                                                                                               \
  template int launch_bn_apply<T>(hipStream_t, const T*, const float*, const float*, const T*, T*, int64_t, int);    \
  template int launch_bn_bwd_reduce<T>(hipStream_t, const BnBwdIn&, const T*, int64_t, int, float*, int*, int);     \
  template int launch_bn_bwd_apply<T>(hipStream_t, const BnBwdIn&, const T*, const float*, T*, int64_t, int);       \
  template int launch_bn_bwd_apply_fin<T>(hipStream_t, const BnBwdIn&, const T*, int64_t, int, const float*, int,  \
                                          int64_t, const float*, const float*, const float*, bool, float*, float*, \
                                          bool, float*, T*);                                                        \
  template int launch_se_squeeze<T>(hipStream_t, const T*, const Pro&, int, int, int, float*, int64_t, int*, T*,   \
                                    const BnFwdFin*);                                                               \
  template int launch_se_bwd_reduce<T>(hipStream_t, const T*, const T*, const Pro&, int, int, int, float*, int64_t, \
                                       float*);                                                                     \
  template int launch_gap<T>(hipStream_t, const T*, const Pro&, int, int, int, float*, const BnFwdFin*);          \
  template int launch_se_bn_bwd_reduce<T>(hipStream_t, const T*, const T*, const float*, const float*, const float*, \
                                          const float*, int, int, int, float*, int64_t, int*);                 \
  template int launch_bn_fold_pw<T>(hipStream_t, const float*, const float*, int, int, T*, T*, float*);             \
  template int launch_col_sums<T>(hipStream_t, const T*, int64_t, int, float*, int64_t, float*);
DFD_BN_INST(float)
DFD_BN_INST(bf16)
DFD_BN_INST(f16)
#undef DFD_BN_INST

}  // namespace dfd
