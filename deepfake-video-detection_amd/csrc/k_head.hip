// Detector head, loss and optimizer kernels (K7, K8 of SURVEY §2.2) on gfx950.
//
//   head   : temporal attention MLP (Linear 1280->64, ReLU, Linear 64->1, Sigmoid),
//            softmax over T, attention-weighted sum, Dropout, fc1 (->256) + ReLU, Dropout, fc2
//            -- src/pretrained_detector.py:65-76, 123-141 -- forward and backward.
//   loss   : weighted 2-class CrossEntropy (ensemble_trainer.py:358, train.py:337), fused fwd/bwd.
//   optim  : global-L2 clip_grad_norm_(max_norm) (ensemble_trainer.py:199) fused into
//            AdamW / Adam (ensemble_trainer.py:146, train.py:323) over the flat fp32 buffer.
//   cast   : fp32 master weights -> compute dtype copies (+ transposed 1x1 weights for dgrad).
#include "kernels.h"
#include "head.h"

namespace dfd {

// ------------------------------------------------------------------ dropout hash (counter based)
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float drop_mul(uint64_t seed, uint32_t stream, int64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  if (p >= 1.f) return 0.f;
  const uint32_t h = mix32((uint32_t)idx ^ mix32((uint32_t)(idx >> 32) ^ mix32((uint32_t)seed ^ mix32(
                          (uint32_t)(seed >> 32) + stream * 0x9E3779B9U))));
  const float u = (float)(h >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.0f / (1.0f - p) : 0.f;
}

// ------------------------------------------------------------------ generic small linear ops
// Y[r][o] = act( sum_i X[r][i]*xm(r,i) * W[o][i] + b[o] ),  xm = dropout multiplier (stream) or 1
// Y[r][o] = post(sum_i drop(X)[r][i] * W[o][i] + b[o]).  A 256-thread block owns 16 rows x 16
// outputs; its 4 waves split K into quarters, each streaming 64-wide chunks through a private
// LDS tile with the next chunk already in registers (X through its dropout mask); lane
// (row = lane>>2, 4 outputs) accumulates in ascending i, the quarters are added in a fixed order.
constexpr int LKC = 64;  // K chunk
__global__ __launch_bounds__(256) void linear_fwd_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                         const float* __restrict__ b, float* __restrict__ Y, int R,
                                                         int I, int O, int relu, uint64_t seed, uint32_t stream,
                                                         float p) {
  __shared__ float xs[4][16][LKC + 1], ws[4][16][LKC + 1];
  __shared__ float red[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.y * 16, o0 = blockIdx.x * 16;
  const int quarter = (I + 3) / 4;
  const int kb = wave * quarter, ke = min(I, kb + quarter);
  const int row = lane >> 2, og = (lane & 3) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float nx[16], nw[16];  // 16 rows x 64 k per operand / 64 lanes
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i, rr = e >> 6, kk = e & 63, k = k0 + kk;
      const int r = r0 + rr, o = o0 + rr;
      const bool xok = r < R && k < ke, wok = o < O && k < ke;
      nx[i] = *(xok ? X + (int64_t)r * I + k : X);  // masked / dropout-scaled when staged
      nw[i] = *(wok ? W + (int64_t)o * I + k : W);
    }
  };
  if (kb < ke) load(kb);
  for (int k0 = kb; k0 < ke; k0 += LKC) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i, rr = e >> 6, kk = e & 63;
      const bool xok = r0 + rr < R && k0 + kk < ke, wok = o0 + rr < O && k0 + kk < ke;
      float x = xok ? nx[i] : 0.f;
      if (p > 0.f && xok) x *= drop_mul(seed, stream, (int64_t)(r0 + rr) * I + k0 + kk, p);
      xs[wave][rr][kk] = x;
      ws[wave][rr][kk] = wok ? nw[i] : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (k0 + LKC < ke) load(k0 + LKC);
    const int kn = min(LKC, ke - k0);
    for (int kk = 0; kk < kn; ++kk) {
      const float x = xs[wave][row][kk];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = fmaf(x, ws[wave][og + q][kk], acc[q]);
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[wave][row * 16 + og + q] = acc[q];
  __syncthreads();
  const int r = r0 + (tid >> 4), o = o0 + (tid & 15);
  if (r < R && o < O) {
    float a = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    if (b) a += b[o];
    if (relu) a = fmaxf(a, 0.f);
    Y[(int64_t)r * O + o] = a;
  }
}

// dX[r][i] = (acc? dX : 0) + sum_o dY[r][o] * W[o][i], then * xm(r,i) (dropout on the input)
__global__ __launch_bounds__(256) void linear_dgrad_kernel(const float* __restrict__ dY, const float* __restrict__ W,
                                                           float* __restrict__ dX, int R, int I, int O, int accumulate,
                                                           uint64_t seed, uint32_t stream, float p) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)R * I) return;
  const int r = (int)(idx / I), i = (int)(idx % I);
  float a = 0.f;
  for (int o = 0; o < O; ++o) a += dY[(int64_t)r * O + o] * W[(int64_t)o * I + i];
  if (p > 0.f) a *= drop_mul(seed, stream, idx, p);
  dX[idx] = accumulate ? dX[idx] + a : a;
}

// dW[o][i] = sum_r dY[r][o] * X[r][i]*xm(r,i);  db[o] = sum_r dY[r][o]
__global__ __launch_bounds__(256) void linear_wgrad_kernel(const float* __restrict__ dY, const float* __restrict__ X,
                                                           float* __restrict__ dW, float* __restrict__ db, int R,
                                                           int I, int O, uint64_t seed, uint32_t stream, float p) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx < (int64_t)O * I) {
    const int o = (int)(idx / I), i = (int)(idx % I);
    float a = 0.f;
    for (int r = 0; r < R; ++r) {
      float x = X[(int64_t)r * I + i];
      if (p > 0.f) x *= drop_mul(seed, stream, (int64_t)r * I + i, p);
      a += dY[(int64_t)r * O + o] * x;
    }
    dW[idx] = a;
  }
  if (db && idx < O) {
    float a = 0.f;
    for (int r = 0; r < R; ++r) a += dY[(int64_t)r * O + idx];
    db[idx] = a;
  }
}

// ------------------------------------------------------------------ fp32 MFMA small GEMM
// C[m][n] (+)= post( sum_k A(m,k) B(k,n) ), A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn],
// on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation).  For the small, deep-K
// products around the head and the squeeze-excite FCs (frames x channels x reduce width), where
// per-output dot-product threads are latency-bound: one workgroup per 16x16 output tile, its
// waves splitting K round-robin in 32-k chunks (operands of a chunk loaded before its MFMAs),
// then a fixed-order LDS reduction over the waves (bit-reproducible).  Options: bias[n],
// post-multiplication by silu'(pre[m][n]), silu(B), counter-hash dropout on B (index k*drop_ld + n), and
// asum[m] (+)= sum_k A(m,k) (the bias gradient of a weight-gradient product) from n-tile 0.
typedef float mf_f32x4 __attribute__((ext_vector_type(4)));
constexpr int MG_MAXW = 16;

// one 16x16 output tile of product `a` (the workgroup's waves split K)
__device__ __forceinline__ void mg_tile(const MfmaGemm& a, int tile, float (&red)[MG_MAXW][5][64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int tn = (a.N + 15) / 16;
  const int m0 = (tile / tn) * 16, n0 = (tile % tn) * 16;
  const int li = lane & 15, lk = lane >> 4;
  const int m = m0 + li, n = n0 + li;
  const bool mok = m < a.M, nok = n < a.N;
  const bool drop = a.p > 0.f && !a.drop_c;
  const bool want_asum = a.asum != nullptr && n0 == 0;
  mf_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float as = 0.f;
  constexpr int U = 8;  // MFMA steps per chunk (32 k)
  for (int k0 = 32 * wave; k0 < a.K; k0 += 32 * nw) {
    float av[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 4 * u + lk;
      const bool kok = k < a.K;
      av[u] = (mok && kok) ? a.A[(int64_t)m * a.sam + (int64_t)k * a.sak] : 0.f;
      float b = (nok && kok) ? a.B[(int64_t)k * a.sbk + (int64_t)n * a.sbn] : 0.f;
      if (a.b_silu) b = siluf_(b);
      if (drop && nok && kok) b *= drop_mul(a.seed, a.stream, (int64_t)k * a.drop_ld + n, a.p);
      bv[u] = b;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    if (want_asum) {
#pragma unroll
      for (int u = 0; u < U; ++u) as += av[u];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][r][lane] = acc[r];
  red[wave][4][lane] = as;
  __syncthreads();
  if (wave != 0) return;
  // D layout: lane holds rows 4*(lane>>4) + r of column lane & 15
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = 0.f;
    for (int w = 0; w < nw; ++w) v += red[w][r][lane];
    const int mm = m0 + 4 * lk + r, nn = n0 + li;
    if (mm >= a.M || nn >= a.N) continue;
    if (a.bias) v += a.bias[nn];
    if (a.relu) v = fmaxf(v, 0.f);
    if (a.dsilu_pre) v *= dsiluf_(a.dsilu_pre[(int64_t)mm * a.ldc + nn]);
    if (a.drop_c && a.p > 0.f) v *= drop_mul(a.seed, a.stream, (int64_t)mm * a.ldc + nn, a.p);
    float* c = a.C + (int64_t)mm * a.ldc + nn;
    *c = a.accumulate ? *c + v : v;
  }
  if (want_asum && lane < 16 && mok) {
    float v = 0.f;
    for (int w = 0; w < nw; ++w) v += (red[w][4][lane] + red[w][4][lane + 16]) + (red[w][4][lane + 32] + red[w][4][lane + 48]);
    a.asum[m] = a.accumulate ? a.asum[m] + v : v;
  }
}

// two independent GEMMs of equal K may share one launch: workgroups [0, tiles0) run a0, the rest a1
__global__ __launch_bounds__(1024) void mfma_small_gemm_kernel(MfmaGemm a0, MfmaGemm a1, int tiles0) {
  __shared__ float red[MG_MAXW][5][64];
  const bool second = (int)blockIdx.x >= tiles0;
  mg_tile(second ? a1 : a0, second ? (int)blockIdx.x - tiles0 : (int)blockIdx.x, red);
}

// up to kMfmaBatch products of equal K in one launch: workgroups [start[k], start[k+1]) run g[k]
struct MfmaGemmBatch {
  MfmaGemm g[kMfmaBatch];
  int start[kMfmaBatch + 1];
  int n;
};
__global__ __launch_bounds__(1024) void mfma_small_gemm_batch_kernel(MfmaGemmBatch b) {
  __shared__ float red[MG_MAXW][5][64];
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.start[k + 1]) ++k;
  mg_tile(b.g[k], (int)blockIdx.x - b.start[k], red);
}

int launch_mfma_small_gemm_batch(hipStream_t s, const MfmaGemm* g, int n) {
  for (int i0 = 0; i0 < n; i0 += kMfmaBatch) {
    MfmaGemmBatch b{};
    int tiles = 0;
    b.n = 0;
    for (int i = i0; i < std::min(n, i0 + kMfmaBatch); ++i) {
      if (g[i].K != g[i0].K) { set_error("mfma_small_gemm_batch: the products need the same K", __FILE__, __LINE__); return -1; }
      if (g[i].M <= 0 || g[i].N <= 0) continue;
      b.g[b.n] = g[i];
      b.start[b.n++] = tiles;
      tiles += cdiv(g[i].M, 16) * cdiv(g[i].N, 16);
    }
    b.start[b.n] = tiles;
    if (tiles == 0) continue;
    const int nw = std::max(1, std::min(MG_MAXW, cdiv(g[i0].K, 64)));
    hipLaunchKernelGGL(mfma_small_gemm_batch_kernel, dim3((unsigned)tiles), dim3(64 * nw), 0, s, b);
    DFD_HIP_CHECK(hipGetLastError());
  }
  return 0;
}

int launch_mfma_small_gemm(hipStream_t s, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                           int64_t sbn, float* C, int64_t ldc, int M, int N, int K, const float* bias,
                           const float* dsilu_pre, float* asum, bool accumulate, uint64_t seed, uint32_t stream,
                           float p, int64_t drop_ld) {
  MfmaGemm g;
  g.A = A; g.sam = sam; g.sak = sak; g.B = B; g.sbk = sbk; g.sbn = sbn; g.C = C; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.bias = bias; g.dsilu_pre = dsilu_pre; g.asum = asum;
  g.accumulate = accumulate ? 1 : 0; g.seed = seed; g.stream = stream; g.p = p; g.drop_ld = drop_ld;
  return launch_mfma_small_gemm(s, g);
}

int launch_mfma_small_gemm(hipStream_t s, const MfmaGemm& g) {
  const int M = g.M, N = g.N, K = g.K;
  if (M <= 0 || N <= 0) return 0;
  const int tiles = cdiv(M, 16) * cdiv(N, 16);
  // waves per tile: enough K-splitting to put ~2 chunks on each wave, at most MG_MAXW
  const int nw = std::max(1, std::min(MG_MAXW, cdiv(K, 64)));
  hipLaunchKernelGGL(mfma_small_gemm_kernel, dim3((unsigned)tiles), dim3(64 * nw), 0, s, g, g, tiles);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int launch_mfma_small_gemm2(hipStream_t s, const MfmaGemm& g0, const MfmaGemm& g1) {
  if (g0.K != g1.K) { set_error("mfma_small_gemm2: the two products need the same K", __FILE__, __LINE__); return -1; }
  const int t0 = (g0.M > 0 && g0.N > 0) ? cdiv(g0.M, 16) * cdiv(g0.N, 16) : 0;
  const int t1 = (g1.M > 0 && g1.N > 0) ? cdiv(g1.M, 16) * cdiv(g1.N, 16) : 0;
  if (t0 + t1 == 0) return 0;
  const int nw = std::max(1, std::min(MG_MAXW, cdiv(g0.K, 64)));
  hipLaunchKernelGGL(mfma_small_gemm_kernel, dim3((unsigned)(t0 + t1)), dim3(64 * nw), 0, s, g0, g1, t0);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// Y[r] = post( dot(X[r], w) + b ) for a single output (the 64->1 attention scorer)
// ------------------------------------------------------------------ temporal attention (per clip)
// e[bt] = sigmoid(w2 . hid[bt] + b2) ; a[b] = softmax_t(e[b]) ; g[b] = sum_t a[b][t] f[bt]
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ F, const float* __restrict__ hid,
                                                       const float* __restrict__ w2, const float* __restrict__ b2,
                                                       int T, int D, int H, int use_attn, float* __restrict__ e,
                                                       float* __restrict__ a, float* __restrict__ g) {
  extern __shared__ float s_a[];  // [T]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (use_attn) {
    for (int t = wave; t < T; t += 4) {
      float v = 0.f;
      for (int j = lane; j < H; j += 64) v += hid[((int64_t)b * T + t) * H + j] * w2[j];
      v = wave_sum(v);
      if (lane == 0) {
        const float ev = sigmoidf_(v + b2[0]);
        e[(int64_t)b * T + t] = ev;
        s_a[t] = ev;
      }
    }
    __syncthreads();
    if (tid == 0) {
      float mx = -INFINITY;
      for (int t = 0; t < T; ++t) mx = fmaxf(mx, s_a[t]);
      float sum = 0.f;
      for (int t = 0; t < T; ++t) { s_a[t] = expf(s_a[t] - mx); sum += s_a[t]; }
      for (int t = 0; t < T; ++t) s_a[t] /= sum;
    }
  } else {
    for (int t = tid; t < T; t += 256) s_a[t] = 1.0f / (float)T;
  }
  __syncthreads();
  for (int t = tid; t < T; t += 256) a[(int64_t)b * T + t] = s_a[t];
  for (int i = tid; i < D; i += 256) {
    float acc = 0.f;
    if (use_attn) {
      for (int t = 0; t < T; ++t) acc += F[((int64_t)b * T + t) * D + i] * s_a[t];
    } else {
      for (int t = 0; t < T; ++t) acc += F[((int64_t)b * T + t) * D + i];
      acc /= (float)T;
    }
    g[(int64_t)b * D + i] = acc;
  }
}

// backward of the attention pooling for clip b:
//   da[t] = dg . f[bt] + dscores[b][t] ; de = a (da - sum a da) ; dpe = de e (1-e)
//   dF[bt] = a[t] dg ;  dhid[bt][j] = dpe[bt] * w2[j] * (hid>0)
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* __restrict__ F, const float* __restrict__ hid,
                                                       const float* __restrict__ w2, const float* __restrict__ e,
                                                       const float* __restrict__ a, const float* __restrict__ dg,
                                                       const float* __restrict__ dscores, int T, int D, int H,
                                                       int use_attn, float* __restrict__ dF, float* __restrict__ dpe,
                                                       float* __restrict__ dhid) {
  extern __shared__ float sm[];  // [2T]
  float* s_da = sm;
  float* s_dpe = sm + T;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < D; i += 256) {
    const float d = dg[(int64_t)b * D + i];
    for (int t = 0; t < T; ++t) dF[((int64_t)b * T + t) * D + i] = a[(int64_t)b * T + t] * d;
  }
  if (!use_attn) return;
  for (int t = wave; t < T; t += 4) {
    float v = 0.f;
    for (int i = lane; i < D; i += 64) v += dg[(int64_t)b * D + i] * F[((int64_t)b * T + t) * D + i];
    v = wave_sum(v);
    if (lane == 0) s_da[t] = v + (dscores ? dscores[(int64_t)b * T + t] : 0.f);
  }
  __syncthreads();
  if (tid == 0) {
    float dot = 0.f;
    for (int t = 0; t < T; ++t) dot += a[(int64_t)b * T + t] * s_da[t];
    for (int t = 0; t < T; ++t) {
      const float at = a[(int64_t)b * T + t], ev = e[(int64_t)b * T + t];
      const float de = at * (s_da[t] - dot);
      const float d = de * ev * (1.f - ev);
      s_dpe[t] = d;
      dpe[(int64_t)b * T + t] = d;
    }
  }
  __syncthreads();
  for (int idx = tid; idx < T * H; idx += 256) {
    const int t = idx / H, j = idx % H;
    const float hv = hid[((int64_t)b * T + t) * H + j];
    dhid[((int64_t)b * T + t) * H + j] = hv > 0.f ? s_dpe[t] * w2[j] : 0.f;
  }
}

// relu'/dropout for fc1 output: d[r][j] *= (h>0) * xm2(r,j)   (in place)
__global__ void relu_drop_bwd_kernel(float* __restrict__ d, const float* __restrict__ h, int64_t n, uint64_t seed,
                                     uint32_t stream, float p) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  d[i] = h[i] > 0.f ? d[i] : 0.f;
}

// ------------------------------------------------------------------ weighted cross entropy
// loss = sum_b w[y_b] * (-log softmax(z_b)[y_b]) / sum_b w[y_b]  (ignore_index rows excluded)
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ y,
                                                     const float* __restrict__ w, int B, int NC, int64_t ignore,
                                                     float* __restrict__ loss, float* __restrict__ wsum) {
  __shared__ double sn[256], sd[256];
  double num = 0.0, den = 0.0;
  for (int b = threadIdx.x; b < B; b += 256) {
    const int64_t lab = y[b];
    if (lab == ignore) continue;
    const float* zb = z + (int64_t)b * NC;
    float mx = -INFINITY;
    for (int k = 0; k < NC; ++k) mx = fmaxf(mx, zb[k]);
    double se = 0.0;
    for (int k = 0; k < NC; ++k) se += exp((double)zb[k] - mx);
    const double lse = mx + log(se);
    const double wb = w ? (double)w[lab] : 1.0;
    num += wb * (lse - (double)zb[lab]);
    den += wb;
  }
  sn[threadIdx.x] = num;
  sd[threadIdx.x] = den;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, d = 0.0;
    for (int i = 0; i < 256; ++i) { a += sn[i]; d += sd[i]; }
    loss[0] = (float)(a / d);
    wsum[0] = (float)d;
  }
}

__global__ void ce_bwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ y, const float* __restrict__ w,
                              int B, int NC, int64_t ignore, const float* __restrict__ wsum,
                              const float* __restrict__ gout, float* __restrict__ dz) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const int64_t lab = y[b];
  const float* zb = z + (int64_t)b * NC;
  float* db = dz + (int64_t)b * NC;
  if (lab == ignore) {
    for (int k = 0; k < NC; ++k) db[k] = 0.f;
    return;
  }
  float mx = -INFINITY;
  for (int k = 0; k < NC; ++k) mx = fmaxf(mx, zb[k]);
  float se = 0.f;
  for (int k = 0; k < NC; ++k) se += expf(zb[k] - mx);
  const float scale = (w ? w[lab] : 1.f) / wsum[0] * gout[0];
  for (int k = 0; k < NC; ++k) db[k] = (expf(zb[k] - mx) / se - (k == lab ? 1.f : 0.f)) * scale;
}

// ------------------------------------------------------------------ grad norm + Adam(W)
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ part) {
  __shared__ double sh[256];
  // four strided elements per iteration, loads issued together, one accumulator each (fixed order)
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t st = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = g[i + u * st];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += (double)v[u] * (double)v[u];
  }
  for (int u = 0; i < n; i += st, ++u) a[u & 3] += (double)g[i] * (double)g[i];
  sh[threadIdx.x] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

// out[0] = total norm, out[1] = clip coefficient min(1, max_norm/(norm+1e-6)) (1 if max_norm <= 0)
// (256 threads: strided partial sums, then a fixed-order tree; deterministic).  With a loss scaler
// (fp16 training) the partials are of the SCALED gradient: the norm is unscaled by the fp32 inverse
// scale (GradScaler.unscale_ then clip_grad_norm_), and scaler[2] = 1 when it is not finite.
__global__ __launch_bounds__(256) void norm_finalize_kernel(const double* __restrict__ part, int nparts, float max_norm,
                                                            float* out, float* __restrict__ scaler) {
  __shared__ double sh[256];
  double v = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) v += part[i];
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double a = sh[0];
  float nrm = (float)sqrt(a);
  if (scaler) {
    // found_inf from the fp64 sum: it is not finite iff an element is (squares of finite floats cannot
    // overflow it), whereas a finite-element norm above FLT_MAX would turn the fp32 narrowing inf
    // and skip a step GradScaler's per-element check keeps
    const bool bad = !isfinite(a);
    scaler[2] = bad ? 1.f : 0.f;
    nrm = bad ? nrm : (float)(sqrt(a) * (double)(1.f / scaler[0]));
  }
  out[0] = nrm;
  float c = 1.f;
  if (max_norm > 0.f) {
    c = max_norm / (nrm + 1e-6f);
    if (c > 1.f) c = 1.f;
  }
  out[1] = c;
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, int64_t n, AdamHyper h,
                                                   const float* __restrict__ coef) {
  const float cf = coef ? coef[1] : 1.f;
  float step_size = h.step_size, bc2_sqrt = h.bc2_sqrt, inv = 1.f;
  if (h.scaler) {
    if (h.scaler[2] != 0.f) return;  // non-finite scaled gradient: the step is skipped (GradScaler.step)
    // bias corrections of the APPLIED step count (skipped steps do not count, as torch's optimizer
    // step is not called for them), in double as torch.optim computes them
    const double t = (double)h.scaler[3] + 1.0;
    step_size = (float)(h.lr / (1.0 - pow(h.beta1d, t)));
    bc2_sqrt = (float)sqrt(1.0 - pow(h.beta2d, t));
    inv = 1.f / h.scaler[0];
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float gi = g[i] * h.grad_scale;
    if (h.scaler) { gi = gi * inv; g[i] = gi; }  // unscale_ in place
    if (coef) { gi = gi * cf; g[i] = gi; }
    float pi = p[i];
    if (h.decoupled) {
      pi = pi * h.decay;
    } else if (h.weight_decay != 0.f) {
      gi = gi + h.weight_decay * pi;
    }
    float mi = m[i];
    mi = mi + h.omb1 * (gi - mi);
    float vi = v[i] * h.beta2 + h.omb2 * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + h.eps;
    pi = pi + (-step_size * mi) / denom;
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

// torch.amp.GradScaler's update (_amp_update_scale_): a non-finite step halves the scale (backoff) and
// restarts the growth count; `interval` finite steps in a row multiply it by `growth`.  Also counts the
// applied optimizer steps (scaler[3]) for the bias corrections.  One thread, after the Adam launches.
__global__ void loss_scale_update_kernel(float* __restrict__ st, float growth, float backoff, int interval) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (st[2] != 0.f) {
    st[0] = st[0] * backoff;
    st[1] = 0.f;
  } else {
    st[3] = st[3] + 1.f;
    const float t = st[1] + 1.f;
    if (t >= (float)interval) {
      const float ns = st[0] * growth;
      if (isfinite(ns)) st[0] = ns;
      st[1] = 0.f;
    } else {
      st[1] = t;
    }
  }
}

// ------------------------------------------------------------------ param cast (+ transpose)
// Transposed segments go through 32x32 LDS tiles: rows read along the input's contiguous axis,
// written along the output's (an output-indexed gather read one 4-B element per 64-B line).
template <typename T>
__global__ __launch_bounds__(256) void cast_params_kernel(const float* __restrict__ params, T* __restrict__ out,
                                                          const CastSeg* __restrict__ segs) {
  __shared__ float tile[32][33];
  const CastSeg sg = segs[blockIdx.y];
  const int64_t n = (int64_t)sg.rows * sg.cols;
  if (!sg.transpose) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
      out[sg.dst + i] = Tr<T>::from_f(params[sg.src + i]);
    return;
  }
  // out[c][r] = in[r][c], in = [rows][cols]
  const int tr = (sg.rows + 31) / 32, tc = (sg.cols + 31) / 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int t = blockIdx.x; t < tr * tc; t += gridDim.x) {
    const int r0 = (t / tc) * 32, c0 = (t % tc) * 32;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = r0 + ty + 8 * k, c = c0 + tx;
      tile[ty + 8 * k][tx] = (r < sg.rows && c < sg.cols) ? params[sg.src + (int64_t)r * sg.cols + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + ty + 8 * k, r = r0 + tx;
      if (r < sg.rows && c < sg.cols) out[sg.dst + (int64_t)c * sg.rows + r] = Tr<T>::from_f(tile[tx][ty + 8 * k]);
    }
    __syncthreads();
  }
}

template <typename T>
int launch_cast_params(hipStream_t s, const float* params, T* out, const CastSeg* segs_dev, int nseg, int max_elems) {
  if (nseg <= 0) return 0;
  const int gx = std::max(1, std::min(64, cdiv(max_elems, 256)));
  hipLaunchKernelGGL((cast_params_kernel<T>), dim3(gx, nseg), dim3(256), 0, s, params, out, segs_dev);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template int launch_cast_params<float>(hipStream_t, const float*, float*, const CastSeg*, int, int);
template int launch_cast_params<bf16>(hipStream_t, const float*, bf16*, const CastSeg*, int, int);
template int launch_cast_params<f16>(hipStream_t, const float*, f16*, const CastSeg*, int, int);

// ------------------------------------------------------------------ host launchers (head.h)
static unsigned nblk(int64_t n) { return (unsigned)std::max<int64_t>(1, cdiv64(n, 256)); }

static dim3 lin_grid(int R, int O) { return dim3((unsigned)cdiv(O, 16), (unsigned)cdiv(R, 16)); }

int head_forward(hipStream_t s, const HeadDims& d, const HeadParams& P, const float* F, HeadWork& w, uint64_t seed,
                 float p, float* logits, float* scores) {
  if (d.use_attn) {
    hipLaunchKernelGGL(linear_fwd_kernel, lin_grid(d.B * d.T, d.H), dim3(256), 0, s, F, P.ta_w1,
                       P.ta_b1, w.hid, d.B * d.T, d.D, d.H, 1, seed, 0u, 0.f);
  }
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(d.B), dim3(256), d.T * sizeof(float), s, F, w.hid, P.ta_w2, P.ta_b2, d.T,
                     d.D, d.H, d.use_attn, w.e, scores, w.g);
  hipLaunchKernelGGL(linear_fwd_kernel, lin_grid(d.B, d.F1), dim3(256), 0, s, w.g, P.fc1_w, P.fc1_b, w.h1,
                     d.B, d.D, d.F1, 1, seed, 1u, p);
  hipLaunchKernelGGL(linear_fwd_kernel, lin_grid(d.B, d.NC), dim3(256), 0, s, w.h1, P.fc2_w, P.fc2_b,
                     logits, d.B, d.F1, d.NC, 0, seed, 2u, p);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int head_backward(hipStream_t s, const HeadDims& d, const HeadParams& P, const float* F, HeadWork& w, uint64_t seed,
                  float p, const float* scores, const float* dlogits, const float* dscores, float* dF, HeadParams& G) {
  // fc2: dW2 = dlogits^T . drop(h1) ; db2 ; dh1 = dlogits . W2 (then * drop2 * relu')
  // dW[o][i] = sum_r dY[r][o] drop(X)[r][i] ;  db = column sums of dY
  DFD_TRY(launch_mfma_small_gemm(s, dlogits, 1, d.NC, w.h1, d.F1, 1, (float*)G.fc2_w, d.F1, d.NC, d.F1, d.B, nullptr,
                                 nullptr, (float*)G.fc2_b, false, seed, 2u, p, d.F1));
  hipLaunchKernelGGL(linear_dgrad_kernel, dim3(nblk((int64_t)d.B * d.F1)), dim3(256), 0, s, dlogits, P.fc2_w, w.dh1,
                     d.B, d.F1, d.NC, 0, seed, 2u, p);
  hipLaunchKernelGGL(relu_drop_bwd_kernel, dim3(nblk((int64_t)d.B * d.F1)), dim3(256), 0, s, w.dh1, w.h1,
                     (int64_t)d.B * d.F1, seed, 0u, 0.f);
  // fc1: dW1 = dh1^T . drop(g) ; db1 ; dg = dh1 . W1 * drop1
  DFD_TRY(launch_mfma_small_gemm(s, w.dh1, 1, d.F1, w.g, d.D, 1, (float*)G.fc1_w, d.D, d.F1, d.D, d.B, nullptr,
                                 nullptr, (float*)G.fc1_b, false, seed, 1u, p, d.D));
  {  // dg = drop1(dh1 . W1): [B][F1] x [F1][D] on fp32 MFMA, the dropout mask on the product (index b*D + i)
    MfmaGemm g{};
    g.A = w.dh1; g.sam = d.F1; g.sak = 1; g.B = P.fc1_w; g.sbk = d.D; g.sbn = 1; g.C = w.dg; g.ldc = d.D;
    g.M = d.B; g.N = d.D; g.K = d.F1; g.seed = seed; g.stream = 1u; g.p = p; g.drop_c = 1;
    DFD_TRY(launch_mfma_small_gemm(s, g));
  }
  // attention pooling
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(d.B), dim3(256), 2 * d.T * sizeof(float), s, F, w.hid, P.ta_w2, w.e,
                     scores, w.dg, dscores, d.T, d.D, d.H, d.use_attn, dF, w.dpe, w.dhid);
  if (d.use_attn) {
    const int R = d.B * d.T;
    DFD_TRY(launch_mfma_small_gemm(s, w.dpe, 1, 1, w.hid, d.H, 1, (float*)G.ta_w2, d.H, 1, d.H, R, nullptr, nullptr,
                                   (float*)G.ta_b2, false, seed, 0u, 0.f, d.H));
    DFD_TRY(launch_mfma_small_gemm(s, w.dhid, 1, d.H, F, d.D, 1, (float*)G.ta_w1, d.D, d.H, d.D, R, nullptr, nullptr,
                                   (float*)G.ta_b1, false, seed, 0u, 0.f, d.D));
    // dF += dhid . W1: [R][H] x [H][D] on fp32 MFMA (the per-output dot-product loop was latency-bound)
    MfmaGemm g{};
    g.A = w.dhid; g.sam = d.H; g.sak = 1; g.B = P.ta_w1; g.sbk = d.D; g.sbn = 1; g.C = dF; g.ldc = d.D;
    g.M = R; g.N = d.D; g.K = d.H; g.accumulate = 1;
    DFD_TRY(launch_mfma_small_gemm(s, g));
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int ce_forward(hipStream_t s, const float* z, const int64_t* y, const float* w, int B, int NC, int64_t ignore,
               float* loss, float* wsum) {
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(1), dim3(256), 0, s, z, y, w, B, NC, ignore, loss, wsum);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int ce_backward(hipStream_t s, const float* z, const int64_t* y, const float* w, int B, int NC, int64_t ignore,
                const float* wsum, const float* gout, float* dz) {
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(nblk(B)), dim3(256), 0, s, z, y, w, B, NC, ignore, wsum, gout, dz);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int grad_norm(hipStream_t s, const float* g, int64_t n, float max_norm, double* part, int nparts, float* out,
              float* scaler) {
  const int gx = std::max(1, std::min<int>(nparts, (int)nblk(n)));
  hipLaunchKernelGGL(sumsq_kernel, dim3(gx), dim3(256), 0, s, g, n, part);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(256), 0, s, part, gx, max_norm, out, scaler);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int loss_scale_update(hipStream_t s, float* scaler, float growth, float backoff, int interval) {
  hipLaunchKernelGGL(loss_scale_update_kernel, dim3(1), dim3(64), 0, s, scaler, growth, backoff, interval);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int adam_step(hipStream_t s, float* p, float* g, float* m, float* v, int64_t n, const AdamHyper& h, const float* coef) {
  const int gx = (int)std::min<int64_t>(nblk(n), 4096);
  hipLaunchKernelGGL(adam_kernel, dim3(gx), dim3(256), 0, s, p, g, m, v, n, h, coef);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
