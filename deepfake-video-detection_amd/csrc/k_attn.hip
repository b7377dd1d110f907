// Fused multi-head attention of the ViT-B/16 trunk (timm Attention, DeepfakeModel's
// ViTFeatureExtractor, src/models.py:88-107), bf16 storage, head dim 64, up to 256 tokens:
//
//   forward   S = scale * Q K^T ; P = softmax_rows(S) ; O = P V          (saves O and the row
//             log-sum-exp L, never S or P)
//   backward  D = rowsum(dO * O) ; P = exp(scale * Q K^T - L) ; dP = dO V^T ; dS = P * (dP - D)
//             dQ = scale * dS K ; dK = scale * dS^T Q ; dV = P^T dO
//
// One workgroup per (image, head) with one wave per 16 tokens (14 waves for 197 tokens): the
// head's K, V (forward), Q, dO (key/value backward) or K, V (query backward) sit in LDS, row-major
// for the MFMA operands indexed by token and transposed for the ones indexed by head dimension.
// Every product runs on v_mfma_f32_16x16x32_bf16.  The probabilities never leave registers: a
// score tile's accumulator layout (lane holds rows 4g..4g+3 of a 16-row block, g = lane / 16, in
// column lane % 16) is used directly as the B operand of the following product, with the
// contraction index k = 8g + j mapped to rows {4g + j of block 2c, 4g + j - 4 of block 2c+1} --
// the A operand is read from LDS in that same order (two 8-B reads per lane).  Softmax
// statistics in fp32; P and dS are rounded to bf16 only as MFMA operands.
//
// The scores of the previous path (bgemm + softmax + bgemm, 3 launches and an S and P round
// trip through HBM per layer, k_vit.hip) remain the fp32 parity path.
#include "kernels.h"

namespace dfd {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int AD = 64;       // head dimension
constexpr int RS = AD + 8;   // LDS row stride (elements) of token-major images

__device__ __forceinline__ f32x4_t mma(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8_t ld16(const bf16* p) { return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p)); }
__device__ __forceinline__ bf16x8_t cat8(const bf16* p0, const bf16* p1) {  // two 8-B halves
  const uint2 a = *reinterpret_cast<const uint2*>(p0), b = *reinterpret_cast<const uint2*>(p1);
  return __builtin_bit_cast(bf16x8_t, make_uint4(a.x, a.y, b.x, b.y));
}
__device__ __forceinline__ bf16x8_t pack8(const float (&x)[2][4]) {  // RNE, as every bf16 store here
  return __builtin_bit_cast(bf16x8_t, make_uint4(pack2bf(x[0][0], x[0][1]), pack2bf(x[0][2], x[0][3]),
                                                 pack2bf(x[1][0], x[1][1]), pack2bf(x[1][2], x[1][3])));
}
// The MFMA operand of head-dimension rows col .. col+15 whose 8 contraction entries are the tokens
// {rlo + 0..3, rhi + 0..3}, read as COLUMNS of a token-major image with ds_read_b64_tr_b16 (lane 4q + pq
// of a 16-lane group supplies row r + q, columns col + 4pq .. +3; lane n receives column col + n of the
// four rows) -- the transposed copy of the image is not needed
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
__device__ __forceinline__ bf16x8_t tr8(const bf16* img, int rlo, int rhi, int col) {
  const int lane = threadIdx.x & 63, q = (lane >> 2) & 3, pq = lane & 3;
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + (rlo + q) * RS + col + 4 * pq));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + (rhi + q) * RS + col + 4 * pq));
  return bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ void st4(bf16* p, const f32x4_t& v, float s) {  // 4 consecutive bf16
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(v[0] * s, v[1] * s), pack2bf(v[2] * s, v[3] * s));
}

// token-major image of one head's 64 columns (rows >= nt zero) and, optionally, its transpose
template <int NP>
__device__ __forceinline__ void load_head(const bf16* __restrict__ src, int64_t ld, int nt, bf16* rows, bf16* tr) {
  constexpr int TS = NP + 8;
  for (int i = threadIdx.x; i < NP * 8; i += blockDim.x) {
    const int t = i >> 3, c8 = (i & 7) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t < nt) v = *reinterpret_cast<const uint4*>(src + (int64_t)t * ld + c8);
    if (rows) *reinterpret_cast<uint4*>(rows + t * RS + c8) = v;
    if (tr) {
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) reinterpret_cast<uint16_t*>(tr)[(c8 + j) * TS + t] = e[j];
    }
  }
}

// Two token-major head images at once (rows >= nt zero), for a workgroup of 64 NB threads: each thread
// moves 16-B chunks t and t + 64 NB of both images (NP * 8 = 128 NB chunks per image), every global
// load issued before the first LDS store
template <int NB>
__device__ __forceinline__ void load_heads2(const bf16* __restrict__ sa, int64_t lda, const bf16* __restrict__ sb,
                                            int64_t ldb, int nt, bf16* ra, bf16* rb) {
  uint4 va[2], vb[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + k * 64 * NB, t = i >> 3, c8 = (i & 7) * 8;
    va[k] = vb[k] = make_uint4(0, 0, 0, 0);
    if (t < nt) {
      va[k] = *reinterpret_cast<const uint4*>(sa + (int64_t)t * lda + c8);
      vb[k] = *reinterpret_cast<const uint4*>(sb + (int64_t)t * ldb + c8);
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + k * 64 * NB, t = i >> 3, c8 = (i & 7) * 8;
    *reinterpret_cast<uint4*>(ra + t * RS + c8) = va[k];
    *reinterpret_cast<uint4*>(rb + t * RS + c8) = vb[k];
  }
}

// D[t] = sum_d dO[t][d] * O[t][d] with four threads per token (16 columns each, the four partial sums
// added by lane shuffles in a fixed order), 64 NB threads = 4 NP tokens' worth (0 beyond nt)
template <int NB>
__device__ __forceinline__ void load_rowdot4(const bf16* __restrict__ dO, int64_t lddo, const bf16* __restrict__ O,
                                             int64_t ldo, int nt, float* out) {
  const int t = threadIdx.x >> 2, c0 = (threadIdx.x & 3) * 16;
  float acc = 0.f;
  if (t < nt) {
    float x[2][8], y[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ld8(dO + (int64_t)t * lddo + c0 + 8 * h, x[h]);
      ld8(O + (int64_t)t * ldo + c0 + 8 * h, y[h]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += x[h][j] * y[h][j];
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  if ((threadIdx.x & 3) == 0) out[t] = acc;
}

// D[t] = sum_d dO[t][d] * O[t][d] for every token of the head (0 beyond nt)
template <int NP>
__device__ __forceinline__ void load_rowdot(const bf16* __restrict__ dO, int64_t lddo, const bf16* __restrict__ O,
                                            int64_t ldo, int nt, float* out) {
  for (int t = threadIdx.x; t < NP; t += blockDim.x) {
    float acc = 0.f;
    if (t < nt) {
#pragma unroll
      for (int c8 = 0; c8 < AD; c8 += 8) {
        float x[8], y[8];
        ld8(dO + (int64_t)t * lddo + c8, x);
        ld8(O + (int64_t)t * ldo + c8, y);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
      }
    }
    out[t] = acc;
  }
}

}  // namespace

// ---------------------------------------------------------------- forward
template <int NB>
__global__ __launch_bounds__(1024) void attn_fwd_kernel(AttnArgs a) {
  constexpr int NP = 16 * NB, TS = NP + 8;
  __shared__ __attribute__((aligned(16))) bf16 Ks[NP * RS];
  __shared__ __attribute__((aligned(16))) bf16 Vs[NP * RS];
  const int bh = blockIdx.x, img = bh / a.heads, h = bh - img * a.heads;
  const int nt = a.nt, lane = threadIdx.x & 63, g = lane >> 4, wave = threadIdx.x >> 6;
  const int64_t row0 = (int64_t)img * nt;
  const bf16* base = a.qkv + row0 * a.ldq + h * AD;
  const int q = wave * 16 + (lane & 15);  // this lane's query (MFMA column)
  bf16x8_t qb[2];  // issued first: in flight with the K / V image loads
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    qb[kk] = q < nt ? ld16(base + (int64_t)q * a.ldq + 32 * kk + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  load_heads2<NB>(base + a.koff, a.ldq, base + a.voff, a.ldq, nt, Ks, Vs);
  __syncthreads();
  if (wave * 16 >= nt) return;
  // S^T blocks: rows key = 16 nb + 4g + r, column q
  f32x4_t st[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) acc = mma(ld16(Ks + (nb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), qb[kk], acc);
    st[nb] = acc;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = nb * 16 + 4 * g + r;
      const float v = key < nt ? st[nb][r] * a.scale : -INFINITY;
      st[nb][r] = v;
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = __expf(st[nb][r] - mx);
      st[nb][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  if (g == 0 && q < nt) a.lse[(int64_t)bh * nt + q] = mx + __logf(sum);
  // O^T[d][q] = sum_key Vt[d][key] P^T[key][q]
  f32x4_t o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NB / 2; ++c) {
    float pv[2][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pv[0][r] = st[2 * c][r] * inv;
      pv[1][r] = st[2 * c + 1][r] * inv;
    }
    const bf16x8_t pb = pack8(pv);
#pragma unroll
    for (int db = 0; db < 4; ++db) o[db] = mma(tr8(Vs, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), pb, o[db]);
  }
  if (q < nt) {
    bf16* orow = a.O + (row0 + q) * a.ldo + h * AD;
#pragma unroll
    for (int db = 0; db < 4; ++db) st4(orow + db * 16 + 4 * g, o[db], 1.f);
  }
}

// ---------------------------------------------------------------- backward: dK, dV (wave = 16 keys)
template <int NB>
__global__ __launch_bounds__(1024) void attn_bwd_kv_kernel(AttnArgs a) {
  constexpr int NP = 16 * NB, TS = NP + 8;
  __shared__ __attribute__((aligned(16))) bf16 Qs[NP * RS];
  __shared__ __attribute__((aligned(16))) bf16 dOs[NP * RS];
  __shared__ float Ls[NP], Dq[NP];
  const int bh = blockIdx.x, img = bh / a.heads, h = bh - img * a.heads;
  const int nt = a.nt, lane = threadIdx.x & 63, g = lane >> 4, wave = threadIdx.x >> 6;
  const int64_t row0 = (int64_t)img * nt;
  const bf16* base = a.qkv + row0 * a.ldq + h * AD;
  const bf16* dob = a.dO + row0 * a.lddo + h * AD;
  load_head<NP>(base, a.ldq, nt, Qs, nullptr);
  load_head<NP>(dob, a.lddo, nt, dOs, nullptr);
  load_rowdot<NP>(dob, a.lddo, a.O + row0 * a.ldo + h * AD, a.ldo, nt, Dq);
  for (int t = threadIdx.x; t < NP; t += blockDim.x) Ls[t] = t < nt ? a.lse[(int64_t)bh * nt + t] : 0.f;
  __syncthreads();
  if (wave * 16 >= nt) return;
  const int key = wave * 16 + (lane & 15);  // MFMA column
  bf16x8_t kb[2], vb[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const bool ok = key < nt;
    kb[kk] = ok ? ld16(base + (int64_t)key * a.ldq + a.koff + 32 * kk + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    vb[kk] = ok ? ld16(base + (int64_t)key * a.ldq + a.voff + 32 * kk + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x4_t dv[4], dk[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) dv[db] = dk[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < NB / 2; ++c) {
    float pv[2][4], sv[2][4];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int qb = 2 * c + hf;
      f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s = mma(ld16(Qs + (qb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), kb[kk], s);
        dp = mma(ld16(dOs + (qb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), vb[kk], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // rows q = 16 qb + 4g + r
        const int qq = qb * 16 + 4 * g + r;
        const float p = qq < nt ? __expf(s[r] * a.scale - Ls[qq]) : 0.f;
        pv[hf][r] = p;
        sv[hf][r] = p * (dp[r] - Dq[qq]);
      }
    }
    const bf16x8_t pb = pack8(pv), sb = pack8(sv);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      dv[db] = mma(tr8(dOs, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), pb, dv[db]);
      dk[db] = mma(tr8(Qs, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), sb, dk[db]);
    }
  }
  if (key < nt) {
    bf16* rowp = a.dqkv + (row0 + key) * a.lddq + h * AD;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      st4(rowp + a.koff + db * 16 + 4 * g, dk[db], a.scale);
      st4(rowp + a.voff + db * 16 + 4 * g, dv[db], 1.f);
    }
  }
}

// ---------------------------------------------------------------- backward: dQ (wave = 16 queries)
template <int NB>
__global__ __launch_bounds__(1024) void attn_bwd_q_kernel(AttnArgs a) {
  constexpr int NP = 16 * NB, TS = NP + 8;
  __shared__ __attribute__((aligned(16))) bf16 Ks[NP * RS];
  __shared__ __attribute__((aligned(16))) bf16 Vs[NP * RS];
  __shared__ float Dq[NP];
  const int bh = blockIdx.x, img = bh / a.heads, h = bh - img * a.heads;
  const int nt = a.nt, lane = threadIdx.x & 63, g = lane >> 4, wave = threadIdx.x >> 6;
  const int64_t row0 = (int64_t)img * nt;
  const bf16* base = a.qkv + row0 * a.ldq + h * AD;
  const bf16* dob = a.dO + row0 * a.lddo + h * AD;
  load_head<NP>(base + a.koff, a.ldq, nt, Ks, nullptr);
  load_head<NP>(base + a.voff, a.ldq, nt, Vs, nullptr);
  load_rowdot<NP>(dob, a.lddo, a.O + row0 * a.ldo + h * AD, a.ldo, nt, Dq);
  __syncthreads();
  if (wave * 16 >= nt) return;
  const int q = wave * 16 + (lane & 15);  // MFMA column
  const bool qok = q < nt;
  bf16x8_t qb[2], ob[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    qb[kk] = qok ? ld16(base + (int64_t)q * a.ldq + 32 * kk + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    ob[kk] = qok ? ld16(dob + (int64_t)q * a.lddo + 32 * kk + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const float L = qok ? a.lse[(int64_t)bh * nt + q] : 0.f, Dv = Dq[q];
  f32x4_t dq[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) dq[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < NB / 2; ++c) {
    float sv[2][4];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int nb = 2 * c + hf;
      f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s = mma(ld16(Ks + (nb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), qb[kk], s);
        dp = mma(ld16(Vs + (nb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), ob[kk], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // rows key = 16 nb + 4g + r
        const int kk2 = nb * 16 + 4 * g + r;
        const float p = (kk2 < nt && qok) ? __expf(s[r] * a.scale - L) : 0.f;
        sv[hf][r] = p * (dp[r] - Dv);
      }
    }
    const bf16x8_t sb = pack8(sv);
#pragma unroll
    for (int db = 0; db < 4; ++db) dq[db] = mma(tr8(Ks, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), sb, dq[db]);
  }
  if (qok) {
    bf16* rowp = a.dqkv + (row0 + q) * a.lddq + h * AD;
#pragma unroll
    for (int db = 0; db < 4; ++db) st4(rowp + db * 16 + 4 * g, dq[db], a.scale);
  }
}

// ---------------------------------------------------------------- backward, one launch
// The two kernels above as two phases of one workgroup: Q, dO, O (row dots) and L are read once for
// the head.  Phase A (dK, dV, wave = 16 keys) runs on the Q / dO images; each wave then takes its 16
// queries' Q and dO operand rows from those images, and the same LDS is refilled with K and V for
// phase B (dQ, wave = 16 queries) -- K and V come back from L2 (the workgroup read them moments
// before).  Same products in the same order as the two-kernel form: bit-identical.
template <int NB>
__global__ __launch_bounds__(1024) void attn_bwd_kernel(AttnArgs a) {
  constexpr int NP = 16 * NB;
  __shared__ __attribute__((aligned(16))) bf16 Xs[NP * RS];  // Q (phase A), K (phase B)
  __shared__ __attribute__((aligned(16))) bf16 Ys[NP * RS];  // dO (phase A), V (phase B)
  __shared__ float Ls[NP], Dq[NP];
  const int bh = blockIdx.x, img = bh / a.heads, h = bh - img * a.heads;
  const int nt = a.nt, lane = threadIdx.x & 63, g = lane >> 4, wave = threadIdx.x >> 6;
  const int64_t row0 = (int64_t)img * nt;
  const bf16* base = a.qkv + row0 * a.ldq + h * AD;
  const bf16* dob = a.dO + row0 * a.lddo + h * AD;
  const int key = wave * 16 + (lane & 15);  // phase A's MFMA column
  bf16x8_t kb[2], vb[2];  // issued first: in flight with the image loads
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const bool ok = key < nt;
    kb[kk] = ok ? ld16(base + (int64_t)key * a.ldq + a.koff + 32 * kk + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    vb[kk] = ok ? ld16(base + (int64_t)key * a.ldq + a.voff + 32 * kk + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  for (int t = threadIdx.x; t < NP; t += blockDim.x) Ls[t] = t < nt ? a.lse[(int64_t)bh * nt + t] : 0.f;
  load_heads2<NB>(base, a.ldq, dob, a.lddo, nt, Xs, Ys);
  load_rowdot4<NB>(dob, a.lddo, a.O + row0 * a.ldo + h * AD, a.ldo, nt, Dq);
  __syncthreads();
  const bool active = wave * 16 < nt;  // the waves past the last token only join the barriers
  bf16* rowp0 = a.dqkv + row0 * a.lddq + h * AD;
  if (active) {  // ---- phase A: dK, dV of keys wave * 16 + (lane & 15)
    f32x4_t dv[4], dk[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) dv[db] = dk[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < NB / 2; ++c) {
      float pv[2][4], sv[2][4];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int qb = 2 * c + hf;
        f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          s = mma(ld16(Xs + (qb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), kb[kk], s);
          dp = mma(ld16(Ys + (qb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), vb[kk], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // rows q = 16 qb + 4g + r
          const int qq = qb * 16 + 4 * g + r;
          const float p = qq < nt ? __expf(s[r] * a.scale - Ls[qq]) : 0.f;
          pv[hf][r] = p;
          sv[hf][r] = p * (dp[r] - Dq[qq]);
        }
      }
      const bf16x8_t pb = pack8(pv), sb = pack8(sv);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        dv[db] = mma(tr8(Ys, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), pb, dv[db]);
        dk[db] = mma(tr8(Xs, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), sb, dk[db]);
      }
    }
    if (key < nt) {
      bf16* rowp = rowp0 + (int64_t)key * a.lddq;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        st4(rowp + a.koff + db * 16 + 4 * g, dk[db], a.scale);
        st4(rowp + a.voff + db * 16 + 4 * g, dv[db], 1.f);
      }
    }
  }
  // this wave's queries for phase B, from the images before they are refilled (rows >= nt are zero)
  const int q = wave * 16 + (lane & 15);
  bf16x8_t qb[2], ob[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    qb[kk] = ld16(Xs + q * RS + 32 * kk + 8 * g);
    ob[kk] = ld16(Ys + q * RS + 32 * kk + 8 * g);
  }
  __syncthreads();
  load_heads2<NB>(base + a.koff, a.ldq, base + a.voff, a.ldq, nt, Xs, Ys);
  __syncthreads();
  if (!active) return;
  // ---- phase B: dQ of queries q
  const bool qok = q < nt;
  const float L = Ls[q], Dv = Dq[q];
  f32x4_t dq[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) dq[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < NB / 2; ++c) {
    float sv[2][4];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int nb = 2 * c + hf;
      f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s = mma(ld16(Xs + (nb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), qb[kk], s);
        dp = mma(ld16(Ys + (nb * 16 + (lane & 15)) * RS + 32 * kk + 8 * g), ob[kk], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // rows key = 16 nb + 4g + r
        const int kk2 = nb * 16 + 4 * g + r;
        const float p = (kk2 < nt && qok) ? __expf(s[r] * a.scale - L) : 0.f;
        sv[hf][r] = p * (dp[r] - Dv);
      }
    }
    const bf16x8_t sb = pack8(sv);
#pragma unroll
    for (int db = 0; db < 4; ++db) dq[db] = mma(tr8(Xs, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), sb, dq[db]);
  }
  if (qok) {
    bf16* rowp = rowp0 + (int64_t)q * a.lddq;
#pragma unroll
    for (int db = 0; db < 4; ++db) st4(rowp + db * 16 + 4 * g, dq[db], a.scale);
  }
}

// ---------------------------------------------------------------- launchers
static int attn_nb(int nt) { return ((nt + 31) / 32) * 2; }  // 16-token blocks, an even count

bool attn_supported(int nt, int head_dim) { return head_dim == AD && nt >= 1 && nt <= 256; }

template <template <int> class K_>
static int attn_go(hipStream_t s, const AttnArgs& a) {
  if (!attn_supported(a.nt, AD)) { set_error("attention: unsupported token count", __FILE__, __LINE__); return -1; }
  const int nb = attn_nb(a.nt);
  const dim3 grid((unsigned)(a.images * a.heads)), block((unsigned)(64 * nb));
  switch (nb) {
#define DFD_ATT(n) \
  case n: hipLaunchKernelGGL(K_<n>::fn, grid, block, 0, s, a); break;
    DFD_ATT(2) DFD_ATT(4) DFD_ATT(6) DFD_ATT(8) DFD_ATT(10) DFD_ATT(12) DFD_ATT(14) DFD_ATT(16)
#undef DFD_ATT
    default: set_error("attention: bad block count", __FILE__, __LINE__); return -1;
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}
template <int N> struct FwdK { static constexpr auto fn = attn_fwd_kernel<N>; };
template <int N> struct KvK { static constexpr auto fn = attn_bwd_kv_kernel<N>; };
template <int N> struct QK { static constexpr auto fn = attn_bwd_q_kernel<N>; };
template <int N> struct BwdK { static constexpr auto fn = attn_bwd_kernel<N>; };

int launch_attn_fwd(hipStream_t s, const AttnArgs& a) { return attn_go<FwdK>(s, a); }
// 1: the one-launch backward (attn_bwd_kernel); 0: the key/value and query kernels (A/B builds)
#ifndef DFD_ATTN_BWD_FUSED
#define DFD_ATTN_BWD_FUSED 1
#endif
int launch_attn_bwd(hipStream_t s, const AttnArgs& a) {
  if (DFD_ATTN_BWD_FUSED) return attn_go<BwdK>(s, a);
  DFD_TRY(attn_go<KvK>(s, a));
  return attn_go<QK>(s, a);
}

}  // namespace dfd
