// Large bf16 GEMMs of the ViT-B/16 trunk (DeepfakeModel, src/models.py:88-107, 222-291; timm
// vit_base_patch16_224 restated in oracle/vit_cpu.py): every linear layer's forward and data
// gradient, C[M][N] = A[M][K] . B[N][K]^T, and every weight gradient, W[P][Q] = sum_m X1[m][p] X2[m][q],
// at M = images * 197 token rows (25,216 at the C5 batch of 128) and N, K, P, Q in {768, 2304, 3072}.
//
// gfx950 design (cdna_hip_programming.md section 5: the 256^2 LDS-DMA template):
//   * 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 each),
//     v_mfma_f32_16x16x32_bf16, fp32 accumulators (128 per lane), one workgroup per CU; 256 x 128
//     tiles (4 x 2 waves of 64 x 64) for the 768-wide products, whose 256-wide tiles fill only
//     1.2 dispatch waves;
//   * operands move HBM -> LDS by global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPR
//     staging), 64-deep K-steps double-buffered (2 x 64 KiB): the next K-step's DMA is in flight
//     while the current one's fragments are read and multiplied;
//   * bank-conflict-free fragment reads through XOR swizzles applied on the DMA SOURCE address
//     (the LDS image of an LDS-DMA is lane-linear): NT operands are [rows][64 k] images (128-B rows)
//     read with ds_read_b128, chunk ^ ((row >> 1) & 7); the weight-gradient operands are [64 m][256]
//     images (512-B rows) read TRANSPOSED with ds_read_b64_tr_b16, chunk ^ (2 (m & 3) + 8 ((m >> 3) & 1));
//   * XCD-aware tile order (tiles that share an A row panel run on one XCD's L2);
//   * epilogue through LDS in two 128-row passes: row-contiguous 16-B stores, with the bias, the
//     residual add, GELU (fc1 stores both Z and gelu(Z)) or the GELU derivative (fc2's data
//     gradient) applied in fp32 and rounded once;
//   * weight gradients split over M into fp32 slabs (one dispatch wave of workgroups), summed in a
//     fixed order (launch_reduce_slabs): the step stays bit-reproducible.
#include "kernels.h"
#include "tail.h"
#include "vit.h"

// 1: fc1's gelu / gelu' epilogue on the branch-free rational erf (common.h erf_rat_); 0: the library
// erff (A/B builds, tools/ab_lib.sh)
#ifndef DFD_GELU_RAT
#define DFD_GELU_RAT 1
#endif

namespace dfd {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(3))) s16x4* lds_s4p;

constexpr int VT = 256;                       // output tile edge
constexpr int VK = 64;                        // K-step (NT) / m-step (TN)
constexpr int VTILE = VT * VK * 2;            // 32 KiB: one operand's K-step image
constexpr int EPS = VT + 4;                   // fp32 epilogue row stride (floats): conflict-free ds_write_b32
constexpr int EPI_BYTES = 128 * EPS * 4;      // one 128-row pass
constexpr int VLDS = 4 * VTILE > EPI_BYTES ? 4 * VTILE : EPI_BYTES;

__device__ const uint4 g_vzero[32] = {};      // 512 B of zeros: the DMA source of rows past the end (TN)

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// wait for this wave's vector-memory operations except the youngest N (LDS counter untouched), and a
// workgroup barrier that does not drain them (__syncthreads would wait for vmcnt(0))
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void lds_bar() {
  asm volatile("" ::: "memory");  // no memory operation moves across (the builtins below touch no memory)
  __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0), visible to the compiler's wait tracking
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------- NT: C = A . B^T
// One K-step image of an operand: [ROWS rows][64 k] bf16, 128-B rows, chunk (16 B) c of row r at
// slot c ^ ((r >> 1) & 7).  Wave w fills rows (ROWS/8) w .. with ROWS/64 DMA instructions of 8 rows.
template <int ROWS = VT>
__device__ __forceinline__ void stage_nt(const bf16* __restrict__ G, int64_t ld, int row0, int rows, int k0, char* img,
                                         int w, int lane) {
  constexpr int IPW = ROWS / 64;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int q = w * IPW + i;
    const int r = 8 * q + (lane >> 3);
    const int gc = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = min(row0 + r, rows - 1);  // rows past the end: any valid row (their outputs are not stored)
    const bf16* src = G + (int64_t)gr * ld + k0 + gc * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)(img + q * 1024), 16, 0, 0);
  }
}

// The A operand of an implicit convolution: row r of the tile = output pixel row0 + r; its 64-deep
// K-step k0 is channels [c0, c0 + 64) of one tap (Cin % 64 == 0), read from the input pixel the tap
// meets, or from the zero page outside the map (and past the last row).  The pixel decomposition
// of the wave's rows (IPW per lane) is computed once per tile: ConvRows.
struct ConvRows {
  int nb[4], iy[4], ix[4];  // n * H, oy * stride - pad, ox * stride - pad (nb < 0: past the last row)
};
__device__ __forceinline__ void conv_rows(const VgemmArgs& a, int row0, int w, int lane, ConvRows& cr) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 8 * (w * 4 + i) + (lane >> 3);
    const int m = row0 + r;
    const int hw = a.Ho * a.Wo, n = m / hw, q = m - n * hw, oy = q / a.Wo, ox = q - oy * a.Wo;
    cr.nb[i] = m < a.M ? n * a.H : -1;
    cr.iy[i] = oy * a.stride - a.pad;
    cr.ix[i] = ox * a.stride - a.pad;
  }
}
__device__ __forceinline__ void stage_conv(const VgemmArgs& a, const ConvRows& cr, int k0, char* img, int w, int lane) {
  const int tap = k0 >> a.cin_log2, c0 = k0 & ((1 << a.cin_log2) - 1);
  const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = w * 4 + i;
    const int r = 8 * q + (lane >> 3);
    const int gc = (lane & 7) ^ ((r >> 1) & 7);
    const int y = cr.iy[i] + kh, x = cr.ix[i] + kw;
    const bool in = cr.nb[i] >= 0 && y >= 0 && y < a.H && x >= 0 && x < a.W;
    const bf16* src = in ? a.A + ((((int64_t)(cr.nb[i] + y) * a.W + x) << a.cin_log2) + c0 + gc * 8)
                         : reinterpret_cast<const bf16*>(g_vzero) + gc * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)(img + q * 1024), 16, 0, 0);
  }
}

// fragment of rows base .. base+15 (base % 16 == 0) at k-chunk 4s + (lane >> 4)
__device__ __forceinline__ s16x8 frag_nt(const char* img, int base, int s, int lane) {
  const int r = base + (lane & 15);
  const int c = (4 * s + (lane >> 4)) ^ ((lane & 15) >> 1);
  return *reinterpret_cast<const s16x8*>(img + r * 128 + (c << 4));
}

// ---------------------------------------------------------------- TN: W = X1^T . X2
// One m-step image of an operand: [64 m][256 cols] bf16, 512-B rows, chunk c of row m at slot
// c ^ (2 (m & 3) + 8 ((m >> 3) & 1)).  Wave w fills rows 8w .. 8w+7 (4 DMA instructions of 2 rows).
__device__ __forceinline__ int tn_swz(int m) { return 2 * (m & 3) + 8 * ((m >> 3) & 1); }

template <int ROWS = VK>
__device__ __forceinline__ void stage_tn(const bf16* __restrict__ G, int64_t ld, int m0, int m_end, int c0, char* img,
                                         int w, int lane) {
  constexpr int IPW = ROWS / 16;  // DMA instructions (2 rows each) per wave
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int q = w * IPW + i;
    const int m = 2 * q + (lane >> 5);
    const int gc = (lane & 31) ^ tn_swz(m);
    const bf16* src = m0 + m < m_end ? G + (int64_t)(m0 + m) * ld + c0 + gc * 8
                                     : reinterpret_cast<const bf16*>(g_vzero) + gc * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)(img + q * 1024), 16, 0, 0);
  }
}

// MFMA operand of output rows base .. base+15 (the image's columns) at k = 32 s + 8 (lane >> 4) + j:
// two transposed reads of 4 m-rows x 16 columns each (ds_read_b64_tr_b16)
__device__ __forceinline__ s16x8 frag_tn(const char* img, int base, int s, int lane) {
  const int h = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int n = base + 4 * pp;
  const int c = n >> 3, half = (n >> 2) & 1;
  const int m1 = 32 * s + 8 * h + qq, m2 = m1 + 4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4p)(img + m1 * 512 + ((c ^ tn_swz(m1)) << 4) + half * 8));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4p)(img + m2 * 512 + ((c ^ tn_swz(m2)) << 4) + half * 8));
  return s16x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
}

// ---------------------------------------------------------------- shared pieces
template <int MI = 8, int NJ = 4>
struct Acc {
  f32x4 v[MI][NJ];
};

// one 64-deep step of a wave's MI x NJ block of 16 x 16 MFMA tiles at (rbase, cbase) of the tile
template <bool TN, int NS = 2, int MI, int NJ>
__device__ __forceinline__ void mma_step(const char* Ai, const char* Bi, int rbase, int cbase, int lane,
                                         Acc<MI, NJ>& acc) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    s16x8 af[MI], bfr[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = TN ? frag_tn(Ai, rbase + 16 * i, s, lane) : frag_nt(Ai, rbase + 16 * i, s, lane);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bfr[j] = TN ? frag_tn(Bi, cbase + 16 * j, s, lane) : frag_nt(Bi, cbase + 16 * j, s, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc.v[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
}

// XP schedule (NT): a sub-step's fragments are read while the previous sub-step's MFMAs run, across
// the K-step barrier too (the next K-step's first fragments are read right after it, under the
// second sub-step's MFMAs) -- the waves of a SIMD no longer all wait on LDS reads at once after each
// barrier
template <int MI, int NJ>
struct Frags {
  s16x8 a[MI], b[NJ];
};
template <int MI, int NJ>
__device__ __forceinline__ void frags_nt(const char* Ai, const char* Bi, int rbase, int cbase, int s, int lane,
                                         Frags<MI, NJ>& f) {
#pragma unroll
  for (int i = 0; i < MI; ++i) f.a[i] = frag_nt(Ai, rbase + 16 * i, s, lane);
#pragma unroll
  for (int j = 0; j < NJ; ++j) f.b[j] = frag_nt(Bi, cbase + 16 * j, s, lane);
}
template <int MI, int NJ>
__device__ __forceinline__ void mma_frags(const Frags<MI, NJ>& f, Acc<MI, NJ>& acc) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[j], acc.v[i][j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

// a wave's accumulators into the fp32 staging image E (row stride eps) at (r0, c0)
template <int MI, int NJ>
__device__ __forceinline__ void epi_put(float* E, const Acc<MI, NJ>& acc, int r0, int c0, int eps, int lane) {
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) E[(r0 + 16 * i + 4 * (lane >> 4) + e) * eps + c0 + 16 * j + (lane & 15)] = acc.v[i][j][e];
}

__device__ __forceinline__ void st8bf(bf16* p, const float (&v)[8]) { st8(p, v); }

// ---------------------------------------------------------------- kernels
// BNT = 64 (ResNet-50 layer1, Cout 64): 8 (M) x 1 (N) waves of 32 x 64.
// BNT = 256: 8 waves as 2 (M) x 4 (N), 128 x 64 each; BNT = 128 (N = 768-wide products: 2.3 instead of
// 1.2 dispatch waves of tiles, so the last wave idles less): 4 (M) x 2 (N) waves of 64 x 64
template <int EP, int BNT, bool CONV = false, bool XP = false>
__global__ __launch_bounds__(512, 1) void vgemm_nt_kernel(VgemmArgs a) {
  constexpr int WMN = BNT == VT ? 2 : BNT == 128 ? 4 : 8, WNN = 8 / WMN;  // waves along M / N
  constexpr int MI = VT / WMN / 16, NJ = BNT / WNN / 16;
  constexpr int BIMG = BNT * VK * 2;                    // B operand's K-step image
  constexpr int STAGE = VTILE + BIMG;
  constexpr int ES = BNT + 4;                           // epilogue row stride (floats)
  // K-step images in flight: 3 for the 128-wide tile (144 KiB; a DMA has two K-steps to land), 2 for
  // the 256-wide one (its K-step is twice as long)
  constexpr int NST = BNT == VT ? 2 : 3;
  constexpr int NPS = VT / 64 + BNT / 64;              // DMA instructions per thread per K-step
  constexpr int SMEM = NST * STAGE > 128 * ES * 4 ? NST * STAGE : 128 * ES * 4;
  static_assert(SMEM <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = uni(tid >> 6), wm = w / WNN, wn = w % WNN;
  const int L = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
  const int tm = L / a.tiles_n, tn = L - tm * a.tiles_n;
  const int row0 = tm * VT, col0 = tn * BNT;
  Acc<MI, NJ> acc;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc.v[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = a.K / VK;
  ConvRows cr;
  if constexpr (CONV) conv_rows(a, row0, w, lane, cr);
  auto stage_a = [&](int k0, char* img) {
    if constexpr (CONV) stage_conv(a, cr, k0, img, w, lane);
    else stage_nt<VT>(a.A, a.lda, row0, a.M, k0, img, w, lane);
  };
  auto stage = [&](int kt, char* img) {
    stage_a(kt * VK, img);
    stage_nt<BNT>(a.B, a.ldb, col0, a.N, kt * VK, img + VTILE, w, lane);
  };
  // counted waits: a K-step's DMA must have landed before the barrier that precedes its reads; the
  // younger K-steps' DMAs (NPS instructions each) stay in flight
  stage(0, smem);
  for (int p = 1; p < NST - 1; ++p)
    if (p < nk) stage(p, smem + p * STAGE);
  if (NST == 3 && nk > 1) vm_wait_n<NPS>();
  else vm_wait_n<0>();
  lds_bar();
  int cb = 0, pb = NST - 1;  // buffers of K-steps kt and kt + NST - 1
  const int rb = wm * (VT / WMN), cbs = wn * (BNT / WNN);
  if constexpr (XP) {
    Frags<MI, NJ> f0, f1;
    frags_nt(smem, smem + VTILE, rb, cbs, 0, lane, f0);
    for (int kt = 0; kt < nk; ++kt) {
      char* cur = smem + cb * STAGE;
      const bool pre = kt + NST - 1 < nk;
      if (pre) stage(kt + NST - 1, smem + pb * STAGE);
      frags_nt(cur, cur + VTILE, rb, cbs, 1, lane, f1);
      // f0's reads (issued before f1's) have landed once at most f1's MI + NJ reads are outstanding
      __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | ((MI + NJ) << 8) | (3 << 14));
      mma_frags(f0, acc);
      if (NST == 3 && pre) vm_wait_n<NPS>();
      else vm_wait_n<0>();
      lds_bar();  // this K-step's reads done everywhere (f1 included); K-step kt + 1 landed
      cb = cb == NST - 1 ? 0 : cb + 1;
      pb = pb == NST - 1 ? 0 : pb + 1;
      // unconditional (after the last K-step it reads a stale image, unused): no branch, so the
      // compiler's LDS wait before f1's MFMAs stays counted
      frags_nt(smem + cb * STAGE, smem + cb * STAGE + VTILE, rb, cbs, 0, lane, f0);
      __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | ((MI + NJ) << 8) | (3 << 14));  // f1 landed before the barrier
      mma_frags(f1, acc);
    }
  } else {
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + cb * STAGE;
    const bool pre = kt + NST - 1 < nk;
    if (pre) stage(kt + NST - 1, smem + pb * STAGE);  // the buffer K-step kt - 1 read (barrier passed)
    mma_step<false>(cur, cur + VTILE, rb, cbs, lane, acc);
    if (NST == 3 && pre) vm_wait_n<NPS>();  // K-step kt + 1 landed; kt + 2 may still be in flight
    else vm_wait_n<0>();
    lds_bar();  // this K-step's reads done everywhere
    cb = cb == NST - 1 ? 0 : cb + 1;
    pb = pb == NST - 1 ? 0 : pb + 1;
  }
  }
  // epilogue: two passes of 128 rows through LDS; a pass's residual / derivative rows are loaded
  // before its staging barrier (their latency under the LDS round trip, not per row)
  constexpr int VPR = BNT / 8, RPS = 512 / VPR, NIT = 128 / RPS;  // 8-column vectors per row, rows per sweep
  constexpr bool LD = (EP & (VG_RESID | VG_DGELU)) != 0;
  float* E = reinterpret_cast<float*>(smem);
  const int v = tid % VPR, rsub = tid / VPR;
  const int c = col0 + 8 * v;
  float bias[8];
  if constexpr ((EP & VG_BIAS) != 0) ld8f(a.bias + c, bias);
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    uint4 xr[LD ? NIT : 1];
    if constexpr (LD) {
      const bf16* src = (EP & VG_RESID) != 0 ? a.R : a.Z;
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int row = min(row0 + pass * 128 + it * RPS + rsub, a.M - 1);
        xr[it] = *reinterpret_cast<const uint4*>(src + (int64_t)row * a.ldc + c);
      }
    }
    const int wr0 = wm * (VT / WMN) - pass * 128;  // this wave's first row within the pass
    if (wr0 >= 0 && wr0 < 128) epi_put(E, acc, wr0, wn * (BNT / WNN), ES, lane);
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rl = it * RPS + rsub;
      const int row = row0 + pass * 128 + rl;
      if (row < a.M) {
        float o[8];
        const float4 x0 = *reinterpret_cast<const float4*>(E + rl * ES + 8 * v);
        const float4 x1 = *reinterpret_cast<const float4*>(E + rl * ES + 8 * v + 4);
        o[0] = x0.x; o[1] = x0.y; o[2] = x0.z; o[3] = x0.w; o[4] = x1.x; o[5] = x1.y; o[6] = x1.z; o[7] = x1.w;
        if constexpr ((EP & VG_BIAS) != 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += bias[j];
        }
        if constexpr (LD) {
          const uint32_t wv[4] = {xr[it].x, xr[it].y, xr[it].z, xr[it].w};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xv = __uint_as_float((j & 1) ? (wv[j >> 1] & 0xffff0000u) : (wv[j >> 1] << 16));
            if constexpr ((EP & VG_RESID) != 0) o[j] += xv;
            else o[j] *= xv;  // VG_DGELU: the stored gelu'
          }
        }
        if constexpr ((EP & VG_RELU) != 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
        }
        if constexpr ((EP & VG_GELU2) != 0) {
          // C = gelu'(z), G = gelu(z) of the stored (rounded) pre-activation z
          float g[8];
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            if (DFD_GELU_RAT) {
              f32x2_t gg, dd;
              gelu_pair2_rat_(f32x2_t{Tr<bf16>::round(o[j]), Tr<bf16>::round(o[j + 1])}, gg, dd);
              g[j] = gg.x; g[j + 1] = gg.y; o[j] = dd.x; o[j + 1] = dd.y;
            } else {
              gelu_pair_(Tr<bf16>::round(o[j]), g[j], o[j]);
              gelu_pair_(Tr<bf16>::round(o[j + 1]), g[j + 1], o[j + 1]);
            }
          }
          st8bf(a.G + (int64_t)row * a.ldc + c, g);
        }
        if constexpr ((EP & VG_GELU) != 0) {
          // inference fc1: C = gelu(z) alone, the same value VG_GELU2 leaves in G (no derivative store)
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            if (DFD_GELU_RAT) {
              f32x2_t gg, dd;
              gelu_pair2_rat_(f32x2_t{Tr<bf16>::round(o[j]), Tr<bf16>::round(o[j + 1])}, gg, dd);
              o[j] = gg.x; o[j + 1] = gg.y;
            } else {
              float gd;
              gelu_pair_(Tr<bf16>::round(o[j]), o[j], gd);
              gelu_pair_(Tr<bf16>::round(o[j + 1]), o[j + 1], gd);
            }
          }
        }
        st8bf(a.C + (int64_t)row * a.ldc + c, o);
      }
    }
    __syncthreads();
  }
}

// TK = 64: two 64-deep m-step images (128 KiB); TK = 32: four 32-deep ones (a DMA has three steps to
// land; one 32-deep MFMA sub-step per barrier) -- DFD_TN_DEPTH, an A/B build switch
#ifndef DFD_TN_DEPTH
#define DFD_TN_DEPTH 64
#endif
template <int TK, bool COOP = false>
__global__ __launch_bounds__(512, 1) void vgemm_tn_kernel(VgemmTnArgs a) {
  constexpr int NST = TK == 64 ? 2 : 4;
  constexpr int OPI = TK * VT * 2;        // one operand's m-step image
  constexpr int NPS = 2 * (TK / 16);      // DMA instructions per thread per m-step (both operands)
  static_assert(NST * 2 * OPI <= VLDS, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[VLDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = uni(tid >> 6), wm = w >> 2, wn = w & 3;
  const int tiles = a.tiles_p * a.tiles_q;
  const int L = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
  const int split = L / tiles, t = L - split * tiles;
  const int tp = t / a.tiles_q, tq = t - tp * a.tiles_q;
  const int p0 = tp * VT, q0 = tq * VT;
  const int m_begin = split * a.mchunk, m_end = min(a.M, m_begin + a.mchunk);
  Acc<8, 4> acc;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc.v[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = m_end > m_begin ? (m_end - m_begin + TK - 1) / TK : 0;
  auto stage = [&](int kt, char* img) {
    stage_tn<TK>(a.X1, a.ld1, m_begin + kt * TK, m_end, p0, img, w, lane);
    stage_tn<TK>(a.X2, a.ld2, m_begin + kt * TK, m_end, q0, img + OPI, w, lane);
  };
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) stage(p, smem + p * 2 * OPI);
  // m-step 0 landed: the younger prologue steps' DMAs stay in flight
  if (NST == 4 && nk > 2) vm_wait_n<2 * NPS>();
  else if (NST == 4 && nk > 1) vm_wait_n<NPS>();
  else vm_wait_n<0>();
  lds_bar();
  // the bias gradient of the linear whose output gradient is X1: colsum[p] = sum_m X1[m][p] as a
  // product with a ones operand (exact products, fixed order) on the workgroups of tile column 0,
  // each wave taking 2 of its half's 8 row blocks (+2 MFMAs and 4 transposed reads per 32-deep
  // step; replaces a separate column-sum pass over X1)
  const bool csum = a.colsum && tq == 0;
  f32x4 cacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const s16x8 ones = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};  // bf16 1.0
  int cb = 0, pb = NST - 1;  // buffers of m-steps kt and kt + NST - 1
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + cb * 2 * OPI;
    if (kt + NST - 1 < nk) stage(kt + NST - 1, smem + pb * 2 * OPI);  // the buffer m-step kt - 1 read
    mma_step<true, TK / 32>(cur, cur + OPI, wm * 128, wn * 64, lane, acc);
    if (csum) {
#pragma unroll
      for (int s2 = 0; s2 < TK / 32; ++s2)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
          cacc[ii] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tn(cur, wm * 128 + 16 * (2 * wn + ii), s2, lane), ones,
                                                             cacc[ii], 0, 0, 0);
    }
    // m-step kt + 1 landed; the younger ones (at most NST - 2) may still be in flight
    const int younger = min(kt + NST - 1, nk - 1) - (kt + 1);
    if (NST == 4 && younger >= 2) vm_wait_n<2 * NPS>();
    else if (NST == 4 && younger == 1) vm_wait_n<NPS>();
    else vm_wait_n<0>();
    lds_bar();
    cb = cb == NST - 1 ? 0 : cb + 1;
    pb = pb == NST - 1 ? 0 : pb + 1;
  }
  const int64_t srow = (int64_t)a.P * a.Q + (a.colsum ? a.P : 0);  // slab row length
  if (csum && (lane & 15) == 0) {
    float* cs = a.slab + (int64_t)split * srow + (int64_t)a.P * a.Q + p0 + wm * 128;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[16 * (2 * wn + ii) + 4 * (lane >> 4) + e] = cacc[ii][e];
  }
  float* E = reinterpret_cast<float*>(smem);
  const int v = tid & 31, rsub = tid >> 5;
  float* out = a.slab + (int64_t)split * srow;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    if (wm == pass) epi_put(E, acc, 0, wn * 64, EPS, lane);
    __syncthreads();
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int rl = it * 16 + rsub;
      const int p = p0 + pass * 128 + rl;
      float* dst = out + (int64_t)p * a.Q + q0 + 8 * v;
      *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(E + rl * EPS + 8 * v);
      *reinterpret_cast<float4*>(dst + 4) = *reinterpret_cast<const float4*>(E + rl * EPS + 8 * v + 4);
    }
    __syncthreads();
  }
  if constexpr (COOP) {
    // every split of this tile has written its slab rows; this split sums its share of the tile's
    // rows over all splits in split order (bit-reproducible: independent of arrival order)
    const int S = a.splits;
    if (S > 1) group_sync(a.bar + 2 * t, a.bar + 2 * t + 1, (unsigned)S);
    const int per = (VT + S - 1) / S;
    const int r0 = min(VT, split * per), r1 = min(VT, r0 + per);
    const int nv = (r1 - r0) * (VT / 4);
    for (int i = tid; i < nv; i += 512) {
      const int rr = r0 + i / (VT / 4), c4 = (i % (VT / 4)) * 4;
      const int64_t off = (int64_t)(p0 + rr) * a.Q + q0 + c4;
      float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
      // 8 splits' loads in flight per round trip, added in split order
      for (int sb = 0; sb < S; sb += 8) {
        float4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          x[u] = sb + u < S ? *reinterpret_cast<const float4*>(a.slab + (int64_t)(sb + u) * srow + off)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (sb + u < S) {
            if (sb + u == 0) sum = x[u];
            else { sum.x += x[u].x; sum.y += x[u].y; sum.z += x[u].z; sum.w += x[u].w; }
          }
      }
      if (a.accumulate) {
        const float4 w0 = *reinterpret_cast<const float4*>(a.W + off);
        sum.x = w0.x + sum.x; sum.y = w0.y + sum.y; sum.z = w0.z + sum.z; sum.w = w0.w + sum.w;
      }
      *reinterpret_cast<float4*>(a.W + off) = sum;
    }
    if (csum) {  // the bias gradient entries p0 + [r0, r1) of this tile row
      for (int i = tid; i < r1 - r0; i += 512) {
        const int64_t off = (int64_t)a.P * a.Q + p0 + r0 + i;
        float sum = a.slab[off];
        for (int sp = 1; sp < S; ++sp) sum += a.slab[(int64_t)sp * srow + off];
        const int64_t o = p0 + r0 + i;
        a.colsum_out[o] = a.accumulate ? a.colsum_out[o] + sum : sum;
      }
    }
  }
}

}  // namespace

bool vgemm_nt_covers(int64_t M, int N, int K) {
  return M > 0 && M < (1ll << 31) && N % 64 == 0 && K % VK == 0 && K > 0;
}
// implicit convolution: a 64-deep K-step is 64 channels of one tap (Cin a power of two >= 64), the
// output width a multiple of the 128-wide tile, KW in {1, 3} (KH <= 3)
bool vgemm_conv_covers(int Cin, int Cout, int KH, int KW) {
  return Cin >= 64 && (Cin & (Cin - 1)) == 0 && Cout % 64 == 0 && (KW == 1 || KW == 3) && KH <= 3 && KH >= 1;
}
bool vgemm_tn_covers(int64_t M, int P, int Q) { return M > 0 && M < (1ll << 31) && P % VT == 0 && Q % VT == 0; }

// the 128-wide tile where 256-wide tiles would leave the last dispatch wave mostly idle: N % 256 != 0,
// or fewer than ~2 waves of 256 x 256 tiles (ViT-B's 768-wide products at M = 25,216: 297 tiles on
// 256 CUs)
static int vgemm_nt_bn(int64_t M, int N) {
  if (N % 128) return 64;
  if (N % VT) return 128;
  const int64_t t256 = cdiv64(M, VT) * (N / VT);
  return t256 < 2 * 256 ? 128 : VT;
}

int launch_vgemm_nt(hipStream_t s, const VgemmArgs& a0, int ep) {
  if (!vgemm_nt_covers(a0.M, a0.N, a0.K)) { set_error("vgemm: shape not covered", __FILE__, __LINE__); return -1; }
  VgemmArgs a = a0;
  const int bn = a0.bn ? a0.bn : vgemm_nt_bn(a.M, a.N);
  if (a.N % bn || (bn != 64 && bn != 128 && bn != VT)) { set_error("vgemm: tile width", __FILE__, __LINE__); return -1; }
  a.tiles_n = a.N / bn;
  const int tiles = cdiv(a.M, VT) * a.tiles_n;
  if (a.conv) {  // implicit convolutions (the ResNet-50 eval 3x3 / strided layers): bias, identity, ReLU
    if (!vgemm_conv_covers(1 << a.cin_log2, a.N, 3, a.KW) || a.K % (1 << a.cin_log2)) {
      set_error("vgemm: convolution shape not covered", __FILE__, __LINE__);
      return -1;
    }
    if (bn == 64) {  // Cout 64 (layer1): the plain K loop
      switch (ep) {
        case VG_BIAS: hipLaunchKernelGGL((vgemm_nt_kernel<VG_BIAS, 64, true>), dim3(tiles), dim3(512), 0, s, a); break;
        case VG_BIAS | VG_RELU:
          hipLaunchKernelGGL((vgemm_nt_kernel<VG_BIAS | VG_RELU, 64, true>), dim3(tiles), dim3(512), 0, s, a); break;
        case VG_BIAS | VG_RESID | VG_RELU:
          hipLaunchKernelGGL((vgemm_nt_kernel<VG_BIAS | VG_RESID | VG_RELU, 64, true>), dim3(tiles), dim3(512), 0, s, a);
          break;
        default: set_error("vgemm: convolution epilogue not instantiated", __FILE__, __LINE__); return -1;
      }
      DFD_HIP_CHECK(hipGetLastError());
      return 0;
    }
    const bool xpc = (tune(TK_VG_XP) & (bn == 128 ? 1 : 2)) != 0;
    switch ((ep * 2 + (bn == 128)) * 2 + xpc) {
#define DFD_VGC(E)                                                                                                   \
  case 4 * (E): hipLaunchKernelGGL((vgemm_nt_kernel<E, VT, true>), dim3(tiles), dim3(512), 0, s, a); break;        \
  case 4 * (E) + 1: hipLaunchKernelGGL((vgemm_nt_kernel<E, VT, true, true>), dim3(tiles), dim3(512), 0, s, a); break; \
  case 4 * (E) + 2: hipLaunchKernelGGL((vgemm_nt_kernel<E, 128, true>), dim3(tiles), dim3(512), 0, s, a); break;   \
  case 4 * (E) + 3: hipLaunchKernelGGL((vgemm_nt_kernel<E, 128, true, true>), dim3(tiles), dim3(512), 0, s, a); break;
      DFD_VGC(VG_BIAS) DFD_VGC(VG_BIAS | VG_RELU) DFD_VGC(VG_BIAS | VG_RESID | VG_RELU)
#undef DFD_VGC
      default: set_error("vgemm: convolution epilogue not instantiated", __FILE__, __LINE__); return -1;
    }
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
  // knob vg_xp: the fragment-pipelined K loop (XP); bit 0 for the 128-wide tile, bit 1 for the 256-wide
  // (the weight-gradient kernel's form of it needs 2 x 24 fragment registers and spills: not built)
  if (bn == 64) {  // 64-wide outputs (ResNet-50 layer1): bias / identity / ReLU epilogues, plain K loop
    switch (ep) {
      case 0: hipLaunchKernelGGL((vgemm_nt_kernel<0, 64>), dim3(tiles), dim3(512), 0, s, a); break;
      case VG_BIAS: hipLaunchKernelGGL((vgemm_nt_kernel<VG_BIAS, 64>), dim3(tiles), dim3(512), 0, s, a); break;
      case VG_BIAS | VG_RESID: hipLaunchKernelGGL((vgemm_nt_kernel<VG_BIAS | VG_RESID, 64>), dim3(tiles), dim3(512), 0, s, a); break;
      case VG_BIAS | VG_RELU: hipLaunchKernelGGL((vgemm_nt_kernel<VG_BIAS | VG_RELU, 64>), dim3(tiles), dim3(512), 0, s, a); break;
      case VG_BIAS | VG_RESID | VG_RELU:
        hipLaunchKernelGGL((vgemm_nt_kernel<VG_BIAS | VG_RESID | VG_RELU, 64>), dim3(tiles), dim3(512), 0, s, a); break;
      default: set_error("vgemm: 64-wide epilogue not instantiated", __FILE__, __LINE__); return -1;
    }
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
  const int64_t xpk = tune(TK_VG_XP);
  const bool xp = (xpk & (bn == 128 ? 1 : 2)) != 0;
  switch ((ep * 2 + (bn == 128)) * 2 + xp) {
#define DFD_VG(E)                                                                                                   \
  case 4 * (E): hipLaunchKernelGGL((vgemm_nt_kernel<E, VT>), dim3(tiles), dim3(512), 0, s, a); break;             \
  case 4 * (E) + 1: hipLaunchKernelGGL((vgemm_nt_kernel<E, VT, false, true>), dim3(tiles), dim3(512), 0, s, a); break; \
  case 4 * (E) + 2: hipLaunchKernelGGL((vgemm_nt_kernel<E, 128>), dim3(tiles), dim3(512), 0, s, a); break;        \
  case 4 * (E) + 3: hipLaunchKernelGGL((vgemm_nt_kernel<E, 128, false, true>), dim3(tiles), dim3(512), 0, s, a); break;
    DFD_VG(0) DFD_VG(VG_BIAS) DFD_VG(VG_BIAS | VG_RESID) DFD_VG(VG_BIAS | VG_GELU2) DFD_VG(VG_BIAS | VG_GELU)
    DFD_VG(VG_DGELU)
    DFD_VG(VG_BIAS | VG_RELU) DFD_VG(VG_BIAS | VG_RESID | VG_RELU)
#undef DFD_VG
    default: set_error("vgemm: epilogue not instantiated", __FILE__, __LINE__); return -1;
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int vgemm_tn_splits(int64_t M, int P, int Q, int64_t slab_cap) {
  const int tiles = (P / VT) * (Q / VT);
  int splits = std::max(1, 256 / std::max(1, tiles));  // one dispatch wave of workgroups
  splits = (int)std::min<int64_t>(splits, cdiv64(M, 4 * VK));  // at least 4 m-steps per split
  splits = (int)std::max<int64_t>(1, std::min<int64_t>(splits, slab_cap / ((int64_t)P * Q)));
  return splits;
}

static int tn_device_cus() {
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

int launch_vgemm_tn(hipStream_t s, const bf16* X1, int64_t ld1, const bf16* X2, int64_t ld2, int64_t M, int P, int Q,
                    float* slab, int64_t slab_cap, float* W, bool accumulate, float* colsum_out, unsigned* bar) {
  if (!vgemm_tn_covers(M, P, Q)) { set_error("vgemm_tn: shape not covered", __FILE__, __LINE__); return -1; }
  const int64_t srow = (int64_t)P * Q + (colsum_out ? P : 0);
  if (srow > slab_cap) { set_error("vgemm_tn: slab too small", __FILE__, __LINE__); return -1; }
  VgemmTnArgs a{};
  a.X1 = X1; a.ld1 = ld1; a.X2 = X2; a.ld2 = ld2; a.M = (int)M; a.P = P; a.Q = Q;
  a.tiles_p = P / VT; a.tiles_q = Q / VT;
  a.colsum = colsum_out != nullptr;
  int splits = vgemm_tn_splits(M, P, Q, slab_cap);
  splits = (int)std::max<int64_t>(1, std::min<int64_t>(splits, slab_cap / srow));
  a.mchunk = (int)(cdiv64(cdiv64(M, splits), VK) * VK);
  splits = (int)cdiv64(M, a.mchunk);
  a.slab = slab;
  const int grid = splits * a.tiles_p * a.tiles_q;
  // cooperative split reduction: one 512-thread, ~128 KiB-LDS workgroup per CU, so the whole grid is
  // co-resident when it has at most one workgroup per CU (vgemm_tn_splits sizes it to one dispatch wave)
  if (bar && grid <= tn_device_cus()) {
    a.bar = bar; a.W = W; a.colsum_out = colsum_out; a.splits = splits; a.accumulate = accumulate ? 1 : 0;
    hipLaunchKernelGGL((vgemm_tn_kernel<DFD_TN_DEPTH, true>), dim3(grid), dim3(512), 0, s, a);
    DFD_HIP_CHECK(hipGetLastError());
    return 0;
  }
  hipLaunchKernelGGL(vgemm_tn_kernel<DFD_TN_DEPTH>, dim3(grid), dim3(512), 0, s, a);
  DFD_HIP_CHECK(hipGetLastError());
  if (!colsum_out) return launch_reduce_slabs(s, slab, splits, (int64_t)P * Q, W, accumulate);
  // a linear's bias gradient stored right after its weight gradient (named_parameters order): one
  // reduction over the whole slab row
  if (colsum_out == W + (int64_t)P * Q) return launch_reduce_slabs(s, slab, splits, srow, W, accumulate);
  DFD_TRY(launch_reduce_slabs_strided(s, slab, splits, (int64_t)P * Q, srow, W, accumulate));
  return launch_reduce_slabs_strided(s, slab + (int64_t)P * Q, splits, P, srow, colsum_out, accumulate);
}

}  // namespace dfd
