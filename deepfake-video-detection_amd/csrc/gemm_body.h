// Tile loops of the 16-bit / fp32 MFMA GEMMs as device functions (pw_gemm_body, pw_wgrad_body), shared by
// the 1x1-convolution kernels of k_gemm.hip (EfficientNet-B0) and the ResNet-50 bf16 training
// convolutions of k_rn16.hip, which run the same loops on an implicit-GEMM gather of the convolution
// input (ConvGather) instead of a dense row-major operand.
#pragma once
#include "kernels.h"

#ifndef DFD_XCD_SWZ
#define DFD_XCD_SWZ 1  // XCD-aware block order of the weight-gradient kernel (A/B knob; -5..-20 us
                       // per 50176/12544-row layer: the 22-126 tiles of one M-split share an L2)
#endif

namespace dfd {

// ---- implicit-GEMM gather of a KHxKW convolution (NHWC source, C % 8 == 0; one tap per k-step) ----
// rows = pixels of the row map (frames x Ho x Wo), k = (ky, kx, c) with c fastest.  Forward / weight
// gradient (dgrad = 0): a row is an OUTPUT pixel and reads source pixel (oy S - P + ky, ox S - P + kx).
// Data gradient (dgrad = 1): a row is an INPUT pixel of the convolution and the source is its output
// gradient, read at ((iy + P - ky) / S, (ix + P - kx) / S) where both divide (S = 1 or 2) -- the
// transposed convolution; with the weights packed [Cin][KH][KW][Cout] the MFMA sequence is the GEMM's.
struct ConvRow {
  int64_t base;  // element offset of the row's frame in the source
  int y, x;      // forward: oy S - P, ox S - P;  dgrad: iy + P, ix + P
  bool ok;       // row < M
};
struct ConvTap {
  int k0, ky, kx;  // first k of the tap, kernel row / column
};
struct ConvGather {
  int C, H, W;      // source tensor: channels, map
  int Ho, Wo;       // row map per frame
  int KW, S, P, dgrad;
  uint32_t mhw, lhw, mw, lw;  // x / (Ho Wo), x / Wo as (mulhi(x, m) + x) >> l
  __device__ __forceinline__ static uint32_t fdiv(uint32_t x, uint32_t m, uint32_t l) {
    return (uint32_t)(((uint64_t)__umulhi(x, m) + x) >> l);
  }
  __device__ __forceinline__ ConvRow row(int64_t gm, int64_t M) const {
    ConvRow r;
    r.ok = gm < M;
    const uint32_t g = r.ok ? (uint32_t)gm : 0u;
    const uint32_t n = fdiv(g, mhw, lhw), q = g - n * (uint32_t)(Ho * Wo), oy = fdiv(q, mw, lw), ox = q - oy * Wo;
    r.base = (int64_t)n * H * W * C;
    if (dgrad) { r.y = (int)oy + P; r.x = (int)ox + P; }
    else { r.y = (int)oy * S - P; r.x = (int)ox * S - P; }
    return r;
  }
  __device__ __forceinline__ ConvTap tap(int k) const {
    const int t = k / C, ky = t / KW;
    return ConvTap{t * C, ky, t - ky * KW};
  }
  // element offset of (row, tap, channel c) in the source; false: zero (padding / no such tap)
  __device__ __forceinline__ bool src(const ConvRow& r, const ConvTap& t, int c, int64_t& off) const {
    int sy, sx;
    bool ok = r.ok;
    if (dgrad) {
      const int ty = r.y - t.ky, tx = r.x - t.kx;
      ok = ok && ty >= 0 && tx >= 0;
      if (S == 2) { ok = ok && ((ty | tx) & 1) == 0; sy = ty >> 1; sx = tx >> 1; }
      else { sy = ty; sx = tx; }
    } else {
      sy = r.y + t.ky; sx = r.x + t.kx;
      ok = ok && sy >= 0 && sx >= 0;
    }
    ok = ok && sy < H && sx < W;
    off = ok ? r.base + ((int64_t)sy * W + sx) * C + c : 0;
    return ok;
  }
};
// host: the divisors of ConvGather (round-up multiplier, 33-bit intermediate)
inline void conv_gather_fdiv(uint32_t d, uint32_t& m, uint32_t& l) {
  l = 0;
  while ((1ull << l) < d) ++l;
  m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d + 1) & 0xffffffffu);
}

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

// Tile shape: BM x BN outputs per workgroup of 4 waves laid out WM x WN (WM * WN = 4); each wave
// owns RB x CB 16x16 MFMA blocks; BK = contraction per k-step (one LDS hand-off, BK / 32 MFMA
// k-slices).  D = global-load pipeline depth: the loads of k-step k + D are issued while step k
// computes (register ring, static stage index via a D-unrolled k loop).
template <typename T, int BM, int BN, int WN, int D, int BK>
struct GemmCfg {
  static constexpr int WM = 4 / WN;
  static constexpr int RB = BM / WM / 16, CB = BN / WN / 16;
  static constexpr int VPR = BK / 8, RPP = 256 / VPR;       // 8-vectors per row, rows per staging pass
  static constexpr int PA = BM / RPP, PB = BN / RPP;        // 8-vectors per thread per k-step
  // LDS row stride (elements) of the A/B tiles.  bf16: unpadded rows whose 16-B chunks are XOR-
  // swizzled by row group (lds_off), so both the staging stores (rows x chunks of one k-step) and
  // the MFMA fragment reads (16 rows, one chunk) hit 16 distinct 4-bank groups; fp32: padded rows.
  static constexpr int AS = sizeof(T) == 2 ? BK : BK + 4;
  static constexpr int CPR = BK / 8;                         // 16-B chunks per bf16 row (4, 8, 16)
  __device__ __forceinline__ static int lds_off(int row, int k) {  // element offset of (row, k), k % 8 == 0
    if constexpr (sizeof(T) == 2) return row * AS + (((k >> 3) ^ ((row / (16 / CPR)) & (CPR - 1))) << 3);
    else return row * AS + k;
  }
  static constexpr int CS = sizeof(T) == 2 ? BN + 8 : BN + 4;    // LDS row stride of the C tile
  static constexpr int AB_BYTES = (BM + BN) * AS * (int)sizeof(T);
  static constexpr int C_BYTES = BM * CS * (int)sizeof(T);
  static constexpr int SMEM = AB_BYTES > C_BYTES ? AB_BYTES : C_BYTES;
  static_assert(WM * WN == 4 && RB >= 1 && CB >= 1 && PA >= 1 && PB >= 1 && BK % 32 == 0, "tile shape");
};

template <typename T>
__device__ __forceinline__ void lds_st8(T* p, const float (&v)[8]) { st8(p, v); }
template <typename T>
__device__ __forceinline__ void lds_ld8(const T* p, float (&v)[8]) { ld8(p, v); }

// The tile loop of one workgroup (the plain kernel below; the ResNet-50 bf16 training convolutions of
// k_rn16.hip): bid / nblk are the workgroup's index and count in its grid, the LDS arrays the
// caller's (st_*: STATS only, pro_lds: BN prologues only).  GA = 1: A is not a dense row-major
// matrix but the implicit-GEMM gather of a convolution (ConvGather, gemm_body.h), one tap per k-step.
// STATS = 1: per-column (sum, sum of squares) of the outputs, one partial row per workgroup;
// STATS = 2: per wave-row group (the BM / WM consecutive rows of one wave row of a tile) the column
// sum and the sum of squared deviations from that group's own column mean: centred partials of
// consecutive BM / WM-row groups, stats row mt * WM + wm (launch_bn_finalize chan_rows = BM / WM;
// empty groups past M write nothing).
// FOLD (fp32): two-level K sum -- each k-step's products go to a fresh tile that is then added to the
// running sum (the ResNet-50 fp32 training convolutions, whose train-mode BatchNorm amplifies rounding).
template <typename T, int MODE, int STATS, int EPI, int BM, int BN, int WN, int D, int BK, int GA = 0, bool FOLD = false>
__device__ __forceinline__ void pw_gemm_body(const T* __restrict__ A, const T* __restrict__ B, T* __restrict__ C,
                                             const T* __restrict__ R, const float* __restrict__ bias,
                                             const T* __restrict__ Z, int64_t M, int N, int K, const Pro& pro,
                                             float* __restrict__ stats, int64_t tiles_m, int ntn, int bid, int nblk,
                                             char* smem, float* st_sum, float* st_sq, float* st_part,
                                             float* pro_lds, const ConvGather& cg = ConvGather{}) {
  constexpr bool RESID = (EPI & EPI_RESID) != 0, BIAS = (EPI & EPI_BIAS) != 0, DGELU = (EPI & EPI_DGELU) != 0;
  using G = GemmCfg<T, BM, BN, WN, D, BK>;
  constexpr int GBK = BK;
  constexpr int WM = G::WM, RB = G::RB, CB = G::CB, PA = G::PA, PB = G::PB;
  constexpr bool GATE = pro_is_gated(MODE);
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + BM * G::AS;
  T* Cs = reinterpret_cast<T*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int rbase = wm * (BM / WM), cbase = wn * (BN / WN);
  // 1-D grid, N tile fastest: the ntn workgroups that share an A row-tile are adjacent in
  // dispatch order, so A is read from HBM once and from L2 by the others.  (XCD swizzle measured
  // slower here: the persistent m-loop already keeps each row tile's ntn workgroups adjacent in time)
  const int nt = bid % ntn;
  const int64_t mg = bid / ntn, mstep = nblk / ntn;
  const int n0 = nt * BN;
  const int nvalid = min(BN, N - n0);
  const int nk = (K + GBK - 1) / GBK;
  if constexpr (STATS == 1) {
    for (int i = tid; i < BN; i += 256) { st_sum[i] = 0.f; st_sq[i] = 0.f; }
  }

  // staging: this thread owns rows srow + RPP i and k-vector skc of each k-step
  const int srow = tid / G::VPR, skc = (tid % G::VPR) * 8;
  Raw8<T> ra[D][PA], rb[D][PB];
  ConvRow crow[GA ? PA : 1];  // GA: this thread's A rows of the current tile, decomposed once per tile
  float pg[GATE ? D : 1][GATE ? PA : 1][8];
  // producer BN scale/shift of all K columns, staged once per workgroup (dynamic LDS, 2K floats)
  if constexpr (pro_is_bn(MODE)) {
    for (int i = tid; i < K; i += 256) {
      pro_lds[i] = pro.scale[i];
      pro_lds[K + i] = pro.shift[i];
    }
    lds_barrier();
  }
  // issue the global loads of k-step k of the tile at row m0 into ring stage d
  auto load = [&](auto dc, int64_t m0, int k) {
    constexpr int d = decltype(dc)::value;
    const int gk = k * GBK + skc;
    const bool kok = gk < K;
    if constexpr (GA) {
      const ConvTap tp = cg.tap(k * GBK);  // one tap per k-step (C % BK == 0)
      const int ci = gk - tp.k0;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        int64_t off;
        const bool ok = cg.src(crow[i], tp, ci, off) && kok;
        raw_ld(ra[d][i], A + off, A, ok);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int64_t gm = m0 + srow + G::RPP * i;
        raw_ld(ra[d][i], A + gm * K + gk, A, gm < M && kok);
      }
    }
#pragma unroll
    for (int i = 0; i < PB; ++i)
      raw_ld(rb[d][i], B + (int64_t)(n0 + srow + G::RPP * i) * K + gk, B, srow + G::RPP * i < nvalid && kok);
    if constexpr (GATE) {
      const int kc = kok ? gk : 0;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int64_t gm = m0 + srow + G::RPP * i;
        const uint32_t f = (uint32_t)(gm < M ? gm : m0) / (uint32_t)pro.rows_per_frame;
        ld8f(pro.gate + (int64_t)f * pro.C + kc, pg[d][i]);
      }
    }
  };
  auto issue_first = [&](int64_t m0) {
    if constexpr (GA) {
#pragma unroll
      for (int i = 0; i < PA; ++i) crow[i] = cg.row(m0 + srow + G::RPP * i, M);
    }
    static_for<D>([&](auto dc) {
      if (decltype(dc)::value < nk) load(dc, m0, decltype(dc)::value);
    });
  };

  // The first D k-steps of the NEXT tile are issued before this tile's epilogue stores: vmcnt
  // counts loads and stores together, so loads issued after the stores would wait for them.
  if (mg < tiles_m) issue_first(mg * BM);
  for (int64_t mt = mg; mt < tiles_m; mt += mstep) {
    const int64_t m0 = mt * BM;
    f32x4_t acc[RB][CB];
#pragma unroll
    for (int a = 0; a < RB; ++a)
#pragma unroll
      for (int b = 0; b < CB; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int kc = 0; kc < nk; kc += D) {
      static_for<D>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        const int k = kc + d;
        if (k >= nk) return;
        const int k0 = k * GBK;
        // ---- registers -> LDS (A through the consumer-side BN/SiLU/gate prologue) ----
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          const int row = srow + G::RPP * i;
          if constexpr (MODE == PRO_NONE) {
            raw_st(As + G::lds_off(row, skc), ra[d][i]);
          } else if constexpr (MODE == PRO_GELU) {
            float x[8];
            raw_to_f(ra[d][i], x);
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = geluf_(x[j]);  // masked lanes hold 0 and gelu(0) = 0
            lds_st8(As + G::lds_off(row, skc), x);
          } else if constexpr (MODE == PRO_GATE) {
            float x[8];
            raw_to_f(ra[d][i], x);  // masked lanes hold 0
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] *= pg[d][i][j];
            lds_st8(As + G::lds_off(row, skc), x);
          } else {
            float x[8], psc[8], psh[8];
            raw_to_f(ra[d][i], x);
            const int kcol = k0 + skc < K ? k0 + skc : 0;
            ld8(pro_lds + kcol, psc);
            ld8(pro_lds + K + kcol, psh);
            if constexpr (GATE) {
#pragma unroll
              for (int j = 0; j < 8; ++j) x[j] = siluf_(x[j] * psc[j] + psh[j]) * pg[d][i][j];
            } else {
#pragma unroll
              for (int j = 0; j < 8; ++j) x[j] = siluf_(x[j] * psc[j] + psh[j]);
            }
            const bool ok = m0 + row < M && k0 + skc < K;
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = ok ? x[j] : 0.f;
            lds_st8(As + G::lds_off(row, skc), x);
          }
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) raw_st(Bs + G::lds_off(srow + G::RPP * i, skc), rb[d][i]);
        lds_barrier();
        if (k + D < nk) load(dc, m0, k + D);
        // ---- MFMA (partial N tiles are zero padded: the sequence is unconditional) ----
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int ks = 0; ks < BK / 32; ++ks) {
            bf16x8_t af[RB];
#pragma unroll
            for (int r_ = 0; r_ < RB; ++r_)
              af[r_] = *reinterpret_cast<const bf16x8_t*>(
                  As + G::lds_off(rbase + r_ * 16 + (lane & 15), ks * 32 + 8 * (lane >> 4)));
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
              const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(
                  Bs + G::lds_off(cbase + cb * 16 + (lane & 15), ks * 32 + 8 * (lane >> 4)));
#pragma unroll
              for (int r_ = 0; r_ < RB; ++r_)
                acc[r_][cb] = mfma16x16x32<T>(af[r_], bfr, acc[r_][cb]);
            }
          }
        } else {
          f32x4_t fold[FOLD ? RB : 1][FOLD ? CB : 1];
          if constexpr (FOLD) {
#pragma unroll
            for (int a = 0; a < RB; ++a)
#pragma unroll
              for (int b = 0; b < CB; ++b) fold[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int s4 = 0; s4 < GBK / 4; ++s4) {
            const int kk = 4 * s4 + (lane >> 4);
            float av[RB];
#pragma unroll
            for (int r_ = 0; r_ < RB; ++r_)
              av[r_] = reinterpret_cast<const float*>(As)[(rbase + r_ * 16 + (lane & 15)) * G::AS + kk];
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
              const float bv = reinterpret_cast<const float*>(Bs)[(cbase + cb * 16 + (lane & 15)) * G::AS + kk];
#pragma unroll
              for (int r_ = 0; r_ < RB; ++r_) {
                if constexpr (FOLD) fold[r_][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r_], bv, fold[r_][cb], 0, 0, 0);
                else acc[r_][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r_], bv, acc[r_][cb], 0, 0, 0);
              }
            }
          }
          if constexpr (FOLD) {
#pragma unroll
            for (int a = 0; a < RB; ++a)
#pragma unroll
              for (int b = 0; b < CB; ++b) acc[a][b] += fold[a][b];
          }
        }
        lds_barrier();
      });
    }
    if (mt + mstep < tiles_m) issue_first((mt + mstep) * BM);

    // ---- epilogue: round, BN-stat partials, stage C tile in LDS ----
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const int col = cbase + cb * 16 + (lane & 15);
      if (cbase + cb * 16 < nvalid) {
        float bcol = 0.f;
        if constexpr (BIAS) bcol = col < nvalid ? bias[n0 + col] : 0.f;
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int r_ = 0; r_ < RB; ++r_) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rbase + r_ * 16 + 4 * (lane >> 4) + r;
            const float v = Tr<T>::round(acc[r_][cb][r] + bcol);
            Cs[row * G::CS + col] = Tr<T>::from_f(v);
            if constexpr (STATS != 0) {
              if (m0 + row < M) { s += v; q += v * v; }
            }
          }
        }
        if constexpr (STATS == 1) {
          s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
          q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
          if (lane < 16) {
            st_part[(wm * 2 + 0) * BN + col] = s;
            st_part[(wm * 2 + 1) * BN + col] = q;
          }
        }
        if constexpr (STATS == 2) {  // this wave's rows: sum, then squared deviations from their mean
          s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
          const int64_t left = M - (m0 + rbase);
          const int nrow = left < BM / WM ? (int)left : BM / WM;
          const float mean = nrow > 0 ? s / (float)nrow : 0.f;
          float m2 = 0.f;
#pragma unroll
          for (int r_ = 0; r_ < RB; ++r_)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = rbase + r_ * 16 + 4 * (lane >> 4) + r;
              const float dv = Tr<T>::round(acc[r_][cb][r] + bcol) - mean;
              if (m0 + row < M) m2 += dv * dv;
            }
          m2 += __shfl_xor(m2, 16, 64);
          m2 += __shfl_xor(m2, 32, 64);
          if (lane < 16 && nrow > 0 && col < nvalid) {
            const int64_t srow = (m0 / BM) * WM + wm;
            stats[(srow * 2 + 0) * N + n0 + col] = s;
            stats[(srow * 2 + 1) * N + n0 + col] = m2;
          }
        }
      }
    }
    lds_barrier();
    if constexpr (STATS == 1) {
      // wave rows in order: bit-reproducible BN statistics
      for (int i = tid; i < nvalid; i += 256) {
        float a = st_part[0 * BN + i], b = st_part[1 * BN + i];
#pragma unroll
        for (int w = 1; w < WM; ++w) { a += st_part[(w * 2 + 0) * BN + i]; b += st_part[(w * 2 + 1) * BN + i]; }
        st_sum[i] += a;
        st_sq[i] += b;
      }
    }
    const int vpr = nvalid >> 3;
    for (int v = tid; v < BM * vpr; v += 256) {
      const int row = v / vpr, cv = (v - row * vpr) * 8;
      const int64_t gm = m0 + row;
      if (gm >= M) continue;
      float x[8];
      lds_ld8(Cs + row * G::CS + cv, x);
      if constexpr (RESID) {
        float r8[8];
        ld8(R + gm * N + n0 + cv, r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] += r8[j];
      }
      if constexpr (DGELU) {
        float z8[8];
        ld8(Z + gm * N + n0 + cv, z8);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] *= dgeluf_(z8[j]);
      }
      st8(C + gm * N + n0 + cv, x);
    }
    lds_barrier();
  }
  if constexpr (STATS == 1) {
    for (int i = tid; i < nvalid; i += 256) {
      stats[(mg * 2 + 0) * N + n0 + i] = st_sum[i];
      stats[(mg * 2 + 1) * N + n0 + i] = st_sq[i];
    }
  }
}

// wgrad: dW[N][K] = sum_m dY[m][n] * pro(X)[m][k].  Output tile 64x64 per workgroup; each of the
// 4 waves streams its own 32-row m-steps through a private LDS region (no block barrier in the
// loop) and the MFMA operands are COLUMN reads of the row-major tiles: ds_read_b64_tr_b16 in
// bf16 mode (two per 8-deep fragment), ds_read_b32 in fp32 mode.  The global loads of m-step
// i+1 are issued (branch-free, masked) before the MFMAs of step i; partial tiles are zero
// padded so the MFMA sequence is unconditional.
constexpr int WT = 64;
constexpr int WMS = 32;

template <typename T> struct WgCfg {
  static constexpr int LS = sizeof(T) == 2 ? WT + 8 : WT + 4;
  static constexpr int WAVE_BYTES = 2 * WMS * LS * (int)sizeof(T);
  static constexpr int SMEM = 4 * WAVE_BYTES > WT * WT * 4 ? 4 * WAVE_BYTES : WT * WT * 4;
};

// PF: m-steps of global loads in flight per wave (a register ring; the loop is unrolled by PF so
// every set is a static register array).  PF = 1 issues step i+1's loads before step i's MFMAs;
// the late-stage shapes (M = 12,544 / 50,176 rows, ~11 steps per workgroup) were ~1.5 us of load
// latency per step with one step in flight, so PF = 2 keeps two.
// One workgroup of the weight gradient: lin / nb its linear index and the workgroup count of its grid
// (tiles x splits), tiles the tile count, smem the caller's LDS (WgCfg<T>::SMEM bytes).  GX = 1: X is
// the implicit-GEMM gather of a convolution input (ConvGather; one tap per 64-wide K tile).
template <typename T, int MODE, int PF, int GX = 0, bool FOLD = false>
__device__ __forceinline__ void pw_wgrad_body(const T* __restrict__ dY, const T* __restrict__ X, int64_t M, int N,
                                              int K, const Pro& pro, float* __restrict__ slab, int tnk,
                                              int64_t m_per_split, int lin, int nb, int tiles, char* smem,
                                              const ConvGather& cg = ConvGather{}) {
  using G = WgCfg<T>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1-D dispatch order over (tile, split), tiles fastest: the tiles of one M-split share an XCD
  const int bid = DFD_XCD_SWZ ? xcd_swizzle(lin, nb) : lin;
  const int split = bid / tiles, tile = bid - split * tiles;
  const int tn = tile / tnk, tk = tile - tn * tnk;
  const int n0 = tn * WT, k0 = tk * WT;
  const int nv = min(WT, N - n0), kv = min(WT, K - k0);
  const int64_t mbeg = (int64_t)split * m_per_split;
  const int64_t mend = min(M, mbeg + m_per_split);
  T* Ys = reinterpret_cast<T*>(smem + wave * G::WAVE_BYTES);
  T* Xs = Ys + WMS * G::LS;

  // this lane stages column vector cv of rows rl + 8 i (i < 4) of every m-step
  const int cv = (lane & 7) * 8, rl = lane >> 3;
  const bool yc = cv < nv, xc = cv < kv;
  const int kc = k0 + (xc ? cv : 0);
  float sc[8], sh[8];
  if constexpr (pro_is_bn(MODE)) {
    ld8f(pro.scale + kc, sc);
    ld8f(pro.shift + kc, sh);
  }
  Raw8<T> ry[PF][4], rx[PF][4];
  float rg[PF][pro_is_gated(MODE) ? 4 : 1][8];
  const ConvTap xtap = GX ? cg.tap(k0) : ConvTap{};  // GX: the tap of this K tile (C % 64 == 0)
  auto load = [&](auto pc, int64_t ms) {
    constexpr int P = decltype(pc)::value;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t gm = ms + rl + 8 * i;
      const bool ok = gm < mend;
      raw_ld(ry[P][i], dY + gm * N + n0 + cv, dY, ok && yc);
      if constexpr (GX) {
        int64_t off;
        const bool sok = cg.src(cg.row(gm, mend), xtap, xc ? cv + (k0 - xtap.k0) : 0, off);
        raw_ld(rx[P][i], X + off, X, ok && xc && sok);
      } else {
        raw_ld(rx[P][i], X + gm * K + k0 + cv, X, ok && xc);
      }
      if constexpr (pro_is_gated(MODE)) {
        const uint32_t f = (uint32_t)(ok ? gm : mbeg) / (uint32_t)pro.rows_per_frame;
        ld8f(pro.gate + (int64_t)f * pro.C + kc, rg[P][i]);
      }
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // one m-step: stage ring slot P (rows from ms) into this wave's LDS region, refill the slot with the
  // step PF ahead, then the MFMAs of the staged step
  auto step = [&](auto pc, int64_t ms) {
    constexpr int P = decltype(pc)::value;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rl + 8 * i;
      raw_st(Ys + row * G::LS + cv, ry[P][i]);
      if constexpr (MODE == PRO_NONE) {
        raw_st(Xs + row * G::LS + cv, rx[P][i]);
      } else {
        float x[8];
        raw_to_f(rx[P][i], x);
        if constexpr (MODE == PRO_BN_SILU_G) {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = siluf_(x[j] * sc[j] + sh[j]) * rg[P][i][j];
        } else if constexpr (MODE == PRO_GATE) {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] *= rg[P][i][j];
        } else if constexpr (MODE == PRO_GELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = geluf_(x[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = siluf_(x[j] * sc[j] + sh[j]);
        }
        const bool ok = ms + row < mend && xc;
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = ok ? x[j] : 0.f;
        lds_st8(Xs + row * G::LS + cv, x);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (ms + PF * 4 * WMS < mend) load(pc, ms + PF * 4 * WMS);
    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
      bf16x8_t bfr[4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const s16x4_t lo =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Xs + (8 * g + q) * G::LS + kb * 16 + 4 * p));
        const s16x4_t hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Xs + (8 * g + 4 + q) * G::LS + kb * 16 + 4 * p));
        bfr[kb] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int nb_ = 0; nb_ < 4; ++nb_) {
        const s16x4_t lo =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Ys + (8 * g + q) * G::LS + nb_ * 16 + 4 * p));
        const s16x4_t hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Ys + (8 * g + 4 + q) * G::LS + nb_ * 16 + 4 * p));
        const bf16x8_t af = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) acc[nb_][kb] = mfma16x16x32<T>(af, bfr[kb], acc[nb_][kb]);
      }
    } else {
      const float* Yf = reinterpret_cast<const float*>(Ys);
      const float* Xf = reinterpret_cast<const float*>(Xs);
      // FOLD: each m-step's products into a fresh tile added to the running sum (two-level M sum)
      f32x4_t fold[FOLD ? 4 : 1][FOLD ? 4 : 1];
      if constexpr (FOLD) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) fold[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s = 0; s < WMS / 4; ++s) {
        const int mm = 4 * s + (lane >> 4);
        float bv[4];
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) bv[kb] = Xf[mm * G::LS + kb * 16 + (lane & 15)];
#pragma unroll
        for (int nb_ = 0; nb_ < 4; ++nb_) {
          const float av = Yf[mm * G::LS + nb_ * 16 + (lane & 15)];
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) {
            if constexpr (FOLD) fold[nb_][kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[kb], fold[nb_][kb], 0, 0, 0);
            else acc[nb_][kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[kb], acc[nb_][kb], 0, 0, 0);
          }
        }
      }
      if constexpr (FOLD) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] += fold[a][b];
      }
    }
    __builtin_amdgcn_wave_barrier();
  };

  int64_t ms = mbeg + wave * WMS;
  static_for<PF>([&](auto pc) {
    constexpr int P = decltype(pc)::value;
    if (ms + P * 4 * WMS < mend) load(pc, ms + P * 4 * WMS);
  });
  for (; ms < mend; ms += PF * 4 * WMS) {
    static_for<PF>([&](auto pc) {
      constexpr int P = decltype(pc)::value;
      if (ms + P * 4 * WMS < mend) step(pc, ms + P * 4 * WMS);
    });
  }
  // ---- cross-wave reduction of the 64x64 tile, waves added in a fixed order (deterministic) ----
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
    lds_barrier();
    if (wave == w) {
#pragma unroll
      for (int nb_ = 0; nb_ < 4; ++nb_)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int idx = (nb_ * 16 + 4 * (lane >> 4) + r) * WT + kb * 16 + (lane & 15);
            red[idx] = (w == 0 ? 0.f : red[idx]) + acc[nb_][kb][r];
          }
    }
  }
  lds_barrier();
  float* out = slab + (int64_t)split * N * K;
  for (int i = tid; i < WT * WT; i += 256) {
    const int nn = i / WT, kk = i - nn * WT;
    if (nn < nv && kk < kv) out[(int64_t)(n0 + nn) * K + k0 + kk] = red[i];
  }
}

}  // namespace dfd
