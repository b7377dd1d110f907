// Pointwise (1x1) convolutions of EfficientNet-B0 as MFMA GEMMs on gfx950.
//
// Replaces aten conv2d(kernel 1x1) for timm's conv_pw / conv_pwl / conv_head
// (reached from src/pretrained_detector.py:116) in all three passes:
//   forward  Y[M][N]  = pro(X)[M][K] . W[N][K]^T   + per-column BN-stat partials (epilogue)
//   dgrad    dX[M][K] = dY[M][N] . (W^T)[K][N]^T   (+ residual gradient in the epilogue)
//   wgrad    dW[N][K] = dY^T . pro(X)              (split over M, deterministic slab reduce)
// where pro() is the consumer-side BatchNorm+SiLU (+SE channel gate) of the producing
// layer, applied while staging A into LDS, so those activations are never materialised.
//
// Layout: NHWC rows, K/N contiguous.  MFMA: v_mfma_f32_16x16x32_bf16 (bf16 mode) or
// v_mfma_f32_16x16x32_f16 (fp16 mode) or v_mfma_f32_16x16x4_f32 (exact fp32 parity mode); C/D layout col=lane&15,
// row=4*(lane>>4)+r for both.
#include "kernels.h"

#include <atomic>

#ifndef DFD_XCD_SWZ
#define DFD_XCD_SWZ 1  // XCD-aware block order of the weight-gradient kernel (A/B knob; -5..-20 us
                       // per 50176/12544-row layer: the 22-126 tiles of one M-split share an L2)
#endif

namespace dfd {

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

template <typename T, int MODE, bool STATS, int EPI, int BM, int BN, int WN, int D, int BK, int OCC>
__global__ __launch_bounds__(256, OCC) void pw_gemm_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                        T* __restrict__ C, const T* __restrict__ R,
                                                        const float* __restrict__ bias, const T* __restrict__ Z,
                                                        int64_t M, int N, int K, Pro pro, float* __restrict__ stats,
                                                        int64_t tiles_m, int ntn) {
  constexpr bool RESID = (EPI & EPI_RESID) != 0, BIAS = (EPI & EPI_BIAS) != 0, DGELU = (EPI & EPI_DGELU) != 0;
  using G = GemmCfg<T, BM, BN, WN, D, BK>;
  constexpr int GBK = BK;
  constexpr int WM = G::WM, RB = G::RB, CB = G::CB, PA = G::PA, PB = G::PB;
  constexpr bool GATE = pro_is_gated(MODE);
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  __shared__ float st_sum[BN];
  __shared__ float st_sq[BN];
  __shared__ float st_part[STATS ? WM : 1][2][BN];  // per-wave-row column partials (fixed-order sum)
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + BM * G::AS;
  T* Cs = reinterpret_cast<T*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int rbase = wm * (BM / WM), cbase = wn * (BN / WN);
  // 1-D grid, N tile fastest: the ntn workgroups that share an A row-tile are adjacent in
  // dispatch order, so A is read from HBM once and from L2 by the others.
  const int bid = blockIdx.x;  // (XCD swizzle measured slower here: the persistent m-loop already
                               // keeps each row tile's ntn workgroups adjacent in time)
  const int nt = bid % ntn;
  const int64_t mg = bid / ntn, mstep = gridDim.x / ntn;
  const int n0 = nt * BN;
  const int nvalid = min(BN, N - n0);
  const int nk = (K + GBK - 1) / GBK;
  if constexpr (STATS) {
    for (int i = tid; i < BN; i += 256) { st_sum[i] = 0.f; st_sq[i] = 0.f; }
  }

  // staging: this thread owns rows srow + RPP i and k-vector skc of each k-step
  const int srow = tid / G::VPR, skc = (tid % G::VPR) * 8;
  Raw8<T> ra[D][PA], rb[D][PB];
  float pg[GATE ? D : 1][GATE ? PA : 1][8];
  // producer BN scale/shift of all K columns, staged once per workgroup (dynamic LDS, 2K floats)
  extern __shared__ float pro_lds[];
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
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int64_t gm = m0 + srow + G::RPP * i;
      raw_ld(ra[d][i], A + gm * K + gk, A, gm < M && kok);
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
              for (int r_ = 0; r_ < RB; ++r_)
                acc[r_][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r_], bv, acc[r_][cb], 0, 0, 0);
            }
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
            if constexpr (STATS) {
              if (m0 + row < M) { s += v; q += v * v; }
            }
          }
        }
        if constexpr (STATS) {
          s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
          q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
          if (lane < 16) {
            st_part[wm][0][col] = s;
            st_part[wm][1][col] = q;
          }
        }
      }
    }
    lds_barrier();
    if constexpr (STATS) {
      // wave rows in order: bit-reproducible BN statistics
      for (int i = tid; i < nvalid; i += 256) {
        float a = st_part[0][0][i], b = st_part[0][1][i];
#pragma unroll
        for (int w = 1; w < WM; ++w) { a += st_part[w][0][i]; b += st_part[w][1][i]; }
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
  if constexpr (STATS) {
    for (int i = tid; i < nvalid; i += 256) {
      stats[(mg * 2 + 0) * N + n0 + i] = st_sum[i];
      stats[(mg * 2 + 1) * N + n0 + i] = st_sq[i];
    }
  }
}

// tile configurations (BM, BN, WN, D, OCC); the gemm_tile knob forces one for experiments (-1 = auto)

template <typename T, int MODE, bool ST, int EP, int BM, int BN, int WN, int D, int BK, int OCC>
static void gemm_go(hipStream_t s, int gx_m, int ntn, size_t dyn, const T* A, const T* B, T* C, const T* R,
                    const float* bias, const T* Z, int64_t M, int N, int K, const Pro& pro, float* stats,
                    int64_t tiles_m) {
  hipLaunchKernelGGL((pw_gemm_kernel<T, MODE, ST, EP, BM, BN, WN, D, BK, OCC>), dim3((unsigned)(gx_m * ntn)),
                     dim3(256), dyn, s, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m, ntn);
}

template <typename T, int MODE, bool ST, int EP>
static int gemm_tiles(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias, const T* Z,
                      int64_t M, int N, int K, const Pro& pro, float* stats, int* stat_rows, size_t dyn) {
  // 0: 128x128 (4x1 waves), 1: 128x64 (4x1), 2: 64x64 (2x2), 3: 32x64 (2x2, 64-deep k-steps).
  // Chosen per shape from tools/kbench on MI355X (tools/gemm_tiles.sh): one 128-wide N tile while
  // N <= 128 (the A prologue then runs once per row tile); 128x64 for narrow N; the 14x14 / 7x7
  // stages (few row tiles) want the small tiles for enough workgroups in flight.
  int cfg = (int)tune(TK_GEMM_TILE);
  if (cfg < 0 || cfg > 12) {
    if (N <= 64) cfg = 1;
    else if (N <= 128) cfg = 0;
    else if (M <= 16384) cfg = N <= 256 ? 3 : 1;
    else if (M <= 65536) cfg = 2;
    else cfg = N <= 160 ? 1 : 2;
  }
  static constexpr int kBM[13] = {128, 128, 64, 32, 128, 64, 64, 128, 64, 64, 64, 32, 128};
  static constexpr int kBN[13] = {128, 64, 64, 64, 64, 64, 64, 128, 192, 128, 320, 192, 192};
  const int bm = kBM[cfg], bn = kBN[cfg];
  const int ntn = cdiv(N, bn);
  const int64_t tiles_m = cdiv64(M, bm);
  const int64_t cap = std::max<int64_t>(1, 1024 / ntn);  // <= 1024 BN-stat partial rows (plan's stats buffer)
  const int gx = (int)std::min<int64_t>(tiles_m, cap);
  constexpr int DW = sizeof(T) == 4 ? 1 : 0;  // fp32 (parity mode): shallower ring, no spills
  constexpr int O64 = (pro_is_gated(MODE) || sizeof(T) == 4) ? 2 : 4;
  if (cfg == 0) gemm_go<T, MODE, ST, EP, 128, 128, 1, 2 - DW, 32, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 1) gemm_go<T, MODE, ST, EP, 128, 64, 1, 3 - DW, 32, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 2) gemm_go<T, MODE, ST, EP, 64, 64, 2, 3, 32, O64>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 3) gemm_go<T, MODE, ST, EP, 32, 64, 2, 2, 64, O64>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  // deeper k-steps (fewer LDS hand-offs per tile) for the long-K late-stage shapes
  else if (cfg == 4) gemm_go<T, MODE, ST, EP, 128, 64, 1, 2 - DW, 64, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 5) gemm_go<T, MODE, ST, EP, 64, 64, 2, 2, 64, O64>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 6) gemm_go<T, MODE, ST, EP, 64, 64, 2, 1, 128, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 7) gemm_go<T, MODE, ST, EP, 128, 128, 1, 1, 64, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  // wide-N tiles (4 waves side by side along N): one tile spans the whole N of the narrow
  // projection / dgrad shapes (N 112..320), so each A row tile is read and put through the
  // producer prologue exactly once
  else if (cfg == 8) gemm_go<T, MODE, ST, EP, 64, 192, 4, 2, 64, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 9) gemm_go<T, MODE, ST, EP, 64, 128, 4, 2, 64, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 10) gemm_go<T, MODE, ST, EP, 64, 320, 4, 2, 32, 1>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else if (cfg == 11) gemm_go<T, MODE, ST, EP, 32, 192, 4, 2, 64, 2>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  else gemm_go<T, MODE, ST, EP, 128, 192, 4, 2, 32, 1>(s, gx, ntn, dyn, A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m);
  if (stat_rows) *stat_rows = gx;
  return 0;
}

template <typename T>
static int gemm_dispatch(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias, const T* Z,
                         int64_t M, int N, int K, int pro_mode, int epi, const Pro& pro, float* stats, int* stat_rows) {
  if (M <= 0) return 0;
  if ((N & 7) || (K & 7)) { set_error("pw_gemm: N and K must be multiples of 8", __FILE__, __LINE__); return -1; }
  if (M > (int64_t)UINT32_MAX) { set_error("pw_gemm: M exceeds 2^32 rows", __FILE__, __LINE__); return -1; }
  if (((epi & EPI_RESID) && !R) || ((epi & EPI_BIAS) && !bias) || ((epi & EPI_DGELU) && !Z)) {
    set_error("pw_gemm: epilogue operand missing", __FILE__, __LINE__);
    return -1;
  }
  const bool st = stats != nullptr;
  const size_t dyn = pro_is_bn(pro_mode) ? 2 * (size_t)K * sizeof(float) : 0;
#define DFD_GEMM_LAUNCH(MODE, ST, EP) \
  gemm_tiles<T, MODE, ST, EP>(s, A, B, C, R, bias, Z, M, N, K, pro, stats, stat_rows, dyn)
  // instantiated combinations: the B0 trunk's (BN prologues, BN-stat epilogue, residual) and the
  // ViT's (bias, bias + residual, GELU prologue + bias + residual, GELU-derivative epilogue)
  if (pro_mode == PRO_NONE && epi == EPI_RESID && !st) DFD_GEMM_LAUNCH(PRO_NONE, false, EPI_RESID);
  else if (pro_mode == PRO_NONE && epi == 0) {
    if (st) DFD_GEMM_LAUNCH(PRO_NONE, true, 0); else DFD_GEMM_LAUNCH(PRO_NONE, false, 0);
  } else if (pro_mode == PRO_BN_SILU && epi == 0) {
    if (st) DFD_GEMM_LAUNCH(PRO_BN_SILU, true, 0); else DFD_GEMM_LAUNCH(PRO_BN_SILU, false, 0);
  } else if (pro_mode == PRO_BN_SILU_G && epi == 0) {
    if (st) DFD_GEMM_LAUNCH(PRO_BN_SILU_G, true, 0); else DFD_GEMM_LAUNCH(PRO_BN_SILU_G, false, 0);
  } else if (pro_mode == PRO_GATE && epi == 0) {
    if (st) DFD_GEMM_LAUNCH(PRO_GATE, true, 0); else DFD_GEMM_LAUNCH(PRO_GATE, false, 0);
  } else if (pro_mode == PRO_NONE && epi == EPI_BIAS && !st) DFD_GEMM_LAUNCH(PRO_NONE, false, EPI_BIAS);
  else if (pro_mode == PRO_NONE && epi == (EPI_BIAS | EPI_RESID) && !st) DFD_GEMM_LAUNCH(PRO_NONE, false, EPI_BIAS | EPI_RESID);
  else if (pro_mode == PRO_GELU && epi == (EPI_BIAS | EPI_RESID) && !st) DFD_GEMM_LAUNCH(PRO_GELU, false, EPI_BIAS | EPI_RESID);
  else if (pro_mode == PRO_NONE && epi == EPI_DGELU && !st) DFD_GEMM_LAUNCH(PRO_NONE, false, EPI_DGELU);
  else {
    set_error("pw_gemm: unsupported prologue/epilogue combination", __FILE__, __LINE__);
    return -1;
  }
#undef DFD_GEMM_LAUNCH
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

template <typename T>
int launch_pw_gemm(hipStream_t s, const T* A, const T* B, T* C, const T* R, int64_t M, int N, int K, int pro_mode,
                   const Pro& pro, float* stats, int* stat_rows) {
  if (R && (pro_mode != PRO_NONE || stats)) {
    set_error("pw_gemm: residual only with plain input", __FILE__, __LINE__);
    return -1;
  }
  if constexpr (is16<T>) {
    // the small-K weight-panel kernel where it measured faster (tools/pw_sk_bench.py, round 4): the
    // forward products with BN statistics (K 80 / 112 / 192: -22 / -14 / -7 %) and the sub-streaming
    // row counts; the streaming kernel keeps the large stat-free data gradients (+31 / +22 % on sk)
    // and K = 320 (+15..+24 %)
    if (pro_mode == PRO_NONE && tune(TK_PW_SK) != 0 && K <= 192 && (stats || M < tune(TK_STREAM_MIN_ROWS))) {
      const int rc = launch_pw_sk(s, A, B, C, R, M, N, K, stats, 1024, stat_rows);
      if (rc <= 0) return rc;
    }
    const int rc = launch_pw_stream(s, A, B, C, R, nullptr, M, N, K, pro_mode, pro, stats, stat_rows);
    if (rc <= 0) return rc;
  }
  return gemm_dispatch<T>(s, A, B, C, R, nullptr, nullptr, M, N, K, pro_mode, R ? EPI_RESID : 0, pro, stats,
                          stat_rows);
}

template <typename T>
int launch_tf_gemm(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias, const T* Z, int64_t M,
                   int N, int K, int pro_mode, int epi) {
  Pro none{};
  if constexpr (is16<T>) {
    if (pro_mode == PRO_NONE && (epi & EPI_BIAS) && !(epi & EPI_DGELU) && bias && (R || !(epi & EPI_RESID))) {
      const int rc = launch_pw_stream(s, A, B, C, (epi & EPI_RESID) ? R : nullptr, bias, M, N, K, PRO_NONE, none,
                                      nullptr, nullptr);
      if (rc <= 0) return rc;
    }
  }
  return gemm_dispatch<T>(s, A, B, C, R, bias, Z, M, N, K, pro_mode, epi, none, nullptr, nullptr);
}

// ------------------------------------------------------------------------------------------
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
template <typename T, int MODE, int PF = 1>
__global__ __launch_bounds__(256, (sizeof(T) == 2 && !pro_is_gated(MODE) && PF == 1) ? 3 : 2) void pw_wgrad_kernel(const T* __restrict__ dY, const T* __restrict__ X, int64_t M,
                                                       int N, int K, Pro pro, float* __restrict__ slab, int tnk,
                                                       int64_t m_per_split) {
  using G = WgCfg<T>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1-D dispatch order over (tile, split), tiles fastest: the tiles of one M-split share an XCD
  const int nb = gridDim.x * gridDim.y, lin = blockIdx.y * gridDim.x + blockIdx.x;
  const int bid = DFD_XCD_SWZ ? xcd_swizzle(lin, nb) : lin;
  const int split = bid / gridDim.x, tile = bid - split * gridDim.x;
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
  auto load = [&](auto pc, int64_t ms) {
    constexpr int P = decltype(pc)::value;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t gm = ms + rl + 8 * i;
      const bool ok = gm < mend;
      raw_ld(ry[P][i], dY + gm * N + n0 + cv, dY, ok && yc);
      raw_ld(rx[P][i], X + gm * K + k0 + cv, X, ok && xc);
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
          for (int kb = 0; kb < 4; ++kb) acc[nb_][kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[kb], acc[nb_][kb], 0, 0, 0);
        }
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

template <typename T>
int launch_pw_wgrad(hipStream_t s, const T* dY, const T* X, int64_t M, int N, int K, int pro_mode, const Pro& pro,
                    float* slab, int64_t slab_cap, float* dW, bool accumulate) {
  if ((N & 7) || (K & 7)) { set_error("pw_wgrad: N and K must be multiples of 8", __FILE__, __LINE__); return -1; }
  if (M > (int64_t)UINT32_MAX) { set_error("pw_wgrad: M exceeds 2^32 rows", __FILE__, __LINE__); return -1; }
  if constexpr (is16<T>) {
    const int rc = launch_pw_wgrad_stream(s, dY, X, M, N, K, pro_mode, pro, slab, slab_cap, dW, accumulate);
    if (rc <= 0) return rc;
  }
  const int tnn = cdiv(N, WT), tnk = cdiv(K, WT);
  const int tiles = tnn * tnk;
#ifndef DFD_WGRAD_SPLIT_WGS
#define DFD_WGRAD_SPLIT_WGS 512  // target workgroups of the M-split (A/B knob; 512 measured best over
                                 // 256/384/1024/2048 on the B0 shapes: less slab traffic)
#endif
  int64_t splits = std::max<int64_t>(1, DFD_WGRAD_SPLIT_WGS / tiles);
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, cdiv64(M, 4 * WMS)));
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, slab_cap / ((int64_t)N * K)));
  int64_t mps = cdiv64(cdiv64(std::max<int64_t>(M, 1), splits), 4 * WMS) * (4 * WMS);
  splits = cdiv64(std::max<int64_t>(M, 1), mps);
  dim3 grid(tiles, (unsigned)splits), block(256);
  // two m-steps of loads in flight for bf16 (knob wg_pf: 1 or 2; DFD_WG_PF the build default)
  // (the gated prologues keep one: their per-step gate rows double the ring and spill)
  const int pf = sizeof(T) == 2 && tune(TK_WG_PF) >= 2 && !pro_is_gated(pro_mode) ? 2 : 1;
#define DFD_WG_GO(MD)                                                                                           \
  do {                                                                                                          \
    if (pf == 2) hipLaunchKernelGGL((pw_wgrad_kernel<T, MD, 2>), grid, block, 0, s, dY, X, M, N, K, pro, slab, tnk, mps); \
    else hipLaunchKernelGGL((pw_wgrad_kernel<T, MD, 1>), grid, block, 0, s, dY, X, M, N, K, pro, slab, tnk, mps);       \
  } while (0)
  if (pro_mode == PRO_NONE) DFD_WG_GO(PRO_NONE);
  else if (pro_mode == PRO_BN_SILU) DFD_WG_GO(PRO_BN_SILU);
  else if (pro_mode == PRO_GELU) DFD_WG_GO(PRO_GELU);
  else if (pro_mode == PRO_GATE) DFD_WG_GO(PRO_GATE);
  else DFD_WG_GO(PRO_BN_SILU_G);
#undef DFD_WG_GO
  DFD_HIP_CHECK(hipGetLastError());
  return launch_reduce_slabs(s, slab, (int)splits, (int64_t)N * K, dW, accumulate);
}

template int launch_pw_gemm<float>(hipStream_t, const float*, const float*, float*, const float*, int64_t, int, int,
                                   int, const Pro&, float*, int*);
template int launch_pw_gemm<bf16>(hipStream_t, const bf16*, const bf16*, bf16*, const bf16*, int64_t, int, int, int,
                                  const Pro&, float*, int*);
template int launch_tf_gemm<float>(hipStream_t, const float*, const float*, float*, const float*, const float*,
                                   const float*, int64_t, int, int, int, int);
template int launch_tf_gemm<bf16>(hipStream_t, const bf16*, const bf16*, bf16*, const bf16*, const float*, const bf16*,
                                  int64_t, int, int, int, int);
template int launch_pw_wgrad<float>(hipStream_t, const float*, const float*, int64_t, int, int, int, const Pro&,
                                    float*, int64_t, float*, bool);
template int launch_pw_wgrad<bf16>(hipStream_t, const bf16*, const bf16*, int64_t, int, int, int, const Pro&, float*,
                                   int64_t, float*, bool);
// fp16 mode (v_mfma_f32_16x16x32_f16): the same 16-bit kernels (tiled, streaming, weight panel)
template int launch_pw_gemm<f16>(hipStream_t, const f16*, const f16*, f16*, const f16*, int64_t, int, int, int,
                                 const Pro&, float*, int*);
template int launch_tf_gemm<f16>(hipStream_t, const f16*, const f16*, f16*, const f16*, const float*, const f16*,
                                 int64_t, int, int, int, int);
template int launch_pw_wgrad<f16>(hipStream_t, const f16*, const f16*, int64_t, int, int, int, const Pro&, float*,
                                  int64_t, float*, bool);

}  // namespace dfd
