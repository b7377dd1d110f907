// ResNet-50 convolutions as implicit-GEMM MFMA kernels on gfx950 (inference, eval-mode BN folded).
//
// Replaces torchvision resnet50's conv + bn (+ identity add) + relu (src/pretrained_detector.py:37-40;
// the app's default EnsembleDetector member, app.py:661,1597) -- every convolution of the trunk:
//     C[M][Cout] = relu?( im2col(X)[M][K] . W[Cout][K]^T + bias (+ R) ),   M = N*Ho*Wo,
//     K = KH*KW*Cin, column k = (kh*KW + kw)*Cin + ci  (the packing of resnet._Conv).
// The im2col is never materialised: each thread's staging load of an 8-channel vector computes
// its source pixel (n, oy*s - pad + kh, ox*s - pad + kw) from the output row and the k index
// (Cin a power of two: shifts, KW in {1, 3}: multiply-shift), zero outside the map.  conv1
// (Cin = 3) keeps its explicit [M][152] gather (rn_stem_im2col, one layer) and runs here as a
// plain GEMM (IMPLICIT = false, as do the 1x1 stride-1 convs that read the activation directly).
//
// Tile: BM x BN per workgroup of 4 waves (WM x WN), 16x16 MFMA blocks (v_mfma_f32_16x16x32_bf16 /
// v_mfma_f32_16x16x4_f32 in the fp32 parity mode), BK-deep k-steps staged global -> registers ->
// LDS through a D-deep register ring (XOR-swizzled 16-B chunks for bf16); epilogue: bias,
// residual, ReLU, one rounding to the storage type, C tile restaged in LDS for 16-B stores.
#include "kernels.h"
#include "vit.h"

namespace dfd {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <typename T, int BM, int BN, int WN, int BK>
struct RnCfg {
  static constexpr int WM = 4 / WN;
  static constexpr int RB = BM / WM / 16, CB = BN / WN / 16;
  static constexpr int VPR = BK / 8, RPP = 256 / VPR;
  static constexpr int PA = BM / RPP, PB = BN / RPP;
  static constexpr int AS = sizeof(T) == 2 ? BK : BK + 4;
  static constexpr int CPR = BK / 8;
  __device__ __forceinline__ static int lds_off(int row, int k) {
    if constexpr (sizeof(T) == 2) return row * AS + (((k >> 3) ^ ((row / (16 / CPR)) & (CPR - 1))) << 3);
    else return row * AS + k;
  }
  static constexpr int CS = sizeof(T) == 2 ? BN + 8 : BN + 4;
  static constexpr int AB_BYTES = (BM + BN) * AS * (int)sizeof(T);
  static constexpr int C_BYTES = BM * CS * (int)sizeof(T);
  static constexpr int SMEM = AB_BYTES > C_BYTES ? AB_BYTES : C_BYTES;
  static_assert(WM * WN == 4 && RB >= 1 && CB >= 1 && PA >= 1 && PB >= 1 && BK % 32 == 0, "tile shape");
};

}  // namespace

template <typename T, int BM, int BN, int WN, int BK, int D, bool IMPLICIT, bool RESID>
__global__ __launch_bounds__(256, 2) void rn_conv_kernel(const T* __restrict__ X, const T* __restrict__ Wt,
                                                       T* __restrict__ C, const T* __restrict__ R,
                                                       const float* __restrict__ bias, int relu, RnConvGeom g,
                                                       int64_t M, int N, int K, int ntn) {
  using G = RnCfg<T, BM, BN, WN, BK>;
  constexpr int WM = G::WM, RB = G::RB, CB = G::CB, PA = G::PA, PB = G::PB;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + BM * G::AS;
  T* Cs = reinterpret_cast<T*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int rbase = wm * (BM / WM), cbase = wn * (BN / WN);
  // N tile fastest within an XCD: the ntn workgroups of one row tile share an L2
  const int bid = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
  const int nt = bid % ntn;
  const int64_t m0 = (int64_t)(bid / ntn) * BM;
  const int n0 = nt * BN;
  const int nvalid = min(BN, N - n0);
  const int nk = (K + BK - 1) / BK;
  const int srow = tid / G::VPR, skc = (tid % G::VPR) * 8;

  // this thread's A rows: source pixel origin (n*H, iy0, ix0) of each output row it stages
  int rn[PA], ry[PA], rx[PA];
  bool rok[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int64_t gm = m0 + srow + G::RPP * i;
    rok[i] = gm < M;
    if constexpr (IMPLICIT) {
      const int64_t gmc = rok[i] ? gm : 0;
      const int hw = g.Ho * g.Wo;
      const int n = (int)(gmc / hw), rem = (int)(gmc - (int64_t)n * hw), oy = rem / g.Wo, ox = rem - oy * g.Wo;
      rn[i] = n * g.H;
      ry[i] = oy * g.stride - g.pad;
      rx[i] = ox * g.stride - g.pad;
    }
  }

  Raw8<T> ra[D][PA], rb[D][PB];
  auto load = [&](auto dc, int k) {
    constexpr int d = decltype(dc)::value;
    const int gk = k * BK + skc;
    const bool kok = gk < K;
    if constexpr (IMPLICIT) {
      const int tap = gk >> g.cin_log2, ci = gk & (g.Cin - 1);
      const int kh = g.KW == 1 ? tap : (tap * 11) >> 5;  // tap / 3 for tap < 9
      const int kw = tap - kh * g.KW;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int iy = ry[i] + kh, ix = rx[i] + kw;
        const bool ok = rok[i] && kok && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
        raw_ld(ra[d][i], X + ((int64_t)(rn[i] + iy) * g.W + ix) * g.Cin + ci, X, ok);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int64_t gm = m0 + srow + G::RPP * i;
        raw_ld(ra[d][i], X + gm * K + gk, X, rok[i] && kok);
      }
    }
#pragma unroll
    for (int i = 0; i < PB; ++i)
      raw_ld(rb[d][i], Wt + (int64_t)(n0 + srow + G::RPP * i) * K + gk, Wt, srow + G::RPP * i < nvalid && kok);
  };

  f32x4_t acc[RB][CB];
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  static_for<D>([&](auto dc) {
    if (decltype(dc)::value < nk) load(dc, decltype(dc)::value);
  });
  for (int kc = 0; kc < nk; kc += D) {
    static_for<D>([&](auto dc) {
      constexpr int d = decltype(dc)::value;
      const int k = kc + d;
      if (k >= nk) return;
#pragma unroll
      for (int i = 0; i < PA; ++i) raw_st(As + G::lds_off(srow + G::RPP * i, skc), ra[d][i]);
#pragma unroll
      for (int i = 0; i < PB; ++i) raw_st(Bs + G::lds_off(srow + G::RPP * i, skc), rb[d][i]);
      lds_barrier();
      if (k + D < nk) load(dc, k + D);
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
              acc[r_][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[r_], bfr, acc[r_][cb], 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int s4 = 0; s4 < BK / 4; ++s4) {
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

  // ---- epilogue: + bias -> C tile (T) in LDS; then 16-B row stores with the residual and ReLU ----
  // (bf16 with a residual rounds twice, bf16(bf16(acc + b) + r), like the B0 dgrad epilogues)
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const int col = cbase + cb * 16 + (lane & 15);
    const float bcol = col < nvalid ? bias[n0 + col] : 0.f;
#pragma unroll
    for (int r_ = 0; r_ < RB; ++r_)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + r_ * 16 + 4 * (lane >> 4) + r;
        Cs[row * G::CS + col] = Tr<T>::from_f(acc[r_][cb][r] + bcol);
      }
  }
  lds_barrier();
  const int vpr = nvalid >> 3;
  for (int v = tid; v < BM * vpr; v += 256) {
    const int row = v / vpr, cv = (v - row * vpr) * 8;
    const int64_t gm = m0 + row;
    if (gm >= M) continue;
    float x[8];
    ld8(Cs + row * G::CS + cv, x);
    if constexpr (RESID) {
      float r8[8];
      ld8(R + gm * N + n0 + cv, r8);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += r8[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = fmaxf(x[j], 0.f);
    }
    st8(C + gm * N + n0 + cv, x);
  }
}

template <typename T, int BM, int BN, int WN, int BK, int D, bool IMPLICIT>
static int rn_go(hipStream_t s, const T* X, const T* Wt, T* C, const T* R, const float* bias, int relu,
                 const RnConvGeom& g, int64_t M, int N, int K) {
  const int ntn = cdiv(N, BN);
  const int64_t tiles = cdiv64(M, BM) * ntn;
  if (tiles > INT32_MAX) { set_error("rn_conv: too many tiles", __FILE__, __LINE__); return -1; }
  if (R)
    hipLaunchKernelGGL((rn_conv_kernel<T, BM, BN, WN, BK, D, IMPLICIT, true>), dim3((unsigned)tiles), dim3(256), 0,
                       s, X, Wt, C, R, bias, relu, g, M, N, K, ntn);
  else
    hipLaunchKernelGGL((rn_conv_kernel<T, BM, BN, WN, BK, D, IMPLICIT, false>), dim3((unsigned)tiles), dim3(256), 0,
                       s, X, Wt, C, R, bias, relu, g, M, N, K, ntn);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// 1: the Cout = 64 convolutions (layer1) on the NT GEMM's 64-wide tile too (A/B build switch; 0: the
// serving line measured 7.92-7.95 ms with them on this kernel vs 8.00-8.13 on the 64-wide tile,
// profiles/r04/ab_vg64_r04u.jsonl -- one 122 KB-LDS workgroup per CU loses to two here)
#ifndef DFD_VG64
#define DFD_VG64 0
#endif

template <typename T>
int launch_rn_conv(hipStream_t s, const T* X, const T* Wt, T* C, const T* R, const float* bias, int relu,
                   const RnConvGeom& g, int64_t M, int N, int K) {
  if (M <= 0) return 0;
  if ((N & 7) || (K & 7)) { set_error("rn_conv: Cout and K must be multiples of 8", __FILE__, __LINE__); return -1; }
  if (!bias) { set_error("rn_conv: bias (folded BN shift) required", __FILE__, __LINE__); return -1; }
  const bool implicit = g.KH > 1 || g.KW > 1 || g.stride > 1;
  if (implicit) {
    if (g.Cin < 8 || (g.Cin & (g.Cin - 1)) || (1 << g.cin_log2) != g.Cin || (g.KW != 1 && g.KW != 3) ||
        g.KH * g.KW * g.Cin != K || (int64_t)g.N * g.Ho * g.Wo != M) {
      set_error("rn_conv: implicit GEMM needs Cin a power of two >= 8, KW 1 or 3 and K = KH*KW*Cin",
                __FILE__, __LINE__);
      return -1;
    }
    if ((int64_t)g.N * g.H >= (1ll << 31)) { set_error("rn_conv: too many rows", __FILE__, __LINE__); return -1; }
    if constexpr (sizeof(T) == 2) {
      // bf16 3x3 and strided convolutions with Cin % 64 == 0 and Cout % 128 == 0: the same LDS-DMA NT
      // kernel, its A tile gathered per tap from the NHWC input (implicit GEMM, K order tap-major as here).
      // Its convolution instantiations carry ReLU (alone or after the identity) or the bias alone; a
      // residual without ReLU (no ResNet-50 layer has one) stays on rn_go below
      const bool ep_ok = relu || !R;
      if (ep_ok && vgemm_conv_covers(g.Cin, N, g.KH, g.KW) && vgemm_nt_covers(M, N, K) && (DFD_VG64 || N % 128 == 0)) {
        VgemmArgs a{};
        a.A = X; a.B = Wt; a.C = C; a.R = R; a.bias = bias;
        a.lda = K; a.ldb = K; a.ldc = N; a.M = (int)M; a.N = N; a.K = K;
        a.conv = 1; a.H = g.H; a.W = g.W; a.Ho = g.Ho; a.Wo = g.Wo; a.cin_log2 = g.cin_log2; a.KW = g.KW;
        a.stride = g.stride; a.pad = g.pad;
        return launch_vgemm_nt(s, a, VG_BIAS | (R ? VG_RESID : 0) | (relu ? VG_RELU : 0));
      }
    }
    if (N <= 64) return rn_go<T, 128, 64, 1, 32, 2, true>(s, X, Wt, C, R, bias, relu, g, M, N, K);
    return rn_go<T, 128, 128, 2, 32, 2, true>(s, X, Wt, C, R, bias, relu, g, M, N, K);
  }
  if constexpr (sizeof(T) == 2) {
    // bf16 1x1 stride-1 convolutions are plain NT GEMMs: the LDS-DMA 256-row-tile kernel of the ViT
    // (k_vgemm.hip) where it covers the shape (Cout % 128, Cin % 64), with the same epilogue order
    // (bias, identity, ReLU in fp32, one rounding)
    if (vgemm_nt_covers(M, N, K) && (DFD_VG64 || N % 128 == 0)) {
      VgemmArgs a{};
      a.A = X; a.B = Wt; a.C = C; a.R = R; a.bias = bias;
      a.lda = K; a.ldb = K; a.ldc = N; a.M = (int)M; a.N = N; a.K = K;
      return launch_vgemm_nt(s, a, VG_BIAS | (R ? VG_RESID : 0) | (relu ? VG_RELU : 0));
    }
  }
  if (N <= 64) return rn_go<T, 128, 64, 1, 32, 2, false>(s, X, Wt, C, R, bias, relu, g, M, N, K);
  return rn_go<T, 128, 128, 2, 32, 2, false>(s, X, Wt, C, R, bias, relu, g, M, N, K);
}

template int launch_rn_conv<float>(hipStream_t, const float*, const float*, float*, const float*, const float*, int,
                                   const RnConvGeom&, int64_t, int, int);
template int launch_rn_conv<bf16>(hipStream_t, const bf16*, const bf16*, bf16*, const bf16*, const float*, int,
                                  const RnConvGeom&, int64_t, int, int);

}  // namespace dfd
