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
#include "gemm_body.h"

#include <atomic>

namespace dfd {


template <typename T, int MODE, bool STATS, int EPI, int BM, int BN, int WN, int D, int BK, int OCC>
__global__ __launch_bounds__(256, OCC) void pw_gemm_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                        T* __restrict__ C, const T* __restrict__ R,
                                                        const float* __restrict__ bias, const T* __restrict__ Z,
                                                        int64_t M, int N, int K, Pro pro, float* __restrict__ stats,
                                                        int64_t tiles_m, int ntn) {
  using G = GemmCfg<T, BM, BN, WN, D, BK>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  __shared__ float st_sum[BN];
  __shared__ float st_sq[BN];
  __shared__ float st_part[STATS ? G::WM : 1][2][BN];  // per-wave-row column partials (fixed-order sum)
  extern __shared__ float pro_lds[];
  pw_gemm_body<T, MODE, STATS, EPI, BM, BN, WN, D, BK>(A, B, C, R, bias, Z, M, N, K, pro, stats, tiles_m, ntn,
                                                        (int)blockIdx.x, (int)gridDim.x, smem, st_sum, st_sq,
                                                        &st_part[0][0][0], pro_lds);
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

template <typename T, int MODE, int PF = 1>
__global__ __launch_bounds__(256, (sizeof(T) == 2 && !pro_is_gated(MODE) && PF == 1) ? 3 : 2) void pw_wgrad_kernel(const T* __restrict__ dY, const T* __restrict__ X, int64_t M,
                                                       int N, int K, Pro pro, float* __restrict__ slab, int tnk,
                                                       int64_t m_per_split) {
  __shared__ __attribute__((aligned(16))) char smem[WgCfg<T>::SMEM];
  pw_wgrad_body<T, MODE, PF>(dY, X, M, N, K, pro, slab, tnk, m_per_split, (int)(blockIdx.y * gridDim.x + blockIdx.x),
                             (int)(gridDim.x * gridDim.y), (int)gridDim.x, smem);
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
