// Small-K 1x1 convolutions of the late EfficientNet-B0 stages (timm conv_pw / conv_pwl / conv_head,
// src/pretrained_detector.py:116) as bf16 GEMMs with the weight panel resident in LDS:
//   C[M][N] = A[M][K] . W[N][K]^T  (+ per-column BN-stat partials | + residual R[M][N])
// for K <= 320 (the expansion convs' forward and the projection convs' data gradient of the 14x14 /
// 7x7 stages: K = cout 80..320, N = mid 480..1152; conv_head 320 -> 1280) at M = 12,544..50,176 rows.
//
// Why a separate kernel: the tiled GEMM (k_gemm.hip) stages 32- or 64-deep k-steps through registers
// with two barriers each, re-stages the weight tile for every row tile, and measured 20-40 us on
// shapes whose HBM floor is 5-12 us (PMC: 7 % MFMA busy, ~45 % of wave time waiting).  Here
//   * a workgroup owns one N panel of BN columns: its weight panel [BN][K] is DMA'd into LDS once;
//   * row tiles of 64 rows x the WHOLE K stream in by LDS-DMA (global_load_lds_dwordx4), double
//     buffered, so the next tile's DMA is in flight while the current tile's MFMAs run: one barrier
//     per tile instead of two per k-step;
//   * K is zero-padded in LDS to a multiple of 32 by DMA-ing from a zero page (K = 80 -> 96, 112 ->
//     128); the XOR swizzle of the 16-B chunks inside each row (applied to the DMA source address, the
//     LDS image being lane-linear) makes the ds_read_b128 fragment reads conflict-free for every row
//     size used (chunks per row 12, 16, 24, 40);
//   * the epilogue rounds to bf16, sums the BN statistics of the rounded values per column in
//     registers over all of the workgroup's tiles (one partial row per workgroup, fixed order ->
//     bit-reproducible), stages the tile in LDS and stores 16-B rows (+ residual);
//   * shapes are taken only when M % 64 == 0 and N % BN == 0 (the 14x14 / 7x7 maps at any frame
//     count that is a multiple of 16 / 64, e.g. the bench's 256): no row or column is masked, so every
//     wave issues a FIXED number of vector-memory operations after the next tile's DMA and a counted
//     s_waitcnt vmcnt retires exactly that DMA while this tile's stores drain.
#include "kernels.h"

namespace dfd {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vp;

constexpr int SK_BM = 64;
__device__ const uint4 g_skzero[64] = {};  // 1 KiB of zeros: the DMA source of the K padding

// 16-B chunk XOR inside a row of KC chunks (conflict-free 16-row ds_read_b128 column reads)
template <int KC>
__device__ __forceinline__ int sk_swz(int r) {
  if constexpr (KC == 12) return (r >> 2) & 3;
  else if constexpr (KC == 16) return r & 15;
  else return (r >> 1) & 7;  // 24, 40 chunks (multiples of 8)
}

// DMA `rows` rows x KC chunks of G (row stride ld elements, kval valid chunks) into img (lane-linear,
// row-major [rows][KC]); rows past `valid_rows` read row valid_rows - 1.  Wave w of `waves` issues
// instructions w, w + waves, ...
template <int KC, typename T>
__device__ __forceinline__ void sk_dma(const T* __restrict__ G, int64_t ld, int64_t row0, int64_t valid_rows,
                                       int kval, int rows, char* img, int w, int waves, int lane) {
  const int ninst = rows * KC / 64;
  for (int q = w; q < ninst; q += waves) {
    const int g = q * 64 + lane;
    const int r = g / KC, p = g - (g / KC) * KC;
    const int sc = p ^ sk_swz<KC>(r);
    int64_t gr = row0 + r;
    gr = gr < valid_rows ? gr : valid_rows - 1;
    const T* src = sc < kval ? G + gr * ld + sc * 8 : reinterpret_cast<const T*>(g_skzero) + 8 * (lane & 7);
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)(img + q * 1024), 16, 0, 0);
  }
}

// wait for this wave's vector-memory operations except the youngest n (LDS / export counters untouched)
template <int N>
__device__ __forceinline__ void vm_wait() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <typename T, int KC, int BN, bool STATS, bool RESID>
__global__ __launch_bounds__(256, 1) void pw_sk_kernel(const T* __restrict__ A, const T* __restrict__ W,
                                                        T* __restrict__ C, const T* __restrict__ R,
                                                        float* __restrict__ stats, int64_t M, int N, int K,
                                                        int panels, int per_panel) {
  constexpr int ROWB = KC * 16;                   // bytes per LDS row
  constexpr int BIMG = BN * ROWB, AIMG = SK_BM * ROWB;
  constexpr int CS = BN + 8;                      // C staging row stride (bf16)
  constexpr int CB = BN / 32, RB = 2;             // 16x16 blocks per wave (2 x 2 waves: 32 x BN/2 each)
  constexpr int NSL = KC / 4;                     // 32-deep k-slices
  constexpr int VPR = BN / 8, ST_PER = SK_BM * VPR / 256;  // 16-B output vectors per row / per thread
  // one LDS array (a second __shared__ object can make hipcc drain vmcnt before LDS reads)
  __shared__ __attribute__((aligned(16))) char smem[BIMG + 2 * AIMG + SK_BM * CS * 2];
  char* Bi = smem;
  char* const Ai0 = smem + BIMG;  // row tile images: Ai0 + buf * AIMG
  T* Cs = reinterpret_cast<T*>(smem + BIMG + 2 * AIMG);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), wm = w >> 1, wn = w & 1;
  const int panel = (int)blockIdx.x % panels, slot = (int)blockIdx.x / panels;
  const int n0 = panel * BN;
  const int kval = K / 8;
  const int64_t tiles = (M + SK_BM - 1) / SK_BM;

  int64_t t = slot;
  sk_dma<KC>(W, K, n0, N, kval, BN, Bi, w, 4, lane);
  if (t < tiles) sk_dma<KC>(A, K, t * SK_BM, M, kval, SK_BM, Ai0, w, 4, lane);
  __syncthreads();

  float cs[CB], cq[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) { cs[j] = 0.f; cq[j] = 0.f; }
  int buf = 0;
  for (; t < tiles; t += per_panel, buf ^= 1) {
    const bool more = t + per_panel < tiles;
    if (more) sk_dma<KC>(A, K, (t + per_panel) * SK_BM, M, kval, SK_BM, Ai0 + (buf ^ 1) * AIMG, w, 4, lane);
    f32x4 acc[RB][CB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* Ac = Ai0 + buf * AIMG;
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      s16x8 af[RB], bfr[CB];
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int r = wm * 32 + 16 * i + (lane & 15);
        const int c = (4 * s + (lane >> 4)) ^ sk_swz<KC>(r);
        af[i] = *reinterpret_cast<const s16x8*>(Ac + r * ROWB + c * 16);
      }
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const int r = wn * (BN / 2) + 16 * j + (lane & 15);
        const int c = (4 * s + (lane >> 4)) ^ sk_swz<KC>(r);
        bfr[j] = *reinterpret_cast<const s16x8*>(Bi + r * ROWB + c * 16);
      }
#pragma unroll
      for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j) acc[i][j] = mfma16x16x32<T>(af[i], bfr[j], acc[i][j]);
    }
    // epilogue: round, BN-stat sums of the rounded values (valid rows), stage the tile
    const int64_t m0 = t * SK_BM;
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const int col = wn * (BN / 2) + 16 * j + (lane & 15);
#pragma unroll
      for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = wm * 32 + 16 * i + 4 * (lane >> 4) + e;
          const float v = Tr<T>::round(acc[i][j][e]);
          Cs[row * CS + col] = Tr<T>::from_f(v);
          if constexpr (STATS) { cs[j] += v; cq[j] += v * v; }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int u = 0; u < ST_PER; ++u) {  // no masks (covers(): M % 64 == 0, N % BN == 0)
      const int v = tid + 256 * u;
      const int row = v / VPR, cv = (v - (v / VPR) * VPR) * 8;
      const int64_t gm = m0 + row;
      float x[8];
      ld8(Cs + row * CS + cv, x);
      if constexpr (RESID) {
        float r8[8];
        ld8(R + gm * N + n0 + cv, r8);
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] += r8[q];
      }
      st8(C + gm * N + n0 + cv, x);
    }
    // the next tile's DMA (issued before this tile's ST_PER stores (+ ST_PER residual loads)) has
    // landed; everyone is done with this tile's A image and with the C staging
    if (more) vm_wait<(RESID ? 2 : 1) * ST_PER>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if constexpr (STATS) {
    // lanes l, l^16, l^32, l^48 hold the same column; then the two row-waves in order (the A images
    // are free: every DMA has landed and the loop's last barrier has passed)
    float (*sred)[2][BN] = reinterpret_cast<float (*)[2][BN]>(smem + BIMG);
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, 64); cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64); cq[j] += __shfl_xor(cq[j], 32, 64);
      if (lane < 16) {
        sred[wm][0][wn * (BN / 2) + 16 * j + lane] = cs[j];
        sred[wm][1][wn * (BN / 2) + 16 * j + lane] = cq[j];
      }
    }
    __syncthreads();
    for (int i = tid; i < BN; i += 256) {
      stats[((int64_t)slot * 2 + 0) * N + n0 + i] = sred[0][0][i] + sred[1][0][i];
      stats[((int64_t)slot * 2 + 1) * N + n0 + i] = sred[0][1][i] + sred[1][1][i];
    }
  }
}

template <int KC, int BN, bool STATS, bool RESID, typename T>
int sk_go(hipStream_t s, const T* A, const T* W, T* C, const T* R, float* stats, int64_t M, int N, int K,
          int max_rows, int* stat_rows) {
  auto kern = pw_sk_kernel<T, KC, BN, STATS, RESID>;
  static const int resident = [&] {
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    return std::max(1, cus * per_cu);
  }();
  const int panels = cdiv(N, BN);
  const int64_t tiles = cdiv64(M, SK_BM);
  int per = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, resident / panels));
  if (STATS) per = std::min(per, max_rows);
  hipLaunchKernelGGL(kern, dim3((unsigned)(panels * per)), dim3(256), 0, s, A, W, C, R, stats, M, N, K, panels, per);
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = per;
  return 0;
}

}  // namespace

// panel width per K: the LDS budget (weight panel + two row tiles + C staging <= 160 KiB) and
// N % BN == 0 for the stage widths 480 / 672 (96), 1152 (128, or 64 at K = 320), 1280 (64)
static int sk_bn(int N, int K) {
  if (K == 320) return N % 64 == 0 ? 64 : 0;
  if (N % 128 == 0) return 128;
  return N % 96 == 0 ? 96 : (N % 64 == 0 ? 64 : 0);
}

bool pw_sk_covers(int64_t M, int N, int K) {
  return M > 0 && M % SK_BM == 0 && M < (1ll << 31) && (K == 80 || K == 112 || K == 192 || K == 320) &&
         sk_bn(N, K) != 0;
}

template <typename T>
int launch_pw_sk(hipStream_t s, const T* A, const T* W, T* C, const T* R, int64_t M, int N, int K, float* stats,
                 int max_rows, int* stat_rows) {
  if (!pw_sk_covers(M, N, K) || (R && stats)) return 1;
  const bool st = stats != nullptr, rs = R != nullptr;
#define DFD_SK(KC_, BN_)                                                                                          \
  return st ? sk_go<KC_, BN_, true, false>(s, A, W, C, R, stats, M, N, K, max_rows, stat_rows)                   \
            : (rs ? sk_go<KC_, BN_, false, true>(s, A, W, C, R, stats, M, N, K, max_rows, stat_rows)             \
                  : sk_go<KC_, BN_, false, false>(s, A, W, C, R, stats, M, N, K, max_rows, stat_rows))
  const int bn = sk_bn(N, K);
  if (K == 80) { if (bn == 128) DFD_SK(12, 128); if (bn == 96) DFD_SK(12, 96); DFD_SK(12, 64); }
  if (K == 112) { if (bn == 128) DFD_SK(16, 128); if (bn == 96) DFD_SK(16, 96); DFD_SK(16, 64); }
  if (K == 192) { if (bn == 128) DFD_SK(24, 128); if (bn == 96) DFD_SK(24, 96); DFD_SK(24, 64); }
  DFD_SK(40, 64);
#undef DFD_SK
}
template int launch_pw_sk<bf16>(hipStream_t, const bf16*, const bf16*, bf16*, const bf16*, int64_t, int, int, float*,
                                int, int*);
template int launch_pw_sk<f16>(hipStream_t, const f16*, const f16*, f16*, const f16*, int64_t, int, int, float*, int,
                               int*);

}  // namespace dfd
