// Streaming pointwise (1x1 conv) GEMM for the tall-skinny layers of EfficientNet-B0 (16-bit: bf16 / fp16).
//
// Same contract as pw_gemm_kernel (k_gemm.hip) -- C[M][N] = pro(A)[M][K] . B[N][K]^T with the
// producer's BN+SiLU(+SE gate) prologue, BN-stat partials of C's columns and the residual add
// of the dgrad -- for the high-resolution layers (M = frames*H*W rows large, K <= 256), where
// the pass is a pure HBM stream: every A row is read once and every C row written once, and the
// weight chunk (<= 128 x 256 bf16) sits in LDS for the whole launch.
//
// Per wave, independent of the other waves (no barrier after the LDS staging):
//   * 16-row groups of A are loaded straight from HBM into MFMA operand fragments
//     (lane = row lane&15, 8 consecutive k at 8*(lane>>4): one 16-B load per lane and k-block),
//     the prologue is applied in registers, the next groups are in flight during the MFMAs;
//   * v_mfma_f32_16x16x32_bf16 computes the TRANSPOSED tile D[n][m] = W[n][:] . A[m][:], so a
//     lane ends up holding 4 consecutive output channels of one row; the rounded tile goes
//     through a wave-private LDS slab (no workgroup barrier) so the global stores are 16 B per
//     lane with consecutive lanes on consecutive bytes of a row (full 128-B lines);
//   * BN-stat partials accumulate per lane across all groups of the wave (fixed order) and are
//     reduced once at the end: 16-lane shuffles, then the 4 waves in order (bit-reproducible).
// The SE gates of the (few) frames a workgroup's rows belong to are staged in LDS with the
// weights and the producer's BN coefficients.  Grid: parts x N-chunks, chunk fastest, so the
// workgroups that read the same A rows are adjacent in dispatch order (A re-reads hit L2).
// Shapes it does not cover go to pw_gemm_kernel.
#include "kernels.h"

#include <algorithm>
#include <atomic>

#ifndef DFD_XCD_SWZ_F
#define DFD_XCD_SWZ_F 1  // XCD-aware block order, streaming forward (A/B knob)
#endif
#ifndef DFD_XCD_SWZ_W
#define DFD_XCD_SWZ_W 1  // XCD-aware block order, streaming weight gradient (A/B knob)
#endif

namespace dfd {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// Row threshold above which the streaming kernel takes a layer (below it the tiled kernel's
// weight reuse wins); settable through dfd_set_tuning("stream_min_rows", v).

template <int NB, int U>
struct StreamTile {
  static constexpr int NC = NB * 16;
  static constexpr int CS = NC + 8;                // LDS row stride of the C slab (elements)
  static constexpr int VPR = NC / 8;               // 16-B vectors per row
  static constexpr int NV = (U * 16 * VPR + 63) / 64;  // vectors per lane per iteration
  static constexpr int SLAB = U * 16 * CS * 2;     // bytes per wave
};

template <typename T, int KB, int U, bool RESID, int NV>
struct StreamRegs {
  Raw8<T> a[U][KB];
  uint4 r[RESID ? NV : 1];
};

template <typename T, int NB, int KB, int U, int MODE, bool STATS, bool RESID, bool BIAS>
__global__ __launch_bounds__(256, 2) void pw_stream_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                           T* __restrict__ C, const T* __restrict__ R,
                                                           const float* __restrict__ bias,
                                                           int64_t M, int N, int K, Pro pro,
                                                           float* __restrict__ stats, int nchunks,
                                                           int64_t groups_per_part, int gate_frames) {
  constexpr int NC = NB * 16, KP = KB * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* Bs = reinterpret_cast<uint4*>(smem);                   // [NB][KB][64] operand fragments
  float* psc = reinterpret_cast<float*>(smem + NB * KB * 1024);  // [KP] producer BN scale
  float* psh = psc + KP;                                         // [KP] producer BN shift
  float* red = psh + KP;                                         // [4][2][NC] stat partials
  float* bl = red + 8 * NC;                                      // [NC] bias
  float* gl = bl + NC;                                           // [gate_frames][KP] SE gates
  using TL = StreamTile<NB, U>;
  T* ct = reinterpret_cast<T*>(gl + gate_frames * KP) + (threadIdx.x >> 6) * (TL::SLAB / 2);  // wave's C slab

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bid = DFD_XCD_SWZ_F ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int chunk = bid % nchunks;
  const int64_t part = bid / nchunks;
  const int n0 = chunk * NC;

  for (int f = tid; f < NB * KB * 64; f += 256) {
    const int ln = f & 63, kb = (f >> 6) % KB, nb = (f >> 6) / KB;
    const int n = n0 + nb * 16 + (ln & 15), k = kb * 32 + 8 * (ln >> 4);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (n < N && k < K) v = *reinterpret_cast<const uint4*>(B + (int64_t)n * K + k);
    Bs[f] = v;
  }
  if constexpr (pro_is_bn(MODE)) {
    for (int k = tid; k < KP; k += 256) {
      psc[k] = k < K ? pro.scale[k] : 0.f;
      psh[k] = k < K ? pro.shift[k] : 0.f;
    }
  }
  if constexpr (BIAS) {
    for (int i = tid; i < NC; i += 256) bl[i] = n0 + i < N ? bias[n0 + i] : 0.f;
  }
  const int64_t G = (M + 15) >> 4;
  const int64_t gbeg = part * groups_per_part;
  const int64_t gend = min(G, gbeg + groups_per_part);
  // SE gates of the frames this part's rows belong to (at most gate_frames, sized at launch)
  int f_first = 0;
  if constexpr (MODE == PRO_BN_SILU_G) {
    if (gbeg < gend) {
      f_first = (int)((gbeg * 16) / pro.rows_per_frame);
      const int f_last = (int)((min(gend * 16, M) - 1) / pro.rows_per_frame);
      const int nfr = min(gate_frames, f_last - f_first + 1);
      for (int i = tid; i < nfr * KP; i += 256) {
        const int fr = i / KP, k = i - fr * KP;
        gl[i] = k < K ? pro.gate[(int64_t)(f_first + fr) * pro.C + k] : 0.f;
      }
    }
  }
  __syncthreads();

  const int lr = lane & 15, lk = 8 * (lane >> 4), ln4 = 4 * (lane >> 4);

  StreamRegs<T, KB, U, RESID, TL::NV> rg;
  auto load = [&](int64_t g0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = (g0 + u) * 16 + lr;
      const bool rok = g0 + u < gend && row < M;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int k = kb * 32 + lk;
        raw_ld(rg.a[u][kb], A + row * K + k, A, rok && k < K);
      }
    }
    if constexpr (RESID) {  // the residual in the store-phase layout (16 B per lane)
#pragma unroll
      for (int i = 0; i < TL::NV; ++i) {
        const int v = lane + 64 * i, rr = v / TL::VPR, cv = (v - rr * TL::VPR) * 8;
        const int64_t row = g0 * 16 + rr;
        const bool ok = rr < U * 16 && g0 * 16 + rr < min(gend * 16, M) && n0 + cv < N;
        rg.r[i] = *reinterpret_cast<const uint4*>(ok ? R + row * N + n0 + cv : R);
      }
    }
  };

  float s_acc[STATS ? NB : 1][4], q_acc[STATS ? NB : 1][4];
  if constexpr (STATS) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s_acc[nb][r] = 0.f; q_acc[nb][r] = 0.f; }
  }

  const int64_t step = 4 * U;
  int64_t g = gbeg + (int64_t)wave * U;
  if (g < gend) load(g);
  for (; g < gend; g += step) {
    // keep the LDS operand/coefficient reads inside the loop (hoisted, they would pin up to
    // 2*KP + 4*NB*KB registers per lane and spill the gated variants)
    asm volatile("" ::: "memory");
    // ---- prologue in registers: raw A -> 16-bit MFMA operands ----
    bf16x8_t af[U][KB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int fr = 0;
      if constexpr (MODE == PRO_BN_SILU_G) {
        const int64_t row = (g + u) * 16 + lr;
        fr = (g + u < gend && row < M) ? (int)((uint32_t)row / (uint32_t)pro.rows_per_frame) - f_first : 0;
      }
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const uint32_t m = rg.a[u][kb].ok ? 0xffffffffu : 0u;
        if constexpr (MODE == PRO_NONE) {
          const uint4 v = make_uint4(rg.a[u][kb].a.x & m, rg.a[u][kb].a.y & m, rg.a[u][kb].a.z & m,
                                     rg.a[u][kb].a.w & m);
          af[u][kb] = __builtin_bit_cast(bf16x8_t, v);
        } else {
          float x[8], sc[8], sh[8];
          raw_to_f(rg.a[u][kb], x);
          const int k = kb * 32 + lk;
          ld8(psc + k, sc);
          ld8(psh + k, sh);
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = siluf_(x[j] * sc[j] + sh[j]);
          if constexpr (MODE == PRO_BN_SILU_G) {
            float gv[8];
            ld8(gl + fr * KP + k, gv);
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] *= gv[j];
          }
          const uint4 v = make_uint4(Tr<T>::pack2(x[0], x[1]) & m, Tr<T>::pack2(x[2], x[3]) & m,
                                     Tr<T>::pack2(x[4], x[5]) & m, Tr<T>::pack2(x[6], x[7]) & m);
          af[u][kb] = __builtin_bit_cast(bf16x8_t, v);
          asm volatile("" ::: "memory");  // one k-block's coefficients live at a time
        }
      }
    }
    uint4 rres[RESID ? TL::NV : 1];
    if constexpr (RESID) {
#pragma unroll
      for (int i = 0; i < TL::NV; ++i) rres[i] = rg.r[i];
    }
    // ---- next groups in flight before the MFMAs and stores of this one ----
    if (g + step < gend) load(g + step);

    f32x4_t acc[U][NB];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[u][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const bf16x8_t wf = __builtin_bit_cast(bf16x8_t, Bs[(nb * KB + kb) * 64 + lane]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          acc[u][nb] = mfma16x16x32<T>(wf, af[u][kb], acc[u][nb]);
      }

    // ---- epilogue: lane = row lr, channels n .. n+3: stats from registers, bf16 into the slab ----
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = (g + u) * 16 + lr;
      const bool rok = g + u < gend && row < M;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = n0 + nb * 16 + ln4;
        if constexpr (BIAS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[u][nb][r] += bl[nb * 16 + ln4 + r];
        }
        const uint2 pk =
            make_uint2(Tr<T>::pack2(acc[u][nb][0], acc[u][nb][1]), Tr<T>::pack2(acc[u][nb][2], acc[u][nb][3]));
        if constexpr (STATS) {
          const bool ok = rok && n < N;
          const float v[4] = {lo2f(pk.x, (T*)nullptr), hi2f(pk.x, (T*)nullptr), lo2f(pk.y, (T*)nullptr),
                              hi2f(pk.y, (T*)nullptr)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float w = ok ? v[r] : 0.f;
            s_acc[nb][r] += w;
            q_acc[nb][r] += w * w;
          }
        }
        *reinterpret_cast<uint2*>(ct + (u * 16 + lr) * TL::CS + nb * 16 + ln4) = pk;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // ---- row-contiguous 16-B stores (+ residual: C = bf16(bf16(acc) + R)) ----
    const int64_t rend = min(gend * 16, M);
#pragma unroll
    for (int i = 0; i < TL::NV; ++i) {
      const int v = lane + 64 * i, rr = v / TL::VPR, cv = (v - rr * TL::VPR) * 8;
      const int64_t row = g * 16 + rr;
      if (rr < U * 16 && row < rend && n0 + cv < N) {
        uint4 o = *reinterpret_cast<const uint4*>(ct + rr * TL::CS + cv);
        if constexpr (RESID) {
          float x[8], y[8];
          ld8(reinterpret_cast<const T*>(&o), x);
          ld8(reinterpret_cast<const T*>(&rres[i]), y);
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] += y[j];
          o = make_uint4(Tr<T>::pack2(x[0], x[1]), Tr<T>::pack2(x[2], x[3]), Tr<T>::pack2(x[4], x[5]),
                         Tr<T>::pack2(x[6], x[7]));
        }
        *reinterpret_cast<uint4*>(C + row * N + n0 + cv) = o;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  if constexpr (STATS) {
    // lanes sharing lane>>4 hold the same 4 channels for 16 different rows
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = s_acc[nb][r], q = q_acc[nb][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s += __shfl_xor(s, o, 64);
          q += __shfl_xor(q, o, 64);
        }
        if (lr == 0) {
          red[(wave * 2 + 0) * NC + nb * 16 + ln4 + r] = s;
          red[(wave * 2 + 1) * NC + nb * 16 + ln4 + r] = q;
        }
      }
    __syncthreads();
    for (int i = tid; i < NC; i += 256) {
      if (n0 + i < N) {
        stats[(part * 2 + 0) * N + n0 + i] =
            ((red[0 * NC + i] + red[2 * NC + i]) + red[4 * NC + i]) + red[6 * NC + i];
        stats[(part * 2 + 1) * N + n0 + i] =
            ((red[1 * NC + i] + red[3 * NC + i]) + red[5 * NC + i]) + red[7 * NC + i];
      }
    }
  }
}

template <typename T, int NB, int KB, int MODE, bool STATS, bool RESID, bool BIAS = false>
static int stream_launch(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias,
                         int64_t M, int N, int K, const Pro& pro, float* stats, int* stat_rows) {
  constexpr int U = KB <= 2 ? 2 : 1;
  using TL = StreamTile<NB, U>;
  auto kern = pw_stream_kernel<T, NB, KB, U, MODE, STATS, RESID, BIAS>;
  const int nchunks = cdiv(N, NB * 16);
  const int64_t G = cdiv64(M, 16);
  const size_t lds_fixed = (size_t)NB * KB * 1024 + 2 * (size_t)KB * 32 * 4 + 9 * (size_t)NB * 16 * 4 + 4 * TL::SLAB;
  // persistent grid: exactly the workgroups that are co-resident (one wave of dispatch, no
  // tail), measured once per instantiation at the LDS size without gate rows
  static const int resident = [&] {
    int dev = 0, cus = 256, per_cu = 2;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds_fixed) != hipSuccess || per_cu < 1)
      per_cu = 1;
    return std::max(1, cus * per_cu);
  }();
  int64_t parts = std::max<int64_t>(1, std::min<int64_t>(std::max(1, resident / nchunks), cdiv64(G, 4 * U)));
  const int64_t gpp = cdiv64(cdiv64(G, parts), 4 * U) * (4 * U);
  parts = cdiv64(G, gpp);
  int gate_frames = 0;
  if (MODE == PRO_BN_SILU_G) {
    // frames one part's rows can touch; past 16 the gate table would crowd the LDS budget
    gate_frames = (int)std::min<int64_t>(cdiv64(M, pro.rows_per_frame), cdiv64(gpp * 16, pro.rows_per_frame) + 1);
    if (gate_frames > 16) return 1;
  }
  const size_t lds = lds_fixed + (size_t)gate_frames * KB * 32 * 4;
  hipLaunchKernelGGL(kern, dim3((unsigned)(parts * nchunks)), dim3(256), lds, s, A, B, C, R, bias, M, N, K, pro,
                     stats, nchunks, gpp, gate_frames);
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = (int)parts;
  return 0;
}

// 0: launched; 1: not covered (shape/mode without an instantiation, or M below the threshold;
// the caller uses the tiled kernel); -1: launch error
template <typename T>
int launch_pw_stream(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias, int64_t M, int N,
                     int K, int pro_mode, const Pro& pro, float* stats, int* stat_rows) {
  if (M <= 0 || M < tune(TK_STREAM_MIN_ROWS) || K > 256 || (N & 7) || (K & 7)) return 1;
  const int nchunks = cdiv(N, 128);
  const int NB = cdiv(cdiv(N, nchunks), 16), KB = cdiv(K, 32);
  const bool st = stats != nullptr, rs = R != nullptr, bs = bias != nullptr;
  if (bs && (st || pro_mode != PRO_NONE)) return 1;
  const int key = NB * 16 + KB;
#define DFD_STREAM_CASE(NB_, KB_, MODE_, ST_, RS_) \
  case NB_ * 16 + KB_:                             \
    return stream_launch<T, NB_, KB_, MODE_, ST_, RS_>(s, A, B, C, R, bias, M, N, K, pro, stats, stat_rows);
#define DFD_STREAM_BIAS(NB_, KB_, RS_) \
  case NB_ * 16 + KB_:                 \
    return stream_launch<T, NB_, KB_, PRO_NONE, false, RS_, true>(s, A, B, C, R, bias, M, N, K, pro, stats, stat_rows);
  if (bs) {  // x . Q + bv (+ skip gradient): the linear part of the conv_pw input gradient (bn_fold_pw)
    if (rs) {
      switch (key) {
        DFD_STREAM_BIAS(2, 1, true)  // 24 -> 24
        DFD_STREAM_BIAS(3, 2, true)  // 40 -> 40
        default: return 1;
      }
    }
    switch (key) {
      DFD_STREAM_BIAS(1, 1, false)  // 16 -> 16
      DFD_STREAM_BIAS(2, 1, false)  // 24 -> 24
      DFD_STREAM_BIAS(3, 2, false)  // 40 -> 40
      default: return 1;
    }
  }
#undef DFD_STREAM_BIAS
  if (pro_mode == PRO_NONE && st && !rs) {  // conv_pw forward (expansion): N = mid, K = cin
    switch (key) {
      DFD_STREAM_CASE(6, 1, PRO_NONE, true, false)  // 16 -> 96
      DFD_STREAM_CASE(5, 1, PRO_NONE, true, false)  // 24 -> 144
      DFD_STREAM_CASE(8, 2, PRO_NONE, true, false)  // 40 -> 240
      DFD_STREAM_CASE(8, 3, PRO_NONE, true, false)  // 80 -> 480
      DFD_STREAM_CASE(7, 4, PRO_NONE, true, false)  // 112 -> 672
      DFD_STREAM_CASE(8, 6, PRO_NONE, true, false)  // 192 -> 1152 (7x7 stages, chunks of 128)
      default: return 1;
    }
  }
  if (pro_mode == PRO_BN_SILU_G && st && !rs) {  // conv_pwl forward: N = cout, K = mid
    switch (key) {
      DFD_STREAM_CASE(1, 1, PRO_BN_SILU_G, true, false)  // 32 -> 16 (stage 0)
      DFD_STREAM_CASE(2, 3, PRO_BN_SILU_G, true, false)  // 96 -> 24
      DFD_STREAM_CASE(2, 5, PRO_BN_SILU_G, true, false)  // 144 -> 24
      DFD_STREAM_CASE(3, 5, PRO_BN_SILU_G, true, false)  // 144 -> 40
      // 240 -> 40 (KB 8) spills at 256 VGPRs: left to the tiled kernel
      default: return 1;
    }
  }
  if (pro_mode == PRO_NONE && !st && !rs) {  // dgrads: conv_pw (N = cin, K = mid), conv_pwl (N = mid, K = cout)
    switch (key) {
      DFD_STREAM_CASE(1, 3, PRO_NONE, false, false)  // 96 -> 16
      DFD_STREAM_CASE(2, 5, PRO_NONE, false, false)  // 144 -> 24
      DFD_STREAM_CASE(3, 8, PRO_NONE, false, false)  // 240 -> 40
      DFD_STREAM_CASE(2, 1, PRO_NONE, false, false)  // 16 -> 32 (stage 0)
      DFD_STREAM_CASE(6, 1, PRO_NONE, false, false)  // 24 -> 96
      DFD_STREAM_CASE(5, 1, PRO_NONE, false, false)  // 24 -> 144
      DFD_STREAM_CASE(5, 2, PRO_NONE, false, false)  // 40 -> 144
      DFD_STREAM_CASE(8, 2, PRO_NONE, false, false)  // 40 -> 240
      DFD_STREAM_CASE(8, 3, PRO_NONE, false, false)  // 80 -> 240 / 480
      DFD_STREAM_CASE(7, 4, PRO_NONE, false, false)  // 112 -> 672
      DFD_STREAM_CASE(8, 6, PRO_NONE, false, false)  // 192 -> 1152
      default: return 1;
    }
  }
  if (pro_mode == PRO_NONE && !st && rs) {  // conv_pw dgrad plus the block's skip gradient
    switch (key) {
      DFD_STREAM_CASE(1, 3, PRO_NONE, false, true)  // 96 -> 16
      DFD_STREAM_CASE(2, 5, PRO_NONE, false, true)  // 144 -> 24
      DFD_STREAM_CASE(3, 8, PRO_NONE, false, true)  // 240 -> 40
      default: return 1;
    }
  }
#undef DFD_STREAM_CASE
  return 1;
}

// ------------------------------------------------------------------------------------------
// Streaming weight gradient for the same layers:  dW[N][K] = sum_m dY[m][n] * pro(X)[m][k].
//
// A workgroup owns one (N-chunk x K-chunk) of dW (<= 16 MFMA blocks of 16x16) for a slice of the
// rows; its 4 waves sweep disjoint 32*S-row steps of that slice, each through a wave-private
// LDS slab (no workgroup barrier inside the loop): the rows are staged with 16-B loads in their
// natural row-major layout (X through the producer's BN+SiLU(+gate) prologue), then read back as
// COLUMNS with ds_read_b64_tr_b16 to form the MFMA operands (the contraction runs over rows).
// The next step's global loads are in flight during the current step's MFMAs.  The four waves'
// accumulators are added in a fixed order and written to the part's slab row; the slabs are
// summed in order afterwards (deterministic).
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

template <int NBW, int KBW, int S>
struct WgsTile {
  static constexpr int NW = NBW * 16, KW = KBW * 16, R = 32 * S;
  static constexpr int YS = NW + 8, XS = KW + 8;  // LDS row strides (elements)
  static constexpr int VY = NW / 8, VX = KW / 8;  // 16-B vectors per row
  static constexpr int NVY = R * VY / 64, NVX = R * VX / 64;
  static constexpr int WAVE_BYTES = R * (YS + XS) * 2;
  static_assert((R * VY) % 64 == 0 && (R * VX) % 64 == 0, "step must be whole wave loads");
};

template <typename T, int NBW, int KBW, int S, int MODE>
__global__ __launch_bounds__(256, 2) void pw_wgrad_stream_kernel(const T* __restrict__ dY,
                                                                 const T* __restrict__ X, int64_t M, int N,
                                                                 int K, Pro pro, float* __restrict__ slab,
                                                                 int nch_n, int nch_k, int64_t rows_per_part,
                                                                 int gate_frames) {
  using TL = WgsTile<NBW, KBW, S>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* psc = reinterpret_cast<float*>(smem);  // [KW]
  float* psh = psc + TL::KW;                     // [KW]
  float* gl = psh + TL::KW;                      // [gate_frames][KW]
  char* wave_base = reinterpret_cast<char*>(gl + gate_frames * TL::KW);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // chunks of one row part share an XCD (and its L2): measured in tools/kbench
  const int bid = DFD_XCD_SWZ_W ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int chunk = bid % (nch_n * nch_k);
  const int64_t part = bid / (nch_n * nch_k);
  const int cn = chunk / nch_k, ck = chunk - cn * nch_k;
  const int n0 = cn * TL::NW, k0 = ck * TL::KW;
  const int64_t mbeg = part * rows_per_part, mend = min(M, mbeg + rows_per_part);
  T* Ys = reinterpret_cast<T*>(wave_base + wave * TL::WAVE_BYTES);
  T* Xs = Ys + TL::R * TL::YS;

  int f_first = 0;
  if constexpr (pro_is_bn(MODE)) {
    for (int i = tid; i < TL::KW; i += 256) {
      const bool ok = k0 + i < K;
      psc[i] = ok ? pro.scale[k0 + i] : 0.f;
      psh[i] = ok ? pro.shift[k0 + i] : 0.f;
    }
    if constexpr (MODE == PRO_BN_SILU_G) {
      if (mbeg < mend) {
        f_first = (int)(mbeg / pro.rows_per_frame);
        const int nfr = min(gate_frames, (int)((mend - 1) / pro.rows_per_frame) - f_first + 1);
        for (int i = tid; i < nfr * TL::KW; i += 256) {
          const int fr = i / TL::KW, k = i - fr * TL::KW;
          gl[i] = k0 + k < K ? pro.gate[(int64_t)(f_first + fr) * pro.C + k0 + k] : 0.f;
        }
      }
    }
  }
  __syncthreads();

  Raw8<T> ry[TL::NVY], rx[TL::NVX];
  auto load = [&](int64_t ms) {
#pragma unroll
    for (int i = 0; i < TL::NVY; ++i) {
      const int v = lane + 64 * i, rr = v / TL::VY, cv = (v - rr * TL::VY) * 8;
      const int64_t row = ms + rr;
      raw_ld(ry[i], dY + row * N + n0 + cv, dY, row < mend && n0 + cv < N);
    }
#pragma unroll
    for (int i = 0; i < TL::NVX; ++i) {
      const int v = lane + 64 * i, rr = v / TL::VX, cv = (v - rr * TL::VX) * 8;
      const int64_t row = ms + rr;
      raw_ld(rx[i], X + row * K + k0 + cv, X, row < mend && k0 + cv < K);
    }
  };

  f32x4_t acc[NBW][KBW];
#pragma unroll
  for (int a = 0; a < NBW; ++a)
#pragma unroll
    for (int b = 0; b < KBW; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int64_t wstep = 4 * TL::R;
  int64_t ms = mbeg + wave * TL::R;
  if (ms < mend) load(ms);
  for (; ms < mend; ms += wstep) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < TL::NVY; ++i) {
      const int v = lane + 64 * i, rr = v / TL::VY, cv = (v - rr * TL::VY) * 8;
      raw_st(Ys + rr * TL::YS + cv, ry[i]);
    }
#pragma unroll
    for (int i = 0; i < TL::NVX; ++i) {
      const int v = lane + 64 * i, rr = v / TL::VX, cv = (v - rr * TL::VX) * 8;
      if constexpr (MODE == PRO_NONE) {
        raw_st(Xs + rr * TL::XS + cv, rx[i]);
      } else {
        float x[8], sc[8], sh[8];
        raw_to_f(rx[i], x);
        ld8(psc + cv, sc);
        ld8(psh + cv, sh);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = siluf_(x[j] * sc[j] + sh[j]);
        if constexpr (MODE == PRO_BN_SILU_G) {
          const int64_t row = ms + rr;
          const int fr = row < mend ? (int)((uint32_t)row / (uint32_t)pro.rows_per_frame) - f_first : 0;
          float gv[8];
          ld8(gl + fr * TL::KW + cv, gv);
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] *= gv[j];
        }
        const uint32_t m = rx[i].ok ? 0xffffffffu : 0u;
        *reinterpret_cast<uint4*>(Xs + rr * TL::XS + cv) =
            make_uint4(Tr<T>::pack2(x[0], x[1]) & m, Tr<T>::pack2(x[2], x[3]) & m, Tr<T>::pack2(x[4], x[5]) & m,
                       Tr<T>::pack2(x[6], x[7]) & m);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (ms + wstep < mend) load(ms + wstep);
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int sub = 0; sub < S; ++sub) {
      const T* Yb = Ys + sub * 32 * TL::YS;
      const T* Xb = Xs + sub * 32 * TL::XS;
      bf16x8_t bfr[KBW];
#pragma unroll
      for (int kb = 0; kb < KBW; ++kb) {
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Xb + (8 * g + q) * TL::XS + kb * 16 + 4 * p));
        const s16x4_t hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Xb + (8 * g + 4 + q) * TL::XS + kb * 16 + 4 * p));
        bfr[kb] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) {
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Yb + (8 * g + q) * TL::YS + nb * 16 + 4 * p));
        const s16x4_t hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Yb + (8 * g + 4 + q) * TL::YS + nb * 16 + 4 * p));
        const bf16x8_t af = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int kb = 0; kb < KBW; ++kb) acc[nb][kb] = mfma16x16x32<T>(af, bfr[kb], acc[nb][kb]);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  // ---- the 4 waves' tiles added in a fixed order, then this part's slab row ----
  float* red = reinterpret_cast<float*>(wave_base);  // [NW][KW], reuses the wave slabs
  static_assert(TL::NW * TL::KW * 4 <= 4 * TL::WAVE_BYTES, "reduction tile exceeds the wave slabs");
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
        for (int kb = 0; kb < KBW; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int idx = (nb * 16 + 4 * (lane >> 4) + r) * TL::KW + kb * 16 + (lane & 15);
            red[idx] = (w == 0 ? 0.f : red[idx]) + acc[nb][kb][r];
          }
    }
  }
  __syncthreads();
  float* out = slab + part * (int64_t)N * K;
  for (int i = tid; i < TL::NW * TL::KW; i += 256) {
    const int nn = i / TL::KW, kk = i - nn * TL::KW;
    if (n0 + nn < N && k0 + kk < K) out[(int64_t)(n0 + nn) * K + k0 + kk] = red[i];
  }
}

template <typename T, int NBW, int KBW, int S, int MODE>
static int wgs_launch(hipStream_t s, const T* dY, const T* X, int64_t M, int N, int K, const Pro& pro,
                      float* slab, int64_t slab_cap, float* dW, bool accumulate) {
  using TL = WgsTile<NBW, KBW, S>;
  auto kern = pw_wgrad_stream_kernel<T, NBW, KBW, S, MODE>;
  const int nch_n = cdiv(N, TL::NW), nch_k = cdiv(K, TL::KW), chunks = nch_n * nch_k;
  const size_t lds_fixed = 2 * (size_t)TL::KW * 4 + 4 * (size_t)TL::WAVE_BYTES;
  static const int resident = [&] {
    int dev = 0, cus = 256, per_cu = 2;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds_fixed) != hipSuccess || per_cu < 1)
      per_cu = 1;
    return std::max(1, cus * per_cu);
  }();
  const int64_t unit = 4 * TL::R;  // one sweep of the 4 waves
  int64_t parts = std::max<int64_t>(1, std::min<int64_t>(std::max(1, resident / chunks), cdiv64(M, unit)));
  parts = std::min<int64_t>(parts, std::max<int64_t>(1, slab_cap / ((int64_t)N * K)));
  const int64_t rpp = cdiv64(cdiv64(M, parts), unit) * unit;
  parts = cdiv64(M, rpp);
  int gate_frames = 0;
  if (MODE == PRO_BN_SILU_G) {
    gate_frames = (int)std::min<int64_t>(cdiv64(M, pro.rows_per_frame), cdiv64(rpp, pro.rows_per_frame) + 1);
    if (gate_frames > 16) return 1;
  }
  const size_t lds = lds_fixed + (size_t)gate_frames * TL::KW * 4;
  hipLaunchKernelGGL(kern, dim3((unsigned)(parts * chunks)), dim3(256), lds, s, dY, X, M, N, K, pro, slab, nch_n,
                     nch_k, rpp, gate_frames);
  DFD_HIP_CHECK(hipGetLastError());
  return launch_reduce_slabs(s, slab, (int)parts, (int64_t)N * K, dW, accumulate);
}

// 0: launched; 1: not covered (the caller uses the tiled wgrad kernel); -1: launch error
template <typename T>
int launch_pw_wgrad_stream(hipStream_t s, const T* dY, const T* X, int64_t M, int N, int K, int pro_mode,
                           const Pro& pro, float* slab, int64_t slab_cap, float* dW, bool accumulate) {
  if (M <= 0 || M < tune(TK_STREAM_MIN_ROWS) || (N & 7) || (K & 7)) return 1;
#define DFD_WGS(NBW_, KBW_, S_, MODE_) \
  return wgs_launch<T, NBW_, KBW_, S_, MODE_>(s, dY, X, M, N, K, pro, slab, slab_cap, dW, accumulate)
  if (pro_mode == PRO_NONE) {  // conv_pw (expansion): N = mid, K = cin;  Gram x^T x: N = K = cin
    if (N == 96 && K == 16) DFD_WGS(6, 1, 2, PRO_NONE);
    if (N == 16 && K == 16) DFD_WGS(1, 1, 4, PRO_NONE);
    if (N == 24 && K == 24) DFD_WGS(2, 2, 2, PRO_NONE);
    if (N == 40 && K == 40) DFD_WGS(3, 3, 2, PRO_NONE);
    if (N == 144 && K == 24) DFD_WGS(5, 2, 2, PRO_NONE);   // N in 2 chunks of 80
    if (N == 240 && K == 40) DFD_WGS(5, 3, 1, PRO_NONE);   // N in 3 chunks of 80
    if (N == 480 && K == 80) DFD_WGS(4, 5, 1, PRO_NONE);   // 14x14 stage: N in chunks of 64 (-1 us)
    return 1;
  }
  if (pro_mode == PRO_BN_SILU_G) {  // conv_pwl: N = cout, K = mid
    if (N == 16 && K == 32) DFD_WGS(1, 2, 4, PRO_BN_SILU_G);
    if (N == 24 && K == 96) DFD_WGS(2, 6, 1, PRO_BN_SILU_G);
    if (N == 24 && K == 144) DFD_WGS(2, 5, 1, PRO_BN_SILU_G);  // K in 2 chunks of 80
    if (N == 40 && (K == 144 || K == 240)) DFD_WGS(3, 5, 1, PRO_BN_SILU_G);
    // 14x14 stage (tools/kbench, against the tiled wgrad): 80x240 31 -> 29 us, 80x480 44 -> 37 us,
    // 112x480 45 -> 38 us, 112x672 55 -> 44 us
    if (N == 80 && (K == 240 || K == 480)) DFD_WGS(5, 4, 1, PRO_BN_SILU_G);   // K in chunks of 64
    if (N == 112 && (K == 480 || K == 672)) DFD_WGS(7, 3, 1, PRO_BN_SILU_G);  // K in chunks of 48
    return 1;
  }
#undef DFD_WGS
  return 1;
}

// bf16 (the performance mode) and fp16 (v_mfma_f32_16x16x32_f16) storage
#define DFD_STREAM_INST(T)                                                                                     \
  template int launch_pw_stream<T>(hipStream_t, const T*, const T*, T*, const T*, const float*, int64_t, int, int, \
                                   int, const Pro&, float*, int*);                                             \
  template int launch_pw_wgrad_stream<T>(hipStream_t, const T*, const T*, int64_t, int, int, int, const Pro&,   \
                                         float*, int64_t, float*, bool);
DFD_STREAM_INST(bf16)
DFD_STREAM_INST(f16)
#undef DFD_STREAM_INST

}  // namespace dfd
