// Fused backward of an MBConv expansion conv (timm conv_pw) through its BatchNorm on the
// high-resolution blocks, bf16 (src/pretrained_detector.py:116 runs the timm blocks).
//
// The BN after conv_pw has the input gradient ge1 = k1*g + k2*y1 + k3 and y1 = x . W^T, so by
// linearity (bn_fold_pw, k_bn.hip) the conv's gradients need only g and the block input x:
//   dX  = g . W1t^T + x . Q^T + bv (+ the block's skip gradient)     W1t = diag(k1) W (as [cin][mid])
//   dW  = diag(k1) T + diag(k2) W G + k3 cs^T                        (pw_wgrad_bn_combine)
//   T   = g^T x   [mid][cin],   G = x^T x   [cin][cin],   cs = 1^T x   [cin]
// The unfused fold path ran five launches over these rows: x . Q (tf GEMM, writing an intermediate),
// the data-gradient GEMM, and three weight-gradient products (g^T x, x^T x, column sums).  Here one
// pass reads every g and x row once and writes dX once; T, G and cs leave as per-part slab rows
// (summed in order by launch_reduce_slabs).
//
// Workgroup = a contiguous range of rows, all channels.  Per 64-row step:
//   staging  g rows [64][MP] (zero-padded to MP = 32*MB), x rows [64][CP] with a ones column at
//            index cin (so G's row cin is cs), the skip gradient rows [64][cin] -- registers (loaded a
//            step ahead) into LDS;
//   dgrad    wave w owns rows 16w..16w+15: D[c][m] = [W1t | Q][c][:] . [g | x][m][:]^T, one MFMA
//            chain over the mid + CP contraction (fragments of W1t and Q preloaded in LDS), so a lane
//            holds 4 consecutive channels of one row; + bv + skip, rounded to bf16, into the LDS C tile;
//   wgrad    T blocks (k-block kb = w, w+4, ..) and G blocks (round-robin) += over the 64 rows (two
//            32-deep MFMA steps, operands read as columns with ds_read_b64_tr_b16);
//   store    the C tile as row-contiguous stores.
// Deterministic: fixed summation orders throughout.
#include "kernels.h"

namespace dfd {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;


template <typename T>
struct PwFoldArgs {
  const T* g;        // [M][mid]
  const T* x;        // [M][cin]
  const T* r;        // [M][cin] skip gradient or nullptr
  const T* w1t;      // [cin][mid]
  const T* q;        // [cin][cin]
  const float* bv;   // [cin]
  T* dx;             // [M][cin]
  float *slabT, *slabG, *slabC;  // [parts][mid*cin], [parts][cin*cin], [parts][cin]
  int64_t M, rows_per_part;
  int mid, cin;
};

template <int MB, int CB, int R>
struct PfTile {
  static_assert(R == 64 || R == 128, "row steps of 64 or 128");
  static constexpr int MP = 32 * MB;                   // mid padded to the contraction
  static constexpr int CP = CB * 16 + 1 <= 32 ? 32 : 64;  // cin + the ones column, padded
  static constexpr int CX = CP / 32;
  static constexpr int NC = MB + CX;                   // dgrad contraction chunks of 32
  static constexpr int GS = MP + 8, XS = CP + 8, RS = CB * 16 + 8;  // LDS row strides (elements)
  static constexpr int VG = MP / 8, VX = CP / 8, VR = CB * 2;       // 16-B vectors per row
  static constexpr int NLG = (R * VG + 255) / 256, NLX = (R * VX + 255) / 256;
  static constexpr int NLR = (R * VR + 255) / 256;
  static constexpr int KPW = (2 * MB + 3) / 4;          // T k-blocks per wave
  static constexpr int GI = CP / 16;                    // G row blocks (cin + ones)
  static constexpr int GPW = (GI * CB + 3) / 4;         // G blocks per wave
  static constexpr int W_BYTES = CB * NC * 1024;
  static constexpr int SMEM = W_BYTES + R * (GS + XS + RS) * 2 + CB * 16 * 4;
};

// waves per SIMD the register allocation must allow (A/B builds: -DPF_WPE=n)
#ifndef PF_WPE
#define PF_WPE 3  // 144-wide: 2 -> 3 waves, 141 -> 135 us without the skip (tools/kbench fused)
#endif
template <typename T, int MB, int CB, bool RES, int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PF_WPE))) void pw_fold_bwd_kernel(PwFoldArgs<T> a) {
  using TL = PfTile<MB, CB, R>;
  __shared__ __attribute__((aligned(16))) char smem[TL::SMEM];
  const uint4* Wf = reinterpret_cast<const uint4*>(smem);  // [CB][NC][64] fragments of [W1t | Q]
  T* Gs = reinterpret_cast<T*>(smem + TL::W_BYTES);   // [R][GS]
  T* Xs = Gs + R * TL::GS;                          // [R][XS] (+ ones column)
  T* Rt = Xs + R * TL::XS;                          // [R][RS] skip gradient in, dX out
  float* bvl = reinterpret_cast<float*>(Rt + R * TL::RS);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mid = a.mid, cin = a.cin;
  const int64_t mbeg = (int64_t)blockIdx.x * a.rows_per_part, mend = min(a.M, mbeg + a.rows_per_part);
  {
    uint4* w = reinterpret_cast<uint4*>(smem);
    for (int i = tid; i < CB * TL::NC * 64; i += 256) {
      const int ln = i & 63, ch = (i >> 6) % TL::NC, cb = (i >> 6) / TL::NC;
      const int c = cb * 16 + (ln & 15), kk = 8 * (ln >> 4);
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (ch < MB) {
        const int k = ch * 32 + kk;
        if (c < cin && k < mid) v = *reinterpret_cast<const uint4*>(a.w1t + (int64_t)c * mid + k);
      } else {
        const int k = (ch - MB) * 32 + kk;
        if (c < cin && k < cin) v = *reinterpret_cast<const uint4*>(a.q + (int64_t)c * cin + k);
      }
      w[i] = v;
    }
    for (int i = tid; i < CB * 16; i += 256) bvl[i] = i < cin ? a.bv[i] : 0.f;
  }

  Raw8<T> rg[TL::NLG], rx[TL::NLX], rr8[RES ? TL::NLR : 1];
  auto load = [&](int64_t m0) {
#pragma unroll
    for (int i = 0; i < TL::NLG; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VG, cv = (v - rr * TL::VG) * 8;
      raw_ld(rg[i], a.g + (m0 + rr) * mid + cv, a.g, rr < R && m0 + rr < mend && cv < mid);
    }
#pragma unroll
    for (int i = 0; i < TL::NLX; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VX, cv = (v - rr * TL::VX) * 8;
      raw_ld(rx[i], a.x + (m0 + rr) * cin + cv, a.x, rr < R && m0 + rr < mend && cv < cin);
    }
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < TL::NLR; ++i) {
        const int v = tid + 256 * i, rr = v / TL::VR, cv = (v - rr * TL::VR) * 8;
        raw_ld(rr8[i], a.r + (m0 + rr) * cin + cv, a.r, rr < R && m0 + rr < mend && cv < cin);
      }
    }
  };

  f32x4_t aT[TL::KPW][CB], aG[TL::GPW];
#pragma unroll
  for (int i = 0; i < TL::KPW; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) aT[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < TL::GPW; ++i) aG[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int kbt = (mid + 15) / 16;  // T k-blocks
  const int gib = (cin + 16) / 16;  // G row blocks: channels 0..cin (cin = the ones column)

  if (mbeg < mend) load(mbeg);
  __syncthreads();
  for (int64_t m0 = mbeg; m0 < mend; m0 += R) {
    // ---- staging ----
#pragma unroll
    for (int i = 0; i < TL::NLG; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VG, cv = (v - rr * TL::VG) * 8;
      if (rr < R) raw_st(Gs + rr * TL::GS + cv, rg[i]);
    }
#pragma unroll
    for (int i = 0; i < TL::NLX; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VX, cv = (v - rr * TL::VX) * 8;
      if (rr < R) {
        uint4 o = make_uint4(0u, 0u, 0u, 0u);
        if (rx[i].ok) o = rx[i].a;
        // the ones column (index cin) of the valid rows: G's row cin becomes the column sums
        if (cv <= cin && cin < cv + 8 && m0 + rr < mend) {
          const int j = cin - cv;
          constexpr uint32_t kOne = std::is_same<T, f16>::value ? 0x3c00u : 0x3f80u;  // 1.0 in the storage type
          const uint32_t one = kOne << ((j & 1) * 16);
          if ((j >> 1) == 0) o.x |= one;
          else if ((j >> 1) == 1) o.y |= one;
          else if ((j >> 1) == 2) o.z |= one;
          else o.w |= one;
        }
        *reinterpret_cast<uint4*>(Xs + rr * TL::XS + cv) = o;
      }
    }
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < TL::NLR; ++i) {
        const int v = tid + 256 * i, rr = v / TL::VR, cv = (v - rr * TL::VR) * 8;
        if (rr < R) raw_st(Rt + rr * TL::RS + cv, rr8[i]);
      }
    }
    lds_barrier();
    if (m0 + R < mend) load(m0 + R);

    // ---- data gradient: the wave's 16-row blocks (w, w + 4, ..), all output channels ----
    auto dgrad_epi = [&](const f32x4_t& acc, int m, int cb) {
      // the ones column met Q's zero column cin (Q is only cin wide): no contribution
      const int c = cb * 16 + 4 * (lane >> 4);
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = acc[j] + bvl[c + j];
      if constexpr (RES) {
        const uint2 rv = *reinterpret_cast<const uint2*>(Rt + m * TL::RS + c);
        v[0] += lo2f(rv.x, (T*)nullptr);
        v[1] += hi2f(rv.x, (T*)nullptr);
        v[2] += lo2f(rv.y, (T*)nullptr);
        v[3] += hi2f(rv.y, (T*)nullptr);
      }
      *reinterpret_cast<uint2*>(Rt + m * TL::RS + c) = make_uint2(Tr<T>::pack2(v[0], v[1]), Tr<T>::pack2(v[2], v[3]));
    };
#pragma unroll
    for (int mj = 0; mj < R / 64; ++mj) {
      f32x4_t ad[CB];
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) ad[cb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int m = (wave + 4 * mj) * 16 + (lane & 15);
#pragma unroll
      for (int ch = 0; ch < TL::NC; ++ch) {
        asm volatile("" ::: "memory");  // one chunk's LDS operands live at a time (occupancy)
        const bf16x8_t bf = ch < MB ? *reinterpret_cast<const bf16x8_t*>(Gs + m * TL::GS + ch * 32 + 8 * (lane >> 4))
                                    : *reinterpret_cast<const bf16x8_t*>(Xs + m * TL::XS + (ch - MB) * 32 +
                                                                          8 * (lane >> 4));
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          ad[cb] = mfma16x16x32<T>(__builtin_bit_cast(bf16x8_t, Wf[(cb * TL::NC + ch) * 64 + lane]), bf, ad[cb]);
      }
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) dgrad_epi(ad[cb], m, cb);
    }

    // ---- weight-gradient products over the step's rows ----
    {
      const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
      for (int sub = 0; sub < R / 32; ++sub) {
        const T* Gb = Gs + sub * 32 * TL::GS;
        const T* Xb = Xs + sub * 32 * TL::XS;
        auto trx = [&](const T* base, int stride, int col) {
          const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + (8 * gq + q) * stride + col + 4 * p));
          const s16x4_t hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + (8 * gq + 4 + q) * stride + col + 4 * p));
          return bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        };
        bf16x8_t xc[CB];
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) xc[cb] = trx(Xb, TL::XS, cb * 16);
#pragma unroll
        for (int i = 0; i < TL::KPW; ++i) {
          const int kb = wave + 4 * i;
          if (kb < kbt) {  // uniform
            const bf16x8_t gk = trx(Gb, TL::GS, kb * 16);
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) aT[i][cb] = mfma16x16x32<T>(gk, xc[cb], aT[i][cb]);
          }
        }
#pragma unroll
        for (int i = 0; i < TL::GPW; ++i) {
          const int b = wave + 4 * i, gi = b / CB, gj = b - gi * CB;
          if (gi < gib) {  // uniform
            const bf16x8_t xr = trx(Xb, TL::XS, gi * 16);
            aG[i] = mfma16x16x32<T>(xr, xc[gj], aG[i]);
          }
        }
      }
    }
    lds_barrier();  // C tile complete; every read of this step's Gs / Xs done
    // ---- dX rows ----
    for (int v = tid; v < R * TL::VR; v += 256) {
      const int rr = v / TL::VR, cv = (v - rr * TL::VR) * 8;
      if (m0 + rr < mend && cv < cin)
        *reinterpret_cast<uint4*>(a.dx + (m0 + rr) * cin + cv) = *reinterpret_cast<const uint4*>(Rt + rr * TL::RS + cv);
    }
    lds_barrier();  // Rt is re-staged by the next step (the prefetched loads stay in flight)
  }

  // ---- this part's slab rows: T[k][c] (k < mid, c < cin), G[c][c'] (c < cin), cs[c'] (G row cin) ----
  const int64_t pidx = blockIdx.x;
#pragma unroll
  for (int i = 0; i < TL::KPW; ++i) {
    const int kb = wave + 4 * i;
    if (kb < kbt) {
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = kb * 16 + 4 * (lane >> 4) + r, c = cb * 16 + (lane & 15);
          if (k < mid && c < cin) a.slabT[pidx * mid * cin + (int64_t)k * cin + c] = aT[i][cb][r];
        }
    }
  }
#pragma unroll
  for (int i = 0; i < TL::GPW; ++i) {
    const int b = wave + 4 * i, gi = b / CB, gj = b - gi * CB;
    if (gi < gib) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = gi * 16 + 4 * (lane >> 4) + r, c2 = gj * 16 + (lane & 15);
        if (c2 < cin) {
          if (c < cin) a.slabG[pidx * cin * cin + (int64_t)c * cin + c2] = aG[i][r];
          else if (c == cin) a.slabC[pidx * cin + c2] = aG[i][r];
        }
      }
    }
  }
}

template <int MB, int CB, int R, typename E>
static int pf_launch(hipStream_t s, PwFoldArgs<E>& a, float* slab, int64_t slab_cap, float* T, float* G, float* cs) {
  const int64_t per = (int64_t)a.mid * a.cin + (int64_t)a.cin * a.cin + a.cin;
  // one dispatch wave: as many parts as workgroups are co-resident (no partial second round), at
  // most what the slab holds
  static const int resident = [] {
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pw_fold_bwd_kernel<E, MB, CB, true, R>, 256, 0) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    return std::max(1, cus * per_cu);
  }();
  int64_t parts = std::min<int64_t>(resident, std::max<int64_t>(1, slab_cap / per));
  parts = std::min<int64_t>(parts, cdiv64(a.M, R));
  a.rows_per_part = cdiv64(cdiv64(a.M, parts), R) * R;
  parts = cdiv64(a.M, a.rows_per_part);
  a.slabT = slab;
  a.slabG = slab + parts * a.mid * a.cin;
  a.slabC = a.slabG + parts * a.cin * a.cin;
  if (a.r)
    hipLaunchKernelGGL((pw_fold_bwd_kernel<E, MB, CB, true, R>), dim3((unsigned)parts), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((pw_fold_bwd_kernel<E, MB, CB, false, R>), dim3((unsigned)parts), dim3(256), 0, s, a);
  DFD_HIP_CHECK(hipGetLastError());
  DFD_TRY(launch_reduce_slabs(s, a.slabT, (int)parts, (int64_t)a.mid * a.cin, T, false));
  DFD_TRY(launch_reduce_slabs(s, a.slabG, (int)parts, (int64_t)a.cin * a.cin, G, false));
  return launch_reduce_slabs(s, a.slabC, (int)parts, a.cin, cs, false);
}

// 0: launched; 1: shape not covered (the caller runs the unfused fold launches); -1: error
template <typename E>
int launch_pw_fold_bwd(hipStream_t s, const E* g, const E* x, const E* r, const E* w1t, const E* q, const float* bv,
                       E* dx, int64_t M, int mid, int cin, float* slab, int64_t slab_cap, float* T, float* G,
                       float* cs) {
  // measured (rocprof, 256 frames, against the five unfused launches): blocks.1.0 430 -> 179 us,
  // blocks.1.1 / 2.0 194 / 183 -> 112 us
  if (M <= 0 || (mid & 7) || (cin & 7) || mid > 160 || cin > 48 || M * std::max(mid, cin) >= (1ll << 31)) return 1;
  PwFoldArgs<E> a{g, x, r, w1t, q, bv, dx, nullptr, nullptr, nullptr, M, 0, mid, cin};
  const int mb = cdiv(mid, 32), cb = cdiv(cin, 16);
  // 64-row steps (128: 1.1-1.8x slower, one wave per SIMD on the 144-wide shapes; tools/kbench fused);
  // the 240-wide shapes (blocks.2.1, 3.0: 40 -> 240) stay on the unfused launches: in 64-row steps
  // 319 registers, one wave per SIMD, 125 -> 199 us on blocks.2.1; in 32-row steps (one accumulator
  // per 16x16 unit) 125 -> 220 us with the skip, 119 -> 133 us without (tools/kbench fused)
#define DFD_PF(MB_, CB_, R_) \
  if (mb == MB_ && cb == CB_) return pf_launch<MB_, CB_, R_>(s, a, slab, slab_cap, T, G, cs)
  DFD_PF(3, 1, 64);  // blocks.1.0: 16 -> 96
  DFD_PF(5, 2, 64);  // blocks.1.1, 2.0: 24 -> 144
#undef DFD_PF
  return 1;
}
template int launch_pw_fold_bwd<bf16>(hipStream_t, const bf16*, const bf16*, const bf16*, const bf16*, const bf16*,
                                      const float*, bf16*, int64_t, int, int, float*, int64_t, float*, float*, float*);
template int launch_pw_fold_bwd<f16>(hipStream_t, const f16*, const f16*, const f16*, const f16*, const f16*,
                                     const float*, f16*, int64_t, int, int, float*, int64_t, float*, float*, float*);

}  // namespace dfd
