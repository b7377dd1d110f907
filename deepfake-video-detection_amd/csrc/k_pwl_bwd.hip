// Fused backward of an MBConv block's projection (timm conv_pwl; conv_pw of the depthwise-separable
// stage-0 block) together with the SE + BN2 backward reduction, bf16 (src/pretrained_detector.py:116
// runs the timm blocks; the step's backward is src/ensemble_trainer.py:197):
//
//   ge2[m][k]        = sum_n gs[m][n] W[n][k]                                   data gradient (stored)
//   dW[n][k]        += sum_m gs[m][n] act[m][k],  act = silu(y2*sc+sh) * gate[f][k]   weight gradient
//   part[q][h][f][k] = per-frame sums D, P1..P4 of (ge2, y2)                    (k_bn.hip FR_SEBN)
//
// gs = dL/d(y3) after the BN3 backward [M][N = cout], y2 = the pre-BN2 depthwise output [M][K = mid].
// The unfused path ran three launches over the expanded tensor -- the dgrad GEMM (writes ge2), the
// weight-gradient GEMM (reads y2) and the SE/BN reduction (reads ge2 and y2): one pass over y2 and
// one write of ge2 here instead of four passes.
//
// Workgroup = (k-chunk of KC = 16*KBC channels) x (part: a chunk of one frame, or whole frames).  Its
// rows run in frame-aligned steps of PB_R = 64 (a step never spans two frames, so the SE gate and the
// per-frame sums are uniform per step).  Per step:
//   staging   gs rows [64][NP] and y2 rows [64][KC] from registers (loaded one step ahead) into LDS:
//             gs as is (zero-padded to NP = 32*NG columns), y2 raw, and act (bf16) for the weight
//             gradient;
//   dgrad     wave w < KBC owns k-block w: the transposed tile D[k][m] = W^T[k][:] . gs[m][:]^T
//             (v_mfma_f32_16x16x32_bf16, W^T fragments preloaded in LDS), so a lane holds 4
//             consecutive channels of one row -- rounded to bf16, put into the LDS C tile, and
//             combined with the same 4 channels of y2 for the SE/BN sums (per-lane accumulators);
//   wgrad     the same wave: dW[n][k-block w] += gs^T . act over the 64 rows (two 32-deep MFMA
//             steps, operands read as columns with ds_read_b64_tr_b16);
//   store     the C tile as row-contiguous 16-B stores.
// At the end of a frame the SE/BN sums of a lane are added over the 16 lanes that share its channels
// (fixed butterfly order) and written; at the end of the part the weight-gradient tile goes to the
// part's slab row (summed in order by launch_reduce_slabs).  Deterministic throughout.
#include "kernels.h"

#include <type_traits>

namespace dfd {


typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
// two channels of a lane's four in natural lane order (x = channel 2h, y = channel 2h + 1): the BN2 /
// SE sums are written on these pairs so that every packed f32 instruction reads both operands in the
// same lane order (see the note at the epilogue)
typedef float pv2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;


template <typename T>
struct PwlBwdArgs {
  const T* gs;   // [M][N] (or, with coef3: the block's output gradient dZ, gs = k1*dZ + k2*y3 + k3)
  const T* y3;   // [M][N] pre-BN3 projection output (with coef3)
  const float* coef3;  // [3][N] BN3 backward coefficients k1, k2, k3, or nullptr (gs given)
  const T* wt;   // [K][N]: row k holds W[:, k] (the cast conv_pwl weight, transposed)
  const T* y2;   // [M][K]
  const float *sc, *sh, *mean, *invstd;  // BN2 (after the depthwise conv) [K]
  const float* gate;                     // SE gate [F][K]
  T* ge2;                                // [M][K]
  float* slab;                           // [parts][N][K]
  float* part;                           // [5][hsplit][F][K]
  int F, HW, N, K;
  int hsplit;  // > 1: part = frame * hsplit + chunk; 1: part = fpp consecutive whole frames
  int fpp;
  int nkc;     // k-chunks
};

template <int NG, int KBC, bool WG, int PB_R>
struct PbTile {
  static_assert(PB_R == 64 || PB_R == 128, "row steps of 64 or 128");
  static constexpr int NP = 32 * NG;   // cout padded to the dgrad contraction
  static constexpr int NBW = NP / 16;  // weight-gradient n-blocks
  static constexpr int KC = 16 * KBC;  // channels per k-chunk
  static constexpr int GS = NP + 8;    // LDS row stride of the gs tile (elements)
  static constexpr int XS = KC + 8;    // row stride of the act / y2 / ge2 tiles
  static constexpr int VG = NP / 8, VK = KC / 8;  // 16-B vectors per row
  static constexpr int NLG = (PB_R * VG + 255) / 256, NLK = (PB_R * VK + 255) / 256;
  static constexpr int W_BYTES = KBC * NG * 1024;
  static constexpr int G_BYTES = PB_R * GS * 2;
  static constexpr int T_BYTES = PB_R * XS * 2;
  static constexpr int SMEM = W_BYTES + G_BYTES + (WG ? 3 : 2) * T_BYTES + 5 * KC * 4 + 3 * NP * 4;
  static_assert(KBC >= 1 && KBC <= 4, "one k-block per wave");
};

template <typename T>
__device__ __forceinline__ void unpack4(uint2 v, float (&f)[4]) {
  f[0] = lo2f(v.x, (T*)nullptr);
  f[1] = hi2f(v.x, (T*)nullptr);
  f[2] = lo2f(v.y, (T*)nullptr);
  f[3] = hi2f(v.y, (T*)nullptr);
}

// WG = false: the data gradient and the SE/BN sums only (no act tile, no weight-gradient
// accumulators, any number of parts); the caller runs the weight gradient separately
// waves per SIMD the register allocation must allow (A/B builds: -DPWL_WPE=n)
#ifndef PWL_RING
#define PWL_RING 1  // 2 sets: neutral at 2 waves per SIMD, and 3 waves do not fit with it
#endif
#ifndef PWL_WPE
#define PWL_WPE 3  // with one prefetch set: 2 -> 3 waves, -13..-16 % (tools/kbench fused)
#endif
template <typename T, int NG, int KBC, bool WG, int PB_R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PWL_WPE))) void pwl_bwd_kernel(PwlBwdArgs<T> a) {
  using TL = PbTile<NG, KBC, WG, PB_R>;
  __shared__ __attribute__((aligned(16))) char smem[TL::SMEM];
  const uint4* Ws = reinterpret_cast<const uint4*>(smem);  // [KBC][NG][64] W^T fragments
  T* Gs = reinterpret_cast<T*>(smem + TL::W_BYTES);  // [R][GS]
  T* Xs = Gs + PB_R * TL::GS;                         // [R][XS] act (WG)
  T* Ys = Xs + (WG ? PB_R * TL::XS : 0);              // [R][XS] raw y2
  T* Cs = Ys + PB_R * TL::XS;                         // [R][XS] ge2
  float* co = reinterpret_cast<float*>(Cs + PB_R * TL::XS);  // [4][KC] sc sh mean invstd
  float* c3 = co + 4 * TL::KC;                                // [3][NP] BN3 k1 k2 k3 (coef3)
  float* gl = c3 + 3 * TL::NP;                                // [KC] SE gate of a one-frame part

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the k-chunks of one part (same gs rows) are dealt to one XCD: gs is fetched once per L2
  const int bid = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
  const int kc = bid % a.nkc, part = bid / a.nkc;
  const int k0 = kc * TL::KC;
  const int K = a.K, N = a.N, HW = a.HW;

  {
    uint4* w = reinterpret_cast<uint4*>(smem);
    for (int i = tid; i < KBC * NG * 64; i += 256) {
      const int ln = i & 63, ng = (i >> 6) % NG, kb = (i >> 6) / NG;
      const int k = k0 + kb * 16 + (ln & 15), n = ng * 32 + 8 * (ln >> 4);
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (k < K && n < N) v = *reinterpret_cast<const uint4*>(a.wt + (int64_t)k * N + n);
      w[i] = v;
    }
    for (int i = tid; i < TL::KC; i += 256) {
      const bool ok = k0 + i < K;
      co[i] = ok ? a.sc[k0 + i] : 0.f;
      co[TL::KC + i] = ok ? a.sh[k0 + i] : 0.f;
      co[2 * TL::KC + i] = ok ? a.mean[k0 + i] : 0.f;
      co[3 * TL::KC + i] = ok ? a.invstd[k0 + i] : 0.f;
    }
    if (a.coef3)
      for (int i = tid; i < 3 * TL::NP; i += 256) {
        const int q = i / TL::NP, n = i - q * TL::NP;
        c3[i] = n < N ? a.coef3[q * N + n] : 0.f;
      }
  }

  // the part's rows
  int fA, nf, pc0, pc1, h;
  if (a.hsplit > 1) {
    fA = part / a.hsplit;
    h = part - fA * a.hsplit;
    nf = 1;
    const int chunk = (HW + a.hsplit - 1) / a.hsplit;
    pc0 = h * chunk;
    pc1 = min(HW, pc0 + chunk);
  } else {
    fA = part * a.fpp;
    h = 0;
    nf = min(a.fpp, a.F - fA);
    pc0 = 0;
    pc1 = HW;
  }
  // a part of one frame (every dispatched shape: HW >= 2048 splits frames) reads its gate from LDS
  const bool gate_lds = nf == 1;
  if (gate_lds)
    for (int i = tid; i < TL::KC; i += 256) gl[i] = k0 + i < K ? a.gate[(int64_t)fA * K + k0 + i] : 0.f;
  const int spf = (pc1 - pc0 + PB_R - 1) / PB_R;
  const int nsteps = nf > 0 && pc1 > pc0 ? nf * spf : 0;

  // NS register sets: the rows of step st + NS are loaded while step st is staged and computed
  constexpr int NS = PWL_RING;
  Raw8<T> rg[NS][TL::NLG], r3[NS][TL::NLG], ry[NS][TL::NLK];
  const bool bn3 = a.coef3 != nullptr;
  auto load = [&](auto setc, int st) {
    constexpr int S = decltype(setc)::value;
    const int f = fA + st / spf, pb = pc0 + (st % spf) * PB_R, pe = min(pc1, pb + PB_R);
    const int64_t rb = (int64_t)f * HW + pb;
#pragma unroll
    for (int i = 0; i < TL::NLG; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VG, cv = (v - rr * TL::VG) * 8;
      const bool ok = rr < PB_R && pb + rr < pe && cv < N;
      raw_ld(rg[S][i], a.gs + (rb + rr) * N + cv, a.gs, ok);
      if (bn3) raw_ld(r3[S][i], a.y3 + (rb + rr) * N + cv, a.y3, ok);
    }
#pragma unroll
    for (int i = 0; i < TL::NLK; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VK, cv = (v - rr * TL::VK) * 8;
      raw_ld(ry[S][i], a.y2 + (rb + rr) * K + k0 + cv, a.y2, rr < PB_R && pb + rr < pe && k0 + cv < K);
    }
  };

  // per-lane constants of the 4 channels this lane holds in the transposed dgrad tile
  const bool cw = wave < KBC;
  const int kl = wave * 16 + 4 * (lane >> 4);  // local channel of r = 0
  pv2 csc[2], csh[2], cmu[2], cis[2];
  float cval[4];
  f32x4_t aw[WG ? TL::NBW : 1];
#pragma unroll
  for (int nb = 0; nb < (WG ? TL::NBW : 1); ++nb) aw[nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  pv2 se[5][2];  // [q][channel pair]
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int hp = 0; hp < 2; ++hp) se[q][hp] = pv2{0.f, 0.f};

  if (nsteps > 0) load(std::integral_constant<int, 0>{}, 0);
  if constexpr (NS == 2)
    if (nsteps > 1) load(std::integral_constant<int, NS - 1>{}, 1);
  __syncthreads();  // fragments and coefficients staged
#pragma unroll
  for (int hp = 0; hp < 2; ++hp) {
    const int c = cw ? kl + 2 * hp : 0, c1 = cw ? c + 1 : 0;
    csc[hp] = pv2{co[c], co[c1]};
    csh[hp] = pv2{co[TL::KC + c], co[TL::KC + c1]};
    cmu[hp] = pv2{co[2 * TL::KC + c], co[2 * TL::KC + c1]};
    cis[hp] = pv2{co[3 * TL::KC + c], co[3 * TL::KC + c1]};
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) cval[r] = cw && k0 + kl + r < K ? 1.f : 0.f;

  auto step = [&](auto setc, int st) {
    constexpr int S = decltype(setc)::value;
    const int f = fA + st / spf, pb = pc0 + (st % spf) * PB_R, pe = min(pc1, pb + PB_R);
    const int64_t rb = (int64_t)f * HW + pb;
    // ---- staging: gs, raw y2 and act into LDS ----
#pragma unroll
    for (int i = 0; i < TL::NLG; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VG, cv = (v - rr * TL::VG) * 8;
      if (rr < PB_R) {
        if (bn3) {  // the BN3 backward apply (bn_bwd_apply's arithmetic), rounded to bf16 like its store
          float z[8], y[8], k1[8], k2[8], k3[8];
          raw_to_f(rg[S][i], z);
          raw_to_f(r3[S][i], y);
          ld8(c3 + cv, k1);
          ld8(c3 + TL::NP + cv, k2);
          ld8(c3 + 2 * TL::NP + cv, k3);
          const uint32_t msk = rg[S][i].ok ? 0xffffffffu : 0u;
#pragma unroll
          for (int j = 0; j < 8; ++j) z[j] = k1[j] * z[j] + k2[j] * y[j] + k3[j];
          *reinterpret_cast<uint4*>(Gs + rr * TL::GS + cv) =
              make_uint4(Tr<T>::pack2(z[0], z[1]) & msk, Tr<T>::pack2(z[2], z[3]) & msk, Tr<T>::pack2(z[4], z[5]) & msk,
                         Tr<T>::pack2(z[6], z[7]) & msk);
        } else {
          raw_st(Gs + rr * TL::GS + cv, rg[S][i]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TL::NLK; ++i) {
      const int v = tid + 256 * i, rr = v / TL::VK, cv = (v - rr * TL::VK) * 8;
      if (rr < PB_R) {
        raw_st(Ys + rr * TL::XS + cv, ry[S][i]);
        if constexpr (!WG) continue;
        float x[8], sc[8], sh[8], gv[8];
        raw_to_f(ry[S][i], x);
        ld8(co + cv, sc);
        ld8(co + TL::KC + cv, sh);
        if (gate_lds) ld8(gl + cv, gv);
        else ld8f(a.gate + (int64_t)f * K + (k0 + cv < K ? k0 + cv : 0), gv);
        const uint32_t msk = ry[S][i].ok ? 0xffffffffu : 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = siluf_(x[j] * sc[j] + sh[j]) * gv[j];
        *reinterpret_cast<uint4*>(Xs + rr * TL::XS + cv) =
            make_uint4(Tr<T>::pack2(x[0], x[1]) & msk, Tr<T>::pack2(x[2], x[3]) & msk, Tr<T>::pack2(x[4], x[5]) & msk,
                       Tr<T>::pack2(x[6], x[7]) & msk);
      }
    }
    lds_barrier();
    if (st + NS < nsteps) load(setc, st + NS);  // rows NS steps ahead in flight during this step's math

    if (cw) {
      // ---- data gradient: D[k][m] = W^T[k][:] . gs[m][:]^T, 4 row blocks ----
      f32x4_t ad[PB_R / 16];
#pragma unroll
      for (int mb = 0; mb < PB_R / 16; ++mb) ad[mb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ng = 0; ng < NG; ++ng) {
        asm volatile("" ::: "memory");  // one chunk's LDS operands live at a time (occupancy)
        const bf16x8_t wf = __builtin_bit_cast(bf16x8_t, Ws[(wave * NG + ng) * 64 + lane]);
#pragma unroll
        for (int mb = 0; mb < PB_R / 16; ++mb) {
          const bf16x8_t gf = *reinterpret_cast<const bf16x8_t*>(Gs + (mb * 16 + (lane & 15)) * TL::GS + ng * 32 +
                                                                 8 * (lane >> 4));
          ad[mb] = mfma16x16x32<T>(wf, gf, ad[mb]);
        }
      }
      // ---- epilogue: bf16 ge2 into the C tile, SE/BN sums against y2 of the same 4 channels ----
      // Written on channel pairs in natural lane order (pv2).  As four scalar channels, the SLP
      // vectoriser of the fp16 instance paired y (hi, lo) against d (lo, hi) and reconciled them with
      // SWAPPED packed-f32 operand selects (v_pk_mul/fma_f32 ... op_sel:[0,1] op_sel_hi:[1,0]: the low
      // lane reads the pair's high register and the high lane its low one) -- exactly the instructions
      // feeding sum(d * silu') and sum(d * silu' * xhat), the only outputs that differed between two
      // identical launches on MI355X (16-185 entries, sign flips; profiles/r05 pwl_det_slp_r05j.txt).
      // Packed operands in one lane order leave the compiler nothing to swap (tests/test_isa_scan.py
      // checks every code object of the library for that form).
#pragma unroll
      for (int mb = 0; mb < PB_R / 16; ++mb) {
        const int m = mb * 16 + (lane & 15);
        const float rv = pb + m < pe ? 1.f : 0.f;
        const uint2 pk = make_uint2(Tr<T>::pack2(ad[mb][0], ad[mb][1]), Tr<T>::pack2(ad[mb][2], ad[mb][3]));
        *reinterpret_cast<uint2*>(Cs + m * TL::XS + kl) = pk;
        float d[4], y[4];
        unpack4<T>(pk, d);
        unpack4<T>(*reinterpret_cast<const uint2*>(Ys + m * TL::XS + kl), y);
        const pv2 rv2 = pv2{rv, rv};
#pragma unroll
        for (int hp = 0; hp < 2; ++hp) {
          const pv2 dd = pv2{d[2 * hp], d[2 * hp + 1]}, yy = pv2{y[2 * hp], y[2 * hp + 1]};
          const pv2 z = yy * csc[hp] + csh[hp];
          const pv2 sg = pv2{sigmoidf_(z.x), sigmoidf_(z.y)};
          const pv2 sp = sg * (1.0f + z * (1.0f - sg)) * rv2;
          const pv2 xh = (yy - cmu[hp]) * cis[hp];
          const pv2 dsp = dd * sp;
          se[0][hp] += dd * (z * sg);  // d = 0 on masked rows (gs rows are zero)
          se[1][hp] += dsp;
          se[2][hp] += sp;
          se[3][hp] += dsp * xh;
          se[4][hp] += sp * xh;
        }
      }
      // ---- weight gradient: dW[n][k-block] += gs^T . act over the 64 rows ----
      const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
      for (int sub = 0; sub < (WG ? PB_R / 32 : 0); ++sub) {
        const T* Gb = Gs + sub * 32 * TL::GS;
        const T* Xb = Xs + sub * 32 * TL::XS;
        const s16x4_t xlo =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Xb + (8 * g + q) * TL::XS + wave * 16 + 4 * p));
        const s16x4_t xhi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Xb + (8 * g + 4 + q) * TL::XS + wave * 16 + 4 * p));
        const bf16x8_t bfr = bf16x8_t{xlo[0], xlo[1], xlo[2], xlo[3], xhi[0], xhi[1], xhi[2], xhi[3]};
#pragma unroll
        for (int nb = 0; nb < TL::NBW; ++nb) {
          if (nb * 16 < N) {  // uniform
            const s16x4_t lo =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(Gb + (8 * g + q) * TL::GS + nb * 16 + 4 * p));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4_t*)(Gb + (8 * g + 4 + q) * TL::GS + nb * 16 + 4 * p));
            const bf16x8_t af = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            aw[WG ? nb : 0] = mfma16x16x32<T>(af, bfr, aw[WG ? nb : 0]);
          }
        }
      }
      // ---- end of a frame: the SE/BN sums of its channels ----
      if (st % spf == spf - 1) {
        const int64_t n = (int64_t)a.F * K;
        float sv[5][4];
#pragma unroll
        for (int qq = 0; qq < 5; ++qq)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = se[qq][r >> 1][r & 1];
            v += __shfl_xor(v, 1, 64);
            v += __shfl_xor(v, 2, 64);
            v += __shfl_xor(v, 4, 64);
            v += __shfl_xor(v, 8, 64);
            sv[qq][r] = v;
          }
        if ((lane & 15) == 0) {
#pragma unroll
          for (int qq = 0; qq < 5; ++qq)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (cval[r] != 0.f) a.part[((int64_t)qq * a.hsplit + h) * n + (int64_t)f * K + k0 + kl + r] = sv[qq][r];
        }
#pragma unroll
        for (int qq = 0; qq < 5; ++qq)
#pragma unroll
          for (int hp = 0; hp < 2; ++hp) se[qq][hp] = pv2{0.f, 0.f};
      }
    }
    lds_barrier();  // C tile complete; every read of this step's Gs / Xs / Ys done
    // ---- ge2: row-contiguous 16-B stores ----
    for (int v = tid; v < PB_R * TL::VK; v += 256) {
      const int rr = v / TL::VK, cv = (v - rr * TL::VK) * 8;
      if (pb + rr < pe && k0 + cv < K)
        *reinterpret_cast<uint4*>(a.ge2 + (rb + rr) * K + k0 + cv) =
            *reinterpret_cast<const uint4*>(Cs + rr * TL::XS + cv);
    }
  };
  for (int st = 0; st < nsteps; st += NS) {
    step(std::integral_constant<int, 0>{}, st);
    if constexpr (NS == 2)
      if (st + 1 < nsteps) step(std::integral_constant<int, NS - 1>{}, st + 1);
  }

  // ---- this part's weight-gradient rows: dW[n][k] of the wave's k-block ----
  if (WG && cw) {
    float* out = a.slab + (int64_t)part * N * K;
    const int k = k0 + wave * 16 + (lane & 15);
#pragma unroll
    for (int nb = 0; nb < (WG ? TL::NBW : 0); ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nn = nb * 16 + 4 * (lane >> 4) + r;
        if (nn < N && k < K) out[(int64_t)nn * K + k] = aw[WG ? nb : 0][r];
      }
  }
}

template <int NG, int KBC, bool WG, int PB_R, typename T>
static int pb_launch(hipStream_t s, PwlBwdArgs<T>& a, int64_t slab_cap, float* dW, bool accumulate, int64_t part_cap,
                     int* hsplit_out) {
  using TL = PbTile<NG, KBC, WG, PB_R>;
  auto kern = pwl_bwd_kernel<T, NG, KBC, WG, PB_R>;
  a.nkc = cdiv(a.K, TL::KC);
  const int64_t per = WG ? (int64_t)a.N * a.K : 0;  // slab floats per part
  int64_t parts;
  if (a.HW >= 2048) {
    // large maps: chunks of a frame (>= 8 steps each); the chunk count minimising dispatch rounds x
    // steps per workgroup (rounds of the co-resident grid): blocks.0.0 (nkc 1) in 3 chunks = one
    // round of 66 steps instead of 4 chunks = 1.3 rounds of 49
    static const int resident = [] {
      int dev = 0, cus = 256, per_cu = 1;
      if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pwl_bwd_kernel<T, NG, KBC, WG, PB_R>, 256, 0) != hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      return std::max(1, cus * per_cu);
    }();
    a.hsplit = 1;
    int64_t best = -1;
    for (int hs = 1; a.HW / hs >= 8 * PB_R; ++hs) {
      if ((int64_t)a.F * hs * per > slab_cap || 5 * (int64_t)hs * a.F * a.K > part_cap) break;
      if (cdiv(a.HW, hs) * (hs - 1) >= a.HW) continue;  // every chunk non-empty (each writes its sums)
      const int64_t wgs = (int64_t)a.F * hs * a.nkc;
      const int64_t cost = cdiv64(wgs, resident) * cdiv(cdiv(a.HW, hs), PB_R);
      if (best < 0 || cost < best) { best = cost; a.hsplit = hs; }
    }
    a.fpp = 1;
    parts = (int64_t)a.F * a.hsplit;
  } else {
    // whole frames per part: ~1024-2048 workgroups (each loads the chunk's weight fragments once);
    // with the weight gradient, as many parts as the slab holds
    a.hsplit = 1;
    const int64_t want = std::max<int64_t>(1, std::min<int64_t>(a.F, cdiv64(WG ? 1024 : 2048, a.nkc)));
    const int64_t cap = WG ? std::max<int64_t>(1, slab_cap / per) : want;
    a.fpp = (int)cdiv64(a.F, std::min(want, cap));
    parts = cdiv64(a.F, a.fpp);
  }
  if (parts * per > slab_cap || 5 * (int64_t)a.hsplit * a.F * a.K > part_cap) return 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)(parts * a.nkc)), dim3(256), 0, s, a);
  DFD_HIP_CHECK(hipGetLastError());
  *hsplit_out = a.hsplit;
  if (!WG) return 2;
  return launch_reduce_slabs(s, a.slab, (int)parts, per, dW, accumulate);
}

// 0: launched (all three outputs); 2: launched without the weight gradient (the caller runs it);
// 1: shape not covered (the caller runs the three unfused launches); -1: error
bool pwl_bwd_covers(int frames, int HW, int N, int K) {
  return frames > 0 && HW > 0 && !(N & 7) && !(K & 15) && N <= 24 && (int64_t)frames * HW * std::max(N, K) < (1ll << 31);
}

template <typename T>
int launch_pwl_bwd(hipStream_t s, const T* gs, const T* y3, const float* coef3, const T* wt, const T* y2,
                   const float* sc, const float* sh, const float* mean, const float* invstd, const float* gate,
                   int frames, int HW, int N, int K, T* ge2, float* slab, int64_t slab_cap, float* dW,
                   bool accumulate, float* part, int64_t part_cap, int* hsplit) {
  if (!pwl_bwd_covers(frames, HW, N, K) || (coef3 && !y3)) return 1;
  PwlBwdArgs<T> a{gs, y3, coef3, wt, y2, sc, sh, mean, invstd, gate, ge2, slab, part, frames, HW, N, K, 1, 1, 1};
  const int ng = cdiv(N, 32);
  const int kbc = K <= 32 ? 2 : 3;
  // 64-row steps: 128-row steps doubled the staging registers to one wave per SIMD and measured
  // 1.3-1.5x slower on every shape (tools/kbench fused)
#define DFD_PB(NG_, KBC_, WG_) \
  if (ng == NG_ && kbc == KBC_) return pb_launch<NG_, KBC_, WG_, 64>(s, a, slab_cap, dW, accumulate, part_cap, hsplit)
  // measured (rocprof, 256 frames): a win only where cout <= 24 (blocks.0.0 231 -> 187 us,
  // blocks.1.1 263 -> 217 us against the three unfused launches).  Wider projections keep the
  // unfused launches: with the weight gradient the k-chunked workgroups re-read gs and the slab caps
  // the parts (blocks.6.0: 88 -> 351 us); without it (data gradient + SE/BN sums only, two passes
  // instead of three) every shape was still slower than the dgrad GEMM + frame_reduce pair it
  // replaces (blocks.6.0 47 -> 132 us, blocks.4.1 51 -> 89 us, blocks.2.1 62 -> 81 us)
  if (N <= 24) {
    DFD_PB(1, 2, true);  // stage 0: 32 -> 16
    DFD_PB(1, 3, true);  // 96/144 -> 24
  }
#undef DFD_PB
  return 1;
}
#define DFD_PWL_INST(T)                                                                                        \
  template int launch_pwl_bwd<T>(hipStream_t, const T*, const T*, const float*, const T*, const T*, const float*, \
                                 const float*, const float*, const float*, const float*, int, int, int, int, T*,   \
                                 float*, int64_t, float*, bool, float*, int64_t, int*);
DFD_PWL_INST(bf16)
DFD_PWL_INST(f16)
#undef DFD_PWL_INST

}  // namespace dfd
