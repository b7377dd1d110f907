// Fused depthwise-conv backward: input gradient, the producer's BN+SiLU backward reduction and
// the weight gradient in ONE pass over (dY, y) per input tile (timm conv_dw inside the MBConv
// blocks run by self.backbone(x_flat), src/pretrained_detector.py:116):
//   dA[p]      = sum_{tap} dY[o(p, tap)] * w[tap]               (o = (p + pad - tap) / S, exact only)
//   g[p]       = dA[p] * silu'(y[p]*scale + shift)               -> out, and stats += [g, g*xhat]
//   dW[tap]   += silu(y[p]*scale + shift) * dY[o(p, tap)]        (every (o, tap) pair is met once)
// The separate dgrad and wgrad kernels read dY and y twice and stage the same tiles twice; here
// the dY tile (+halo) is staged once into LDS and each (pixel, tap) product feeds both sums.
//
// Thread = (channel vector of VW channels, pixel slot); a thread visits P pixels of the tile.
// Stride 2: a thread's pixels share their row and column parity, so only the taps of that
// parity class are valid for it (k3: <= 2x2, k5: <= 3x3) and its weight-gradient accumulators
// are NA x NA x VW registers.  Stride 1 uses VW = 4 (k5: 25 x 4 accumulators) except
// the 8x28 tile (VW = 8); fewer registers there buy co-resident workgroups.  At the end the
// accumulators are reduced over the lanes of a class (shuffles), then over the 4 waves in a fixed
// order (LDS) into the workgroup's slab row (summed by the deterministic slab reducer).
#include "dw_common.h"

#include <atomic>

// which tiles bound the tap loop's LDS-read hoisting to one kernel row (compiler fence per row):
// 1 = k5 stride 1 (without it the 14x14 k5 tile spills), 2 = k3 stride 1, 4 = stride 2
#ifndef DFD_DWB_ROWFENCE
#define DFD_DWB_ROWFENCE 1
#endif
#ifndef DFD_DWB_ALT
#define DFD_DWB_ALT 0  // tile-choice A/B knob (bits: see launch_dw_bwd)
#endif
#ifndef DFD_DWB_PF1
#define DFD_DWB_PF1 1  // bit mask of the stride-1 tiles that also prefetch the next tile (A/B knob)
#endif
namespace dfd {

// 1: fused (default); 0: the two kernels (dgrad, wgrad)
bool dw_bwd_fused_enabled() { return tune(TK_DW_BWD_FUSED) != 0; }
// 1: the stride-1 blocks take dw_bwd1_kernel (k_dw_bwd1.hip) with both BN backward passes fused

bool dw_bwd1_enabled() {
  return dw_bwd_fused_enabled() && tune(TK_DW_BWD1) != 0;
}
// 1: the stride-1 forward takes dw_fwd1_kernel (k_dw_fwd1.hip, channel pairs)
bool dw_fwd1_enabled() { return tune(TK_DW_FWD1) != 0; }

template <int TH, int TW, int K, int S, int VW>
struct DwB {
  static constexpr int NV = DCG / VW;   // channel vectors per 32-channel group
  static constexpr int NPT = 256 / NV;  // pixel slots
  static constexpr int NPX = TH * TW;
  static constexpr int P = (NPX + NPT - 1) / NPT;
  static constexpr int GH = (TH - 1 + K - 1) / S + 2, GW = (TW - 1 + K - 1) / S + 2, NG = GH * GW;
  static constexpr int NA = S == 1 ? K : (K + 1) / 2;  // taps per axis one thread can touch
  static constexpr int TPW = 64 / NV;                  // pixel slots per wave
  static constexpr int NCLS = S == 2 ? 4 : 1;          // tap parity classes
  static constexpr int RED = 4 * NCLS * NA * NA * DCG; // [wave][class][NA][NA][32] floats
  static constexpr int TGF = NG * DCG > RED ? NG * DCG : RED;  // LDS floats of the dY tile / scratch
  static_assert(S == 1 || ((NPT % TW) == 0 && ((NPT / TW) % 2) == 0 && (TH % 2) == 0 && (TW % 2) == 0),
                "stride 2: a thread's pixels must share their parity class");
};

// VW-channel vector load / store helpers (VW = 8: 16 B bf16 / 32 B fp32; VW = 4: 8 B / 16 B)
template <typename T, int VW> struct RawV;
template <typename T> struct RawV<T, 8> {
  Raw8<T> r;
  __device__ __forceinline__ void ld(const T* p, const T* safe, bool ok) { raw_ld(r, p, safe, ok); }
  __device__ __forceinline__ void to_f(float (&v)[8]) const { raw_to_f(r, v); }
};
template <typename T> struct RawV16x4 {  // 4 channels of a 16-bit type (bf16 / f16)
  uint2 a; bool ok;
  __device__ __forceinline__ void ld(const T* p, const T* safe, bool o) {
    a = *reinterpret_cast<const uint2*>(o ? p : safe); ok = o;
  }
  __device__ __forceinline__ void to_f(float (&v)[4]) const {
    const uint32_t m = ok ? 0xffffffffu : 0u, x = a.x & m, y = a.y & m;
    v[0] = lo2f(x, (T*)nullptr); v[1] = hi2f(x, (T*)nullptr);
    v[2] = lo2f(y, (T*)nullptr); v[3] = hi2f(y, (T*)nullptr);
  }
};
template <> struct RawV<bf16, 4> : RawV16x4<bf16> {};
template <> struct RawV<f16, 4> : RawV16x4<f16> {};
template <> struct RawV<float, 4> {
  float4 a; bool ok;
  __device__ __forceinline__ void ld(const float* p, const float* safe, bool o) {
    a = *reinterpret_cast<const float4*>(o ? p : safe); ok = o;
  }
  __device__ __forceinline__ void to_f(float (&v)[4]) const {
    v[0] = ok ? a.x : 0.f; v[1] = ok ? a.y : 0.f; v[2] = ok ? a.z : 0.f; v[3] = ok ? a.w : 0.f;
  }
};
template <int VW> __device__ __forceinline__ void ldsv(const float* p, float (&v)[VW]) {
#pragma unroll
  for (int j = 0; j < VW; j += 4) {
    const float4 q = *reinterpret_cast<const float4*>(p + j);
    v[j] = q.x; v[j + 1] = q.y; v[j + 2] = q.z; v[j + 3] = q.w;
  }
}
__device__ __forceinline__ void stv(bf16* p, const float (&v)[8]) { st8(p, v); }
__device__ __forceinline__ void stv(float* p, const float (&v)[8]) { st8(p, v); }
__device__ __forceinline__ void stv(f16* p, const float (&v)[8]) { st8(p, v); }
__device__ __forceinline__ void stv(bf16* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
}
__device__ __forceinline__ void stv(f16* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2h(v[0], v[1]), pack2h(v[2], v[3]));
}
__device__ __forceinline__ void stv(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

template <typename T, int TH, int TW, int K, int S, int VW, bool PF>
__global__ __launch_bounds__(256, 2) void dw_bwd_kernel(DwGeom g, const T* __restrict__ dY, const float* __restrict__ w,
                                                     T* __restrict__ out, const T* __restrict__ Yp, BnBwdIn bn,
                                                     float* __restrict__ stats, float* __restrict__ slab, int ntiles,
                                                     int groups, int tiles_x, int tiles_y) {
  using D = DwB<TH, TW, K, S, VW>;
  constexpr int NA = D::NA;
  __shared__ __attribute__((aligned(16))) float tg[D::TGF];  // dY tile; the reduction scratch at the end
  __shared__ __attribute__((aligned(16))) float wts[K * K * DCG];
  __shared__ __attribute__((aligned(16))) float bnc[4][DCG];  // producer BN scale, shift, mean, invstd
  const int tid = threadIdx.x, vec = tid % D::NV, tp = tid / D::NV;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = blockIdx.x % groups;
  const int c0 = grp * DCG, C = g.C;
  const int c = c0 + vec * VW;
  const bool cok = c < C;
  const int c8 = c0 + (tid & 3) * 8;  // the dY staging's own 8-channel mapping
  const bool cok8 = c8 < C;
  for (int i = tid; i < K * K * DCG; i += 256) {
    const int tap = i / DCG, cl = i - tap * DCG;
    wts[i] = (c0 + cl < C) ? w[(int64_t)(c0 + cl) * K * K + tap] : 0.f;
  }
  if (tid < DCG) {
    const bool ok = c0 + tid < C;
    bnc[0][tid] = ok ? bn.scale[c0 + tid] : 1.f;
    bnc[1][tid] = ok ? bn.shift[c0 + tid] : 0.f;
    bnc[2][tid] = ok ? bn.mean[c0 + tid] : 0.f;
    bnc[3][tid] = ok ? bn.invstd[c0 + tid] : 1.f;
  }
  // parity class of this thread's pixels (tile origins are even for stride 2)
  const int kh0 = S == 2 ? (((tp / TW) + g.pad) & 1) : 0, kw0 = S == 2 ? (((tp % TW) + g.pad) & 1) : 0;
  const int nah = S == 2 ? (K - kh0 + 1) / 2 : K, naw = S == 2 ? (K - kw0 + 1) / 2 : K;

  float accw[NA][NA][VW];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NA; ++b)
#pragma unroll
      for (int j = 0; j < VW; ++j) accw[a][b][j] = 0.f;
  float st_s[VW], st_q[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }

  const int tpf = tiles_x * tiles_y;
  const int tstep = gridDim.x / groups;
  // one tile's global loads -- the dY tile (+halo, 8-channel vectors for the LDS staging) and the
  // producer values of this thread's P pixels -- issued together; with PF the next tile's are in
  // flight while the current tile computes
  constexpr int NLD = (D::NG * 4 + 255) / 256;
  Raw8<T> rd[NLD];
  RawV<T, VW> ry[PF ? D::P : 1];  // PF: all of the next tile's pixels; else loaded per pixel below
  auto issue = [&](int t) {
    const int f = t / tpf, r = t - (t / tpf) * tpf, ty = r / tiles_x;
    const int iy0 = ty * TH, ix0 = (r - ty * tiles_x) * TW;
    const int gy0 = floordiv(iy0 + g.pad - (K - 1), S), gx0 = floordiv(ix0 + g.pad - (K - 1), S);
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = tid + 256 * i, pixl = e >> 2;
      const int oy = gy0 + pixl / D::GW, ox = gx0 + pixl % D::GW;
      const bool in = t < ntiles && pixl < D::NG && cok8 && oy >= 0 && oy < g.Ho && ox >= 0 && ox < g.Wo;
      raw_ld(rd[i], dY + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * C + c8, dY, in);
    }
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < D::P; ++i) {
        const int p = tp + D::NPT * i;
        const int iy = iy0 + p / TW, ix = ix0 + (p - (p / TW) * TW);
        const bool ok = t < ntiles && p < D::NPX && iy < g.H && ix < g.W && cok;
        ry[i].ld(Yp + (((int64_t)f * g.H + iy) * g.W + ix) * C + c, Yp, ok);
      }
    }
  };
  int t = blockIdx.x / groups;
  if (PF && t < ntiles) issue(t);
  for (; t < ntiles; t += tstep) {
    const int f = t / tpf, r = t - (t / tpf) * tpf;
    const int ty = r / tiles_x, tx = r - (r / tiles_x) * tiles_x;
    const int iy0 = ty * TH, ix0 = tx * TW;
    const int gy0 = floordiv(iy0 + g.pad - (K - 1), S), gx0 = floordiv(ix0 + g.pad - (K - 1), S);
    if (!PF) issue(t);
    lds_barrier();  // the previous tile's pixels are done with tg
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = tid + 256 * i, pixl = e >> 2;
      if (pixl < D::NG) {
        float x[8];
        raw_to_f(rd[i], x);
        st8(tg + pixl * DCG + (tid & 3) * 8, x);
      }
    }
    RawV<T, VW> ryc[PF ? D::P : 1];
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < D::P; ++i) ryc[i] = ry[i];
    } else {  // without the tile prefetch (register budget): pixel i+1's load flies during pixel i
      const int iy = iy0 + tp / TW, ix = ix0 + tp % TW;
      ryc[0].ld(Yp + (((int64_t)f * g.H + iy) * g.W + ix) * C + c, Yp, tp < D::NPX && iy < g.H && ix < g.W && cok);
    }
    lds_barrier();
    if (PF && t + tstep < ntiles) issue(t + tstep);
    // one input pixel: taps -> g (+ stats) and the weight-gradient sums
    auto pixel = [&](int i, const RawV<T, VW>& ryi) {
      const int p = tp + D::NPT * i;
      const int iy = iy0 + p / TW, ix = ix0 + (p - (p / TW) * TW);
      const bool ok = p < D::NPX && iy < g.H && ix < g.W && cok;
      if (ok) {
        float y[VW], av[VW], sp[VW], acc[VW], sc[VW], sh[VW];
        ryi.to_f(y);
        ldsv<VW>(&bnc[0][vec * VW], sc);
        ldsv<VW>(&bnc[1][vec * VW], sh);
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          const float z = y[j] * sc[j] + sh[j];
          const float sg = sigmoidf_(z);
          av[j] = z * sg;
          sp[j] = sg * (1.0f + z * (1.0f - sg));
          acc[j] = 0.f;
        }
#pragma unroll
        for (int ah = 0; ah < NA; ++ah) {
          if (ah >= nah) break;
          if constexpr ((DFD_DWB_ROWFENCE & (S == 2 ? 4 : K == 5 ? 1 : 2)) != 0)
            asm volatile("" ::: "memory");  // one kernel row's LDS reads in flight at a time
          const int kh = kh0 + S * ah;
          const int tyv = iy + g.pad - kh;
          const int gyl = (S == 2 ? (tyv >> 1) : tyv) - gy0;
#pragma unroll
          for (int aw = 0; aw < NA; ++aw) {
            if (aw >= naw) break;
            const int kw = kw0 + S * aw;
            const int txv = ix + g.pad - kw;
            const int gxl = (S == 2 ? (txv >> 1) : txv) - gx0;
            float x[VW], wv[VW];
            ldsv<VW>(tg + (gyl * D::GW + gxl) * DCG + vec * VW, x);
            ldsv<VW>(wts + (kh * K + kw) * DCG + vec * VW, wv);
#pragma unroll
            for (int j = 0; j < VW; ++j) {
              acc[j] = fmaf(x[j], wv[j], acc[j]);
              accw[ah][aw][j] = fmaf(av[j], x[j], accw[ah][aw][j]);
            }
          }
        }
        float mu[VW], is[VW];
        ldsv<VW>(&bnc[2][vec * VW], mu);
        ldsv<VW>(&bnc[3][vec * VW], is);
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          const float gg = Tr<T>::round(acc[j] * sp[j]);
          acc[j] = gg;
          st_s[j] += gg;
          st_q[j] += gg * (y[j] - mu[j]) * is[j];
        }
        stv(out + (((int64_t)f * g.H + iy) * g.W + ix) * C + c, acc);
      }
    };
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < D::P; ++i) {
        asm volatile("" ::: "memory");  // one pixel's LDS reads live at a time
        pixel(i, ryc[i]);
      }
    } else {
#pragma unroll 1
      for (int i = 0; i < D::P; ++i) {
        RawV<T, VW> rn;
        const int p2 = tp + D::NPT * (i + 1);
        const int iy2 = iy0 + p2 / TW, ix2 = ix0 + (p2 - (p2 / TW) * TW);
        const bool ok2 = i + 1 < D::P && p2 < D::NPX && iy2 < g.H && ix2 < g.W && cok;
        rn.ld(Yp + (((int64_t)f * g.H + iy2) * g.W + ix2) * C + c, Yp, ok2);
        pixel(i, ryc[0]);
        ryc[0] = rn;
      }
    }
  }

  // ---- reductions: lanes of one (vector, parity class) by shuffles, then the waves in order ----
  // BN-backward partials: every lane of a vector (any class)
#pragma unroll
  for (int j = 0; j < VW; ++j) {
#pragma unroll
    for (int o = D::NV; o < 64; o <<= 1) {
      st_s[j] += __shfl_xor(st_s[j], o, 64);
      st_q[j] += __shfl_xor(st_q[j], o, 64);
    }
  }
  // weight-gradient partials: xor over the pixel-slot bits that keep the parity class (stride 2:
  // slot bit 0 = column parity, and the row-parity bit when a wave spans two rows of slots)
#pragma unroll
  for (int bo = D::NV; bo < 64; bo <<= 1) {
    const int slot_bit = bo / D::NV;
    if (S == 2 && (slot_bit == 1 || slot_bit == TW)) continue;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NA; ++b)
#pragma unroll
        for (int j = 0; j < VW; ++j) accw[a][b][j] += __shfl_xor(accw[a][b][j], bo, 64);
  }
  lds_barrier();
  float* red = tg;  // [wave][kh0*2+kw0][NA][NA][32]
  float* sred = wts;  // [wave][2][32] (the weights are no longer needed)
  __syncthreads();
  const int slot_l = lane / D::NV;  // pixel slot within the wave
  bool leader = true;               // lowest lane of its (vector, class) group
#pragma unroll
  for (int bo = D::NV; bo < 64; bo <<= 1) {
    const int slot_bit = bo / D::NV;
    if (S == 2 && (slot_bit == 1 || slot_bit == TW)) continue;
    if (slot_l & slot_bit) leader = false;
  }
  if (leader) {
    const int cls = S == 2 ? kh0 * 2 + kw0 : 0;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NA; ++b)
#pragma unroll
        for (int j = 0; j < VW; ++j)
          red[((((wave * D::NCLS + cls) * NA + a) * NA + b) * DCG) + vec * VW + j] =
              (a < nah && b < naw) ? accw[a][b][j] : 0.f;
  }
  if (slot_l == 0) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      sred[(wave * 2 + 0) * DCG + vec * VW + j] = st_s[j];
      sred[(wave * 2 + 1) * DCG + vec * VW + j] = st_q[j];
    }
  }
  __syncthreads();
  // stride 1 has one class; for stride 2 a wave's leaders cover exactly the classes of its slots,
  // and a class absent from a wave is skipped through `present`
  const int64_t row = blockIdx.x / groups;
  if (tid < 2 * DCG) {
    const int which = tid / DCG, cl = tid - which * DCG;
    const float v = ((sred[(0 * 2 + which) * DCG + cl] + sred[(1 * 2 + which) * DCG + cl]) +
                     sred[(2 * 2 + which) * DCG + cl]) + sred[(3 * 2 + which) * DCG + cl];
    if (c0 + cl < C) stats[(row * 2 + which) * C + c0 + cl] = v;
  }
  float* sout = slab + row * (int64_t)C * K * K;
  for (int i = tid; i < K * K * DCG; i += 256) {
    const int tap = i / DCG, cl = i - tap * DCG;
    const int kh = tap / K, kw = tap - (tap / K) * K;
    const int ch = S == 2 ? (kh & 1) : 0, cw = S == 2 ? (kw & 1) : 0;
    const int a = S == 2 ? kh >> 1 : kh, b = S == 2 ? kw >> 1 : kw;
    // the class (ch, cw) is present in wave w iff some slot of w has that parity
    float v = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) {
      bool present = true;
      if constexpr (S == 2) {
        // slots of wave wv: [wv*TPW, (wv+1)*TPW); class of slot s: kh0 = (s/TW + pad) & 1, kw0 = (s%TW + pad) & 1
        present = false;
        for (int sl = wv * D::TPW; sl < (wv + 1) * D::TPW && sl < D::NPT; ++sl) {
          if ((((sl / TW) + g.pad) & 1) == ch && (((sl % TW) + g.pad) & 1) == cw) { present = true; break; }
        }
      }
      if (present) v += red[((((wv * D::NCLS + (S == 2 ? ch * 2 + cw : 0)) * NA + a) * NA + b) * DCG) + cl];
    }
    if (c0 + cl < C) sout[(int64_t)(c0 + cl) * K * K + tap] = v;
  }
}

template <int TH, int TW, int K> constexpr int pf1_bit() {
  return (TH == 16 && K == 3) ? 1 : (TH == 8 && K == 3) ? 2 : (TH == 14 && K == 3) ? 4 : (TH == 7 && K == 3) ? 8
       : (TH == 14 && K == 5) ? 16 : 32;
}
template <typename T, int TH, int TW, int K, int S, int VW,
          bool PF = (S == 2 || (DFD_DWB_PF1 & pf1_bit<TH, TW, K>()) != 0)>
static int bwd_launch(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* out, const T* Yp,
                      const BnBwdIn& bn, float* stats, int* stat_rows, float* slab, int64_t slab_cap, float* dW,
                      bool accumulate) {
  const int tiles_x = cdiv(g.W, TW), tiles_y = cdiv(g.H, TH);
  const int ntiles = g.frames * tiles_x * tiles_y;
  const int groups = cdiv(g.C, DCG);
  const int64_t per = (int64_t)g.C * K * K;
  // persistent grid of exactly the co-resident workgroups (one dispatch wave: measured faster than
  // two waves of 1024 on every B0 shape)
  auto kern = dw_bwd_kernel<T, TH, TW, K, S, VW, PF>;
  const int resident = resident_wgs<dw_bwd_kernel<T, TH, TW, K, S, VW, PF>, 256>();
  int64_t rows = std::min<int64_t>(ntiles, std::max(1, resident / groups));
  rows = std::max<int64_t>(1, std::min<int64_t>(rows, slab_cap / per));
  const int gx = (int)(rows * groups);
  hipLaunchKernelGGL(kern, dim3(gx), dim3(256), 0, s, g, dY, w, out, Yp, bn, stats,
                     slab, ntiles, groups, tiles_x, tiles_y);
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = (int)rows;
  return launch_reduce_slabs(s, slab, (int)rows, per, dW, accumulate);
}

// 0: launched; 1: no fused configuration for this layer (use launch_dw_dgrad + launch_dw_wgrad)
template <typename T>
int launch_dw_bwd(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* out, const T* Yp,
                  const BnBwdIn* bn, float* stats, int* stat_rows, float* slab, int64_t slab_cap, float* dW,
                  bool accumulate) {
  if (!bn || !Yp || !stats) { set_error("dw bwd: the fused BN-backward inputs are required", __FILE__, __LINE__); return -1; }
  if (!dw_bwd_fused_enabled()) return 1;
  const int H = g.H, W = g.W;
  if (g.k == 3 && g.s == 2) {
    if (H >= 56 && !(DFD_DWB_ALT & 1)) return bwd_launch<T, 16, 16, 3, 2, 8>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
    return bwd_launch<T, 8, 8, 3, 2, 8>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
  }
  if (g.k == 5 && g.s == 2)
    return bwd_launch<T, 8, 8, 5, 2, 8>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
  if (g.k == 3 && g.s == 1) {
    if (H % 16 == 0 && W % 16 == 0 && !(DFD_DWB_ALT & 8))
      return bwd_launch<T, 16, 16, 3, 1, 4>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
    if (H % 8 == 0 && W % 28 == 0 && !(DFD_DWB_ALT & 2))
      return bwd_launch<T, 8, 28, 3, 1, 8>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
    if (H % 14 == 0 && W % 14 == 0)
      return bwd_launch<T, 14, 14, 3, 1, 4>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
    return bwd_launch<T, 7, 7, 3, 1, 4>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
  }
  if (g.k == 5 && g.s == 1) {
    if (H % 14 == 0 && W % 14 == 0 && !(DFD_DWB_ALT & 4))
      return bwd_launch<T, 14, 14, 5, 1, 4>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
    return bwd_launch<T, 7, 7, 5, 1, 4>(s, g, dY, w, out, Yp, *bn, stats, stat_rows, slab, slab_cap, dW, accumulate);
  }
  return 1;
}

template int launch_dw_bwd<float>(hipStream_t, const DwGeom&, const float*, const float*, float*, const float*,
                                  const BnBwdIn*, float*, int*, float*, int64_t, float*, bool);
template int launch_dw_bwd<bf16>(hipStream_t, const DwGeom&, const bf16*, const float*, bf16*, const bf16*,
                                 const BnBwdIn*, float*, int*, float*, int64_t, float*, bool);
template int launch_dw_bwd<f16>(hipStream_t, const DwGeom&, const f16*, const float*, f16*, const f16*,
                                 const BnBwdIn*, float*, int*, float*, int64_t, float*, bool);

}  // namespace dfd
