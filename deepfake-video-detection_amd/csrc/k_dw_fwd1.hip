// Stride-1 depthwise-conv FORWARD in the channel-pair form of k_dw_bwd1.hip (timm conv_dw inside
// the blocks run by self.backbone(x_flat), src/pretrained_detector.py:116), with the producer's
// BN1 + SiLU applied while staging and the BN2 statistics of the output in the epilogue:
//   staging  act[p] = silu(y1[p] * sc1 + sh1)   (fp32 LDS, zero outside the map; packed fp32 math,
//            halo pixels outside the map skipped)
//   strips   y2[o]  = sum_tap act[o - pad + tap] * w[tap] -> out (rounded to T),
//            stats += [y2, y2^2]  (BN2 partial sums, fixed order)
// Thread = (channel pair, strip of RS outputs of one row): per kernel row the strip's RS+K-1
// activation pairs are read once (ds_read_b64) and feed RS*K packed FMAs.  Tiles as in the backward:
// 8x28 (k3, 112/56 maps), 14x14 (28/14 maps), two stacked 7x7 frames.  Replaces the 8-channel
// strip / tile kernels on these shapes (VALU-issue bound: fewer instructions per output).
#include "dw1_common.h"
#include "bnfin.h"

#ifndef DFD_FWD1_PF
#define DFD_FWD1_PF 0  // next-tile register prefetch of the staged window (A/B knob)
#endif

namespace dfd {

template <typename T, int K, int TH, int TW, int RS, int FR = 1, int S = 1, int RB = 1>
struct Dwf1 {
  // TH x TW OUTPUT tile; the staged input window is ((TH-1)S+K) x ((TW-1)S+K) (+ FR stacked frames)
  static constexpr int PAD = K / 2;
  static constexpr int GH1 = (TH - 1) * S + K, GW = (TW - 1) * S + K;
  static constexpr int GH = FR * GH1, NG = GH * GW;
  static constexpr int NLD = (NG * 4 + 255) / 256;
  // RB = 2: a thread's strip covers two adjacent output rows (stride 1): the K+1 input rows feed
  // both rows' K kernel rows, so each staged row is read once per two outputs
  static constexpr int SPR = TW / RS, SPF = (TH / RB) * SPR, NSTRIP = FR * SPF;
  static_assert(TH % RB == 0 && (RB == 1 || S == 1), "row blocking: stride 1, whole row pairs");
  static constexpr int RW = (RS - 1) * S + K;
  static constexpr int NP = DCG / 2;
  // act row stride (float2 pairs): the four strips of a wave read rows S apart; stride 1: an odd
  // pixel count puts consecutive rows in opposite bank halves; stride 2: a half-pixel pad does so
  // for rows two apart
  static constexpr int ARS = S == 1 ? (GW | 1) * NP : GW * NP + NP / 2;
  static constexpr int RED = 4 * 2 * DCG * 4;
  static constexpr int AB = GH * ARS * 8 > RED ? GH * ARS * 8 : RED;
  static constexpr int LDS = AB + K * K * DCG * 4 + 2 * DCG * 4;
  static constexpr int OCC = (sizeof(T) == 2 && S == 1) ? 3 : 2;  // = the kernel's launch bounds
  static_assert(TW % RS == 0, "strips tile the row");
  static_assert(LDS * OCC <= 160 * 1024, "LDS footprint sets the occupancy");
};

template <typename T, int K, int TH, int TW, int RS, int FR, int S, int RB>
__global__ __launch_bounds__(256, (sizeof(T) == 2 && S == 1) ? 3 : 2) void dw_fwd1_kernel(
    DwGeom g, const T* __restrict__ Y1, const float* __restrict__ w, Pro bn1, T* __restrict__ out,
    float* __restrict__ stats, int ntiles, int groups, int tiles_x, int tiles_y, int xcd, BnFwdFin fin) {
  using D = Dwf1<T, K, TH, TW, RS, FR, S, RB>;
  static_assert(D::AB >= kBnFinScratch * 8, "the staging area holds the BN1 finalize scratch");
  __shared__ __attribute__((aligned(16))) char araw[D::AB];        // staged activations; reduction scratch
  __shared__ __attribute__((aligned(16))) float wts[K * K * DCG];  // [tap][ch]
  __shared__ __attribute__((aligned(16))) float cst[2][DCG];       // BN1 scale, shift
  float* acts = reinterpret_cast<float*>(araw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bid = xcd ? xcd_swizzle((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int grp = bid % groups;
  const int c0 = grp * DCG, C = g.C;
  for (int i = tid; i < K * K * DCG; i += 256) {
    const int tap = i / DCG, cl = i - tap * DCG;
    wts[i] = (c0 + cl < C) ? w[(int64_t)(c0 + cl) * K * K + tap] : 0.f;
  }
  // BN1 scale / shift: finalized here from the producer's stat rows (bnfin.h; the first workgroup of
  // the channel group stores them and the running statistics), or read from the finalize launch's output
  const int nc = C - c0 < DCG ? C - c0 : DCG;
  if (fin.rows > 0) bn_fin_wg(fin, C, c0, nc, bid / groups == 0, cst[0], cst[1], reinterpret_cast<double*>(araw));
  for (int i = tid; i < 2 * DCG; i += 256) {
    const int k = i / DCG, cl = i - k * DCG, c = c0 + cl;
    if (fin.rows > 0 && cl < nc) continue;
    cst[k][cl] = c < C ? (k ? bn1.shift[c] : bn1.scale[c]) : (k ? 0.f : 1.f);
  }
  const int tpf = tiles_x * tiles_y;
  const int tstep = gridDim.x / groups;
  const int fstride = g.H * g.W * C;          // input frame
  const int ostride = g.Ho * g.Wo * C;        // output frame
  const int v8 = tid & 3, c8 = c0 + v8 * 8;
  const bool cok8 = c8 < C;
  const int cp = tid & 15, slot = tid >> 4;
  const int ch = c0 + 2 * cp;
  const bool cokp = ch < C;
  v2f ss = {0.f, 0.f}, sq = {0.f, 0.f};

  // raw loads of a tile's staged window (one 8-channel vector per lane and pass)
  auto stage_load = [&](int t, Raw8<T> (&ry)[D::NLD]) {
    const int f = (t / tpf) * FR, r = t - (t / tpf) * tpf, ty = r / tiles_x;
    const int iy0 = ty * TH, ix0 = (r - ty * tiles_x) * TW;
    const T* yf = Y1 + (int64_t)f * fstride;
#pragma unroll
    for (int i = 0; i < D::NLD; ++i) {
      const int pixl = (tid >> 2) + 64 * i;
      const int fi = FR > 1 ? pixl / (D::GH1 * D::GW) : 0, pf = pixl - fi * (D::GH1 * D::GW);
      const int oy = iy0 * S - D::PAD + pf / D::GW, ox = ix0 * S - D::PAD + pf % D::GW;
      const bool in = pixl < D::NG && cok8 && f + fi < g.frames && oy >= 0 && oy < g.H && ox >= 0 && ox < g.W;
      const uint32_t o = in ? (uint32_t)(fi * fstride + (oy * g.W + ox) * C + c8) : 0u;
      raw_ld(ry[i], yf + o, yf, in);
    }
  };
  // RB = 2: the channel pair's K x K weights in registers for the whole launch
  v2f wreg[RB == 2 ? K : 1][RB == 2 ? K : 1];
  if constexpr (RB == 2) {
    lds_barrier();  // wts written
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) wreg[kh][kw] = lds2(wts + (kh * K + kw) * DCG + 2 * cp);
  }
  Raw8<T> ry[D::NLD];
  if (DFD_FWD1_PF && bid / groups < ntiles) stage_load(bid / groups, ry);
  for (int t = bid / groups; t < ntiles; t += tstep) {
    const int f = (t / tpf) * FR, r = t - (t / tpf) * tpf, ty = r / tiles_x;
    const int iy0 = ty * TH, ix0 = (r - ty * tiles_x) * TW;
    if (!DFD_FWD1_PF) stage_load(t, ry);
    lds_barrier();  // the previous tile's strips are done with acts
#pragma unroll
    for (int i = 0; i < D::NLD; ++i) {
      const int pixl = (tid >> 2) + 64 * i;
      asm volatile("" ::: "memory");  // BN1 constants re-read per pixel (few live registers)
      if (pixl < D::NG) {
        float* dst = acts + (pixl / D::GW) * D::ARS * 2 + (pixl % D::GW) * DCG + v8 * 8;
        float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (ry[i].ok) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cq = v8 * 8 + 2 * q;
            const v2f z = fma2(raw8_pair(ry[i], q), lds2(&cst[0][cq]), lds2(&cst[1][cq]));
            const v2f a = z * sigmoid2(z);
            o[2 * q] = a.x;
            o[2 * q + 1] = a.y;
          }
        }
        st8(dst, o);
      }
    }
    lds_barrier();
    // the next tile's window loads fly while this tile's strips run (issued before its stores)
    if (DFD_FWD1_PF && t + tstep < ntiles) stage_load(t + tstep, ry);
    if constexpr (RB == 1) {
#pragma unroll 1
    for (int s = slot; s < D::NSTRIP; s += 16) {
      const int fi = FR > 1 ? s / D::SPF : 0, sf = s - fi * D::SPF;
      const int pr = sf % TH, xs = (sf / TH) * RS;
      const int iy = iy0 + pr;  // output row
      // output tiles never cross the map (try_dw_fwd1: exact tilings): only the channel bound and a
      // missing last stacked frame mask the epilogue; frame base + 32-bit byte offsets
      T* outf = out + (int64_t)f * ostride;
      const uint32_t sb = (uint32_t)((fi * ostride + (iy * g.Wo + ix0 + xs) * C + ch) * sizeof(T));
      const bool rok = cokp && f + fi < g.frames;
      v2f acc[RS];
#pragma unroll
      for (int px = 0; px < RS; ++px) acc[px] = v2f{0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        asm volatile("" ::: "memory");
        const float* rowp = acts + (fi * D::GH1 + pr * S + kh) * D::ARS * 2 + xs * S * DCG + 2 * cp;
        v2f ar[D::RW], wr[K];
#pragma unroll
        for (int j = 0; j < D::RW; ++j) ar[j] = lds2(rowp + j * DCG);
#pragma unroll
        for (int kw = 0; kw < K; ++kw) wr[kw] = lds2(wts + (kh * K + kw) * DCG + 2 * cp);
#pragma unroll
        for (int kw = 0; kw < K; ++kw)
#pragma unroll
          for (int px = 0; px < RS; ++px) acc[px] = fma2(ar[px * S + kw], wr[kw], acc[px]);
#pragma unroll
        for (int px = 0; px < RS; ++px) asm volatile("" : "+v"(acc[px]));
      }
      if (rok) {
#pragma unroll
        for (int px = 0; px < RS; ++px) {
          const v2f v = round2(acc[px], (T*)nullptr);
          ss += v;
          sq = fma2(v, v, sq);
          st2(boff(outf, sb + px * (uint32_t)(C * sizeof(T))), v);
        }
      }
    }
    } else {
    // two output rows per strip; the weights live in registers (loaded once per launch): per two
    // rows K+1 staged-row reads instead of 2K row + 2K weight-row reads.  Same kh-then-kw FMA order
    // per output as RB = 1 (bit-identical results)
#pragma unroll 1
    for (int s = slot; s < D::NSTRIP; s += 16) {
      const int fi = FR > 1 ? s / D::SPF : 0, sf = s - fi * D::SPF;
      const int pr = (sf % (TH / 2)) * 2, xs = (sf / (TH / 2)) * RS;
      const int iy = iy0 + pr;
      T* outf = out + (int64_t)f * ostride;
      const uint32_t sb = (uint32_t)((fi * ostride + (iy * g.Wo + ix0 + xs) * C + ch) * sizeof(T));
      const bool rok = cokp && f + fi < g.frames;
      v2f acc0[RS], acc1[RS];
#pragma unroll
      for (int px = 0; px < RS; ++px) acc0[px] = acc1[px] = v2f{0.f, 0.f};
#pragma unroll
      for (int ih = 0; ih <= K; ++ih) {
        asm volatile("" ::: "memory");
        const float* rowp = acts + (fi * D::GH1 + pr + ih) * D::ARS * 2 + xs * DCG + 2 * cp;
        v2f ar[D::RW];
#pragma unroll
        for (int j = 0; j < D::RW; ++j) ar[j] = lds2(rowp + j * DCG);
        if (ih < K) {
#pragma unroll
          for (int kw = 0; kw < K; ++kw)
#pragma unroll
            for (int px = 0; px < RS; ++px) acc0[px] = fma2(ar[px + kw], wreg[ih < K ? ih : 0][kw], acc0[px]);
        }
        if (ih > 0) {
#pragma unroll
          for (int kw = 0; kw < K; ++kw)
#pragma unroll
            for (int px = 0; px < RS; ++px) acc1[px] = fma2(ar[px + kw], wreg[ih > 0 ? ih - 1 : 0][kw], acc1[px]);
        }
#pragma unroll
        for (int px = 0; px < RS; ++px) asm volatile("" : "+v"(acc0[px]), "+v"(acc1[px]));
      }
      if (rok) {
        const uint32_t rowb = (uint32_t)(g.Wo * C * sizeof(T));
#pragma unroll
        for (int px = 0; px < RS; ++px) {
          const v2f v = round2(acc0[px], (T*)nullptr);
          ss += v;
          sq = fma2(v, v, sq);
          st2(boff(outf, sb + px * (uint32_t)(C * sizeof(T))), v);
        }
#pragma unroll
        for (int px = 0; px < RS; ++px) {
          const v2f v = round2(acc1[px], (T*)nullptr);
          ss += v;
          sq = fma2(v, v, sq);
          st2(boff(outf, sb + rowb + px * (uint32_t)(C * sizeof(T))), v);
        }
      }
    }
    }
  }
  // ---- BN2 partial sums: lanes sharing a channel pair, then the 4 waves, in a fixed order ----
  lane_sum4(ss);
  lane_sum4(sq);
  lds_barrier();
  float* red = reinterpret_cast<float*>(araw);  // [4 waves][2][32]
  if (lane < 16) {
    *reinterpret_cast<v2f*>(red + (wave * 2 + 0) * DCG + 2 * cp) = ss;
    *reinterpret_cast<v2f*>(red + (wave * 2 + 1) * DCG + 2 * cp) = sq;
  }
  lds_barrier();
  if (tid < 2 * DCG) {
    const int which = tid / DCG, cl = tid - which * DCG;
    const float v = ((red[(0 * 2 + which) * DCG + cl] + red[(1 * 2 + which) * DCG + cl]) +
                     red[(2 * 2 + which) * DCG + cl]) + red[(3 * 2 + which) * DCG + cl];
    const int64_t row = bid / groups;
    if (stats && c0 + cl < C) stats[(row * 2 + which) * C + c0 + cl] = v;
  }
}

template <typename T, int K, int TH, int TW, int RS, int FR = 1, int S = 1, int RB = 1>
static int fwd1_launch(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                       int* stat_rows, const BnFwdFin* fin) {
  const int tiles_x = cdiv(g.Wo, TW), tiles_y = cdiv(g.Ho, TH);
  if (FR > 1 && (tiles_x != 1 || tiles_y != 1)) { set_error("dw_fwd1: frame stacking needs whole-map tiles", __FILE__, __LINE__); return -1; }
  const int ntiles = cdiv(g.frames, FR) * tiles_x * tiles_y;
  const int groups = cdiv(g.C, DCG);
  const int resident = resident_wgs<dw_fwd1_kernel<T, K, TH, TW, RS, FR, S, RB>, 256>();
  int64_t rows = std::min<int64_t>(ntiles, std::max(1, resident / groups));
  rows = std::min<int64_t>(rows, 1024);  // the plan's BN-stat partial rows
  // XCD-aware order where it measured faster (kbench A/B: 56x56 s1 -16 %, 14x14 c480 -2..-6 %); the
  // 14x14 k5 c672 (+7 %), stacked 7x7 (+7..12 %) and single-group layers keep dispatch order
  const int xcd = DFD_DW_XCD >= 0 ? DFD_DW_XCD : (groups > 1 && (g.Ho >= 28 || (g.Ho == 14 && g.C <= 480)));
  hipLaunchKernelGGL((dw_fwd1_kernel<T, K, TH, TW, RS, FR, S, RB>), dim3((unsigned)(rows * groups)), dim3(256), 0, s, g, X, w,
                     pro, Y, stats, ntiles, groups, tiles_x, tiles_y, xcd, fin ? *fin : BnFwdFin{});
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = (int)rows;
  return 0;
}

// 1: launched, 0: shape not covered, -1: error
template <typename T>
int try_dw_fwd1(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                int* stat_rows, const BnFwdFin* fin) {
  if ((g.k != 3 && g.k != 5) || g.pad != g.k / 2 || (g.s != 1 && g.s != 2)) return 0;
  if (g.Ho != (g.H + 2 * g.pad - g.k) / g.s + 1 || g.Wo != (g.W + 2 * g.pad - g.k) / g.s + 1) return 0;
  // 32-bit element offsets into the input frames; 32-bit byte offsets within two output frames
  if ((g.C & 1) || (int64_t)g.H * g.W * g.C >= (1ll << 31) || (int64_t)g.Ho * g.Wo * g.C * 8 >= (1ll << 32) ||
      !dw_fwd1_enabled())
    return 0;
  const int H = g.Ho, W = g.Wo;  // output map
  // two output rows per strip (knob dw_rb bit 0, default on: kbench dw_fwd over the 16 layers
  // 1,037-1,042 -> 1,010-1,023 us, round 4)
  const bool rb = (tune(TK_DW_RB) & 1) != 0;
  int rc;
  if (g.s == 2) {
    // k3 stride 2 (112->56, 28->14): the 8x8 tile kernel is as fast or faster (kbench: 214 vs 246,
    // 42 vs 42 us); k5: 153 -> 126 and 43 -> 35 us
    if (g.k == 3) return 0;
    if (H == 7 && W == 7)
      rc = g.k == 3 ? fwd1_launch<T, 3, 7, 7, 7, 2, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin)
                    : fwd1_launch<T, 5, 7, 7, 7, 2, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin);
    else if (H % 7 == 0 && W % 14 == 0)
      rc = g.k == 3 ? fwd1_launch<T, 3, 7, 14, 7, 1, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin)
                    : fwd1_launch<T, 5, 7, 14, 7, 1, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin);
    else
      return 0;
  } else if (H == 7 && W == 7) {
    rc = g.k == 3 ? fwd1_launch<T, 3, 7, 7, 7, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin)
                  : fwd1_launch<T, 5, 7, 7, 7, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin);
  } else if (g.k == 3 && H % 8 == 0 && W % 28 == 0 && W >= 112) {  // 56x56: the 8-channel strip kernel is 6% faster
    rc = rb ? fwd1_launch<T, 3, 8, 28, 7, 1, 1, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin)
            : fwd1_launch<T, 3, 8, 28, 7>(s, g, X, w, Y, pro, stats, stat_rows, fin);
  } else if (H % 14 == 0 && W % 14 == 0) {
    if (rb)
      rc = g.k == 3 ? fwd1_launch<T, 3, 14, 14, 7, 1, 1, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin)
                    : fwd1_launch<T, 5, 14, 14, 7, 1, 1, 2>(s, g, X, w, Y, pro, stats, stat_rows, fin);
    else
      rc = g.k == 3 ? fwd1_launch<T, 3, 14, 14, 7>(s, g, X, w, Y, pro, stats, stat_rows, fin)
                    : fwd1_launch<T, 5, 14, 14, 7>(s, g, X, w, Y, pro, stats, stat_rows, fin);
  } else {
    return 0;
  }
  return rc == 0 ? 1 : -1;
}

template int try_dw_fwd1<float>(hipStream_t, const DwGeom&, const float*, const float*, float*, const Pro&, float*,
                                int*, const BnFwdFin*);
template int try_dw_fwd1<bf16>(hipStream_t, const DwGeom&, const bf16*, const float*, bf16*, const Pro&, float*,
                               int*, const BnFwdFin*);
template int try_dw_fwd1<f16>(hipStream_t, const DwGeom&, const f16*, const float*, f16*, const Pro&, float*,
                               int*, const BnFwdFin*);

}  // namespace dfd
