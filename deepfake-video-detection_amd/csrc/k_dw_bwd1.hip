// Stride-1 depthwise-conv backward, one launch per MBConv block, with BOTH neighbouring BatchNorm
// backward passes fused (timm conv_dw inside the blocks run by self.backbone(x_flat),
// src/pretrained_detector.py:116):
//   staging  dY[o]  = k1*g2 + k2*y2 + k3,  g2 = (dZ*gate[f] + bc[f]) * silu'(y2*sc2 + sh2)
//            (the backward of BN2+SiLU and the SE gate after the depthwise conv -- formerly a
//            separate bn_bwd_apply pass reading dZ, y2 and writing dY)
//   strips   dA[p]  = sum_tap dY[p + pad - tap] * w[tap]
//            g1[p]  = dA * silu'(y1*sc1 + sh1) -> out,   stats += [g1, g1*xhat1]  (BN1 backward sums)
//            dW[tap] += act[p] * dY[p + pad - tap],  act = silu(y1*sc1 + sh1)
// Design (MI355X, wave64).  The kernel is VALU-issue bound, so it is built to spend the fewest
// instructions per output element:
//   * one workgroup = one TH x TW tile of one frame x 32 channels; dY (+halo) is staged ONCE into
//     LDS (fp32: no unpacking in the inner loop) through the fused BN2 backward, computed with packed
//     fp32 math (v_pk_fma_f32) and skipped for halo pixels outside the map;
//   * thread = (channel pair, strip of RS pixels).  Per kernel row the strip's RS+K-1 dY pairs are
//     read once and feed BOTH the data gradient (acc[p] += dY * w) and the weight gradient
//     (dW[row][tap] += act[p] * dY): the activations never go to LDS and no second pass re-reads dY;
//   * the K*K x 2 weight-gradient accumulators stay in registers for the whole launch and are
//     reduced once at the end (lanes, then waves, in a fixed order: bit-reproducible).
#include "dw1_common.h"

namespace dfd {

template <typename T, int K, int TH, int TW, int RS, int FR = 1, int RB = 1>
struct Dw1 {
  // FR > 1: the tile is FR whole frames (TH x TW = the map), stacked with their own halos -- fills
  // the 16 strip slots on 7x7 maps
  static constexpr int PAD = K / 2;
  static constexpr int GH1 = TH + K - 1, GW = TW + K - 1;
  static constexpr int GH = FR * GH1, NG = GH * GW;
  static constexpr int NLD = (NG * 4 + 255) / 256;  // 8-channel vector loads per thread per tensor
  static constexpr int SPR = TW / RS;               // strips per tile row
  // RB = 2: a strip covers two adjacent rows; the K+1 staged dY rows it reads feed both rows' K
  // kernel rows (each staged row read once per two outputs)
  static constexpr int SPF = (TH / RB) * SPR;       // strips per frame
  static_assert(TH % RB == 0, "row blocking: whole row pairs");
  static constexpr int NSTRIP = FR * SPF;
  static constexpr int RW = RS + K - 1;             // dY pairs per strip row
  static_assert(TW % RS == 0, "strips tile the row");
  static constexpr int NP = DCG / 2;                // channel pairs per pixel
  // rows hold an odd number of pixels: strips are numbered row-fastest, so the two 16-lane slot
  // groups of each 32-lane half of a ds_read_b64 read consecutive rows, in opposite bank halves
  static constexpr int DRS = (GW | 1) * NP;         // dys row stride (float2 pairs)
  static constexpr int RED = 4 * (K * K + 2) * DCG * 4;  // end-of-launch reduction scratch (bytes)
  static constexpr int DYB = GH * DRS * 8 > RED ? GH * DRS * 8 : RED;
  static constexpr int LDS = DYB + K * K * DCG * 4 + 9 * DCG * 4 + FR * 2 * DCG * 4;
  static constexpr int OCC = (sizeof(T) == 2 && K == 3) ? 3 : 2;  // workgroups per CU (= the kernel's launch bounds)
  static_assert(LDS * OCC <= 160 * 1024, "LDS footprint sets the occupancy");
};

template <typename T, int K, int TH, int TW, int RS, int FR, bool PF, int RB>
__global__ __launch_bounds__(256, (sizeof(T) == 2 && K == 3 && !PF && RB == 1) ? 3 : 2) void dw_bwd1_kernel(
    DwGeom g, const T* __restrict__ dZ, const T* __restrict__ Y2, Dw1Bn2 b2, const float* __restrict__ w,
    const T* __restrict__ Y1, BnBwdIn bn1, T* __restrict__ out, float* __restrict__ stats, float* __restrict__ slab,
    int ntiles, int groups, int tiles_x, int tiles_y, int xcd) {
  using D = Dw1<T, K, TH, TW, RS, FR, RB>;
  __shared__ __attribute__((aligned(16))) char dyraw[D::DYB];  // staged dY (fp32 pairs); reduction scratch
  __shared__ __attribute__((aligned(16))) float gbl[FR][2][DCG];   // the tile frames' SE gate and bc
  __shared__ __attribute__((aligned(16))) float wts[K * K * DCG];  // [tap][ch]
  __shared__ __attribute__((aligned(16))) float cst[9][DCG];       // sc2 sh2 k1 k2 k3 | sc1 sh1 mean1 invstd1
  float* dys = reinterpret_cast<float*>(dyraw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bid = xcd ? xcd_swizzle((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int grp = bid % groups;
  const int c0 = grp * DCG, C = g.C;
  for (int i = tid; i < K * K * DCG; i += 256) {
    const int tap = i / DCG, cl = i - tap * DCG;
    wts[i] = (c0 + cl < C) ? w[(int64_t)(c0 + cl) * K * K + tap] : 0.f;
  }
  for (int i = tid; i < 9 * DCG; i += 256) {
    const int k = i / DCG, cl = i - k * DCG, c = c0 + cl;
    const bool ok = c < C;
    float v = 0.f;
    switch (k) {
      case 0: v = ok ? b2.sc[c] : 0.f; break;
      case 1: v = ok ? b2.sh[c] : 0.f; break;
      case 2: v = ok ? b2.coef[c] : 0.f; break;
      case 3: v = ok ? b2.coef[C + c] : 0.f; break;
      case 4: v = ok ? b2.coef[2 * C + c] : 0.f; break;
      case 5: v = ok ? bn1.scale[c] : 1.f; break;
      case 6: v = ok ? bn1.shift[c] : 0.f; break;
      case 7: v = ok ? bn1.mean[c] : 0.f; break;
      default: v = ok ? bn1.invstd[c] : 1.f; break;
    }
    cst[k][cl] = v;
  }
  const int tpf = tiles_x * tiles_y;
  const int tstep = gridDim.x / groups;
  const int fstride = g.H * g.W * C;  // elements per frame (< 2^31: checked by the launcher)
  const int v8 = tid & 3, c8 = c0 + v8 * 8;
  const bool cok8 = c8 < C;
  const int cp = tid & 15, slot = tid >> 4;  // channel pair; strip slot
  const int ch = c0 + 2 * cp;
  const bool cokp = ch < C;
  constexpr int NSI = (D::NSTRIP + 15) / 16;  // strips per slot and tile

  // ---- weight-gradient accumulators and BN1 sums, live for the whole launch ----
  v2f dw[K][K];
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = 0; b < K; ++b) dw[a][b] = v2f{0.f, 0.f};
  v2f ss = {0.f, 0.f}, sq = {0.f, 0.f};

  // staging loads of tile t: dZ, y2 + halo (this thread's 8 channels); frame base + 32-bit offsets.
  // A tile past the end (the prefetch after a workgroup's last tile) loads nothing.
  Raw8<T> rz[D::NLD], r2[D::NLD];
  auto stage_ld = [&](int t) {
    const int f = (t / tpf) * FR, r = t - (t / tpf) * tpf, ty = r / tiles_x;
    const int iy0 = ty * TH, ix0 = (r - ty * tiles_x) * TW;
    const bool live = f < g.frames;
    const T* zf = dZ + (int64_t)(live ? f : 0) * fstride;
    const T* yf = Y2 + (int64_t)(live ? f : 0) * fstride;
#pragma unroll
    for (int i = 0; i < D::NLD; ++i) {
      const int pixl = (tid >> 2) + 64 * i;
      const int fi = FR > 1 ? pixl / (D::GH1 * D::GW) : 0, pf = pixl - fi * (D::GH1 * D::GW);
      const int oy = iy0 - D::PAD + pf / D::GW, ox = ix0 - D::PAD + pf % D::GW;
      const bool in = pixl < D::NG && cok8 && f + fi < g.frames && oy >= 0 && oy < g.H && ox >= 0 && ox < g.W;
      const uint32_t o = in ? (uint32_t)(fi * fstride + (oy * g.W + ox) * C + c8) : 0u;
      raw_ld(rz[i], zf + o, zf, in);
      raw_ld(r2[i], yf + o, yf, in);
    }
  };
  // PF: software pipeline -- the next tile's staging loads are in flight during this tile's strips
  // (they reuse rz / r2, free once committed), and each strip's y1 is loaded before the commit
  if (PF) stage_ld(bid / groups);

  for (int t = bid / groups; t < ntiles; t += tstep) {
    const int f = (t / tpf) * FR, r = t - (t / tpf) * tpf, ty = r / tiles_x;  // first frame of the tile
    const int iy0 = ty * TH, ix0 = (r - ty * tiles_x) * TW;
    if (!PF) stage_ld(t);
    // the tile frames' SE gate and squeeze-path gradient (tiny, L2-resident) -> LDS
    for (int i = tid; i < FR * 2 * DCG; i += 256) {
      const int fi = i / (2 * DCG), w2 = (i / DCG) & 1, cl = i % DCG;
      const bool ok = c0 + cl < C && f + fi < g.frames;
      gbl[fi][w2][cl] = ok ? (w2 ? b2.bc : b2.gate)[(int64_t)(f + fi) * C + c0 + cl] : 0.f;
    }
    // strip geometry: tiles never cross the map (dw_bwd1_covers: exact tilings), so only the channel
    // bound and, with stacked frames, a missing last frame mask anything: such lanes read pixel 0 of
    // frame f (pixel stride 0; their zero dY gives zero dW terms) and skip the epilogue
    const T* y1f = Y1 + (int64_t)f * fstride;
    T* outf = out + (int64_t)f * fstride;
    auto strip_at = [&](int s, int& fi, int& pr, int& xs, bool& rok, uint32_t& sb, uint32_t& pb) {
      fi = FR > 1 ? s / D::SPF : 0;
      const int sf = s - fi * D::SPF;
      pr = (sf % (TH / RB)) * RB;
      xs = (sf / (TH / RB)) * RS;
      rok = cokp && f + fi < g.frames && s < D::NSTRIP;
      pb = rok ? (uint32_t)(C * sizeof(T)) : 0u;
      sb = rok ? (uint32_t)((fi * fstride + ((iy0 + pr) * g.W + ix0 + xs) * C + ch) * sizeof(T)) : 0u;
    };
    const uint32_t rowb = (uint32_t)(g.W * C * sizeof(T));  // next row of a strip (RB = 2)
    Raw2<T> ryp[PF ? NSI : 1][RB][RS];
    if (PF) {
#pragma unroll
      for (int si = 0; si < NSI; ++si) {
        int fi, pr, xs;
        bool rok;
        uint32_t sb, pb;
        strip_at(slot + 16 * si, fi, pr, xs, rok, sb, pb);
#pragma unroll
        for (int rr = 0; rr < RB; ++rr)
#pragma unroll
          for (int px = 0; px < RS; ++px) raw2_ld(ryp[PF ? si : 0][rr][px], boff(y1f, sb + (rok ? rr * rowb : 0u) + px * pb));
      }
    }
    lds_barrier();  // the previous tile's strips are done with dys; gbl written
    // ---- commit: the fused BN2 backward into fp32 LDS (zero outside the map) ----
#pragma unroll
    for (int i = 0; i < D::NLD; ++i) {
      const int pixl = (tid >> 2) + 64 * i;
      asm volatile("" ::: "memory");  // the BN2 constants are re-read per pixel (few live registers)
      if (pixl < D::NG) {
        float* dst = dys + (pixl / D::GW) * D::DRS * 2 + (pixl % D::GW) * DCG + v8 * 8;
        if (rz[i].ok) {
          const int fi = FR > 1 ? pixl / (D::GH1 * D::GW) : 0;
          float o[8];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cq = v8 * 8 + 2 * q;
            const v2f gtq = lds2(&gbl[fi][0][cq]), bcq = lds2(&gbl[fi][1][cq]);
            const v2f z = raw8_pair(rz[i], q), y = raw8_pair(r2[i], q);
            const v2f tz = fma2(y, lds2(&cst[0][cq]), lds2(&cst[1][cq]));
            const v2f sg = sigmoid2(tz);
            const v2f ds = sg * fma2(tz, 1.0f - sg, v2f{1.f, 1.f});
            const v2f g2 = fma2(z, gtq, bcq) * ds;
            const v2f v = round2(fma2(lds2(&cst[2][cq]), g2, fma2(lds2(&cst[3][cq]), y, lds2(&cst[4][cq]))),
                                 (T*)nullptr);
            o[2 * q] = v.x;
            o[2 * q + 1] = v.y;
          }
          st8(dst, o);
        } else {
          const float zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          st8(dst, zero);
        }
      }
    }
    if (PF) stage_ld(t + tstep);
    lds_barrier();

    // ---- strips: data gradient + weight gradient from one read of each dY row ----
    const v2f sc1 = lds2(&cst[5][2 * cp]), sh1 = lds2(&cst[6][2 * cp]);
    const v2f is1 = lds2(&cst[8][2 * cp]), mi1 = -lds2(&cst[7][2 * cp]) * is1;  // xhat = y*is + mi
#pragma unroll
    for (int si = 0; si < NSI; ++si) {
      const int s = slot + 16 * si;
      if (NSI * 16 > D::NSTRIP && s >= D::NSTRIP) break;
      int fi, pr, xs;
      bool rok;
      uint32_t sb, pb;
      strip_at(s, fi, pr, xs, rok, sb, pb);
      Raw2<T> ry[RB][RS];
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int px = 0; px < RS; ++px) {
          if (PF) ry[rr][px] = ryp[PF ? si : 0][rr][px];
          else raw2_ld(ry[rr][px], boff(y1f, sb + (rok ? rr * rowb : 0u) + px * pb));
        }
      // activations (weight-gradient operand) and sigmoids (for silu') of the strip
      v2f act[RB][RS], sg[RB][RS];
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int px = 0; px < RS; ++px) {
          const v2f z = fma2(raw2_f(ry[rr][px]), sc1, sh1);
          sg[rr][px] = sigmoid2(z);
          act[rr][px] = z * sg[rr][px];
        }
      v2f acc[RB][RS];
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int px = 0; px < RS; ++px) acc[rr][px] = v2f{0.f, 0.f};
      // staged row pr + ih feeds row rr of the strip through kernel row kh = K - 1 - ih + rr; ih
      // descending = kh ascending per output (RB = 1: the kernel-row order of the original loop)
#pragma unroll
      for (int ih = K + RB - 2; ih >= 0; --ih) {
        asm volatile("" ::: "memory");  // one staged row's LDS operands live at a time
        const float* rowp = dys + (fi * D::GH1 + pr + ih) * D::DRS * 2 + xs * DCG + 2 * cp;
        v2f dr[D::RW];
#pragma unroll
        for (int j = 0; j < D::RW; ++j) dr[j] = lds2(rowp + j * DCG);
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
          const int kh = K - 1 - ih + rr;
          if (kh < 0 || kh >= K) continue;
          v2f wr[K];
#pragma unroll
          for (int kw = 0; kw < K; ++kw) wr[kw] = lds2(wts + (kh * K + kw) * DCG + 2 * cp);
#pragma unroll
          for (int kw = 0; kw < K; ++kw)
#pragma unroll
            for (int px = 0; px < RS; ++px) {
              acc[rr][px] = fma2(dr[px + K - 1 - kw], wr[kw], acc[rr][px]);
              dw[kh][kw] = fma2(act[rr][px], dr[px + K - 1 - kw], dw[kh][kw]);
            }
          // the row's FMAs complete here (otherwise they sink into the per-pixel epilogue and every
          // row's operands stay live at once)
#pragma unroll
          for (int kw = 0; kw < K; ++kw) asm volatile("" : "+v"(dw[kh][kw]));
        }
#pragma unroll
        for (int rr = 0; rr < RB; ++rr)
#pragma unroll
          for (int px = 0; px < RS; ++px) asm volatile("" : "+v"(acc[rr][px]));
      }
      // ---- epilogue: g1 = dA * silu'(z1) -> out, BN1 backward sums ----
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int px = 0; px < RS; ++px) pin2(ry[rr][px]);
      if (rok) {
#pragma unroll
        for (int rr = 0; rr < RB; ++rr)
#pragma unroll
          for (int px = 0; px < RS; ++px) {
            // silu'(z) = s (1 + z (1 - s)) = s + act (1 - s)
            const v2f dsl = fma2(act[rr][px], 1.0f - sg[rr][px], sg[rr][px]);
            const v2f gg = round2(acc[rr][px] * dsl, (T*)nullptr);
            ss += gg;
            sq = fma2(gg, fma2(raw2_f(ry[rr][px]), is1, mi1), sq);
            st2(boff(outf, sb + rr * rowb + px * pb), gg);
          }
      }
    }
  }

  // ---- fixed-order reductions: lanes of a wave sharing a channel pair, then the 4 waves ----
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = 0; b < K; ++b) {
      dw[a][b].x += __shfl_xor(dw[a][b].x, 16, 64);
      dw[a][b].y += __shfl_xor(dw[a][b].y, 16, 64);
      dw[a][b].x += __shfl_xor(dw[a][b].x, 32, 64);
      dw[a][b].y += __shfl_xor(dw[a][b].y, 32, 64);
    }
  ss.x += __shfl_xor(ss.x, 16, 64); ss.y += __shfl_xor(ss.y, 16, 64);
  ss.x += __shfl_xor(ss.x, 32, 64); ss.y += __shfl_xor(ss.y, 32, 64);
  sq.x += __shfl_xor(sq.x, 16, 64); sq.y += __shfl_xor(sq.y, 16, 64);
  sq.x += __shfl_xor(sq.x, 32, 64); sq.y += __shfl_xor(sq.y, 32, 64);
  lds_barrier();
  float* red = reinterpret_cast<float*>(dyraw);  // [4 waves][K*K + 2][32]
  if (lane < 16) {
    float* rw = red + wave * (K * K + 2) * DCG + 2 * cp;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = 0; b < K; ++b) *reinterpret_cast<v2f*>(rw + (a * K + b) * DCG) = dw[a][b];
    *reinterpret_cast<v2f*>(rw + (K * K) * DCG) = ss;
    *reinterpret_cast<v2f*>(rw + (K * K + 1) * DCG) = sq;
  }
  lds_barrier();
  const int64_t row = bid / groups;
  float* sout = slab + row * (int64_t)C * K * K;
  for (int i = tid; i < (K * K + 2) * DCG; i += 256) {
    const int e = i / DCG, cl = i - e * DCG;
    constexpr int E = (K * K + 2) * DCG;
    const float v = ((red[i] + red[E + i]) + red[2 * E + i]) + red[3 * E + i];
    if (c0 + cl < C) {
      if (e < K * K) sout[(int64_t)(c0 + cl) * K * K + e] = v;
      else stats[(row * 2 + (e - K * K)) * C + c0 + cl] = v;
    }
  }
}

template <typename T, int K, int TH, int TW, int RS, int FR = 1, bool PF = false, int RB = 1>
static int bwd1_launch(hipStream_t s, const DwGeom& g, const T* dZ, const T* Y2, const Dw1Bn2& b2, const float* w,
                       const T* Y1, const BnBwdIn& bn1, T* out, float* stats, int* stat_rows, float* slab,
                       int64_t slab_cap, float* dW, bool accumulate) {
  const int tiles_x = cdiv(g.W, TW), tiles_y = cdiv(g.H, TH);
  if (FR > 1 && (tiles_x != 1 || tiles_y != 1)) { set_error("dw_bwd1: frame stacking needs whole-map tiles", __FILE__, __LINE__); return -1; }
  const int ntiles = cdiv(g.frames, FR) * tiles_x * tiles_y;
  const int groups = cdiv(g.C, DCG);
  const int64_t per = (int64_t)g.C * K * K;
  auto kern = dw_bwd1_kernel<T, K, TH, TW, RS, FR, PF, RB>;
  const int resident = resident_wgs<dw_bwd1_kernel<T, K, TH, TW, RS, FR, PF, RB>, 256>();
  int64_t rows = std::min<int64_t>(ntiles, std::max(1, resident / groups));
  rows = std::max<int64_t>(1, std::min<int64_t>(rows, slab_cap / per));
  rows = std::min<int64_t>(rows, 1024);  // the plan's BN-stat partial rows
  const int gx = (int)(rows * groups);
  // XCD-aware order where it measured faster (kbench A/B, interleaved: 56x56 -12 %, 14x14 k3 -10 %,
  // 28x28 / 14x14 k5 -2..-4 %); one channel group (112x112 c32) and the stacked 7x7 tiles +4 %
  const int xcd = DFD_DW_XCD >= 0 ? DFD_DW_XCD : (groups > 1 && g.H >= 14);
  hipLaunchKernelGGL(kern, dim3(gx), dim3(256), 0, s, g, dZ, Y2, b2, w, Y1, bn1, out, stats, slab, ntiles, groups,
                     tiles_x, tiles_y, xcd);
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = (int)rows;
  return launch_reduce_slabs(s, slab, (int)rows, per, dW, accumulate);
}

bool dw_bwd1_covers(const DwGeom& g) {
  if (g.s != 1 || (g.k != 3 && g.k != 5) || g.pad != g.k / 2 || g.Ho != g.H || g.Wo != g.W) return false;
  if (!dw_bwd1_enabled()) return false;
  // channel-pair accesses; 32-bit byte offsets within the tile's frames (FR <= 2; fp32 bound for
  // both dtypes) -- checked here so the caller falls back to the split path instead of failing
  if (g.C % 2 || (int64_t)g.H * g.W * g.C * 8 >= (1ll << 32)) return false;
  if (g.H == 7 && g.W == 7) return true;  // two stacked frames per tile
  if (g.k == 3) return (g.H % 8 == 0 && g.W % 28 == 0) || (g.H % 14 == 0 && g.W % 14 == 0);
  return g.H % 14 == 0 && g.W % 14 == 0;
}

// 0: launched; 1: shape not covered (use the BN2 apply + launch_dw_bwd path)
template <typename T>
int launch_dw_bwd1(hipStream_t s, const DwGeom& g, const T* dZ, const T* Y2, const float* gate, const float* bc,
                   const float* sc2, const float* sh2, const float* coef2, const float* w, const T* Y1,
                   const BnBwdIn& bn1, T* out, float* stats, int* stat_rows, float* slab, int64_t slab_cap, float* dW,
                   bool accumulate) {
  if (!dw_bwd1_covers(g)) return 1;
  const Dw1Bn2 b2{gate, bc, sc2, sh2, coef2};
  const int H = g.H, W = g.W;
  // bf16: the software-pipelined form (knob dw_pf, default on: kbench dw_bwd1 over the 12 stride-1
  // layers 1,377-1,380 -> 1,350-1,357 us, round 4) where its registers fit the launch bounds;
  // two-row strips (knob dw_rb bit 1, default off: 1,397 us) on the even-height tiles
  const bool pf = sizeof(T) == 2 && tune(TK_DW_PF) != 0;
  const bool rb = sizeof(T) == 2 && (tune(TK_DW_RB) & 2) != 0;
#define DFD_BWD1_(K_, TH_, TW_, RS_, FR_, RB_, PFOK_)                                                           \
  return pf && (PFOK_) ? bwd1_launch<T, K_, TH_, TW_, RS_, FR_, sizeof(T) == 2 && (PFOK_), RB_>(                  \
                             s, g, dZ, Y2, b2, w, Y1, bn1, out, stats, stat_rows, slab, slab_cap, dW, accumulate) \
                       : bwd1_launch<T, K_, TH_, TW_, RS_, FR_, false, RB_>(s, g, dZ, Y2, b2, w, Y1, bn1, out, stats, \
                                                                            stat_rows, slab, slab_cap, dW, accumulate)
  // (bf16 only; k5 two-row strips leave no registers for the prefetch)
#define DFD_BWD1(K_, TH_, TW_, RS_, FR_)                                                                 \
  do {                                                                                                   \
    if (rb && (TH_) % 2 == 0)                                                                            \
      DFD_BWD1_(K_, TH_, TW_, RS_, FR_, ((TH_) % 2 == 0 && sizeof(T) == 2 ? 2 : 1), (K_) == 3);         \
    DFD_BWD1_(K_, TH_, TW_, RS_, FR_, 1, true);                                                          \
  } while (0)
  if (H == 7 && W == 7) {
    if (g.k == 3) DFD_BWD1(3, 7, 7, 7, 2);
    DFD_BWD1(5, 7, 7, 7, 2);
  }
  if (g.k == 3) {
    if (H % 8 == 0 && W % 28 == 0) DFD_BWD1(3, 8, 28, 7, 1);
    if (H % 14 == 0 && W % 14 == 0) DFD_BWD1(3, 14, 14, 7, 1);
    return 1;
  }
  if (H % 14 == 0 && W % 14 == 0) DFD_BWD1(5, 14, 14, 7, 1);
#undef DFD_BWD1_
#undef DFD_BWD1
  return 1;
}

template int launch_dw_bwd1<float>(hipStream_t, const DwGeom&, const float*, const float*, const float*, const float*,
                                   const float*, const float*, const float*, const float*, const float*,
                                   const BnBwdIn&, float*, float*, int*, float*, int64_t, float*, bool);
template int launch_dw_bwd1<bf16>(hipStream_t, const DwGeom&, const bf16*, const bf16*, const float*, const float*,
                                  const float*, const float*, const float*, const float*, const bf16*,
                                  const BnBwdIn&, bf16*, float*, int*, float*, int64_t, float*, bool);
template int launch_dw_bwd1<f16>(hipStream_t, const DwGeom&, const f16*, const f16*, const float*, const float*,
                                  const float*, const float*, const float*, const float*, const f16*,
                                  const BnBwdIn&, f16*, float*, int*, float*, int64_t, float*, bool);

}  // namespace dfd
