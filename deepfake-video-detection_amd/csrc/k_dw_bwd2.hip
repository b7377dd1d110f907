// STRIDE-2 depthwise-conv backward of a whole MBConv block in one launch, in the channel-pair form
// of k_dw_bwd1.hip (timm conv_dw of the first block of a stage, src/pretrained_detector.py:116):
//   staging  dY[o] = k1*g2 + k2*y2 + k3, g2 = (dZ*gate + bc) * silu'(y2*sc2 + sh2)   (OUTPUT res)
//   strips   for each INPUT pixel p and tap (kh,kw) with o = (p + pad - tap)/2 integral:
//              dA[p]       += dY[o] * w[tap]
//              dW[kh][kw]  += act[p] * dY[o],      act = silu(y1*sc1 + sh1)
//            g1[p] = dA * silu'(y1*sc1 + sh1) -> out,  stats += [g1, g1*xhat1]
// Tile = TH x TW INPUT pixels (x FR stacked frames) x 32 channels; its dY window
// (TH/2+2) x (TW/2+2) per frame is staged once (fp32).  Thread = (channel pair, strip of RS input
// pixels of one row).  Which taps meet a pixel depends on its parity: the column parity is static
// (strips start at even x) and the row parity is uniform per wave:
//   * 8 x 56 tiles (blocks.1.0 112->56 k3, blocks.2.0 56->28 k5): two passes of the 16 slots, the
//     row parity flips between them, so every wave runs the same number of kernel rows (even rows
//     meet ceil(K/2) of them, odd rows floor(K/2));
//   * whole-frame tiles (blocks.3.0 28->14 k3; blocks.5.0 14->7 k5 with 4 stacked frames): strips
//     numbered parity-major (all even-row strips, then the odd ones; 4 | #even strips), so every
//     pass but the one at the boundary has a single parity.
// Replaces the BN2 apply pass + dw_bwd_kernel on these layers.
#include "dw1_common.h"

namespace dfd {

template <typename T, int K, int TH, int TW, int RS, int FR>
struct Dw2 {
  static constexpr int PAD = K / 2;
  static constexpr int GH1 = TH / 2 + 2, GW = TW / 2 + 2;  // staged dY window per frame (output res)
  static constexpr int NG1 = GH1 * GW, GH = FR * GH1, NG = FR * NG1;
  static constexpr int NLD = (NG * 4 + 255) / 256;
  static constexpr int CH = NLD < 3 ? NLD : 3;      // staging loads in flight per tensor
  static constexpr int SPR = TW / RS;
  static constexpr int HE = TH / 2;                 // even (= odd) input rows per frame
  static constexpr int NE = FR * HE * SPR;          // even-row strips; the odd ones follow
  static constexpr int NSTRIP = 2 * NE;
  static constexpr bool BAL = FR == 1 && TH == 8 && SPR == 4;  // the two-pass balanced map
  static constexpr int NPASS = BAL ? 2 : (NSTRIP + 15) / 16;
  static constexpr int RWO = RS / 2 + 2;  // staged dY columns a strip touches
  static constexpr int NP = DCG / 2;
  static constexpr int DRS = (GW | 1) * NP;  // pairs per staged row: odd pixel count (banks)
  static constexpr int RED = 4 * (K * K + 2) * DCG * 4;
  static constexpr int DYB = GH * DRS * 8 > RED ? GH * DRS * 8 : RED;
  static_assert(TH % 2 == 0 && TW % RS == 0 && RS % 2 == 0, "even tiles and strips");
  static_assert(BAL || NE % 4 == 0, "a wave's 4 slots never straddle the parity boundary");
  static_assert(GH * DRS * 8 + (K * K + 9 + 2 * FR) * DCG * 4 <= 80 * 1024, "two workgroups per CU");
};

template <typename T, int K, int TH, int TW, int RS, int FR>
__global__ __launch_bounds__(256, 2) void dw_bwd2_kernel(
    DwGeom g, const T* __restrict__ dZ, const T* __restrict__ Y2, Dw1Bn2 b2, const float* __restrict__ w,
    const T* __restrict__ Y1, BnBwdIn bn1, T* __restrict__ out, float* __restrict__ stats, float* __restrict__ slab,
    int ntiles, int groups, int tiles_x, int tiles_y, int xcd) {
  using D = Dw2<T, K, TH, TW, RS, FR>;
  __shared__ __attribute__((aligned(16))) char dyraw[D::DYB];
  __shared__ __attribute__((aligned(16))) float wts[K * K * DCG];
  __shared__ __attribute__((aligned(16))) float cst[9][DCG];  // sc2 sh2 k1 k2 k3 | sc1 sh1 mean1 invstd1
  __shared__ __attribute__((aligned(16))) float gbl[FR][2][DCG];  // the tile frames' SE gate and bc
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
  const int istride = g.H * g.W * C, ostride = g.Ho * g.Wo * C;
  const int v8 = tid & 3, c8 = c0 + v8 * 8;
  const bool cok8 = c8 < C;
  const int cp = tid & 15, slot = tid >> 4;
  const int ch = c0 + 2 * cp;
  const bool cokp = ch < C;

  v2f dw[K][K];
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = 0; b < K; ++b) dw[a][b] = v2f{0.f, 0.f};
  v2f ss = {0.f, 0.f}, sq = {0.f, 0.f};

  for (int t = bid / groups; t < ntiles; t += tstep) {
    const int f = (t / tpf) * FR, r = t - (t / tpf) * tpf, ty = r / tiles_x;  // first frame of the tile
    const int iy0 = ty * TH, ix0 = (r - ty * tiles_x) * TW;  // input tile origin (even)
    const int ob = iy0 / 2 - 1, oxb = ix0 / 2 - 1;             // staged dY window origin
    // staging in chunks of at most CH 8-channel loads per tensor in flight (the stacked-frame tiles
    // would otherwise hold 2 x 6 raw vectors next to the launch-long dW accumulators)
    const T* zf = dZ + (int64_t)f * ostride;
    const T* yf = Y2 + (int64_t)f * ostride;
#pragma unroll
    for (int base = 0; base < D::NLD; base += D::CH) {
      Raw8<T> rz[D::CH], r2[D::CH];
#pragma unroll
      for (int u = 0; u < D::CH; ++u) {
        const int pixl = (tid >> 2) + 64 * (base + u);
        const int fi = FR > 1 ? pixl / D::NG1 : 0, pf = pixl - fi * D::NG1;
        const int oy = ob + pf / D::GW, ox = oxb + pf % D::GW;
        const bool in = base + u < D::NLD && pixl < D::NG && cok8 && f + fi < g.frames && oy >= 0 && oy < g.Ho &&
                        ox >= 0 && ox < g.Wo;
        const uint32_t o = in ? (uint32_t)(fi * ostride + (oy * g.Wo + ox) * C + c8) : 0u;
        raw_ld(rz[u], zf + o, zf, in);
        raw_ld(r2[u], yf + o, yf, in);
      }
      if (base == 0) {
        for (int i = tid; i < FR * 2 * DCG; i += 256) {
          const int fi = i / (2 * DCG), w2 = (i / DCG) & 1, cl = i % DCG;
          const bool ok = c0 + cl < C && f + fi < g.frames;
          gbl[fi][w2][cl] = ok ? (w2 ? b2.bc : b2.gate)[(int64_t)(f + fi) * C + c0 + cl] : 0.f;
        }
        lds_barrier();  // the previous tile's strips are done with dys; gbl written
      }
#pragma unroll
      for (int u = 0; u < D::CH; ++u) {
        const int pixl = (tid >> 2) + 64 * (base + u);
        asm volatile("" ::: "memory");
        if (base + u < D::NLD && pixl < D::NG) {
          float* dst = dys + (pixl / D::GW) * D::DRS * 2 + (pixl % D::GW) * DCG + v8 * 8;
          float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if (rz[u].ok) {
            const int fi = FR > 1 ? pixl / D::NG1 : 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int cq = v8 * 8 + 2 * q;
              const v2f z = raw8_pair(rz[u], q), y = raw8_pair(r2[u], q);
              const v2f tz = fma2(y, lds2(&cst[0][cq]), lds2(&cst[1][cq]));
              const v2f sg = sigmoid2(tz);
              const v2f ds = sg * fma2(tz, 1.0f - sg, v2f{1.f, 1.f});
              const v2f g2 = fma2(z, lds2(&gbl[fi][0][cq]), lds2(&gbl[fi][1][cq])) * ds;
              const v2f v = round2(fma2(lds2(&cst[2][cq]), g2, fma2(lds2(&cst[3][cq]), y, lds2(&cst[4][cq]))),
                                   (T*)nullptr);
              o[2 * q] = v.x;
              o[2 * q + 1] = v.y;
            }
          }
          st8(dst, o);
        }
      }
    }
    lds_barrier();

    const v2f sc1 = lds2(&cst[5][2 * cp]), sh1 = lds2(&cst[6][2 * cp]);
    const v2f is1 = lds2(&cst[8][2 * cp]), mi1 = -lds2(&cst[7][2 * cp]) * is1;
    const T* y1f = Y1 + (int64_t)f * istride;
    T* outf = out + (int64_t)f * istride;
#pragma unroll 1
    for (int it = 0; it < D::NPASS; ++it) {
      int fi = 0, par, pr, xs;
      if constexpr (D::BAL) {
        // wave w, slot q, pass it -> row 2q + par, par = (w&1)^it; column (w>>1) + 2 it.  Over the
        // two passes the 32 (row, column) strips are each visited once; a wave's 4 slots read 4
        // consecutive staged rows (odd row stride: opposite bank halves)
        par = (wave & 1) ^ it;
        pr = 2 * (slot & 3) + par;
        xs = ((wave >> 1) + 2 * it) * RS;
      } else {
        const int s = slot + 16 * it;  // parity-major: [even-row strips of all frames][odd ...]
        if (s >= D::NSTRIP) continue;  // uniform per wave (NSTRIP % 4 == 0)
        par = s >= D::NE;
        const int e = s - par * D::NE;
        fi = e / (D::HE * D::SPR);
        const int e2 = e - fi * (D::HE * D::SPR);
        pr = 2 * (e2 % D::HE) + par;   // consecutive slots: consecutive staged rows
        xs = (e2 / D::HE) * RS;
      }
      // tiles never cross the map (covers()): only the channel bound and a missing last stacked
      // frame mask anything.  Such lanes read pixel 0 of frame f (pixel stride 0; their staged dY is
      // zero, so their dW terms are too) and skip the epilogue
      const bool rok = cokp && f + fi < g.frames;
      const uint32_t pb = rok ? (uint32_t)(C * sizeof(T)) : 0u;
      const uint32_t sb =
          rok ? (uint32_t)((fi * istride + ((iy0 + pr) * g.W + ix0 + xs) * C + ch) * sizeof(T)) : 0u;
      Raw2<T> ry[RS];
#pragma unroll
      for (int px = 0; px < RS; ++px) raw2_ld(ry[px], boff(y1f, sb + px * pb));
      v2f act[RS], sg[RS];
#pragma unroll
      for (int px = 0; px < RS; ++px) {
        const v2f z = fma2(raw2_f(ry[px]), sc1, sh1);
        sg[px] = sigmoid2(z);
        act[px] = z * sg[px];
      }
      v2f acc[RS];
#pragma unroll
      for (int px = 0; px < RS; ++px) acc[px] = v2f{0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        // output row (pr + pad - kh) / 2 exists for one row parity; uniform per wave
        if (((pr + D::PAD - kh) & 1) == 0) {
          asm volatile("" ::: "memory");
          const int srow = fi * D::GH1 + (pr + D::PAD - kh) / 2 + 1;  // staged row (window origin iy0/2 - 1)
          const float* rowp = dys + srow * D::DRS * 2 + (xs / 2) * DCG + 2 * cp;
          v2f dr[D::RWO], wr[K];
#pragma unroll
          for (int j = 0; j < D::RWO; ++j) dr[j] = lds2(rowp + j * DCG);
#pragma unroll
          for (int kw = 0; kw < K; ++kw) wr[kw] = lds2(wts + (kh * K + kw) * DCG + 2 * cp);
#pragma unroll
          for (int kw = 0; kw < K; ++kw)
#pragma unroll
            for (int px = 0; px < RS; ++px) {
              if (((px + D::PAD - kw) & 1) == 0) {  // static: strips start at even x
                const int j = (px + D::PAD - kw) / 2 + 1;
                acc[px] = fma2(dr[j], wr[kw], acc[px]);
                dw[kh][kw] = fma2(act[px], dr[j], dw[kh][kw]);
              }
            }
#pragma unroll
          for (int px = 0; px < RS; ++px) asm volatile("" : "+v"(acc[px]));
#pragma unroll
          for (int kw = 0; kw < K; ++kw) asm volatile("" : "+v"(dw[kh][kw]));
        }
      }
#pragma unroll
      for (int px = 0; px < RS; ++px) pin2(ry[px]);
      if (rok) {
#pragma unroll
        for (int px = 0; px < RS; ++px) {
          const v2f dsl = fma2(act[px], 1.0f - sg[px], sg[px]);
          const v2f gg = round2(acc[px] * dsl, (T*)nullptr);
          ss += gg;
          sq = fma2(gg, fma2(raw2_f(ry[px]), is1, mi1), sq);
          st2(boff(outf, sb + px * pb), gg);
        }
      }
    }
  }

#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = 0; b < K; ++b) lane_sum4(dw[a][b]);
  lane_sum4(ss);
  lane_sum4(sq);
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

template <typename T, int K, int TH, int TW, int RS, int FR>
static int bwd2_launch(hipStream_t s, const DwGeom& g, const T* dZ, const T* Y2, const Dw1Bn2& b2, const float* w,
                       const T* Y1, const BnBwdIn& bn1, T* out, float* stats, int* stat_rows, float* slab,
                       int64_t slab_cap, float* dW, bool accumulate) {
  const int tiles_x = g.W / TW, tiles_y = g.H / TH;
  const int ntiles = cdiv(g.frames, FR) * tiles_x * tiles_y;
  const int groups = cdiv(g.C, DCG);
  const int64_t per = (int64_t)g.C * K * K;
  const int resident = resident_wgs<dw_bwd2_kernel<T, K, TH, TW, RS, FR>, 256>();
  int64_t rows = std::min<int64_t>(ntiles, std::max(1, resident / groups));
  rows = std::max<int64_t>(1, std::min<int64_t>(rows, slab_cap / per));
  rows = std::min<int64_t>(rows, 1024);
  // XCD-aware order: faster on every stride-2 layer (kbench A/B, interleaved: blocks.1.0 -3 %,
  // 2.0 -11 %, 3.0 -20 %, 5.0 -3 %)
  const int xcd = DFD_DW_XCD >= 0 ? DFD_DW_XCD : (groups > 1);
  hipLaunchKernelGGL((dw_bwd2_kernel<T, K, TH, TW, RS, FR>), dim3((unsigned)(rows * groups)), dim3(256), 0, s, g, dZ,
                     Y2, b2, w, Y1, bn1, out, stats, slab, ntiles, groups, tiles_x, tiles_y, xcd);
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = (int)rows;
  return launch_reduce_slabs(s, slab, (int)rows, per, dW, accumulate);
}

// tile configuration for a stride-2 layer: 0 none, 1 8x56 tiles, 2 whole 28x28 frames (k3),
// 3 four stacked 14x14 frames (k5)
static int dw2_config(const DwGeom& g) {
  if (g.s != 2 || (g.k != 3 && g.k != 5) || g.pad != g.k / 2) return 0;
  if (g.Ho != (g.H + 2 * g.pad - g.k) / 2 + 1 || g.Wo != (g.W + 2 * g.pad - g.k) / 2 + 1) return 0;
  // channel pairs; 32-bit byte offsets within the (up to 4) frames of a tile, fp32 bound
  if ((g.C & 1) || (int64_t)g.H * g.W * g.C * 16 >= (1ll << 32)) return 0;
  if (g.H % 8 == 0 && g.W % 56 == 0) return 1;
  if (g.k == 3 && g.H == 28 && g.W == 28) return 2;
  if (g.k == 5 && g.H == 14 && g.W == 14) return 3;
  return 0;
}

bool dw_bwd2_covers(const DwGeom& g) { return dw2_config(g) != 0 && dw_bwd1_enabled(); }

template <typename T>
int launch_dw_bwd2(hipStream_t s, const DwGeom& g, const T* dZ, const T* Y2, const float* gate, const float* bc,
                   const float* sc2, const float* sh2, const float* coef2, const float* w, const T* Y1,
                   const BnBwdIn& bn1, T* out, float* stats, int* stat_rows, float* slab, int64_t slab_cap, float* dW,
                   bool accumulate) {
  if (!dw_bwd2_covers(g)) return 1;
  const Dw1Bn2 b2{gate, bc, sc2, sh2, coef2};
  switch (dw2_config(g)) {
    case 1:
      if (g.k == 3)
        return bwd2_launch<T, 3, 8, 56, 14, 1>(s, g, dZ, Y2, b2, w, Y1, bn1, out, stats, stat_rows, slab, slab_cap, dW,
                                               accumulate);
      return bwd2_launch<T, 5, 8, 56, 14, 1>(s, g, dZ, Y2, b2, w, Y1, bn1, out, stats, stat_rows, slab, slab_cap, dW,
                                             accumulate);
    case 2:
      return bwd2_launch<T, 3, 28, 28, 14, 1>(s, g, dZ, Y2, b2, w, Y1, bn1, out, stats, stat_rows, slab, slab_cap, dW,
                                              accumulate);
    default:
      return bwd2_launch<T, 5, 14, 14, 14, 4>(s, g, dZ, Y2, b2, w, Y1, bn1, out, stats, stat_rows, slab, slab_cap, dW,
                                              accumulate);
  }
}

template int launch_dw_bwd2<float>(hipStream_t, const DwGeom&, const float*, const float*, const float*, const float*,
                                   const float*, const float*, const float*, const float*, const float*,
                                   const BnBwdIn&, float*, float*, int*, float*, int64_t, float*, bool);
template int launch_dw_bwd2<bf16>(hipStream_t, const DwGeom&, const bf16*, const bf16*, const float*, const float*,
                                  const float*, const float*, const float*, const float*, const bf16*,
                                  const BnBwdIn&, bf16*, float*, int*, float*, int64_t, float*, bool);
template int launch_dw_bwd2<f16>(hipStream_t, const DwGeom&, const f16*, const f16*, const float*, const float*,
                                  const float*, const float*, const float*, const float*, const f16*,
                                  const BnBwdIn&, f16*, float*, int*, float*, int64_t, float*, bool);

}  // namespace dfd
