// Depthwise conv forward, stride 1, register-blocked "strip" kernel (timm conv_dw,
// src/pretrained_detector.py:116).
//
// The tile kernels (k_dw_fwd.hip) read one 32-B input vector and one 32-B weight vector from
// LDS per 8-channel FMA -- LDS bandwidth (256 B/clk/CU for ds_read_b128) bounds them.  Here a
// thread owns a STRIP of R consecutive outputs of one row (8 channels): per kernel row it
// loads the R+K-1 input vectors once into registers and each weight vector once, and applies
// them to all R outputs -- (R+K-1 + K) LDS reads per R*K FMAs instead of 2*R*K.
//
// Workgroup = CV channel vectors (8*CV channels) x a TH x TW output tile; thread (vec = tid % CV,
// slot = tid / CV) computes strips slot, slot + NT/CV, ...  The input tile (+halo) is staged once
// into LDS (element type LT) through the producer's BN+SiLU, pixel stride padded by 16 B (bank
// spread).  PF: the next tile's global loads are issued before this tile's strips (register
// budget permitting); OCC: minimum resident workgroups per CU (__launch_bounds__).
#include "dw_common.h"

namespace dfd {

template <typename LT, int K, int TH, int TW, int R, int CV, int NT>
struct StripCfg {
  static constexpr int CVW = CV * 8;
  static constexpr int PS = CVW + 16 / (int)sizeof(LT);  // LDS pixel stride (elements), +16 B pad
  static constexpr int IH = TH + K - 1, IW = TW + K - 1, NIN = IH * IW;
  static constexpr int SPR = TW / R, NS = TH * SPR;
  static constexpr int SLOTS = NT / CV;
  static constexpr int NSP = (NS + SLOTS - 1) / SLOTS;
  static constexpr int NLD = (NIN * CV + NT - 1) / NT;
  static constexpr int TIN_B = NIN * PS * (int)sizeof(LT), RED_B = SLOTS * CVW * 2 * 4;
  static constexpr int TIN_ALLOC = (TIN_B > RED_B ? TIN_B : RED_B) / (int)sizeof(LT);
  static constexpr int LDS = TIN_ALLOC * (int)sizeof(LT) + K * K * CVW * 4;
  static_assert(TW % R == 0, "strip width must divide the tile width");
  static_assert(NT % CV == 0, "threads must be a multiple of the channel vectors");
};

template <typename T, typename LT, int K, int TH, int TW, int R, int CV, int NT, int OCC, bool PF, bool STATS>
__global__ __launch_bounds__(NT, OCC) void dw_fwd_strip_kernel(DwGeom g, const T* __restrict__ X, const float* __restrict__ w,
                                                          T* __restrict__ Y, Pro pro, float* __restrict__ stats,
                                                          int ntiles, int groups, int tiles_x, int tiles_y) {
  using Cf = StripCfg<LT, K, TH, TW, R, CV, NT>;
  __shared__ __attribute__((aligned(16))) LT tin[Cf::TIN_ALLOC];  // input tile; BN-stat scratch at the end
  __shared__ __attribute__((aligned(16))) float wts[K * K * Cf::CVW];
  const int tid = threadIdx.x, vec = tid % CV, slot = tid / CV;
  const int grp = blockIdx.x % groups;
  const int c0 = grp * Cf::CVW, C = g.C;
  const int c = c0 + vec * 8;
  const bool cok = c < C;
  for (int i = tid; i < K * K * Cf::CVW; i += NT) {
    const int tap = i / Cf::CVW, cl = i - tap * Cf::CVW;
    wts[i] = (c0 + cl < C) ? w[(int64_t)(c0 + cl) * K * K + tap] : 0.f;
  }
  // staging: element e -> (pixel e / CV, vector e % CV) with its own BN coefficients
  float ssc[8], ssh[8];
  {
    const int sv = tid % CV;  // NT % CV == 0: the staging vector of a thread is fixed
    const int sc_c = c0 + sv * 8;
    if (sc_c < C) {
      ld8f(pro.scale + sc_c, ssc);
      ld8f(pro.shift + sc_c, ssh);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { ssc[j] = 1.f; ssh[j] = 0.f; }
    }
  }
  float st_s[8], st_q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
  const int tpf = tiles_x * tiles_y;
  const int tstep = gridDim.x / groups;
  // tile t -> (frame, origin); its input loads (+halo, masked) go to registers
  auto issue = [&](int t, Raw8<T>* raw, int& f, int& oy0, int& ox0) {
    f = t / tpf;
    const int r = t - f * tpf, ty = r / tiles_x;
    oy0 = ty * TH;
    ox0 = (r - ty * tiles_x) * TW;
    const int y0 = oy0 - g.pad, x0 = ox0 - g.pad;
#pragma unroll
    for (int i = 0; i < Cf::NLD; ++i) {
      const int e = tid + NT * i, pix = e / CV, v = e - (e / CV) * CV;
      const int iy = y0 + pix / Cf::IW, ix = x0 + pix % Cf::IW;
      const bool in = t < ntiles && pix < Cf::NIN && c0 + v * 8 < C && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
      raw_ld(raw[i], X + (((int64_t)f * g.H + iy) * g.W + ix) * C + c0 + v * 8, X, in);
    }
  };
  Raw8<T> raw[Cf::NLD];
  int nf, noy, nox;
  issue(blockIdx.x / groups, raw, nf, noy, nox);
  for (int t = blockIdx.x / groups; t < ntiles; t += tstep) {
    if (!PF && t != (int)(blockIdx.x / groups)) issue(t, raw, nf, noy, nox);
    const int f = nf, oy0 = noy, ox0 = nox;
    lds_barrier();  // previous tile's strips are done with tin
#pragma unroll
    for (int i = 0; i < Cf::NLD; ++i) {
      const int e = tid + NT * i, pix = e / CV, v = e - (e / CV) * CV;
      if (pix < Cf::NIN) {
        float x[8];
        raw_to_f(raw[i], x);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = raw[i].ok ? siluf_(x[j] * ssc[j] + ssh[j]) : 0.f;
        st8(tin + pix * Cf::PS + v * 8, x);
      }
    }
    lds_barrier();
    // the next tile's global loads fly while this tile computes (register budget permitting)
    if (PF && t + tstep < ntiles) issue(t + tstep, raw, nf, noy, nox);
    // ---- strips ----
#pragma unroll
    for (int q = 0; q < Cf::NSP; ++q) {
      const int s = slot + Cf::SLOTS * q;
      if (Cf::NS % Cf::SLOTS != 0 && s >= Cf::NS) break;
      const int sy = s / Cf::SPR, sx = (s - (s / Cf::SPR) * Cf::SPR) * R;
      float acc[R][8];
#pragma unroll
      for (int rr = 0; rr < R; ++rr)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[rr][j] = 0.f;
#pragma unroll 1
      for (int kh = 0; kh < K; ++kh) {
        // the K weights of this kernel row stay in registers; each input vector of the row is
        // read once and scattered into the (up to K) outputs whose window covers it
        float wv[K][8];
#pragma unroll
        for (int kw = 0; kw < K; ++kw) ld8(wts + (kh * K + kw) * Cf::CVW + vec * 8, wv[kw]);
        const LT* row = tin + ((sy + kh) * Cf::IW + sx) * Cf::PS + vec * 8;
#pragma unroll
        for (int i = 0; i < R + K - 1; ++i) {
          float xv[8];
          ld8(row + i * Cf::PS, xv);
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            const int rr = i - kw;
            if (rr >= 0 && rr < R) {
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[rr][j] = fmaf(xv[j], wv[kw][j], acc[rr][j]);
            }
          }
        }
      }
      const int oy = oy0 + sy;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int ox = ox0 + sx + rr;
        if (cok && oy < g.Ho && ox < g.Wo) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[rr][j] = Tr<T>::round(acc[rr][j]);
          st8(Y + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * C + c, acc[rr]);
          if constexpr (STATS) {
#pragma unroll
            for (int j = 0; j < 8; ++j) { st_s[j] += acc[rr][j]; st_q[j] += acc[rr][j] * acc[rr][j]; }
          }
        }
      }
    }
  }
  if constexpr (STATS) {
    // per channel: threads with equal vec -> LDS [slots][CVW] then a fixed-order column sum
    lds_barrier();
    float* red = reinterpret_cast<float*>(tin);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(slot * 2 + 0) * Cf::CVW + vec * 8 + j] = st_s[j];
      red[(slot * 2 + 1) * Cf::CVW + vec * 8 + j] = st_q[j];
    }
    lds_barrier();
    float* out = stats + (int64_t)(blockIdx.x / groups) * 2 * C;
    for (int i = tid; i < 2 * Cf::CVW; i += NT) {
      const int which = i / Cf::CVW, cl = i - which * Cf::CVW;
      float a = 0.f;
      for (int sl = 0; sl < Cf::SLOTS; ++sl) a += red[(sl * 2 + which) * Cf::CVW + cl];
      if (c0 + cl < C) out[(int64_t)which * C + c0 + cl] = a;
    }
  }
}

template <typename T, typename LT, int K, int TH, int TW, int R, int CV, int NT, int OCC, bool PF>
static int strip_launch(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                        int* stat_rows) {
  using Cf = StripCfg<LT, K, TH, TW, R, CV, NT>;
  static_assert(Cf::LDS <= 64 * 1024, "strip tile does not fit LDS");
  const int tiles_x = cdiv(g.Wo, TW), tiles_y = cdiv(g.Ho, TH);
  const int ntiles = g.frames * tiles_x * tiles_y;
  const int groups = cdiv(g.C, Cf::CVW);
  // grid: up to 4096 workgroups for the 8x28 k3 tile; the others run exactly the co-resident
  // workgroups (one dispatch wave; measured 4-9% faster there, 5% slower on 8x28 k3)
  int cap = 4096;
  if (!(K == 3 && TH == 8)) {
    const int res = stats ? resident_wgs<dw_fwd_strip_kernel<T, LT, K, TH, TW, R, CV, NT, OCC, PF, true>, NT>()
                          : resident_wgs<dw_fwd_strip_kernel<T, LT, K, TH, TW, R, CV, NT, OCC, PF, false>, NT>();
    cap = std::min(4096, res);
  }
  const int per_group = std::min(ntiles, std::max(1, cap / groups));
  const int gx = per_group * groups;
  if (stats)
    hipLaunchKernelGGL((dw_fwd_strip_kernel<T, LT, K, TH, TW, R, CV, NT, OCC, PF, true>), dim3(gx), dim3(NT), 0, s, g, X, w, Y, pro,
                       stats, ntiles, groups, tiles_x, tiles_y);
  else
    hipLaunchKernelGGL((dw_fwd_strip_kernel<T, LT, K, TH, TW, R, CV, NT, OCC, PF, false>), dim3(gx), dim3(NT), 0, s, g, X, w, Y,
                       pro, stats, ntiles, groups, tiles_x, tiles_y);
  if (stat_rows) *stat_rows = per_group;
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

// Returns 1 if a strip configuration covers this stride-1 layer (and launched it), 0 if not.
// Configurations measured on MI355X (tools/kbench dw_fwd, 256 frames bf16; the tile kernel in
// parentheses): 112x112 k3 116 us (149), 56x56 k3 162 (203), 28x28 k5 127 (157), 14x14 k3 36 (41),
// 14x14 k5 63-83 (76-104).  Candidates that lost: bf16 LDS staging (the unpack costs more VALU
// than the halved LDS traffic saves), 2-wide strips at 4 blocks/CU (spills), and 7x7 maps (the
// 7-wide strips leave the halo-heavy tile LDS-bound; the tile kernel is 15 % faster there).
template <typename T>
int try_dw_fwd_strip(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                     int* stat_rows) {
  if (g.s != 1 || g.Ho != g.H || g.Wo != g.W) return 0;
  const int H = g.Ho, W = g.Wo;
  int rc;
  if (W % 28 == 0 && H % 8 == 0 && g.k == 3)
    rc = strip_launch<T, float, 3, 8, 28, 4, 4, 256, 2, true>(s, g, X, w, Y, pro, stats, stat_rows);
  else if (W % 28 == 0 && H % 7 == 0 && g.k == 5)
    rc = strip_launch<T, float, 5, 7, 28, 4, 4, 256, 2, true>(s, g, X, w, Y, pro, stats, stat_rows);
  else if (W % 14 == 0 && H % 14 == 0 && g.k == 3)
    rc = strip_launch<T, float, 3, 14, 14, 7, 4, 128, 2, false>(s, g, X, w, Y, pro, stats, stat_rows);
  else if (W % 14 == 0 && H % 14 == 0 && g.k == 5) {
    if constexpr (sizeof(T) == 2)  // the fp32 instance spills: fp32 (parity) mode keeps the tile kernel
      rc = strip_launch<T, float, 5, 14, 14, 7, 4, 128, 2, false>(s, g, X, w, Y, pro, stats, stat_rows);
    else
      return 0;
  } else {
    return 0;
  }
  return rc == 0 ? 1 : -1;
}

template int try_dw_fwd_strip<float>(hipStream_t, const DwGeom&, const float*, const float*, float*, const Pro&, float*,
                                     int*);
template int try_dw_fwd_strip<bf16>(hipStream_t, const DwGeom&, const bf16*, const float*, bf16*, const Pro&, float*,
                                    int*);
template int try_dw_fwd_strip<f16>(hipStream_t, const DwGeom&, const f16*, const float*, f16*, const Pro&, float*,
                                    int*);

}  // namespace dfd
