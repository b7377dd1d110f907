// EfficientNet-B0 stem: conv2d 3->32, k3, s2, pad 1 (timm conv_stem), forward with BN-stat
// epilogue and weight gradient.  The input frames are read IN PLACE with arbitrary
// (frame, channel, row, col) strides -- the reference hands over channels-last-strided
// (B*T,3,H,W) tensors (app.py:2084-2086) -- so no transpose/copy precedes it.  They
// are either fp32 (normalised by the caller) or the raw uint8 face crops of the .npz feed
// (data_prepare.py:278-281), normalised while staging the tile (InputFmt): 1 B instead of 4 B
// per input element in both the forward and the weight-gradient pass.
#include "kernels.h"

namespace dfd {

constexpr int ST = 16;                // output tile edge
constexpr int SIE = (ST - 1) * 2 + 3; // 33: input tile edge
constexpr int SNIN = 3 * SIE * SIE;   // 3267 input floats per tile
constexpr int SNLD = (SNIN + 255) / 256;
constexpr int SCO = 32;               // output channels
constexpr int SP = ST * ST / 64;      // output pixels per thread (fwd)

struct StemTiles {
  int tiles_x, tiles_y;
  __device__ void coords(int64_t t, int& f, int& oy0, int& ox0) const {
    const int64_t tpf = (int64_t)tiles_x * tiles_y;
    f = (int)(t / tpf);
    const int rem = (int)(t - (int64_t)f * tpf);
    oy0 = (rem / tiles_x) * ST;
    ox0 = (rem - (rem / tiles_x) * tiles_x) * ST;
  }
};

// input tile [pix][ci] (pix = row*SIE + col) of frame f at origin (iy0, ix0): branch-free
// masked loads through the caller's strides, all issued together (register prefetch).
// uint8 frames (InputFmt.u8 = 1): the raw bytes are loaded here and normalised in stem_store
// through a 3 x 256 table in LDS.  Dense NHWC uint8 (u8 = 2, the .npz crops / the app's permute):
// each tile row is 33 px x 3 B = 99 contiguous bytes, loaded as <= 26 aligned dwords per row
// (4 loads per lane instead of 13 byte loads), staged as bytes in LDS and unpacked in stem_store.
// The loads stay in flight across the current tile's math in both cases.
constexpr int SRW = 26;                // dwords per staged row (99 B + alignment slack)
constexpr int SNW = SIE * SRW;         // 858 dwords per tile
constexpr int SNWL = (SNW + 255) / 256;
static_assert(SNWL <= SNLD, "the dword path reuses the tile's load registers");
// FMT: -1 = the input format read at run time; 2 = dense NHWC uint8 only (no strided-path registers)
template <int FMT = -1>
__device__ __forceinline__ void stem_load(const StemGeom& g, const void* __restrict__ x, int f, int iy0, int ix0,
                                          float (&r)[SNLD], uint32_t& okm) {
  okm = 0u;
  const int tid = threadIdx.x;
  if (FMT == 2 || (FMT < 0 && g.in.u8 == 2)) {
    const int xa = max(ix0, 0), xb = min(ix0 + SIE - 1, g.W - 1);
    const int off0 = (xa * 3) & ~3;
    const int nw = ((xb * 3 + 2) - off0) / 4 + 1;
    const uint8_t* base = static_cast<const uint8_t*>(x) + (int64_t)f * g.sf + off0;
#pragma unroll
    for (int i = 0; i < SNWL; ++i) {
      const int w = tid + 256 * i, row = w / SRW, k = w - row * SRW, iy = iy0 + row;
      const bool ok = w < SNW && k < nw && iy >= 0 && iy < g.H;
      const uint32_t v = *reinterpret_cast<const uint32_t*>(ok ? base + (int64_t)iy * g.sh + 4 * k
                                                               : static_cast<const uint8_t*>(x));
      r[i] = __uint_as_float(ok ? v : 0u);
    }
    return;
  }
  if constexpr (FMT == 2) return;
#pragma unroll
  for (int i = 0; i < SNLD; ++i) {
    const int e = tid + 256 * i;
    const int pix = e / 3, ci = e - 3 * (e / 3);
    const int iy = iy0 + pix / SIE, ix = ix0 + pix % SIE;
    const bool ok = e < SNIN && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
    const int64_t o = ok ? ((int64_t)f * g.sf + ci * g.sc + (int64_t)iy * g.sh + (int64_t)ix * g.sw) : 0;
    if (g.in.u8)
      r[i] = (float)static_cast<const uint8_t*>(x)[o];
    else
      r[i] = static_cast<const float*>(x)[o];
    okm |= ok ? (1u << i) : 0u;
  }
}
// The normalised value of every (channel, byte) pair: (v / 255 - mean) / std in fp32 with correctly
// rounded divisions -- torch's operations in torch's order -- computed once per workgroup (768
// entries) instead of two divisions per staged element.  Visible after the caller's next barrier.
constexpr int SLUT = 3 * 256;
__device__ __forceinline__ void stem_lut_init(const StemGeom& g, float* lut) {
  if (!g.in.u8) return;
  for (int i = threadIdx.x; i < SLUT; i += 256) {
    const int c = i >> 8;
    const float m = c == 0 ? g.in.mean[0] : c == 1 ? g.in.mean[1] : g.in.mean[2];
    const float sd = c == 0 ? g.in.stdv[0] : c == 1 ? g.in.stdv[1] : g.in.stdv[2];
    lut[i] = ((float)(i & 255) / 255.0f - m) / sd;
  }
}
// tin[pix][ci] of the tile at input origin (iy0, ix0); the dword path stages its bytes in u8s
// (an extra LDS barrier: every thread of the workgroup calls this uniformly).
template <int FMT = -1>
__device__ __forceinline__ void stem_store(const StemGeom& g, const float* lut, uint32_t* u8s, float* tin,
                                           const float (&r)[SNLD], uint32_t okm, int iy0, int ix0) {
  if (FMT == 2 || (FMT < 0 && g.in.u8 == 2)) {
#pragma unroll
    for (int i = 0; i < SNWL; ++i) {
      const int w = threadIdx.x + 256 * i;
      if (w < SNW) u8s[w] = __float_as_uint(r[i]);
    }
    lds_barrier();
    const uint8_t* bytes = reinterpret_cast<const uint8_t*>(u8s);
    const int off0 = (max(ix0, 0) * 3) & ~3;
#pragma unroll
    for (int i = 0; i < SNLD; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int pix = e / 3, ci = e - 3 * (e / 3);
      const int row = pix / SIE, ix = ix0 + pix % SIE, iy = iy0 + row;
      const bool ok = e < SNIN && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
      const int b = ok ? bytes[row * (SRW * 4) + ix * 3 + ci - off0] : 0;
      if (e < SNIN) tin[e] = ok ? lut[ci * 256 + b] : 0.f;  // zero padding AFTER normalisation
    }
    return;
  }
  if constexpr (FMT == 2) return;
#pragma unroll
  for (int i = 0; i < SNLD; ++i) {
    const int e = threadIdx.x + 256 * i;
    float v = r[i];
    if (g.in.u8) v = lut[(e - 3 * (e / 3)) * 256 + (int)v];
    if (e < SNIN) tin[e] = ((okm >> i) & 1u) ? v : 0.f;  // zero padding AFTER normalisation, as conv2d pads
  }
}

template <typename T, bool STATS>
__global__ __launch_bounds__(256, 2) void stem_fwd_kernel(StemGeom g, const void* __restrict__ x,
                                                       const float* __restrict__ w, T* __restrict__ Y,
                                                       float* __restrict__ stats, int64_t ntiles) {
  __shared__ float tin[SNIN];
  __shared__ float lut[SLUT];  // uint8 input: normalised value per (channel, byte)
  __shared__ uint32_t u8s[SNW];  // dense uint8 input: the tile's rows as staged dwords
  stem_lut_init(g, lut);
  __shared__ __attribute__((aligned(16))) float wts[27][SCO];  // [ci*9+tap][co]
  __shared__ float red[2][4][SCO];
  const int tid = threadIdx.x, vec = tid & 3, pt = tid >> 2;
  for (int i = tid; i < 27 * SCO; i += 256) {
    const int co = i / 27, r = i % 27;  // w[co][ci][kh][kw], r = ci*9 + kh*3 + kw
    wts[r][co] = w[i];
  }
  const StemTiles tl{(g.Wo + ST - 1) / ST, (g.Ho + ST - 1) / ST};
  float st_s[8], st_q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
  float nxt[SNLD];
  uint32_t nok = 0u;
  int64_t t = blockIdx.x;
  if (t < ntiles) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    stem_load(g, x, f, oy0 * 2 - 1, ox0 * 2 - 1, nxt, nok);
  }
  for (; t < ntiles; t += gridDim.x) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    lds_barrier();
    stem_store(g, lut, u8s, tin, nxt, nok, oy0 * 2 - 1, ox0 * 2 - 1);
    lds_barrier();
    if (t + gridDim.x < ntiles) {  // next tile in flight during this tile's math and stores
      int f2, oy2, ox2;
      tl.coords(t + gridDim.x, f2, oy2, ox2);
      stem_load(g, x, f2, oy2 * 2 - 1, ox2 * 2 - 1, nxt, nok);
    }
    float acc[SP][8];
#pragma unroll
    for (int i = 0; i < SP; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
#pragma unroll 3
    for (int tap = 0; tap < 27; ++tap) {
      const int ci = tap / 9, kh = (tap % 9) / 3, kw = tap % 3;
      float wv[8];
      ld8(&wts[tap][vec * 8], wv);
#pragma unroll
      for (int i = 0; i < SP; ++i) {
        const int p = pt + 64 * i, ly = p / ST, lx = p % ST;
        const float xv = tin[((ly * 2 + kh) * SIE + lx * 2 + kw) * 3 + ci];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(xv, wv[j], acc[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < SP; ++i) {
      const int p = pt + 64 * i, oy = oy0 + p / ST, ox = ox0 + p % ST;
      const bool ok = oy < g.Ho && ox < g.Wo;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = Tr<T>::round(acc[i][j]);
      if (ok) st8(Y + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * SCO + vec * 8, acc[i]);
      if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = ok ? acc[i][j] : 0.f;
          st_s[j] += v;
          st_q[j] += v * v;
        }
      }
    }
  }
  if constexpr (STATS) {
    // fixed-order reduction: lanes with the same vec (shuffles), then the 4 waves through LDS
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) {
        st_s[j] += __shfl_xor(st_s[j], o, 64);
        st_q[j] += __shfl_xor(st_q[j], o, 64);
      }
    if (lane < 4) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { red[0][wave][vec * 8 + j] = st_s[j]; red[1][wave][vec * 8 + j] = st_q[j]; }
    }
    lds_barrier();
    if (tid < 2 * SCO) {
      const int which = tid / SCO, c = tid % SCO;
      stats[((int64_t)blockIdx.x * 2 + which) * SCO + c] =
          red[which][0][c] + red[which][1][c] + red[which][2][c] + red[which][3][c];
    }
  }
}

// The BN after the stem (batch statistics) backward, applied while staging the wgrad's dY tile:
// dY = k1*g + k2*y + k3 per channel (coef = [k1; k2; k3], bn_bwd_finalize) -- the separate
// bn_bwd_apply pass over the 112x112x32 map (read g, y; write dY) is not needed.
// coefficients staged in LDS (bnk[3][32], visible after the loop's first barrier)
__device__ __forceinline__ void stem_bn_coef(const float* coef, float (*bnk)[SCO]) {
  if (coef && threadIdx.x < 3 * SCO) bnk[threadIdx.x / SCO][threadIdx.x % SCO] = coef[threadIdx.x];
}
template <typename T>
__device__ __forceinline__ void stem_bn_apply(bool ok, float (&d)[8], const Raw8<T>& ry, const float (*bnk)[SCO],
                                              int v) {
  float y[8], k1[8], k2[8], k3[8];
  raw_to_f(ry, y);
  ld8(&bnk[0][v * 8], k1);
  ld8(&bnk[1][v * 8], k2);
  ld8(&bnk[2][v * 8], k3);
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = ok ? k1[j] * d[j] + k2[j] * y[j] + k3[j] : 0.f;
}

// dW[co][ci][kh][kw] = sum dY[f,oy,ox,co] * x[f,ci,2oy-1+kh,2ox-1+kw]
// thread (co = tid & 31, sub = tid >> 5) accumulates all 27 taps over pixels p = sub (mod 8);
// the next tile's input and dY are loaded into registers while the current tile is reduced.
template <typename T>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(StemGeom g, const void* __restrict__ x,
                                                         const T* __restrict__ dY, const T* __restrict__ Yb,
                                                         const float* __restrict__ coef, float* __restrict__ slab,
                                                         int64_t ntiles) {
  __shared__ float tin[SNIN];
  __shared__ float lut[SLUT];  // uint8 input: normalised value per (channel, byte)
  __shared__ uint32_t u8s[SNW];  // dense uint8 input: the tile's rows as staged dwords
  stem_lut_init(g, lut);
  __shared__ __attribute__((aligned(16))) float tg[ST * ST * SCO];  // [pix][co]; reused as red[8][27][32]
  const int tid = threadIdx.x, co = tid & 31, sub = tid >> 5;
  const StemTiles tl{(g.Wo + ST - 1) / ST, (g.Ho + ST - 1) / ST};
  float acc[27];
#pragma unroll
  for (int r = 0; r < 27; ++r) acc[r] = 0.f;
  float nx[SNLD];
  uint32_t nxok = 0u;
  Raw8<T> nd[4];  // 256 px x 4 vectors / 256 threads
  Raw8<T> ny[4];  // fused BN backward: the stem's pre-BN output at the same pixels
  __shared__ __attribute__((aligned(16))) float bnk[3][SCO];
  stem_bn_coef(coef, bnk);
  auto load = [&](int64_t t) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    stem_load(g, x, f, oy0 * 2 - 1, ox0 * 2 - 1, nx, nxok);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, pix = e >> 2, v = e & 3;
      const int oy = oy0 + pix / ST, ox = ox0 + pix % ST;
      const int64_t o = (((int64_t)f * g.Ho + oy) * g.Wo + ox) * SCO + v * 8;
      raw_ld(nd[i], dY + o, dY, oy < g.Ho && ox < g.Wo);
      if (coef) raw_ld(ny[i], Yb + o, Yb, oy < g.Ho && ox < g.Wo);
    }
  };
  int64_t t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    lds_barrier();
    stem_store(g, lut, u8s, tin, nx, nxok, oy0 * 2 - 1, ox0 * 2 - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, pix = e >> 2, v = e & 3;
      float d[8];
      raw_to_f(nd[i], d);
      if (coef) stem_bn_apply(nd[i].ok, d, ny[i], bnk, v);
      st8(&tg[pix * SCO + v * 8], d);
    }
    lds_barrier();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);
    for (int p = sub; p < ST * ST; p += 8) {
      const int ly = p / ST, lx = p % ST;
      const float d = tg[p * SCO + co];
#pragma unroll
      for (int tap = 0; tap < 27; ++tap) {
        const int ci = tap / 9, kh = (tap % 9) / 3, kw = tap % 3;
        acc[tap] = fmaf(d, tin[((ly * 2 + kh) * SIE + lx * 2 + kw) * 3 + ci], acc[tap]);
      }
    }
  }
  lds_barrier();
  float* red = tg;  // [8][27][32] = 6912 floats <= 8192
#pragma unroll
  for (int r = 0; r < 27; ++r) red[(sub * 27 + r) * SCO + co] = acc[r];
  lds_barrier();
  float* out = slab + (int64_t)blockIdx.x * 27 * SCO;
  for (int i = tid; i < 27 * SCO; i += 256) {
    const int c = i / 27, r = i % 27;
    float a = 0.f;
    for (int sb = 0; sb < 8; ++sb) a += red[(sb * 27 + r) * SCO + c];
    out[i] = a;
  }
}

// 16-bit modes: the same weight gradient as a GEMM on v_mfma_f32_16x16x32_bf16 / _f16 --
// dW[co][tap] = sum_p dY[p][co] * patch[p][tap], K = pixels.  Per 16x16-pixel tile the dY tile
// ([pix][co], 16-B row writes) and the im2col tile ([pix][tap], 27 taps padded to 32, bf16 as the
// bf16 conv consumes its input) are staged in LDS; each wave takes 32-pixel k-steps and reads both
// operands as columns with ds_read_b64_tr_b16 (the pw_wgrad_kernel pattern): per pixel the LDS
// traffic is 27 reads + 4 writes instead of 28 reads per (pixel, channel) of the FMA kernel.
constexpr int SWL = 40;  // LDS row stride (bf16) of the [pix][32] operand tiles
typedef short stw_bf16x8_t __attribute__((ext_vector_type(8)));
typedef short stw_s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) stw_s16x4_t stw_lds_s16x4_t;
typedef float stw_f32x4_t __attribute__((ext_vector_type(4)));

template <typename T>
__global__ __launch_bounds__(256, 2) void stem_wgrad_mfma_kernel(StemGeom g, const void* __restrict__ x,
                                                              const T* __restrict__ dY, const T* __restrict__ Yb,
                                                              const float* __restrict__ coef,
                                                              float* __restrict__ slab, int64_t ntiles) {
  __shared__ float tin[SNIN];
  __shared__ float lut[SLUT];  // uint8 input: normalised value per (channel, byte)
  __shared__ uint32_t u8s[SNW];  // dense uint8 input: the tile's rows as staged dwords
  stem_lut_init(g, lut);
  __shared__ __attribute__((aligned(16))) T ys[ST * ST * SWL];  // dY tile [pix][co]; reused for the reduction
  __shared__ __attribute__((aligned(16))) T xs[ST * ST * SWL];  // im2col tile [pix][tap]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const StemTiles tl{(g.Wo + ST - 1) / ST, (g.Ho + ST - 1) / ST};
  stw_f32x4_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = stw_f32x4_t{0.f, 0.f, 0.f, 0.f};
  float nx[SNLD];
  uint32_t nxok = 0u;
  Raw8<T> nd[4];  // 256 px x 4 vectors / 256 threads
  Raw8<T> ny[4];  // fused BN backward: the stem's pre-BN output at the same pixels
  __shared__ __attribute__((aligned(16))) float bnk[3][SCO];
  stem_bn_coef(coef, bnk);
  auto load = [&](int64_t t) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    stem_load(g, x, f, oy0 * 2 - 1, ox0 * 2 - 1, nx, nxok);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, pix = e >> 2, v = e & 3;
      const int oy = oy0 + pix / ST, ox = ox0 + pix % ST;
      const int64_t o = (((int64_t)f * g.Ho + oy) * g.Wo + ox) * SCO + v * 8;
      raw_ld(nd[i], dY + o, dY, oy < g.Ho && ox < g.Wo);
      if (coef) raw_ld(ny[i], Yb + o, Yb, oy < g.Ho && ox < g.Wo);
    }
  };
  const int gq = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  int64_t t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    lds_barrier();
    stem_store(g, lut, u8s, tin, nx, nxok, oy0 * 2 - 1, ox0 * 2 - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, pix = e >> 2, v = e & 3;
      if (coef) {
        float d[8];
        raw_to_f(nd[i], d);
        stem_bn_apply(nd[i].ok, d, ny[i], bnk, v);
        st8(ys + pix * SWL + v * 8, d);
      } else {
        raw_st(ys + pix * SWL + v * 8, nd[i]);  // masked pixels store zeros
      }
    }
    lds_barrier();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);
    {  // im2col: thread = output pixel of the tile, 27 taps (+5 zero pads) as 4 x 16 B
      const int ly = tid / ST, lx = tid % ST;
      float v[32];
#pragma unroll
      for (int tap = 0; tap < 32; ++tap) {
        if (tap < 27) {
          const int ci = tap / 9, kh = (tap % 9) / 3, kw = tap % 3;
          v[tap] = tin[((ly * 2 + kh) * SIE + lx * 2 + kw) * 3 + ci];
        } else {
          v[tap] = 0.f;
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float w8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w8[j] = v[8 * c + j];
        st8(xs + tid * SWL + 8 * c, w8);
      }
    }
    lds_barrier();
    // this wave's two 32-pixel k-steps: D[co][tap] += dY^T . patches
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p0 = (wave * 2 + ks) * 32;
      stw_bf16x8_t bfr[2], afr[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const stw_s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (stw_lds_s16x4_t*)(xs + (p0 + 8 * gq + q) * SWL + b * 16 + 4 * pq));
        const stw_s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (stw_lds_s16x4_t*)(xs + (p0 + 8 * gq + 4 + q) * SWL + b * 16 + 4 * pq));
        bfr[b] = stw_bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const stw_s16x4_t alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (stw_lds_s16x4_t*)(ys + (p0 + 8 * gq + q) * SWL + b * 16 + 4 * pq));
        const stw_s16x4_t ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (stw_lds_s16x4_t*)(ys + (p0 + 8 * gq + 4 + q) * SWL + b * 16 + 4 * pq));
        afr[b] = stw_bf16x8_t{alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma16x16x32<T>(afr[a], bfr[b], acc[a][b]);
    }
  }
  // ---- the 4 waves' 32x32 partials in a fixed order into this workgroup's slab row ----
  lds_barrier();
  float* red = reinterpret_cast<float*>(ys);  // [4][32 co][32 tap] = 16 KB <= 20 KB
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = a * 16 + 4 * (lane >> 4) + r, tap = b * 16 + (lane & 15);
        red[(wave * 32 + co) * 32 + tap] = acc[a][b][r];
      }
  lds_barrier();
  float* out = slab + (int64_t)blockIdx.x * 27 * SCO;
  for (int i = tid; i < 27 * SCO; i += 256) {
    const int co = i / 27, tap = i % 27;
    out[i] = ((red[(0 * 32 + co) * 32 + tap] + red[(1 * 32 + co) * 32 + tap]) + red[(2 * 32 + co) * 32 + tap]) +
             red[(3 * 32 + co) * 32 + tap];
  }
}

// bf16 mode forward on v_mfma_f32_16x16x32_bf16: the 27 taps (+5 zero pads) are ONE 32-deep
// k-step, so per 16-pixel block and 16 output channels a single MFMA computes the transposed
// tile D[co][pix] = W[co][:] . patch[pix][:] (lanes then hold 4 consecutive channels of one
// pixel).  Per 16x16 tile: fp32 input + halo -> LDS (as the FMA kernel), im2col as bf16 rows
// (thread = pixel), 8 MFMAs per wave, rounded tile through an LDS slab for 16-B row stores,
// BN-stat partials from the rounded values (per lane, fixed-order reduction at the end).
constexpr int SFC = SCO + 8;  // LDS row stride (bf16) of the output slab
// OCC workgroups per CU (knob stem_occ, default 3: the output slab aliases the im2col tile, 44 KB of
// LDS, and the dense-uint8 instantiation fits 168 VGPRs; 2 is the previous occupancy)
template <typename T, int OCC, int FMT>
__global__ __launch_bounds__(256, OCC) void stem_fwd_mfma_kernel(StemGeom g, const void* __restrict__ x,
                                                            const float* __restrict__ w, T* __restrict__ Y,
                                                            float* __restrict__ stats, int64_t ntiles) {
  __shared__ float tin[SNIN];
  __shared__ float lut[SLUT];  // uint8 input: normalised value per (channel, byte)
  __shared__ uint32_t u8s[SNW];  // dense uint8 input: the tile's rows as staged dwords
  stem_lut_init(g, lut);
  __shared__ __attribute__((aligned(16))) T xs[ST * ST * SWL];  // im2col [pix][tap]
  // the output slab [pix][co] shares xs: a wave writes the output rows of the 16-pixel blocks whose
  // im2col rows it has just read (same pixels, same row stride), so no other wave's operand is hit
  static_assert(SFC == SWL, "slab and im2col rows alias");
  T* const ct = xs;
  __shared__ __attribute__((aligned(16))) T wsb[SCO * SWL];     // weights [co][tap]
  __shared__ float red[2][4][SCO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < SCO * 32; i += 256) {
    const int co = i / 32, tap = i % 32;  // w[co][ci][kh][kw], tap = ci*9 + kh*3 + kw
    wsb[co * SWL + tap] = Tr<T>::from_f(tap < 27 ? w[co * 27 + tap] : 0.f);
  }
  lds_barrier();
  stw_bf16x8_t wf[2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
    wf[a] = *reinterpret_cast<const stw_bf16x8_t*>(wsb + (a * 16 + (lane & 15)) * SWL + 8 * (lane >> 4));
  const StemTiles tl{(g.Wo + ST - 1) / ST, (g.Ho + ST - 1) / ST};
  const bool stats_on = stats != nullptr;
  float s_acc[2][4], q_acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s_acc[a][r] = 0.f; q_acc[a][r] = 0.f; }
  float nxt[SNLD];
  uint32_t nok = 0u;
  int64_t t = blockIdx.x;
  if (t < ntiles) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    stem_load<FMT>(g, x, f, oy0 * 2 - 1, ox0 * 2 - 1, nxt, nok);
  }
  for (; t < ntiles; t += gridDim.x) {
    int f, oy0, ox0;
    tl.coords(t, f, oy0, ox0);
    lds_barrier();
    stem_store<FMT>(g, lut, u8s, tin, nxt, nok, oy0 * 2 - 1, ox0 * 2 - 1);
    lds_barrier();
    if (t + gridDim.x < ntiles) {  // next tile in flight during this tile's math and stores
      int f2, oy2, ox2;
      tl.coords(t + gridDim.x, f2, oy2, ox2);
      stem_load<FMT>(g, x, f2, oy2 * 2 - 1, ox2 * 2 - 1, nxt, nok);
    }
    {  // im2col: thread = output pixel, 27 taps + 5 zero pads as 4 x 16 B
      const int ly = tid / ST, lx = tid % ST;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float w8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tap = 8 * c + j;
          if (tap < 27) {
            const int ci = tap / 9, kh = (tap % 9) / 3, kw = tap % 3;
            w8[j] = tin[((ly * 2 + kh) * SIE + lx * 2 + kw) * 3 + ci];
          } else {
            w8[j] = 0.f;
          }
        }
        st8(xs + tid * SWL + 8 * c, w8);
      }
    }
    lds_barrier();
    // this wave's 4 blocks of 16 pixels x 2 blocks of 16 channels
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      const int p0 = (wave * 4 + pb) * 16;
      const stw_bf16x8_t pf = *reinterpret_cast<const stw_bf16x8_t*>(xs + (p0 + (lane & 15)) * SWL + 8 * (lane >> 4));
      const int pix = p0 + (lane & 15);
      const int oy = oy0 + pix / ST, ox = ox0 + pix % ST;
      const bool ok = oy < g.Ho && ox < g.Wo;
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        stw_f32x4_t d = {0.f, 0.f, 0.f, 0.f};
        d = mfma16x16x32<T>(wf[a], pf, d);
        const uint2 pk = make_uint2(Tr<T>::pack2(d[0], d[1]), Tr<T>::pack2(d[2], d[3]));
        if (stats_on) {
          const float v[4] = {lo2f(pk.x, (T*)nullptr), hi2f(pk.x, (T*)nullptr), lo2f(pk.y, (T*)nullptr),
                              hi2f(pk.y, (T*)nullptr)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float vv = ok ? v[r] : 0.f;
            s_acc[a][r] += vv;
            q_acc[a][r] += vv * vv;
          }
        }
        *reinterpret_cast<uint2*>(ct + pix * SFC + a * 16 + 4 * (lane >> 4)) = pk;
      }
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // 256 px x 4 vectors of 8 channels
      const int e = tid + 256 * i, pix = e >> 2, v = e & 3;
      const int oy = oy0 + pix / ST, ox = ox0 + pix % ST;
      if (oy < g.Ho && ox < g.Wo)
        *reinterpret_cast<uint4*>(Y + (((int64_t)f * g.Ho + oy) * g.Wo + ox) * SCO + v * 8) =
            *reinterpret_cast<const uint4*>(ct + pix * SFC + v * 8);
    }
  }
  if (stats_on) {
    // lanes with equal lane >> 4 hold the same 4 channels (per a): shuffles over lane & 15, then
    // the 4 waves in order through LDS
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sv = s_acc[a][r], qv = q_acc[a][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          sv += __shfl_xor(sv, o, 64);
          qv += __shfl_xor(qv, o, 64);
        }
        if ((lane & 15) == 0) {
          red[0][wave][a * 16 + 4 * (lane >> 4) + r] = sv;
          red[1][wave][a * 16 + 4 * (lane >> 4) + r] = qv;
        }
      }
    lds_barrier();
    if (tid < 2 * SCO) {
      const int which = tid / SCO, c = tid % SCO;
      stats[((int64_t)blockIdx.x * 2 + which) * SCO + c] =
          ((red[which][0][c] + red[which][1][c]) + red[which][2][c]) + red[which][3][c];
    }
  }
}

template <typename T>
int launch_stem_fwd(hipStream_t s, const StemGeom& g, const void* x, const float* w, T* Y, float* stats,
                    int* stat_rows) {
  const int64_t ntiles = (int64_t)g.frames * cdiv(g.Ho, ST) * cdiv(g.Wo, ST);
  // dense uint8 frames only: the strided-input instantiation spills at 168 VGPRs
  const bool occ3 = sizeof(T) == 2 && tune(TK_STEM_OCC) == 3 && g.in.u8 == 2;
  const int gx = (int)std::min<int64_t>(ntiles, occ3 ? 768 : 1024);  // whole rounds of co-resident workgroups
  if constexpr (sizeof(T) == 2) {
    const bool dense = g.in.u8 == 2;
    if (occ3)
      hipLaunchKernelGGL((stem_fwd_mfma_kernel<T, 3, 2>), dim3(gx), dim3(256), 0, s, g, x, w, Y, stats, ntiles);
    else if (dense)
      hipLaunchKernelGGL((stem_fwd_mfma_kernel<T, 2, 2>), dim3(gx), dim3(256), 0, s, g, x, w, Y, stats, ntiles);
    else
      hipLaunchKernelGGL((stem_fwd_mfma_kernel<T, 2, -1>), dim3(gx), dim3(256), 0, s, g, x, w, Y, stats, ntiles);
  } else {  // fp32 parity mode: exact fp32 products
    if (stats)
      hipLaunchKernelGGL((stem_fwd_kernel<T, true>), dim3(gx), dim3(256), 0, s, g, x, w, Y, stats, ntiles);
    else
      hipLaunchKernelGGL((stem_fwd_kernel<T, false>), dim3(gx), dim3(256), 0, s, g, x, w, Y, stats, ntiles);
  }
  DFD_HIP_CHECK(hipGetLastError());
  if (stat_rows) *stat_rows = gx;
  return 0;
}

template <typename T>
int launch_stem_wgrad(hipStream_t s, const StemGeom& g, const void* x, const T* dY, const T* Yb, const float* coef,
                      float* slab, int64_t slab_cap, float* dW, bool accumulate) {
  const int64_t ntiles = (int64_t)g.frames * cdiv(g.Ho, ST) * cdiv(g.Wo, ST);
  int gx = (int)std::min<int64_t>(ntiles, 1024);
  gx = (int)std::max<int64_t>(1, std::min<int64_t>(gx, slab_cap / (27 * SCO)));
  if constexpr (sizeof(T) == 2)
    hipLaunchKernelGGL((stem_wgrad_mfma_kernel<T>), dim3(gx), dim3(256), 0, s, g, x, dY, Yb, coef, slab, ntiles);
  else  // fp32 parity mode: exact fp32 products
    hipLaunchKernelGGL((stem_wgrad_kernel<T>), dim3(gx), dim3(256), 0, s, g, x, dY, Yb, coef, slab, ntiles);
  DFD_HIP_CHECK(hipGetLastError());
  return launch_reduce_slabs(s, slab, gx, 27 * SCO, dW, accumulate);
}

template int launch_stem_fwd<float>(hipStream_t, const StemGeom&, const void*, const float*, float*, float*, int*);
template int launch_stem_fwd<bf16>(hipStream_t, const StemGeom&, const void*, const float*, bf16*, float*, int*);
template int launch_stem_fwd<f16>(hipStream_t, const StemGeom&, const void*, const float*, f16*, float*, int*);
template int launch_stem_wgrad<float>(hipStream_t, const StemGeom&, const void*, const float*, const float*,
                                      const float*, float*, int64_t, float*, bool);
template int launch_stem_wgrad<bf16>(hipStream_t, const StemGeom&, const void*, const bf16*, const bf16*,
                                     const float*, float*, int64_t, float*, bool);
template int launch_stem_wgrad<f16>(hipStream_t, const StemGeom&, const void*, const f16*, const f16*,
                                     const float*, float*, int64_t, float*, bool);

}  // namespace dfd
