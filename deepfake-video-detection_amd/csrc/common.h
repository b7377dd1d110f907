// Shared device helpers for the gfx950 (MI355X) kernels of the EfficientNet-B0 hot path.
//
// Storage types: `float` (fp32 parity mode) and `bf16` (raw 16-bit brain-float, the
// performance mode).  All arithmetic accumulates in fp32.  Activations are NHWC
// ("[M][C]", M = frames*H*W rows, C contiguous), every channel count on the path is a
// multiple of 8, so the unit of every global access is an 8-element vector
// (16 B for bf16, 2 x 16 B for fp32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace dfd {

// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1 (static register-array indices)
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}


struct bf16 {
  uint16_t x;
};

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
// hardware round-to-nearest-even (v_cvt_pk_bf16_f32; NaN stays NaN)
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{lo, hi}), bf16x2_t));
}
__device__ __forceinline__ uint16_t f2bf(float f) { return (uint16_t)(pack2bf(f, 0.f) & 0xffffu); }

// IEEE half (fp16 storage mode, v_mfma_f32_16x16x32_f16): conversions round to nearest even
// (v_cvt_f16_f32; NaN stays NaN, overflow -> inf, which the loss scaler sees)
struct f16 {
  uint16_t x;
};
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float h2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ uint32_t pack2h(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, f16x2_t{(_Float16)lo, (_Float16)hi});
}
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
// the low / high 16-bit element of a packed word as fp32
__device__ __forceinline__ float lo2f(uint32_t w, f16*) { return h2f((uint16_t)(w & 0xffffu)); }
__device__ __forceinline__ float hi2f(uint32_t w, f16*) { return h2f((uint16_t)(w >> 16)); }
__device__ __forceinline__ float lo2f(uint32_t w, struct bf16*) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi2f(uint32_t w, struct bf16*) { return __uint_as_float(w & 0xffff0000u); }

template <typename T> struct Tr;
template <> struct Tr<float> {
  static constexpr int kDtype = 0;
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
  __device__ __forceinline__ static float round(float v) { return v; }
};
template <> struct Tr<bf16> {
  static constexpr int kDtype = 1;
  __device__ __forceinline__ static float to_f(bf16 v) { return bf2f(v.x); }
  __device__ __forceinline__ static bf16 from_f(float v) { return bf16{f2bf(v)}; }
  __device__ __forceinline__ static float round(float v) { return bf2f(f2bf(v)); }
  __device__ __forceinline__ static uint32_t pack2(float lo, float hi) { return pack2bf(lo, hi); }
};
template <> struct Tr<f16> {
  static constexpr int kDtype = 2;
  __device__ __forceinline__ static float to_f(f16 v) { return h2f(v.x); }
  __device__ __forceinline__ static f16 from_f(float v) { return f16{f2h(v)}; }
  __device__ __forceinline__ static float round(float v) { return h2f(f2h(v)); }
  __device__ __forceinline__ static uint32_t pack2(float lo, float hi) { return pack2h(lo, hi); }
};
// 16-bit storage types (bf16, f16): the MFMA operand paths; is_bf16: the kernels that exist for bf16 only
template <typename T> constexpr bool is16 = sizeof(T) == 2;
template <typename T> constexpr bool is_bf16 = std::is_same<T, bf16>::value;

// 16 x 16 x 32 MFMA on 8 packed 16-bit operands per lane (bf16 or fp16 by storage type)
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4m_t __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ f32x4m_t mfma16x16x32(s16x8_t a, s16x8_t b, f32x4m_t c) {
  if constexpr (std::is_same<T, f16>::value) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
  } else {
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
  }
}

// ---- 8-element vector load/store (p must be 16-B aligned for bf16, 32-B for fp32) ----
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void ld8(const bf16* p, float (&v)[8]) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xffff0000u);
  v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xffff0000u);
  v[4] = __uint_as_float(a.z << 16); v[5] = __uint_as_float(a.z & 0xffff0000u);
  v[6] = __uint_as_float(a.w << 16); v[7] = __uint_as_float(a.w & 0xffff0000u);
}
__device__ __forceinline__ void ld8(const f16* p, float (&v)[8]) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  v[0] = lo2f(a.x, (f16*)nullptr); v[1] = hi2f(a.x, (f16*)nullptr);
  v[2] = lo2f(a.y, (f16*)nullptr); v[3] = hi2f(a.y, (f16*)nullptr);
  v[4] = lo2f(a.z, (f16*)nullptr); v[5] = hi2f(a.z, (f16*)nullptr);
  v[6] = lo2f(a.w, (f16*)nullptr); v[7] = hi2f(a.w, (f16*)nullptr);
}
__device__ __forceinline__ void st8(f16* p, const float (&v)[8]) {
  uint4 a;
  a.x = pack2h(v[0], v[1]); a.y = pack2h(v[2], v[3]);
  a.z = pack2h(v[4], v[5]); a.w = pack2h(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = a;
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void st8(bf16* p, const float (&v)[8]) {
  uint4 a;
  a.x = pack2bf(v[0], v[1]); a.y = pack2bf(v[2], v[3]);
  a.z = pack2bf(v[4], v[5]); a.w = pack2bf(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = a;
}
__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) { ld8(p, v); }

// ---- raw (unconverted) 8-element vectors for register prefetch ----
// Masked loads are branch-free and wait-free: a masked-off lane loads from `safe` (a valid
// address of the same tensor) and carries ok = false; the zero is selected when the value is
// CONSUMED (raw_to_f / raw_st), after the wait the consumer needs anyway.  A guarded
// `if (ok) ld8(...)`, or zeroing the destination right after the load, makes hipcc emit a
// branch and an s_waitcnt vmcnt(0) per load, serialising every global round trip.
template <typename T> struct Raw8;
template <> struct Raw8<bf16> { uint4 a; bool ok; };
template <> struct Raw8<float> { float4 a, b; bool ok; };
template <> struct Raw8<f16> { uint4 a; bool ok; };
__device__ __forceinline__ void raw_ld(Raw8<f16>& r, const f16* p, const f16* safe, bool ok) {
  r.a = *reinterpret_cast<const uint4*>(ok ? p : safe);
  r.ok = ok;
}
__device__ __forceinline__ void raw_to_f(const Raw8<f16>& r, float (&v)[8]) {
  const uint32_t m = r.ok ? 0xffffffffu : 0u;
  const uint32_t x = r.a.x & m, y = r.a.y & m, z = r.a.z & m, w = r.a.w & m;
  v[0] = lo2f(x, (f16*)nullptr); v[1] = hi2f(x, (f16*)nullptr);
  v[2] = lo2f(y, (f16*)nullptr); v[3] = hi2f(y, (f16*)nullptr);
  v[4] = lo2f(z, (f16*)nullptr); v[5] = hi2f(z, (f16*)nullptr);
  v[6] = lo2f(w, (f16*)nullptr); v[7] = hi2f(w, (f16*)nullptr);
}
__device__ __forceinline__ void raw_st(f16* p, const Raw8<f16>& r) {
  const uint32_t m = r.ok ? 0xffffffffu : 0u;
  *reinterpret_cast<uint4*>(p) = make_uint4(r.a.x & m, r.a.y & m, r.a.z & m, r.a.w & m);
}

__device__ __forceinline__ void raw_ld(Raw8<bf16>& r, const bf16* p, const bf16* safe, bool ok) {
  r.a = *reinterpret_cast<const uint4*>(ok ? p : safe);
  r.ok = ok;
}
__device__ __forceinline__ void raw_ld(Raw8<float>& r, const float* p, const float* safe, bool ok) {
  const float* q = ok ? p : safe;
  r.a = *reinterpret_cast<const float4*>(q);
  r.b = *reinterpret_cast<const float4*>(q + 4);
  r.ok = ok;
}
__device__ __forceinline__ void raw_to_f(const Raw8<bf16>& r, float (&v)[8]) {
  const uint32_t m = r.ok ? 0xffffffffu : 0u;
  const uint32_t x = r.a.x & m, y = r.a.y & m, z = r.a.z & m, w = r.a.w & m;
  v[0] = __uint_as_float(x << 16); v[1] = __uint_as_float(x & 0xffff0000u);
  v[2] = __uint_as_float(y << 16); v[3] = __uint_as_float(y & 0xffff0000u);
  v[4] = __uint_as_float(z << 16); v[5] = __uint_as_float(z & 0xffff0000u);
  v[6] = __uint_as_float(w << 16); v[7] = __uint_as_float(w & 0xffff0000u);
}
__device__ __forceinline__ void raw_to_f(const Raw8<float>& r, float (&v)[8]) {
  v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w;
  v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
  if (!r.ok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
}
__device__ __forceinline__ void raw_st(bf16* p, const Raw8<bf16>& r) {
  const uint32_t m = r.ok ? 0xffffffffu : 0u;
  *reinterpret_cast<uint4*>(p) = make_uint4(r.a.x & m, r.a.y & m, r.a.z & m, r.a.w & m);
}
__device__ __forceinline__ void raw_st(float* p, const Raw8<float>& r) {
  float v[8];
  raw_to_f(r, v);
  st8(p, v);
}

// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch): remap the
// dispatch index so that LOGICALLY consecutive blocks share one XCD and its L2 (blocks that read the
// same operand tile then fetch it once per XCD instead of once per block).  A speed hint only:
// correctness never depends on the placement.
__device__ __forceinline__ int xcd_swizzle(int b, int n) {
  const int full = n & ~7;
  if (b >= full) return b;
  return (b & 7) * (full >> 3) + (b >> 3);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads (prefetches stay in flight) or stores.  __syncthreads() carries a
// workgroup-scope fence that drains vmcnt to 0 whenever a global store is pending.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// ---- activations ----
// v_exp_f32 + v_rcp_f32 (1 ulp); an IEEE division here costs ~10 VALU ops per element
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float siluf_(float x) { return x * sigmoidf_(x); }
// d/dx silu(x) = s (1 + x (1 - s))
__device__ __forceinline__ float dsiluf_(float x) {
  const float s = sigmoidf_(x);
  return s * (1.0f + x * (1.0f - s));
}

// ---- wave reductions (wave64) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ __forceinline__ int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Activation-prologue modes for kernels that consume a pre-BN tensor Y:
//   PRO_NONE      a = y
//   PRO_BN_SILU   a = silu(y*scale[c] + shift[c])
//   PRO_BN_SILU_G a = silu(y*scale[c] + shift[c]) * gate[frame][c]
//   PRO_GELU      a = gelu(y)   (exact erf form; ViT MLP, no per-channel parameters)
//   PRO_GATE      a = y * gate[frame][c]   (y already activated: a materialised silu(bn(.)))
enum ProMode { PRO_NONE = 0, PRO_BN_SILU = 1, PRO_BN_SILU_G = 2, PRO_GELU = 3, PRO_GATE = 4 };
constexpr bool pro_is_gated(int mode) { return mode == PRO_BN_SILU_G || mode == PRO_GATE; }
constexpr bool pro_is_bn(int mode) { return mode == PRO_BN_SILU || mode == PRO_BN_SILU_G; }

// torch.nn.functional.gelu (approximate='none'): 0.5 x (1 + erf(x / sqrt 2)) and its derivative
__device__ __forceinline__ float geluf_(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float dgeluf_(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
// gelu(x) and gelu'(x) from one erf (the same expressions as geluf_ / dgeluf_: identical values)
// erf as a branch-free odd/even rational minimax form on [-4, 4] (|x| > 4: +-1 in fp32): 12 FMAs and a
// division, max |error| 4e-7 against the correctly rounded fp32 erf (CPU check over N(0, 1.5^2)
// inputs: 0.3 % of bf16-rounded gelu values move one ulp, all of them |gelu| < 1e-2 but 0.006 %).
// For the bf16 GEMM epilogue (fc1's gelu / gelu' pair), where the library erff's range branches
// diverge inside every wave.
__device__ __forceinline__ float erf_rat_(float x) {
  x = fminf(fmaxf(x, -4.f), 4.f);
  const float x2 = x * x;
  float p = fmaf(x2, -2.72614225801306e-10f, 2.77068142495902e-08f);
  p = fmaf(x2, p, -2.10102402082508e-06f);
  p = fmaf(x2, p, -5.69250639462346e-05f);
  p = fmaf(x2, p, -7.34990630326855e-04f);
  p = fmaf(x2, p, -2.95459980854025e-03f);
  p = fmaf(x2, p, -1.60960333262415e-02f);
  p *= x;
  float q = fmaf(x2, -1.45660718464996e-05f, -2.13374055278905e-04f);
  q = fmaf(x2, q, -1.68282697438203e-03f);
  q = fmaf(x2, q, -7.37332916720468e-03f);
  q = fmaf(x2, q, -1.42647390514189e-02f);
  return p / q;
}
__device__ __forceinline__ void gelu_pair_rat_(float x, float& g, float& d) {
  const float e = 1.0f + erf_rat_(x * 0.70710678118654752f);
  g = 0.5f * x * e;
  d = 0.5f * e + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
// the same pair for two values at once: the polynomial chains as packed-f32 FMAs (v_pk_fma_f32, two
// lanes per instruction), the quotient by v_rcp_f32 (1 ulp) instead of the IEEE division sequence,
// exp(-x^2 / 2) from the scaled argument's square.  For fc1's epilogue, whose per-element VALU work
// ran longer than the tile's stores (k_vgemm.hip).
__device__ __forceinline__ void gelu_pair2_rat_(f32x2_t x, f32x2_t& g, f32x2_t& d) {
  const f32x2_t u = x * 0.70710678118654752f;
  const f32x2_t uc = {fminf(fmaxf(u.x, -4.f), 4.f), fminf(fmaxf(u.y, -4.f), 4.f)};
  const f32x2_t x2 = uc * uc;
  auto fma2 = [](f32x2_t a, f32x2_t b, f32x2_t c) { return __builtin_elementwise_fma(a, b, c); };
  auto splat = [](float v) { return f32x2_t{v, v}; };
  f32x2_t p = fma2(x2, splat(-2.72614225801306e-10f), splat(2.77068142495902e-08f));
  p = fma2(x2, p, splat(-2.10102402082508e-06f));
  p = fma2(x2, p, splat(-5.69250639462346e-05f));
  p = fma2(x2, p, splat(-7.34990630326855e-04f));
  p = fma2(x2, p, splat(-2.95459980854025e-03f));
  p = fma2(x2, p, splat(-1.60960333262415e-02f));
  p *= uc;
  f32x2_t q = fma2(x2, splat(-1.45660718464996e-05f), splat(-2.13374055278905e-04f));
  q = fma2(x2, q, splat(-1.68282697438203e-03f));
  q = fma2(x2, q, splat(-7.37332916720468e-03f));
  q = fma2(x2, q, splat(-1.42647390514189e-02f));
  const f32x2_t e = fma2(p, f32x2_t{__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)}, splat(1.0f));
  g = (x * 0.5f) * e;
  const f32x2_t uu = u * u;
  const f32x2_t ex = {__expf(-uu.x), __expf(-uu.y)};
  d = fma2(x * 0.39894228040143268f, ex, e * 0.5f);
}
__device__ __forceinline__ void gelu_pair_(float x, float& g, float& d) {
  const float e = 1.0f + erff(x * 0.70710678118654752f);
  g = 0.5f * x * e;
  d = 0.5f * e + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

struct Pro {
  const float* scale;  // [C]
  const float* shift;  // [C]
  const float* gate;   // [frames][C]
  int rows_per_frame;  // H*W of the consumed tensor
  int C;
};

template <int MODE>
__device__ __forceinline__ void apply_pro8(const Pro& pr, int64_t row, int c0, float (&v)[8]) {
  if constexpr (MODE == PRO_NONE) {
    return;
  } else {
    float sc[8], sh[8];
    ld8f(pr.scale + c0, sc);
    ld8f(pr.shift + c0, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = siluf_(v[j] * sc[j] + sh[j]);
    if constexpr (MODE == PRO_BN_SILU_G) {
      const int64_t f = row / pr.rows_per_frame;
      float g[8];
      ld8f(pr.gate + f * pr.C + c0, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= g[j];
    }
  }
}

// producer BN+SiLU(+gate) on 8 channels with per-lane preloaded scale/shift; gate row given
template <int MODE>
__device__ __forceinline__ void pro8_pre(float (&v)[8], const float (&sc)[8], const float (&sh)[8], const float* gate) {
  if constexpr (MODE != PRO_NONE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * sc[j] + sh[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * sigmoidf_(v[j]);
    if constexpr (MODE == PRO_BN_SILU_G) {
      float g[8];
      ld8f(gate, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= g[j];
    }
  }
}

}  // namespace dfd

#define DFD_TRY(x) do { if ((x) != 0) return -1; } while (0)

#define DFD_HIP_CHECK(expr)                                                     \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      dfd::set_error(hipGetErrorString(_e), __FILE__, __LINE__);                \
      return -1;                                                                \
    }                                                                           \
  } while (0)

namespace dfd {
void set_error(const char* msg, const char* file, int line);
}
