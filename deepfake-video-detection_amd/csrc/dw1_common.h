// Shared helpers of the channel-pair depthwise kernels (k_dw_fwd1.hip, k_dw_bwd1.hip): a lane owns
// two adjacent channels, held as a packed fp32 pair (v_pk_fma_f32 math), loaded from NHWC global
// memory as one dword (bf16) or dwordx2 (fp32).
#pragma once
#include "dw_common.h"

#ifndef DFD_DW_XCD
// XCD-aware workgroup order of the channel-pair depthwise kernels: the channel groups of one
// spatial tile (and consecutive tiles) are dealt to workgroups that share an XCD (A/B knob)
#define DFD_DW_XCD -1  // -1: per-shape rule in the launchers; 0 / 1: force off / on
#endif

namespace dfd {

typedef float v2f __attribute__((ext_vector_type(2)));

struct Dw1Bn2 {           // the fused BN2(+SiLU, SE gate) backward of the staging
  const float* gate;      // [frames][C]
  const float* bc;        // [frames][C]
  const float* sc;        // BN2 scale (gamma*invstd), shift
  const float* sh;
  const float* coef;      // [3][C]: k1, k2, k3 of bn_bwd_finalize_frames
};

// raw two-channel global load and its unpacking
template <typename T> struct Raw2;
template <> struct Raw2<bf16> { uint32_t v; };
template <> struct Raw2<float> { float2 v; };
__device__ __forceinline__ void raw2_ld(Raw2<bf16>& r, const bf16* p) { r.v = *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ void raw2_ld(Raw2<float>& r, const float* p) { r.v = *reinterpret_cast<const float2*>(p); }
__device__ __forceinline__ v2f raw2_f(const Raw2<bf16>& r) {
  return v2f{__uint_as_float(r.v << 16), __uint_as_float(r.v & 0xffff0000u)};
}
__device__ __forceinline__ v2f raw2_f(const Raw2<float>& r) { return v2f{r.v.x, r.v.y}; }
// "redefine" a raw pair at this point: values derived from it cannot be hoisted above (keeps the
// 1-VGPR bf16 pair live instead of its 2-VGPR fp32 expansion across a long loop)
__device__ __forceinline__ void pin2(Raw2<bf16>& r) { asm volatile("" : "+v"(r.v)); }
__device__ __forceinline__ void pin2(Raw2<float>& r) { asm volatile("" : "+v"(r.v.x), "+v"(r.v.y)); }
// pairs of an 8-element raw vector
__device__ __forceinline__ v2f raw8_pair(const Raw8<bf16>& r, int q) {
  const uint32_t w = q == 0 ? r.a.x : q == 1 ? r.a.y : q == 2 ? r.a.z : r.a.w;
  return v2f{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
__device__ __forceinline__ v2f raw8_pair(const Raw8<float>& r, int q) {
  return q == 0 ? v2f{r.a.x, r.a.y} : q == 1 ? v2f{r.a.z, r.a.w} : q == 2 ? v2f{r.b.x, r.b.y} : v2f{r.b.z, r.b.w};
}
__device__ __forceinline__ v2f round2(v2f v, bf16*) {
  const uint32_t w = pack2bf(v.x, v.y);
  return v2f{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
__device__ __forceinline__ v2f round2(v2f v, float*) { return v; }
__device__ __forceinline__ void st2(bf16* p, v2f v) { *reinterpret_cast<uint32_t*>(p) = pack2bf(v.x, v.y); }
__device__ __forceinline__ void st2(float* p, v2f v) { *reinterpret_cast<float2*>(p) = make_float2(v.x, v.y); }
// fp16 storage (the half-precision mode): the same helpers with IEEE-half packing
template <> struct Raw2<f16> { uint32_t v; };
__device__ __forceinline__ void raw2_ld(Raw2<f16>& r, const f16* p) { r.v = *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ v2f raw2_f(const Raw2<f16>& r) { return v2f{lo2f(r.v, (f16*)nullptr), hi2f(r.v, (f16*)nullptr)}; }
__device__ __forceinline__ void pin2(Raw2<f16>& r) { asm volatile("" : "+v"(r.v)); }
__device__ __forceinline__ v2f raw8_pair(const Raw8<f16>& r, int q) {
  const uint32_t w = q == 0 ? r.a.x : q == 1 ? r.a.y : q == 2 ? r.a.z : r.a.w;
  return v2f{lo2f(w, (f16*)nullptr), hi2f(w, (f16*)nullptr)};
}
__device__ __forceinline__ v2f round2(v2f v, f16*) {
  const uint32_t w = pack2h(v.x, v.y);
  return v2f{lo2f(w, (f16*)nullptr), hi2f(w, (f16*)nullptr)};
}
__device__ __forceinline__ void st2(f16* p, v2f v) { *reinterpret_cast<uint32_t*>(p) = pack2h(v.x, v.y); }
// base + a 32-bit BYTE offset: the uniform frame base stays in SGPRs and each access is one
// global_load/store with a 32-bit VGPR offset (no per-lane 64-bit address arithmetic)
template <typename T> __device__ __forceinline__ const T* boff(const T* base, uint32_t off) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
}
template <typename T> __device__ __forceinline__ T* boff(T* base, uint32_t off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}
__device__ __forceinline__ v2f lds2(const float* p) { return *reinterpret_cast<const v2f*>(p); }
__device__ __forceinline__ v2f sigmoid2(v2f z) { return v2f{sigmoidf_(z.x), sigmoidf_(z.y)}; }
__device__ __forceinline__ v2f fma2(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }

// the final fixed-order reduction helper: lanes l, l^16, l^32, l^48 of a wave hold the same channel
// pair; (a+b)+(c+d) is the same sum on every lane (commutative adds)
__device__ __forceinline__ void lane_sum4(v2f& v) {
  v.x += __shfl_xor(v.x, 16, 64);
  v.y += __shfl_xor(v.y, 16, 64);
  v.x += __shfl_xor(v.x, 32, 64);
  v.y += __shfl_xor(v.y, 32, 64);
}

}  // namespace dfd
