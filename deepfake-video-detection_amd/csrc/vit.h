// ViT-B/16 + SimpleGCN (DeepfakeModel, src/models.py:88-107, 199-291) launchers: attention /
// LayerNorm / token kernels (k_vit.hip) and the model orchestration (vit.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace dfd {

constexpr int VIT_PATCH = 16;
constexpr int VIT_SM_PER_LANE = 4;  // softmax rows up to 256 wide (197 tokens, ld 200)
constexpr int VIT_LN_VEC = 2;       // LayerNorm rows up to 2 x 64 x 8 = 1024 wide
constexpr int VIT_LN_MAXC = 1024;

// operand addressing of the batched GEMM: batch b -> (b / inner) * s_outer + (b % inner) * s_inner
struct BgOp {
  int64_t ld;
  int inner;
  int64_t s_outer, s_inner;
  __host__ __device__ int64_t off(int b) const { return (int64_t)(b / inner) * s_outer + (int64_t)(b % inner) * s_inner; }
};

// fp32 image batch (B, N, 3, H, W) with element strides
struct VitImg {
  int nodes, H, W;
  int64_t sb, sn, sc, sh, sw;
};

struct VitCastSeg {
  const float* src;  // [rows][cols] fp32
  void* dst;         // T [rows][cols] or, transposed, [cols][rows]
  int rows, cols, transpose;
};
struct VitCast {
  VitCastSeg seg[8];
};

template <typename T>
int launch_bgemm(hipStream_t s, bool ta, bool tb, int batch, int M, int N, int K, float alpha, const T* A,
                 const BgOp& a, const T* B, const BgOp& b, T* C, const BgOp& c);
template <typename T>
int launch_softmax_fwd(hipStream_t s, const T* S, T* P, int64_t rows, int n, int ld);
template <typename T>
int launch_softmax_bwd(hipStream_t s, const T* P, const T* dP, T* dS, int64_t rows, int n, int ld, float scale);
template <typename T, typename O>
int launch_ln_fwd(hipStream_t s, const T* X, int64_t ldx, const float* g, const float* b, O* Y, int64_t ldy, float* mean,
                  float* rstd, int64_t rows, int C, float eps);
template <typename T, typename D>
int launch_ln_bwd(hipStream_t s, const T* X, int64_t ldx, const D* dY, int64_t ldd, const float* g, const float* mean,
                  const float* rstd, const T* dres, T* dX, int64_t rows, int C, float* part, int64_t part_cap,
                  float* dgamma, float* dbeta, bool accumulate);
template <typename T>
int launch_patch_gather(hipStream_t s, const float* x, const VitImg& im, int images, T* A);
template <typename T>
int launch_tokens_fwd(hipStream_t s, const T* PE, const float* cls, const float* pos, int images, int ntok, int D, T* X0);
template <typename T>
int launch_tokens_bwd(hipStream_t s, const T* dX0, int images, int ntok, int D, T* dPE, float* dpos, float* dcls);
template <typename T>
int launch_colsum(hipStream_t s, const T* X, int64_t M, int N, float* part, int64_t part_cap, float* out,
                  bool accumulate);
template <typename T>
int launch_wcast(hipStream_t s, const VitCast& cs, int nseg, int max_rows, int max_cols);
int launch_gcn_mix(hipStream_t s, const float* A, const float* F, int B, int N, int D, bool transpose, float* H);
int launch_relu_drop(hipStream_t s, float* Y, float* D, int64_t n, uint64_t seed, uint32_t st, float p);
int launch_relu_drop_bwd(hipStream_t s, const float* Y, const float* dD, float* dY, int64_t n, uint64_t seed,
                         uint32_t st, float p);
int launch_node_mean(hipStream_t s, const float* H, int B, int N, int D, float* G);
int launch_node_mean_bwd(hipStream_t s, const float* dG, int B, int N, int D, float* dH);

int launch_gelu(hipStream_t s, const bf16* Z, bf16* out, int64_t n, bool backward);

template <typename T>
__device__ __forceinline__ void lds_st8v(T* p, const float (&v)[8]) { st8(p, v); }

}  // namespace dfd
