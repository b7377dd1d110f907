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
  const float* src;  // [rows][cols] fp32, read once
  void* dst;         // T [rows][cols] (null: not wanted)
  void* dst_t;       // T [cols][rows], the transpose (null: not wanted)
  int rows, cols;
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
int launch_wcast(hipStream_t s, const VitCast& cs, int nseg);
int launch_gcn_mix(hipStream_t s, const float* A, const float* F, int B, int N, int D, bool transpose, float* H);
int launch_relu_drop(hipStream_t s, float* Y, float* D, int64_t n, uint64_t seed, uint32_t st, float p);
int launch_relu_drop_bwd(hipStream_t s, const float* Y, const float* dD, float* dY, int64_t n, uint64_t seed,
                         uint32_t st, float p);
int launch_node_mean(hipStream_t s, const float* H, int B, int N, int D, float* G);
int launch_node_mean_bwd(hipStream_t s, const float* dG, int B, int N, int D, float* dH);

enum GeluPass { GELU_PAIR = 0, GELU_MULD = 1 };
int launch_gelu(hipStream_t s, bf16* Z, bf16* out, int64_t n, int mode);

// The large bf16 GEMMs of the trunk (k_vgemm.hip): 256 x 256 / 256 x 128 tiles, LDS-DMA double buffering.
// NT: C[M][N] = A[M][K] . B[N][K]^T with the epilogue flags below (fp32, rounded once);
// TN: W[P][Q] = sum_m X1[m][p] X2[m][q] (fp32, split over m into slabs summed in a fixed order).
// VG_GELU2: Z = the rounded pre-activation, G = gelu(Z) and C = gelu'(Z) (the MLP backward needs only
// the derivative: computing it here, where erf(Z) is at hand, keeps the erf out of the backward);
// VG_DGELU: C *= Z[m][n] with Z the derivative a VG_GELU2 launch stored
// VG_RELU: relu after the bias and residual (the ResNet-50 eval 1x1 convolutions, k_rnconv.hip)
enum VgEpi { VG_BIAS = 1, VG_RESID = 2, VG_GELU2 = 4, VG_DGELU = 8, VG_RELU = 16, VG_GELU = 32 };
struct VgemmArgs {
  const bf16* A;
  const bf16* B;
  bf16* C;
  const bf16* R;      // residual [M][ldc] (VG_RESID)
  const float* bias;  // [N] (VG_BIAS)
  const bf16* Z;      // gelu'(pre-activation) [M][ldc] (VG_DGELU)
  bf16* G;            // gelu(pre-activation) [M][ldc] (VG_GELU2)
  int64_t lda, ldb, ldc;
  int M, N, K, tiles_n;
  int bn;             // tile width 256 / 128; 0: chosen by shape (launch_vgemm_nt)
  // implicit convolution (conv != 0): A is the NHWC input [N][H][W][Cin] (Cin = 2^cin_log2, a multiple of
  // 64), row m = output pixel (n, oy, ox), column k = (kh * KW + kw) * Cin + ci; zero outside the map
  int conv, H, W, Ho, Wo, cin_log2, KW, stride, pad;
};
struct VgemmTnArgs {
  const bf16* X1;
  const bf16* X2;
  float* slab;        // [split][P*Q (+ P when colsum)]
  int64_t ld1, ld2;
  int M, P, Q, tiles_p, tiles_q, mchunk;
  int colsum;         // also sum X1's columns (a linear's bias gradient) into the slab rows' tail
  // cooperative split reduction (coop launches): the splits of a tile meet at a group barrier and each
  // sums its share of the tile's rows over all splits (fixed order) into W (+ colsum_out)
  unsigned* bar;      // 2 zeroed counters per tile
  float* W;
  float* colsum_out;
  int splits, accumulate;
};
bool vgemm_nt_covers(int64_t M, int N, int K);
bool vgemm_conv_covers(int Cin, int Cout, int KH, int KW);
bool vgemm_tn_covers(int64_t M, int P, int Q);
int launch_vgemm_nt(hipStream_t s, const VgemmArgs& a, int ep);
int vgemm_tn_splits(int64_t M, int P, int Q, int64_t slab_cap);
// colsum_out (optional): colsum_out[p] = sum_m X1[m][p] in the same launch (the slab then needs
// splits x (P*Q + P) floats: vgemm_tn_splits(M, P, Q + 1, ...) x P x (Q + 1) is enough)
// bar (optional): 2 x (P/256) x (Q/256) zeroed unsigned counters (zero again when the launch ends): the
// split partial sums are then reduced inside the launch (cooperative, when the grid fits the device at
// once) instead of by separate slab-reduction launches
int launch_vgemm_tn(hipStream_t s, const bf16* X1, int64_t ld1, const bf16* X2, int64_t ld2, int64_t M, int P, int Q,
                    float* slab, int64_t slab_cap, float* W, bool accumulate, float* colsum_out = nullptr,
                    unsigned* bar = nullptr);
// counters launch_vgemm_tn's cooperative form needs for a P x Q product
inline int vgemm_tn_bar_count(int P, int Q) { return 2 * (P / 256) * (Q / 256); }

template <typename T>
__device__ __forceinline__ void lds_st8v(T* p, const float (&v)[8]) { st8(p, v); }

}  // namespace dfd
