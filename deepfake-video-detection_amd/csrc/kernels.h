// Internal launcher declarations (host side).  Every launcher enqueues on `stream`
// and returns 0 on success / -1 with dfd::set_error() on failure.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

#include "bnfin.h"
#include "common.h"

namespace dfd {

// ---------------- pointwise (1x1 conv) GEMMs: k_gemm.hip ----------------
// C[M][N] = pro(A)[M][K] * B[N][K]^T (+ R[M][N]); optional BN-stat partials of C's columns
// into stats[gridDim.x][2][N] (rows written = *stat_rows).
template <typename T>
int launch_pw_gemm(hipStream_t s, const T* A, const T* B, T* C, const T* R, int64_t M, int N, int K,
                   int pro_mode, const Pro& pro, float* stats, int* stat_rows);
// Streaming variant for tall-skinny 16-bit layers (k_pw_stream.hip; T = bf16 / f16): 0 launched, 1 not
// covered (shape/mode without an instantiation, or M below the streaming threshold), -1 error.
template <typename T>
int launch_pw_stream(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias, int64_t M, int N,
                     int K, int pro_mode, const Pro& pro, float* stats, int* stat_rows);
template <typename T>
int launch_pw_wgrad_stream(hipStream_t s, const T* dY, const T* X, int64_t M, int N, int K, int pro_mode,
                           const Pro& pro, float* slab, int64_t slab_cap, float* dW, bool accumulate);
// Fused projection backward (k_pwl_bwd.hip, T = bf16 / f16): ge2 = gs . W (wt = W^T [K][N]), the weight gradient
// dW[N][K] (+)= gs^T . (silu(y2*sc+sh) * gate) through the slab, and the per-frame SE + BN2 backward
// sums part[5][*hsplit][frames][K] of launch_se_bn_bwd_reduce.  With coef3 (the BN3 backward
// coefficients [3][N]) gs is the block's output gradient dZ and the kernel applies the BN3 backward
// gs = k1*dZ + k2*y3 + k3 while staging (no separate apply pass).  0 launched, 1 not covered, -1 error.
bool pwl_bwd_covers(int frames, int HW, int N, int K);
template <typename T>
int launch_pwl_bwd(hipStream_t s, const T* gs, const T* y3, const float* coef3, const T* wt, const T* y2,
                   const float* sc, const float* sh, const float* mean, const float* invstd, const float* gate,
                   int frames, int HW, int N, int K, T* ge2, float* slab, int64_t slab_cap, float* dW,
                   bool accumulate, float* part, int64_t part_cap, int* hsplit);
// Fused conv_pw backward through its BN on the fold path (k_pw_fold_bwd.hip, T = bf16 / f16): dx = g . w1t^T +
// x . q^T + bv (+ r), and the partial products T = g^T x, G = x^T x, cs = 1^T x summed into T / G / cs
// (launch_reduce_slabs) for pw_wgrad_bn_combine.  0 launched, 1 not covered, -1 error.
template <typename E>
int launch_pw_fold_bwd(hipStream_t s, const E* g, const E* x, const E* r, const E* w1t, const E* q,
                       const float* bv, E* dx, int64_t M, int mid, int cin, float* slab, int64_t slab_cap, float* T,
                       float* G, float* cs);
// Kernel-selection knobs.  No process-wide mutable state is consulted on a model path: every knob
// has a compile-time default (tune_default), a plan's forward/backward installs the plan's own
// overrides (dfd_b0_plan_set_tuning) for the enqueuing thread (TuningScope), and the kernel test
// seams (dfd_pw_conv, dfd_pw_conv_wgrad, dfd_vgemm) install a snapshot of the seam overrides of dfd_set_tuning.
// Concurrent plans -- e.g. inference on a ThreadPoolExecutor worker (app.py:127-129) next to a
// training step -- therefore never read each other's knobs.
enum TuneKey { TK_STREAM_MIN_ROWS = 0, TK_FOLD_MIN_ROWS, TK_DW_BWD_FUSED, TK_GEMM_TILE, TK_DW_BWD1, TK_DW_FWD1,
               TK_WGRAD_STREAM, TK_MBCONV7, TK_PWL_FUSED, TK_FOLD_FUSED, TK_PW_SK, TK_DW_PF, TK_DW_RB, TK_STEM_OCC, TK_VG_XP,
               TK_TAIL_FIN, TK_WG_PF, TK_COUNT };
constexpr int64_t kTuneUnset = INT64_MIN;
struct Tuning {
  int64_t v[TK_COUNT];
  Tuning() { for (auto& x : v) x = kTuneUnset; }
};
// defaults: streaming 1x1 kernels from 40,000 rows; BN-folded conv_pw backward from 100,000 rows;
// fused depthwise backward / channel-pair kernels on; tiled-GEMM config automatic (-1); weight
// gradients on the main stream; fused 7x7 MBConv off; fused projection / fold backward on; small-K
// weight-panel GEMM (k_pw_sk.hip) on for K <= 192; depthwise prefetch / row blocking on; the stem
// forward at 3 workgroups per CU (120 -> 91 us, profiles/r04 kernel_stats_r04h*); the vgemm NT
// fragment-pipelined K loop for the 128-wide tile only (in-model A/B, profiles/r04 ab_vg_xp_r04l:
// the 256-wide form is faster in the L2-warm microbenchmark but not in the ViT step)
#ifndef DFD_VG_XP_DEFAULT  // A/B builds of k_vgemm.o only (tools/ab_lib.sh): the one reader of TK_VG_XP
#define DFD_VG_XP_DEFAULT 1
#endif
// tail_fin: BN finalizes in the producers' last-arriving workgroups (tail.h) instead of their own
// launches (bit 0: the SE-backward chain's BN2 finalize); bit 1: the SE excitation's first product
// split over its channel slices (k_bn.hip SeSplit); bit 2: BN backward finalize inside the apply pass
// (bn_bwd_apply_fin) where the producer wrote <= 256 stat rows; bit 3: forward BN finalize inside the
// consumer (depthwise forward, SE squeeze, global average pool) where the producer wrote <= 128 rows
// (kBnFinRowsMax)
#ifndef DFD_TAIL_FIN_DEFAULT
#define DFD_TAIL_FIN_DEFAULT 15
#endif
// wg_pf: m-steps of loads in flight in the tiled 1x1 weight gradient (pw_wgrad_kernel, bf16)
#ifndef DFD_WG_PF
#define DFD_WG_PF 1
#endif
constexpr int64_t kTuneDefault[TK_COUNT] = {40000, 100000, 1, -1, 1, 1, 0, 0, 1, 1, 1, 1, 1, 3, DFD_VG_XP_DEFAULT,
                                            DFD_TAIL_FIN_DEFAULT, DFD_WG_PF};
extern const char* const kTuneNames[TK_COUNT];
int64_t tune_override(TuneKey k);  // the calling thread's override, or kTuneUnset
inline int64_t tune(TuneKey k) {
  const int64_t o = tune_override(k);
  return o == kTuneUnset ? kTuneDefault[k] : o;
}
struct TuningScope {
  const Tuning* prev;
  explicit TuningScope(const Tuning* t);
  ~TuningScope();
};
// Transformer form of the same kernel: C = pro(A) * B^T  (+bias[n]) (+R) (* gelu'(Z) elementwise),
// pro_mode PRO_NONE or PRO_GELU; epi a mask of GemmEpi.
enum GemmEpi { EPI_RESID = 1, EPI_BIAS = 2, EPI_DGELU = 4 };
// ---------------- ResNet-50 ensemble member (inference): k_resnet.hip ----------------
struct InputFmt;
template <typename T>
int launch_rn_im2col(hipStream_t s, const T* x, int N, int H, int W, int C, int kh, int kw, int stride, int pad,
                     int Kp, T* out);
template <typename T>
int launch_rn_stem_im2col(hipStream_t s, const void* x, const InputFmt& in, const int64_t* strides, int N, int H,
                          int W, T* out);
// conv1 7x7/2 + folded BN + ReLU as an implicit GEMM (bf16; Ho, Wo multiples of 16): Wt [64][152]
int launch_rn_stem_conv(hipStream_t s, const void* x, const InputFmt& in, const int64_t* strides, int N, int H, int W,
                        const bf16* Wt, const float* bias, bf16* out);
template <typename T>
int launch_rn_maxpool(hipStream_t s, const T* x, int N, int H, int W, int C, T* out);
template <typename T>
int launch_rn_avgpool(hipStream_t s, const T* x, int N, int HW, int C, float* out);
// ResNet-50 training pieces (k_rntrain.hip, fp32)
// centred BN apply: out = relu?((y - mean) * sc + beta (+ r))
int rn_bn_act(hipStream_t s, const float* y, const float* mean, const float* sc, const float* beta, const float* r,
              int relu, int64_t M, int C, float* out);
int rn_relu_bwd(hipStream_t s, const float* dout, const float* out, int64_t n, float* g);
int rn_gap_bwd(hipStream_t s, const float* dfeat, const float* out, int N, int HW, int C, float* g);
int rn_bn_train_bwd(hipStream_t s, const float* g, const float* y, int64_t M, int C, const float* mean,
                    const float* invstd, const float* scale, const float* shift, const float* gamma, float* dgamma,
                    float* dbeta, float* stats, float* coef, float* dy);

// Fused 7x7-stage MBConv forward (k_mbconv7.hip): one workgroup per frame, the expanded tensor in LDS
struct Mb7Bn {
  const float* gamma;
  const float* beta;
  float* run_mean;
  float* run_var;
  float* mean;
  float* invstd;
  float* scale;
  float* shift;
};
struct Mb7Args {
  int frames, cin, mid, cout, rd, k, skip, training;
  float momentum, eps;
  const bf16* x;     // block input [F*49][cin]
  const bf16* w1;    // conv_pw [mid][cin] (compute-dtype copy)
  const float* wdw;  // conv_dw [mid][k*k] fp32
  const float* wr;   // SE reduce [rd][mid], bias [rd]; expand [mid][rd], bias [mid]
  const float* br;
  const float* we;
  const float* be;
  const bf16* w3;    // conv_pwl [cout][mid]
  Mb7Bn bn[3];       // bn1, bn2, bn3
  bf16 *y1, *y2, *s2, *y3, *xo;     // saved tensors (training) and the block output
  float *sq, *rpre, *gate, *part;   // SE saved vectors; per-frame BN partial sums [F][2][C]
  unsigned* bar;                    // zeroed grid-barrier counter of this launch
  int* abort;                       // zeroed; set if the grid was not co-resident
  unsigned long long* ts;           // development timing: per-workgroup phase timestamps (nullptr: off)
};
bool mbconv7_supported(int frames, int H, int W, int cin, int mid, int cout, int rd, int k, int s);
int launch_mbconv7_fwd(hipStream_t s, const Mb7Args& a);

// Fused multi-head attention, bf16, head dim 64, <= 256 tokens (k_attn.hip): one workgroup per
// (image, head).  qkv rows of `nt` tokens per image, q / k / v of head h at columns h*64, koff +
// h*64, voff + h*64; O / dO [rows][ldo] with head h at h*64; lse [images*heads][nt] fp32.
struct AttnArgs {
  int images, heads, nt;
  float scale;
  const bf16* qkv;
  int64_t ldq;
  int koff, voff;
  bf16* O;          // forward output (read by the backward for rowsum(dO * O))
  int64_t ldo;
  float* lse;       // forward output / backward input
  const bf16* dO;   // backward input
  int64_t lddo;
  bf16* dqkv;       // backward output, qkv's layout
  int64_t lddq;
};
bool attn_supported(int nt, int head_dim);
// ViT bf16 GEMM backend (vit.cpp): bit 0 own weight-gradient kernels, bit 1 own linears; previous value
int launch_attn_fwd(hipStream_t s, const AttnArgs& a);
int launch_attn_bwd(hipStream_t s, const AttnArgs& a);

// ResNet-50 convolutions as implicit-GEMM MFMA kernels (k_rnconv.hip): C = relu?(conv(X) + bias (+ R))
struct RnConvGeom {
  int N, H, W, Cin, KH, KW, stride, pad, Ho, Wo, cin_log2;
};
template <typename T>
int launch_rn_conv(hipStream_t s, const T* X, const T* Wt, T* C, const T* R, const float* bias, int relu,
                   const RnConvGeom& g, int64_t M, int N, int K);
// plain library GEMMs through hipBLASLt (blaslt.cpp): C = A . B^T + bias (+ R); dW (+)= dY^T . X
int64_t blaslt_calls();  // library GEMM calls so far (the measurement seam only)
int blaslt_linear(hipStream_t s, const bf16* A, const bf16* B, bf16* C, const bf16* R, const float* bias, int64_t M,
                  int N, int K);
int blaslt_wgrad(hipStream_t s, const bf16* dY, const bf16* X, float* dW, int64_t M, int N, int K, bool accumulate);
int blaslt_wgrad_split(hipStream_t s, const bf16* dY, const bf16* X, float* dW, int64_t M, int N, int K, int splits,
                       float* slab, int64_t slab_floats);
int blaslt_gemm(hipStream_t s, int dtype, const void* A, const void* B, void* C, const void* R, const float* bias,
                bool relu, int64_t M, int N, int K);

// small-K (80 / 112 / 192 / 320) 16-bit 1x1 GEMM with the weight panel resident in LDS and LDS-DMA row
// tiles (k_pw_sk.hip; T = bf16 / f16): 0 launched, 1 not covered; stats as launch_pw_gemm (one partial
// row per workgroup, at most max_rows rows), R (residual) or stats, not both
bool pw_sk_covers(int64_t M, int N, int K);
template <typename T>
int launch_pw_sk(hipStream_t s, const T* A, const T* W, T* C, const T* R, int64_t M, int N, int K, float* stats,
                 int max_rows, int* stat_rows);
template <typename T>
int launch_tf_gemm(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias, const T* Z, int64_t M,
                   int N, int K, int pro_mode, int epi);
// dW[N][K] = sum_m dY[m][n] * pro(X)[m][k]  -> written (or added) into dW (fp32) via slabs
template <typename T>
int launch_pw_wgrad(hipStream_t s, const T* dY, const T* X, int64_t M, int N, int K, int pro_mode,
                    const Pro& pro, float* slab, int64_t slab_cap, float* dW, bool accumulate);

// ---------------- depthwise convs: k_dw.hip ----------------
struct DwGeom {
  int frames, H, W, C, k, s, pad, Ho, Wo;
};
// Y[n,ho,wo,c] = sum_taps pro(X)[n, ho*s-pad+kh, wo*s-pad+kw, c] * w[c][kh][kw]
// fin (optional): the input BN's train-mode finalize from its producer's stat rows -- inside the kernel
// where the rows are few and the channel-pair kernel runs (bnfin.h), else as its own launch first
template <typename T>
int launch_dw_fwd(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro,
                  int pro_mode, float* stats, int* stat_rows, const BnFwdFin* fin = nullptr);
struct BnBwdIn;
// dA = dgrad(dY).  With bn != null (fused backward of the producer's BN+SiLU): writes
// g = dA * silu'(Yp*scale+shift) and per-channel partials of g, g*xhat into stats rows.
template <typename T>
int launch_dw_dgrad(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* out, const T* Yp,
                    const BnBwdIn* bn, float* stats, int* stat_rows);
template <typename T>
int launch_dw_wgrad(hipStream_t s, const DwGeom& g, const T* dY, const T* X, const Pro& pro,
                    int pro_mode, float* slab, int64_t slab_cap, float* dW, bool accumulate);
// fused dgrad (+ producer BN+SiLU backward reduction) + wgrad, k_dw_bwd.hip: 0 launched, 1 not
// covered (use the two kernels above), -1 error
template <typename T>
int launch_dw_bwd(hipStream_t s, const DwGeom& g, const T* dY, const float* w, T* out, const T* Yp,
                  const BnBwdIn* bn, float* stats, int* stat_rows, float* slab, int64_t slab_cap, float* dW,
                  bool accumulate);
bool dw_bwd_fused_enabled();
// stride-1 depthwise backward with the BN2 (after the conv) and BN1 (before it) backward fused,
// k_dw_bwd1.hip: 0 launched, 1 not covered (BN2 apply + launch_dw_bwd instead)
template <typename T>
int launch_dw_bwd1(hipStream_t s, const DwGeom& g, const T* dZ, const T* Y2, const float* gate, const float* bc,
                   const float* sc2, const float* sh2, const float* coef2, const float* w, const T* Y1,
                   const BnBwdIn& bn1, T* out, float* stats, int* stat_rows, float* slab, int64_t slab_cap, float* dW,
                   bool accumulate);
bool dw_bwd1_enabled();
bool dw_bwd1_covers(const DwGeom& g);  // a tile configuration exists and the knob is on
// the stride-2 counterpart, k_dw_bwd2.hip (same contract; rides the dw_bwd1 knob)
template <typename T>
int launch_dw_bwd2(hipStream_t s, const DwGeom& g, const T* dZ, const T* Y2, const float* gate, const float* bc,
                   const float* sc2, const float* sh2, const float* coef2, const float* w, const T* Y1,
                   const BnBwdIn& bn1, T* out, float* stats, int* stat_rows, float* slab, int64_t slab_cap, float* dW,
                   bool accumulate);
bool dw_bwd2_covers(const DwGeom& g);
// k_dw_fwd1.hip: 1 launched, 0 not covered, -1 error
template <typename T>
int try_dw_fwd1(hipStream_t s, const DwGeom& g, const T* X, const float* w, T* Y, const Pro& pro, float* stats,
                int* stat_rows, const BnFwdFin* fin = nullptr);
bool dw_fwd1_enabled();

// ---------------- BatchNorm / SE / pooling: k_bn.hip ----------------
// finalize training stats: mean/invstd/scale/shift + running update (momentum); eval: from running
// chan_rows > 0: stats rows are centred (sum, M2) partials of consecutive chan_rows-row tiles
// (conv_forward's epilogue: kConvStatRows), merged in fp64 (Chan); 0: plain (sum, sum of squares)
// all of a plan's eval-mode BatchNorms in one launch (float offsets into params P, BN buffers bnb and
// the fp32 view of the workspace)
constexpr int kEvalBnMax = 64;
struct EvalBnEntry {
  int C, w, b, rm, rv, mean, invstd, scale, shift;
};
struct EvalBnTable {
  int n;
  EvalBnEntry e[kEvalBnMax];
};
int launch_bn_eval_all(hipStream_t s, const float* P, const float* bnb, float* wsf, const EvalBnTable& t, float eps);
int launch_bn_finalize(hipStream_t s, const float* stats, int rows, int64_t count, int C, const float* gamma,
                       const float* beta, float* run_mean, float* run_var, float momentum, float eps,
                       bool training, float* mean, float* invstd, float* scale, float* shift, int chan_rows = 0);
// the same from a BnFwdFin descriptor (the consumer-side finalize's fallback)
int launch_bn_finalize_fin(hipStream_t s, const BnFwdFin& f, int C);
constexpr int kConvStatRows = 64;  // rows per BN partial of conv_forward (k_conv.hip CG_T)
// X = Y*scale + shift (+ R)
template <typename T>
int launch_bn_apply(hipStream_t s, const T* Y, const float* scale, const float* shift, const T* R, T* X,
                    int64_t M, int C);
// BN backward, phase 1: per-channel partials of g and g*xhat, where
//   dA = dZ * gate[f][c] (if gate) + bc[f][c]*bc_scale (if bc);  g = dA * act'(y)  (act = SiLU or identity)
struct BnBwdIn {
  const void* dZ;       // [M][C] T or null
  const float* gate;    // [frames][C] or null
  const float* bc;      // [frames][C] broadcast term or null
  float bc_scale;
  int rows_per_frame;
  bool silu;
  const float* mean;    // saved batch mean   (or running mean in eval)
  const float* invstd;  // saved batch invstd (or running invstd in eval)
  const float* scale;   // gamma*invstd
  const float* shift;   // beta - mean*scale
};
template <typename T>
int launch_bn_bwd_reduce(hipStream_t s, const BnBwdIn& in, const T* Y, int64_t M, int C, float* stats,
                         int* stat_rows, int max_rows = 0);  // max_rows > 0: at most that many partial rows
// phase 2 (finalize): dgamma/dbeta into grads, coefficients k1,k2,k3 for dY = k1*g + k2*y + k3
int launch_bn_bwd_finalize(hipStream_t s, const float* stats, int rows, int64_t count, int C,
                           const float* gamma, const float* mean, const float* invstd, bool training,
                           float* dgamma, float* dbeta, bool accumulate, float* coef /*[3][C]*/,
                           bool centred = false /* k3 without the k2*mean term: dY = k1*g + k2*(y-mean) + k3 */);
// phase 3: dY = k1*g + k2*y + k3   (dY may alias dZ)
template <typename T>
int launch_bn_bwd_apply(hipStream_t s, const BnBwdIn& in, const T* Y, const float* coef, T* dY, int64_t M,
                        int C);
// phases 2 + 3 in one launch when the producer wrote <= 256 stat rows (k_bn.hip): dbeta / dgamma (and
// coef, if non-null) and dY = k1*g + k2*y + k3; 1 launched, 0 not covered (finalize + apply instead)
template <typename T>
int launch_bn_bwd_apply_fin(hipStream_t s, const BnBwdIn& in, const T* Y, int64_t M, int C, const float* stats, int rows,
                            int64_t count, const float* gamma, const float* mean, const float* invstd, bool training,
                            float* dgamma, float* dbeta, bool accumulate, float* coef, T* dY);
// SE squeeze partials: part[h][f][c] = sum over pixel chunk h of pro(Y)   (pro = BN+SiLU), h < *hsplit
// s_out: optional materialised silu(bn(Y)); fin: the BN's finalize (inside the launch where the stat rows
// are few, else its own launch first)
template <typename T>
int launch_se_squeeze(hipStream_t s, const T* Y, const Pro& pro, int frames, int HW, int C, float* part,
                      int64_t part_cap, int* hsplit, T* s_out, const BnFwdFin* fin = nullptr);
// scratch of the split SE excitation (k_bn.hip se_chain_kernel SPLIT): zeroed counters (2 per 16-frame
// tile) and partial first products; nullptr (or too small) runs the unsplit form
struct SeScratch {
  unsigned* bar;
  int bar_slots;
  float* tp;
  int64_t tp_cap;  // floats
  // a timed-out slice barrier raises these (tail.h SyncAbort): a zeroed device word the waiters poll
  // and the plan's sticky host word, checked on every later call of the plan
  int* abort_dev = nullptr;
  int* abort_host = nullptr;
};
// SE excitation: sq = inv_hw * sum_h part (stored) ; r = silu(Wr sq + br) ; gate = sigmoid(We r + be) ; saves rpre
int launch_se_fc_fwd(hipStream_t s, const float* part, int hsplit, float inv_hw, float* sq, const float* wr,
                     const float* br, const float* we, const float* be, int frames, int C, int rd, float* rpre,
                     float* gate, const SeScratch* sc = nullptr);
// SE backward reduce: dgate[f][c] = sum_hw dZ * pro(Y)   (pro = BN+SiLU, no gate)
template <typename T>
int launch_se_bwd_reduce(hipStream_t s, const T* dZ, const T* Y, const Pro& pro, int frames, int HW, int C,
                         float* part, int64_t part_cap, float* dgate);
// SE FC backward: from dgate -> dsq (written, scaled by 1/HW into bc), grads of wr,br,we,be.
// tmp_de: frames*C floats; tmp_dr: 2*frames*rd floats
// (de = dgate g (1-g) from the q = 0 partials of launch_se_bn_bwd_reduce, stored to `de`)
// defer2 != nullptr: the two weight-gradient products are returned there (MfmaGemm[2]) for a later
// launch_mfma_small_gemm_batch instead of being launched (de and tmp_dz must then stay intact)
// bnf != nullptr: the BN(+SiLU) backward finalize of launch_bn_bwd_finalize_frames (dbeta, dgamma, coef
// from gate, bc and the partials part[1..4]) runs in the same launch, in each channel slice's
// last-arriving workgroup (tail.h; ctr: >= cdiv(C, 256) zeroed counters, rows: frame-tile scratch)
struct MfmaGemm;
struct BnFramesFin {
  double* rows;
  int64_t rows_cap;  // floats
  unsigned* ctr;
  int ctr_slots;
  int64_t count;
  const float *gamma, *mean, *invstd;
  bool training, accumulate;
  float *dgamma, *dbeta, *coef;
};
int launch_se_fc_bwd(hipStream_t s, const float* part, int hsplit, const float* gate, float* de, const float* sq,
                     const float* rpre, const float* wr, const float* we, int frames, int C, int rd, float inv_hw,
                     float* tmp_dz, float* bc_out, float* gwr, float* gbr, float* gwe, float* gbe, bool accumulate,
                     MfmaGemm* defer2 = nullptr, const BnFramesFin* bnf = nullptr, const SeScratch* sc = nullptr);
// SE + BN(+SiLU) backward sums in one pass over (dZ, Y): per-frame partials part[5][hsplit][frames][C] -- q = 0
// the SE gate gradient (added by launch_se_fc_bwd), q = 1..4 the sums bn_bwd_finalize_frames combines with the
// gate and bc (k_bn.hip)
template <typename T>
int launch_se_bn_bwd_reduce(hipStream_t s, const T* dZ, const T* Y, const float* scale, const float* shift,
                            const float* mean, const float* invstd, int frames, int HW, int C, float* part,
                            int64_t part_cap, int* hsplit);
int launch_bn_bwd_finalize_frames(hipStream_t s, float* part, int hsplit, const float* gate, const float* bc,
                                  int frames, int C, int64_t count, const float* gamma, const float* mean,
                                  const float* invstd, bool training, float* dgamma, float* dbeta, bool accumulate,
                                  float* coef);
// conv_pw backward through its BN (no activation), by linearity (k_bn.hip): fold the BN-backward
// coefficients coef = [k1; k2; k3] into the dgrad operands, combine the weight-gradient terms
template <typename T>
int launch_bn_fold_pw(hipStream_t s, const float* W, const float* coef, int mid, int cin, T* w1t, T* q, float* bv);
int launch_pw_wgrad_bn_combine(hipStream_t s, const float* Tg, const float* G, const float* cs, const float* W,
                               const float* coef, int mid, int cin, float* dW, bool accumulate);
template <typename T>
int launch_col_sums(hipStream_t s, const T* X, int64_t M, int C, float* part, int64_t part_cap, float* out);
// fp32 MFMA small GEMM (k_head.hip): C[m][n] (+)= post( sum_k A(m,k) B(k,n) ),
// A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn] (silu(B) if b_silu, dropout on B if p > 0);
// post: + bias[n], * silu'(dsilu_pre[m][n]);  asum[m] (+)= sum_k A(m,k) when non-null
struct MfmaGemm {
  const float* A = nullptr; int64_t sam = 0, sak = 0;
  const float* B = nullptr; int64_t sbk = 0, sbn = 0;
  float* C = nullptr; int64_t ldc = 0;
  int M = 0, N = 0, K = 0;
  const float* bias = nullptr;
  const float* dsilu_pre = nullptr;  // [M][ldc]
  float* asum = nullptr;             // [M]
  int accumulate = 0;
  int b_silu = 0;
  int relu = 0;    // post: max(., 0) after the bias
  int drop_c = 0;  // the dropout (p, seed, stream) multiplies C[m][n] (index m*ldc + n) instead of B
  uint64_t seed = 0; uint32_t stream = 0; float p = 0.f; int64_t drop_ld = 0;
};
int launch_mfma_small_gemm(hipStream_t s, const MfmaGemm& g);
int launch_mfma_small_gemm2(hipStream_t s, const MfmaGemm& g0, const MfmaGemm& g1);  // one launch, same K
// test seam: CU-holding workgroups spinning for a bounded time (k_test.hip, dfd_test_occupy)
int launch_occupy(hipStream_t s, int workgroups, int64_t microseconds);
// n independent products of equal K in one launch per kMaxBatch (workgroup ranges per product)
constexpr int kMfmaBatch = 8;
int launch_mfma_small_gemm_batch(hipStream_t s, const MfmaGemm* g, int n);
int launch_mfma_small_gemm(hipStream_t s, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                           int64_t sbn, float* C, int64_t ldc, int M, int N, int K, const float* bias,
                           const float* dsilu_pre, float* asum, bool accumulate, uint64_t seed, uint32_t stream,
                           float p, int64_t drop_ld);
// head global average pool: feat[f][c] = mean_hw silu(Y*scale+shift)
template <typename T>
int launch_gap(hipStream_t s, const T* Y, const Pro& pro, int frames, int HW, int C, float* feat,
               const BnFwdFin* fin = nullptr);
// sum `splits` slabs of n floats into out (= or +=)
// Deferred weight-gradient reductions: while a SlabDefer is active on the calling thread, slab
// reductions on `stream` whose output lies inside [lo, hi) (the gradient buffer) are queued and
// flush() runs them as one launch.  The caller keeps every queued slab region intact until then.
struct SlabJob {
  const float* slab;
  int64_t n;
  float* out;
  int splits, accumulate;
};
// With an aux stream (the backward's weight-gradient stream), jobs queued from either stream are
// reduced on `stream`; flush() first makes `stream` wait for everything enqueued on `aux`, and
// afterwards makes `aux` wait for the reduction (the slab regions are then free on both streams).
struct SlabDefer {
  static constexpr int kMax = 16;
  hipStream_t stream;
  const float* lo;
  const float* hi;
  SlabJob jobs[kMax];
  int n = 0;
  hipStream_t aux = nullptr;
  hipEvent_t ev_aux = nullptr, ev_main = nullptr;
  int flush();
};
SlabDefer* set_slab_defer(SlabDefer* d);  // returns the previous one
int launch_reduce_slabs(hipStream_t s, const float* slab, int splits, int64_t n, float* out, bool accumulate);
// the same with slab rows `stride` floats apart
int launch_reduce_slabs_strided(hipStream_t s, const float* slab, int splits, int64_t n, int64_t stride, float* out,
                                bool accumulate);

// ---------------- stem (3->32, k3 s2): k_stem.hip ----------------
// Input frames of the trunk: fp32 (already normalised by the caller, app.py:2084-2085) or raw
// uint8 pixels normalised in the stem's load as ((v / 255) - mean[c]) / std[c] -- the same fp32
// operations, in the same order, as the reference's `.float() / 255.0` + imagenet_normalize
// (app.py:1772-1780), so both formats give bit-identical stem inputs.
struct InputFmt {
  int u8;                 // 0: fp32 frames, 1: uint8 pixels (any strides), 2: dense NHWC uint8
  float mean[3], stdv[3]; // u8 only (mean 0 / std 1: the /255-only feed of train.py:59)
};
struct StemGeom {
  int frames, H, W, Ho, Wo;
  int64_t sf, sc, sh, sw;  // element strides of the input (frame, channel, row, col)
  InputFmt in;
};
template <typename T>
int launch_stem_fwd(hipStream_t s, const StemGeom& g, const void* x, const float* w, T* Y, float* stats,
                    int* stat_rows);
template <typename T>
int launch_stem_wgrad(hipStream_t s, const StemGeom& g, const void* x, const T* dY, const T* Yb, const float* coef,
                      float* slab, int64_t slab_cap, float* dW, bool accumulate);  // coef: fused BN backward

// ---------------- input pipeline: k_input.hip ----------------
int launch_collate_gather(hipStream_t s, const uint8_t* src, const int64_t* sel, int64_t nsel, int64_t frame_bytes,
                          bool f32, void* out);

// ---------------- misc: k_misc.hip ----------------
struct CastSeg {
  int64_t src, dst;  // element offsets
  int rows, cols;    // transpose a [rows][cols] matrix into [cols][rows] if transpose
  int transpose;
};
template <typename T>
int launch_cast_params(hipStream_t s, const float* params, T* out, const CastSeg* segs_dev, int nseg,
                       int max_elems);

}  // namespace dfd
