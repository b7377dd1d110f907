// DeepfakeModel (src/models.py:222-291) on MI355X: the timm vit_base_patch16_224 trunk
// (ViTFeatureExtractor, src/models.py:88-107; restated in oracle/vit_cpu.py) and the SimpleGCN +
// classifier head (src/models.py:199-219, 274-291), forward and backward, behind the C ABI
// dfd_vit_* / dfd_gcn_head_* (include/dfd_hip.h).
//
// Trunk data layout: token rows [images * 197][768] (row = image * 197 + token), storage T
// (bf16 or fp32), fp32 accumulation everywhere.  Per block the forward keeps what the backward
// reads: block input x, LN1 output h1, qkv [rows][2304], softmax probabilities P
// [images*12*197][200] (rows padded to 200 for 16-B vector reads), attention output O, the
// post-attention stream xm, LN2 output h2 and the fc1 pre-activation Z [rows][3072] (bf16: fc1's
// epilogue also stores G = gelu(Z), read by fc2 and by its weight gradient; fp32: GELU is re-applied
// by fc2's operand prologue).  The bf16 linear layers are the LDS-DMA 256 x 256 MFMA GEMMs of
// k_vgemm.hip (bias / residual / GELU / GELU-derivative epilogues), the fp32 parity mode and the
// shapes they do not cover run launch_tf_gemm (k_gemm.hip); weights are cast per step to T in both
// [out][in] (forward) and [in][out] (dgrad) layouts; weight gradients are split-M slab GEMMs
// reduced in a fixed order, so a step is bit-reproducible.  No library GEMM.
#include "../../include/dfd_hip.h"

#include <atomic>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "kernels.h"
#include "rnn.h"
#include "vit.h"

namespace dfd {
namespace {

constexpr int D = 768, HEADS = 12, DH = 64, FF = 3072, D3 = 3 * D, SLD = 200;
constexpr float LN_EPS = 1e-6f;

struct VitDims {
  int dtype, depth, images, H, W;
  int ntok() const { return (H / VIT_PATCH) * (W / VIT_PATCH) + 1; }
  int64_t rows() const { return (int64_t)images * ntok(); }
};

int vit_check(const VitDims& d) {
  if (d.dtype != 0 && d.dtype != 1) { set_error("vit: dtype must be 0 (fp32) or 1 (bf16)", __FILE__, __LINE__); return -1; }
  if (d.depth < 1 || d.depth > 12) { set_error("vit: depth must be 1..12", __FILE__, __LINE__); return -1; }
  if (d.images < 1 || d.H % VIT_PATCH || d.W % VIT_PATCH || d.ntok() != 197) {
    set_error("vit: vit_base_patch16_224 takes 224x224 images (197 tokens)", __FILE__, __LINE__);
    return -1;
  }
  return 0;
}

// byte layout of the trunk workspace (kept forward -> backward) and backward scratch
struct VitLayout {
  struct Blk {
    int64_t x, h1, mu1, rs1, qkv, P, O, xm, h2, mu2, rs2, Z, G;
    int64_t wqkv, wqkvT, wp, wpT, w1, w1T, w2, w2T;
  };
  std::vector<Blk> blk;
  int64_t wpe, ape, pe, xfin, mu_f, rs_f, S, total;
  // scratch
  int64_t dx, dxm, dh, dZ, dqkv, dO, dS, part, slab, dpe, bar, stotal;
  int64_t dx2, dxm2, dZ2, dqkv2;  // bf16: the second set of the side stream's double-buffered inputs
  int64_t part_cap, slab_cap;
};

constexpr int kVitBars = 256;  // >= vgemm_tn_bar_count of every ViT-B weight gradient (3072 x 768: 72)
// 1: bf16 work off the critical chain runs on a second stream -- the forward's weight casts
// (vit_forward_t) and the backward's weight gradients, GEMM + split reduction (vit_backward_t);
// 0: everything on the caller's stream (A/B builds)
#ifndef DFD_VIT_SIDE
#define DFD_VIT_SIDE 1
#endif
#ifndef DFD_VIT_TN_COOP
#define DFD_VIT_TN_COOP 0  // 1: the weight gradients' split partials reduced inside the GEMM launch (measured slower, DESIGN r5)
#endif

VitLayout vit_layout(const VitDims& d) {
  VitLayout L;
  const int64_t es = d.dtype == 1 ? 2 : 4;
  const int64_t M = d.rows(), M0 = (int64_t)d.images * (d.ntok() - 1);
  const int64_t SR = (int64_t)d.images * HEADS * d.ntok();  // score rows
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    const int64_t o = off;
    off += (bytes + 255) / 256 * 256 + 256;  // +256: slack for padded vector reads at the very end
    return o;
  };
  L.blk.resize(d.depth);
  L.wpe = take(es * D * D);
  for (auto& b : L.blk) {
    b.wqkv = take(es * D3 * D);
    b.wqkvT = take(es * D3 * D);
    b.wp = take(es * D * D);
    b.wpT = take(es * D * D);
    b.w1 = take(es * FF * D);
    b.w1T = take(es * FF * D);
    b.w2 = take(es * FF * D);
    b.w2T = take(es * FF * D);
  }
  L.ape = take(es * M0 * D);
  L.pe = take(es * M0 * D);
  for (auto& b : L.blk) {
    b.x = take(es * M * D);
    b.h1 = take(es * M * D);
    b.mu1 = take(4 * M);
    b.rs1 = take(4 * M);
    b.qkv = take(es * M * D3);
    b.P = take(es * SR * SLD);
    b.O = take(es * M * D);
    b.xm = take(es * M * D);
    b.h2 = take(es * M * D);
    b.mu2 = take(4 * M);
    b.rs2 = take(4 * M);
    b.Z = take(es * M * FF);
    b.G = d.dtype == 1 ? take(es * M * FF) : 0;  // gelu(Z), written by fc1's epilogue (bf16)
  }
  L.xfin = take(es * M * D);
  L.mu_f = take(4LL * d.images);
  L.rs_f = take(4LL * d.images);
  L.S = take(es * SR * SLD);
  L.total = off;
  // scratch
  off = 0;
  L.dx = take(es * M * D);
  L.dxm = take(es * M * D);
  L.dh = take(es * M * D);
  L.dZ = take(es * M * FF);
  L.dqkv = take(es * M * D3);
  L.dO = take(es * M * D);
  L.dS = take(es * SR * SLD);
  L.dpe = take(es * M0 * D);
  if (d.dtype == 1) {
    L.dx2 = take(es * M * D);
    L.dxm2 = take(es * M * D);
    L.dZ2 = take(es * M * FF);
    L.dqkv2 = take(es * M * D3);
  } else {
    L.dx2 = L.dx;
    L.dxm2 = L.dxm;
    L.dZ2 = L.dZ;
    L.dqkv2 = L.dqkv;
  }
  L.part_cap = 2LL * 1024 * FF;
  L.part = take(4 * L.part_cap);
  L.slab_cap = 16LL * FF * D;
  L.slab = take(4 * L.slab_cap);
  L.bar = take(4 * kVitBars);  // the weight-gradient GEMMs' split-barrier counters (zeroed per backward)
  L.stotal = off;
  return L;
}

// parameter table: 0 cls_token, 1 pos_embed, 2 patch w, 3 patch b, then 12 per block
// (norm1 w,b, qkv w,b, proj w,b, norm2 w,b, fc1 w,b, fc2 w,b), then norm w,b
inline int vit_nparams(int depth) { return 4 + 12 * depth + 2; }

template <typename T>
struct Ws {
  char* base;
  template <typename U = T>
  U* at(int64_t off) const { return reinterpret_cast<U*>(base + off); }
};

// The bf16 side stream (the forward's weight casts, the backward's weight gradients): one non-blocking
// stream per device, created on first use and kept for the process (never destroyed: every forward /
// backward joins its last work), with the events of the fork / join points; `mu` serialises the
// enqueues that share it.
struct VitSide {
  std::mutex mu;
  int dev = -1;
  hipStream_t s = nullptr;
  hipEvent_t fork[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};  // per layer parity: the side's work of that layer
  hipEvent_t tail = nullptr;
  hipEvent_t cast[13] = {};  // forward: the patch embedding's (0) and layer l's (l + 1) weight casts
};
VitSide* vit_side() {
  static VitSide g[64];
  static std::mutex init_mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("vit: no device for the side stream", __FILE__, __LINE__);
    return nullptr;
  }
  VitSide& v = g[dev];
  const std::lock_guard<std::mutex> lk(init_mu);
  if (v.dev == dev) return &v;
  std::vector<hipEvent_t*> evs = {&v.fork[0], &v.fork[1], &v.done[0], &v.done[1], &v.tail};
  for (hipEvent_t& e : v.cast) evs.push_back(&e);
  // the lowest priority: the data-gradient chain's workgroups dispatch first when both streams wait
  int least = 0, greatest = 0;
  bool ok = hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
            hipStreamCreateWithPriority(&v.s, hipStreamNonBlocking, least) == hipSuccess;
  for (hipEvent_t* e : evs) ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    set_error("vit: side stream / event creation failed", __FILE__, __LINE__);
    return nullptr;
  }
  v.dev = dev;
  return &v;
}

// with a side stream the casts run there, after everything enqueued on s so far, and cast[i] marks the
// patch embedding's (i = 0) and layer i - 1's weights ready
template <typename T>
int cast_weights(hipStream_t s, const VitDims& d, const VitLayout& L, const float* const* P, const Ws<T>& w,
                 VitSide* vs = nullptr) {
  hipStream_t cs = s;
  if (vs) {
    cs = vs->s;
    DFD_HIP_CHECK(hipEventRecord(vs->fork[0], s));
    DFD_HIP_CHECK(hipStreamWaitEvent(cs, vs->fork[0], 0));
  }
  VitCast pe{};
  pe.seg[0] = {P[2], w.at(L.wpe), nullptr, D, D};
  DFD_TRY(launch_wcast<T>(cs, pe, 1));
  if (vs) DFD_HIP_CHECK(hipEventRecord(vs->cast[0], cs));
  for (int l = 0; l < d.depth; ++l) {
    const float* const* q = P + 4 + 12 * l;
    const auto& b = L.blk[l];
    VitCast c{};
    c.seg[0] = {q[2], w.at(b.wqkv), w.at(b.wqkvT), D3, D};
    c.seg[1] = {q[4], w.at(b.wp), w.at(b.wpT), D, D};
    c.seg[2] = {q[8], w.at(b.w1), w.at(b.w1T), FF, D};
    c.seg[3] = {q[10], w.at(b.w2), w.at(b.w2T), D, FF};
    DFD_TRY(launch_wcast<T>(cs, c, 4));
    if (vs) DFD_HIP_CHECK(hipEventRecord(vs->cast[l + 1], cs));
  }
  return 0;
}

// attention operand addressing inside qkv [rows][2304] / O [rows][768] / scores [b][197][200]
// (the head's column offset is the batch's inner stride; q/k/v sit at column offsets 0/768/1536)
inline BgOp op_tok(int ld) { return BgOp{ld, HEADS, (int64_t)197 * ld, DH}; }
inline BgOp op_score() { return BgOp{SLD, 1, (int64_t)197 * SLD, 0}; }

// the fused attention's view of one layer's qkv / O / log-sum-exp buffers (bf16 path)
template <typename T>
inline AttnArgs attn_args(int images, int nt, const T* qkv, T* O, float* lse) {
  AttnArgs a{};
  a.images = images; a.heads = HEADS; a.nt = nt; a.scale = 0.125f;
  a.qkv = reinterpret_cast<const bf16*>(qkv); a.ldq = D3; a.koff = D; a.voff = 2 * D;
  a.O = reinterpret_cast<bf16*>(O); a.ldo = D; a.lse = lse;
  return a;
}

// C[M][N] = A . B^T (+ bias) (+ R), epi a mask of VgEpi.  bf16 MLP: VG_GELU2 leaves G = gelu(pre) and
// C = gelu'(pre); VG_DGELU multiplies by that stored derivative (Z).  fp32: C = pre-activation and
// EPI_DGELU takes gelu' of Z itself (the fp32 forward keeps Z).
template <typename T>
int lin(hipStream_t s, const T* A, const T* B, T* C, const T* R, const float* bias, int64_t M, int N, int K,
        int epi_extra = 0, const T* Z = nullptr, T* G = nullptr) {
  const int epi = (bias ? VG_BIAS : 0) | (R ? VG_RESID : 0) | epi_extra;
  if constexpr (sizeof(T) == 2) {
    // the NT kernel's 64-wide tile carries only the bias / identity / ReLU epilogues: 128-multiples here
    if (vgemm_nt_covers(M, N, K) && N % 128 == 0) {
      VgemmArgs a{};
      a.A = A; a.B = B; a.C = C; a.R = R; a.bias = bias; a.Z = Z; a.G = G;
      a.lda = K; a.ldb = K; a.ldc = N; a.M = (int)M; a.N = N; a.K = K;
      return launch_vgemm_nt(s, a, epi);
    }
    // uncovered shapes: the GEMM, then the same GELU arithmetic as a pass
    const int base = (bias ? EPI_BIAS : 0) | (R ? EPI_RESID : 0);
    if (epi_extra & VG_GELU2) {
      DFD_TRY(launch_tf_gemm<T>(s, A, B, C, R, bias, nullptr, M, N, K, PRO_NONE, base));
      return launch_gelu(s, C, G, M * N, GELU_PAIR);
    }
    if (epi_extra & VG_DGELU) {
      DFD_TRY(launch_tf_gemm<T>(s, A, B, C, R, bias, nullptr, M, N, K, PRO_NONE, base));
      return launch_gelu(s, const_cast<T*>(Z), C, M * N, GELU_MULD);
    }
  }
  return launch_tf_gemm<T>(s, A, B, C, R, bias, Z, M, N, K, PRO_NONE,
                           (bias ? EPI_BIAS : 0) | (R ? EPI_RESID : 0) | ((epi_extra & VG_DGELU) ? EPI_DGELU : 0));
}
// dW[N][K] = dY^T . X, and the bias gradient dB[N] = sum_m dY[m] (in the same launch on the own
// bf16 kernel; a column-sum pass otherwise)
template <typename T>
int wgrad(hipStream_t s, const T* dY, const T* X, int64_t M, int N, int K, float* slab, int64_t slab_cap, float* dW,
          float* dB, float* part, int64_t part_cap, unsigned* bar) {
  if constexpr (sizeof(T) == 2)
    if (vgemm_tn_covers(M, N, K))
      return launch_vgemm_tn(s, dY, N, X, K, M, N, K, slab, slab_cap, dW, false, dB,
                             DFD_VIT_TN_COOP && bar && vgemm_tn_bar_count(N, K) <= kVitBars ? bar : nullptr);
  Pro none{};
  DFD_TRY(launch_pw_wgrad<T>(s, dY, X, M, N, K, PRO_NONE, none, slab, slab_cap, dW, false));
  return launch_colsum<T>(s, dY, M, N, part, part_cap, dB, false);
}

// keep_backward = 0 (inference): fc1 stores gelu(pre) alone where the own GEMM covers it (the
// derivative the backward would read is not written); the outputs are the same bits either way
template <typename T>
int vit_forward_t(hipStream_t s, const VitDims& d, const VitLayout& L, const float* const* P, const float* x,
                  const VitImg& im, char* work, float* feats, bool keep_backward = true) {
  const Ws<T> w{work};
  const int nt = d.ntok(), I = d.images, BH = I * HEADS;
  const int64_t M = d.rows(), M0 = (int64_t)I * (nt - 1), SR = (int64_t)BH * nt;
  // bf16: the weight casts run ahead on the side stream; each layer waits for its own (the last wait
  // joins the side stream's work)
  const bool side = DFD_VIT_SIDE && sizeof(T) == 2;
  VitSide* vs = nullptr;
  std::unique_lock<std::mutex> lk;
  if (side) {
    vs = vit_side();
    if (!vs) return -1;
    lk = std::unique_lock<std::mutex>(vs->mu);
  }
  auto ready = [&](int i) -> int {
    if (vs) DFD_HIP_CHECK(hipStreamWaitEvent(s, vs->cast[i], 0));
    return 0;
  };
  DFD_TRY(cast_weights<T>(s, d, L, P, w, vs));
  // patch embedding (Conv2d 16x16/16 as a GEMM over gathered patches) + cls + pos
  DFD_TRY(launch_patch_gather<T>(s, x, im, I, w.at(L.ape)));
  DFD_TRY(ready(0));
  DFD_TRY(lin<T>(s, w.at(L.ape), w.at(L.wpe), w.at(L.pe), nullptr, P[3], M0, D, D));
  DFD_TRY(launch_tokens_fwd<T>(s, w.at(L.pe), P[0], P[1], I, nt, D, w.at(L.blk[0].x)));
  for (int l = 0; l < d.depth; ++l) {
    const float* const* q = P + 4 + 12 * l;
    const auto& b = L.blk[l];
    T* xnext = l + 1 < d.depth ? w.at(L.blk[l + 1].x) : w.at(L.xfin);
    DFD_TRY((launch_ln_fwd<T, T>(s, w.at(b.x), D, q[0], q[1], w.at(b.h1), D, w.template at<float>(b.mu1),
                                w.template at<float>(b.rs1), M, D, LN_EPS)));
    DFD_TRY(ready(l + 1));
    DFD_TRY(lin<T>(s, w.at(b.h1), w.at(b.wqkv), w.at(b.qkv), nullptr, q[3], M, D3, D));
    T* qkv = w.at(b.qkv);
    // S = (q * 64^-0.5) k^T ; P = softmax(S) ; O = P v
    if constexpr (sizeof(T) == 2) {  // fused (k_attn.hip): O and the row log-sum-exp (in b.P's space)
      DFD_TRY(launch_attn_fwd(s, attn_args(I, nt, qkv, w.at(b.O), w.template at<float>(b.P))));
    } else {
      DFD_TRY(launch_bgemm<T>(s, false, true, BH, nt, nt, DH, 0.125f, qkv, op_tok(D3), qkv + D, op_tok(D3),
                              w.at(L.S), op_score()));
      DFD_TRY(launch_softmax_fwd<T>(s, w.at(L.S), w.at(b.P), SR, nt, SLD));
      DFD_TRY(launch_bgemm<T>(s, false, false, BH, nt, DH, nt, 1.f, w.at(b.P), op_score(), qkv + 2 * D, op_tok(D3),
                              w.at(b.O), op_tok(D)));
    }
    // xm = x + proj(O) ; x' = xm + fc2(gelu(fc1(LN2(xm))))
    DFD_TRY(lin<T>(s, w.at(b.O), w.at(b.wp), w.at(b.xm), w.at(b.x), q[5], M, D, D));
    DFD_TRY((launch_ln_fwd<T, T>(s, w.at(b.xm), D, q[6], q[7], w.at(b.h2), D, w.template at<float>(b.mu2),
                                w.template at<float>(b.rs2), M, D, LN_EPS)));
    if constexpr (sizeof(T) == 2) {  // fc1 stores Z and G = gelu(Z) (inference: G alone); fc2 reads G
      if (!keep_backward && vgemm_nt_covers(M, FF, D) && FF % 128 == 0)
        DFD_TRY(lin<T>(s, w.at(b.h2), w.at(b.w1), w.at(b.G), nullptr, q[9], M, FF, D, VG_GELU));
      else
        DFD_TRY(lin<T>(s, w.at(b.h2), w.at(b.w1), w.at(b.Z), nullptr, q[9], M, FF, D, VG_GELU2, nullptr, w.at(b.G)));
      DFD_TRY(lin<T>(s, w.at(b.G), w.at(b.w2), xnext, w.at(b.xm), q[11], M, D, FF));
    } else {  // fp32: GELU re-applied in fc2's operand prologue
      DFD_TRY(lin<T>(s, w.at(b.h2), w.at(b.w1), w.at(b.Z), nullptr, q[9], M, FF, D));
      DFD_TRY(launch_tf_gemm<T>(s, w.at(b.Z), w.at(b.w2), xnext, w.at(b.xm), q[11], nullptr, M, D, FF, PRO_GELU,
                                EPI_BIAS | EPI_RESID));
    }
  }
  // final norm, CLS rows only (global_pool='token')
  const float* const* fn = P + 4 + 12 * d.depth;
  return launch_ln_fwd<T, float>(s, w.at(L.xfin), (int64_t)nt * D, fn[0], fn[1], feats, D, w.template at<float>(L.mu_f),
                                 w.template at<float>(L.rs_f), I, D, LN_EPS);
}

template <typename T>
int vit_backward_t(hipStream_t s, const VitDims& d, const VitLayout& L, const float* const* P, char* work,
                   char* scratch, const float* dfeats, float* const* G) {
  const Ws<T> w{work};
  const Ws<T> sc{scratch};
  const int nt = d.ntok(), I = d.images, BH = I * HEADS;
  const int64_t M = d.rows(), M0 = (int64_t)I * (nt - 1), SR = (int64_t)BH * nt;
  float* part = sc.template at<float>(L.part);
  float* slab = sc.template at<float>(L.slab);
  unsigned* bar = sc.template at<unsigned>(L.bar);
  // bf16: the weight gradients (vgemm TN + its split reduction, all through the one slab) run on the
  // side stream in enqueue order while this stream runs the data-gradient chain.  The side waits at
  // two forks per layer (after dZ; after dqkv); the gradient inputs it reads are double-buffered by
  // layer parity, so this stream overwrites them only two layers later, after waiting for that
  // layer's side work (done[parity], long finished by then); one join at the end.
  const bool side = DFD_VIT_SIDE && sizeof(T) == 2;
  VitSide* vs = nullptr;
  std::unique_lock<std::mutex> lk;
  if (side) {
    vs = vit_side();
    if (!vs) return -1;
    lk = std::unique_lock<std::mutex>(vs->mu);
  }
  hipStream_t ss = side ? vs->s : s;
  int nfork = 0;
  auto fork = [&]() -> int {  // the side stream waits for everything enqueued on s so far
    if (!side) return 0;
    hipEvent_t e = vs->fork[nfork++ & 1];
    DFD_HIP_CHECK(hipEventRecord(e, s));
    DFD_HIP_CHECK(hipStreamWaitEvent(ss, e, 0));
    return 0;
  };
  auto join = [&](hipEvent_t e) -> int {  // s waits for everything enqueued on the side so far
    if (!side) return 0;
    DFD_HIP_CHECK(hipEventRecord(e, ss));
    DFD_HIP_CHECK(hipStreamWaitEvent(s, e, 0));
    return 0;
  };
  auto wgd = [&](const T* dY, const T* X, int64_t Mr, int N, int K, float* dW, float* dB) -> int {
    if (side && vgemm_tn_covers(Mr, N, K))
      return wgrad<T>(ss, dY, X, Mr, N, K, slab, L.slab_cap, dW, dB, part, L.part_cap, bar);
    DFD_TRY(join(vs ? vs->tail : nullptr));  // the other forms share slab / part with this stream
    return wgrad<T>(s, dY, X, Mr, N, K, slab, L.slab_cap, dW, dB, part, L.part_cap, bar);
  };
  DFD_HIP_CHECK(hipMemsetAsync(bar, 0, 4 * kVitBars, s));  // zero at rest from here on (group_sync)
  T* const dxb[2] = {sc.at(L.dx), sc.at(L.dx2)};
  T* const dxmb[2] = {sc.at(L.dxm), sc.at(L.dxm2)};
  T* const dZb[2] = {sc.at(L.dZ), sc.at(L.dZ2)};
  T* const dqkvb[2] = {sc.at(L.dqkv), sc.at(L.dqkv2)};
  T* dh = sc.at(L.dh);
  // final norm: only the CLS rows receive gradient (into the last layer's input-gradient buffer)
  T* dx0 = dxb[(d.depth - 1) & 1];
  DFD_HIP_CHECK(hipMemsetAsync(dx0, 0, sizeof(T) * M * D, s));
  const float* const* fn = P + 4 + 12 * d.depth;
  float* const* gn = G + 4 + 12 * d.depth;
  DFD_TRY((launch_ln_bwd<T, float>(s, w.at(L.xfin), (int64_t)nt * D, dfeats, D, fn[0], w.template at<float>(L.mu_f),
                                  w.template at<float>(L.rs_f), nullptr, dx0, I, D, part, L.part_cap, gn[0], gn[1],
                                  false)));
  Pro none{};
  for (int l = d.depth - 1; l >= 0; --l) {
    const float* const* q = P + 4 + 12 * l;
    float* const* g = G + 4 + 12 * l;
    const auto& b = L.blk[l];
    const int par = l & 1;
    T* qkv = w.at(b.qkv);
    T* dx = dxb[par];        // this layer's output gradient (side: fc2's weight gradient reads it)
    T* dxo = dxb[par ^ 1];   // its input gradient, the next layer down's dx
    T* dZ = dZb[par];
    T* dxm = dxmb[par];
    T* dqkv = dqkvb[par];
    T* dO = sc.at(L.dO);
    T* dS = sc.at(L.dS);
    // ---- MLP: dZ = (dx W2) * gelu'(Z); dW2 = dx^T gelu(Z); dh2 = dZ W1 ----
    DFD_TRY(lin<T>(s, dx, w.at(b.w2T), dZ, nullptr, nullptr, M, FF, D, VG_DGELU, w.at(b.Z)));
    DFD_TRY(fork());
    if constexpr (sizeof(T) == 2) {  // G = gelu(Z) kept by the forward
      DFD_TRY(wgd(dx, w.at(b.G), M, D, FF, g[10], g[11]));
    } else {
      DFD_TRY(launch_pw_wgrad<T>(s, dx, w.at(b.Z), M, D, FF, PRO_GELU, none, slab, L.slab_cap, g[10], false));
      DFD_TRY(launch_colsum<T>(s, dx, M, D, part, L.part_cap, g[11], false));
    }
    DFD_TRY(wgd(dZ, w.at(b.h2), M, FF, D, g[8], g[9]));
    DFD_TRY(lin<T>(s, dZ, w.at(b.w1T), dh, nullptr, nullptr, M, D, FF));
    // LN2: dxm = dx + LN2'(dh2)
    DFD_TRY((launch_ln_bwd<T, T>(s, w.at(b.xm), D, dh, D, q[6], w.template at<float>(b.mu2),
                                w.template at<float>(b.rs2), dx, dxm, M, D, part, L.part_cap, g[6], g[7], false)));
    // ---- attention projection ----
    DFD_TRY(lin<T>(s, dxm, w.at(b.wpT), dO, nullptr, nullptr, M, D, D));
    // ---- attention core: dP = dO v^T ; dS = scale P (dP - rowdot) ; dq = dS k ; dk = dS^T q ; dv = P^T dO
    if constexpr (sizeof(T) == 2) {  // fused (k_attn.hip): recomputes P from the saved log-sum-exp
      AttnArgs at = attn_args(I, nt, qkv, w.at(b.O), w.template at<float>(b.P));
      at.dO = dO;
      at.lddo = D;
      at.dqkv = dqkv;
      at.lddq = D3;
      DFD_TRY(launch_attn_bwd(s, at));
    } else {
      DFD_TRY(launch_bgemm<T>(s, false, true, BH, nt, nt, DH, 1.f, dO, op_tok(D), qkv + 2 * D, op_tok(D3), dS,
                              op_score()));
      DFD_TRY(launch_softmax_bwd<T>(s, w.at(b.P), dS, dS, SR, nt, SLD, 0.125f));
      DFD_TRY(launch_bgemm<T>(s, false, false, BH, nt, DH, nt, 1.f, dS, op_score(), qkv + D, op_tok(D3), dqkv,
                              op_tok(D3)));
      DFD_TRY(launch_bgemm<T>(s, true, false, BH, nt, DH, nt, 1.f, dS, op_score(), qkv, op_tok(D3), dqkv + D,
                              op_tok(D3)));
      DFD_TRY(launch_bgemm<T>(s, true, false, BH, nt, DH, nt, 1.f, w.at(b.P), op_score(), dO, op_tok(D),
                              dqkv + 2 * D, op_tok(D3)));
    }
    DFD_TRY(fork());
    DFD_TRY(wgd(dxm, w.at(b.O), M, D, D, g[4], g[5]));
    DFD_TRY(wgd(dqkv, w.at(b.h1), M, D3, D, g[2], g[3]));
    if (side) DFD_HIP_CHECK(hipEventRecord(vs->done[par], ss));
    // ---- qkv projection and LN1: dx_l = dxm + LN1'(dqkv Wqkv) ----
    DFD_TRY(lin<T>(s, dqkv, w.at(b.wqkvT), dh, nullptr, nullptr, M, D, D3));
    // dxo was the layer above's dx, read by that layer's side work: wait for it (long done)
    if (side && l + 1 < d.depth) DFD_HIP_CHECK(hipStreamWaitEvent(s, vs->done[par ^ 1], 0));
    DFD_TRY((launch_ln_bwd<T, T>(s, w.at(b.x), D, dh, D, q[0], w.template at<float>(b.mu1), w.template at<float>(b.rs1),
                                dxm, dxo, M, D, part, L.part_cap, g[0], g[1], false)));
  }
  // tokens: dcls, dpos, patch rows -> patch-embedding weight / bias
  T* dpe = sc.at(L.dpe);
  DFD_TRY(launch_tokens_bwd<T>(s, dxb[1], I, nt, D, dpe, G[1], G[0]));
  DFD_TRY(fork());
  DFD_TRY(wgd(dpe, w.at(L.ape), M0, D, D, G[2], G[3]));
  return join(vs ? vs->tail : nullptr);
}

// ------------------------------------------------------------------------------------------
// GCN head (fp32): feats [B*N][Dv] -> logits [B][C].  work (floats):
//   H1 [BN][Dv] | Y1 [BN][hid] (post-ReLU) | D1 [BN][hid] | Y2 [BN][out] (post-ReLU) | G [B][out] |
//   C1 [B][64] (post-ReLU) | Dc [B][64]
struct HeadDims {
  int B, N, Dv, hid, out, classes;
};
struct HeadLayout {
  int64_t H1, Y1, D1, Y2, Gm, C1, Dc, total;
  // backward scratch
  int64_t dl, dDc, dC1, dG, dY2, dD1, dY1, dH1, part, stotal;
};
HeadLayout head_layout(const HeadDims& h) {
  HeadLayout L;
  const int64_t BN = (int64_t)h.B * h.N;
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) / 64 * 64; return r; };
  L.H1 = take(BN * h.Dv);
  L.Y1 = take(BN * h.hid);
  L.D1 = take(BN * h.hid);
  L.Y2 = take(BN * h.out);
  L.Gm = take((int64_t)h.B * h.out);
  L.C1 = take((int64_t)h.B * 64);
  L.Dc = take((int64_t)h.B * 64);
  L.total = o;
  o = 0;
  L.dl = take((int64_t)h.B * h.classes);
  L.dDc = take((int64_t)h.B * 64);
  L.dC1 = take((int64_t)h.B * 64);
  L.dG = take((int64_t)h.B * h.out);
  L.dY2 = take(BN * h.out);
  L.dD1 = take(BN * h.hid);
  L.dY1 = take(BN * h.hid);
  L.dH1 = take(BN * h.Dv);
  L.part = take(4096);
  L.stotal = o;
  return L;
}

__global__ void colsum_f32_kernel(const float* __restrict__ X, int M, int N, float* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int m = 0; m < M; ++m) s += X[(int64_t)m * N + n];
  out[n] = s;
}
int colsum_f32(hipStream_t s, const float* X, int M, int N, float* out) {
  hipLaunchKernelGGL(colsum_f32_kernel, dim3((unsigned)cdiv(N, 256)), dim3(256), 0, s, X, M, N, out);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

constexpr uint32_t ST_GCN = 40, ST_CLS = 41;  // dropout streams of gcn.dropout and classifier[2]

int head_forward(hipStream_t s, const HeadDims& h, const float* const* P, const float* feats, const float* A,
                 float* work, bool training, uint64_t seed, float p, float* logits) {
  const HeadLayout L = head_layout(h);
  const int BN = h.B * h.N;
  const float pd = training ? p : 0.f;
  float* H1 = work + L.H1;
  float* Y1 = work + L.Y1;
  float* D1 = work + L.D1;
  float* Y2 = work + L.Y2;
  float* Gm = work + L.Gm;
  float* C1 = work + L.C1;
  float* Dc = work + L.Dc;
  DFD_TRY(launch_gcn_mix(s, A, feats, h.B, h.N, h.Dv, false, H1));
  DFD_TRY(launch_sgemm(s, false, false, H1, h.Dv, P[0], h.Dv, Y1, h.hid, BN, h.hid, h.Dv, 0.f, P[1]));
  DFD_TRY(launch_relu_drop(s, Y1, D1, (int64_t)BN * h.hid, seed, ST_GCN, pd));
  DFD_TRY(launch_sgemm(s, false, false, D1, h.hid, P[2], h.hid, Y2, h.out, BN, h.out, h.hid, 0.f, P[3]));
  DFD_TRY(launch_relu_drop(s, Y2, nullptr, (int64_t)BN * h.out, 0, 0, 0.f));
  DFD_TRY(launch_node_mean(s, Y2, h.B, h.N, h.out, Gm));
  DFD_TRY(launch_sgemm(s, false, false, Gm, h.out, P[4], h.out, C1, 64, h.B, 64, h.out, 0.f, P[5]));
  DFD_TRY(launch_relu_drop(s, C1, Dc, (int64_t)h.B * 64, seed, ST_CLS, pd));
  return launch_sgemm(s, false, false, Dc, 64, P[6], 64, logits, h.classes, h.B, h.classes, 64, 0.f, P[7]);
}

int head_backward(hipStream_t s, const HeadDims& h, const float* const* P, const float* A, const float* work,
                  float* scratch, uint64_t seed, float p, const float* dlogits, float* const* G, float* dfeats) {
  const HeadLayout L = head_layout(h);
  const int BN = h.B * h.N;
  const float* H1 = work + L.H1;
  const float* Y1 = work + L.Y1;
  const float* D1 = work + L.D1;
  const float* Y2 = work + L.Y2;
  const float* Gm = work + L.Gm;
  const float* C1 = work + L.C1;
  const float* Dc = work + L.Dc;
  float* dDc = scratch + L.dDc;
  float* dC1 = scratch + L.dC1;
  float* dG = scratch + L.dG;
  float* dY2 = scratch + L.dY2;
  float* dD1 = scratch + L.dD1;
  float* dY1 = scratch + L.dY1;
  float* dH1 = scratch + L.dH1;
  // classifier[3]
  DFD_TRY(launch_sgemm(s, true, true, dlogits, h.classes, Dc, 64, G[6], 64, h.classes, 64, h.B, 0.f, nullptr));
  DFD_TRY(colsum_f32(s, dlogits, h.B, h.classes, G[7]));
  DFD_TRY(launch_sgemm(s, false, true, dlogits, h.classes, P[6], 64, dDc, 64, h.B, 64, h.classes, 0.f, nullptr));
  DFD_TRY(launch_relu_drop_bwd(s, C1, dDc, dC1, (int64_t)h.B * 64, seed, ST_CLS, p));
  // classifier[0]
  DFD_TRY(launch_sgemm(s, true, true, dC1, 64, Gm, h.out, G[4], h.out, 64, h.out, h.B, 0.f, nullptr));
  DFD_TRY(colsum_f32(s, dC1, h.B, 64, G[5]));
  DFD_TRY(launch_sgemm(s, false, true, dC1, 64, P[4], h.out, dG, h.out, h.B, h.out, 64, 0.f, nullptr));
  // node mean, gcn.fc2 (+ReLU)
  DFD_TRY(launch_node_mean_bwd(s, dG, h.B, h.N, h.out, dY2));
  DFD_TRY(launch_relu_drop_bwd(s, Y2, dY2, dY2, (int64_t)BN * h.out, 0, 0, 0.f));
  DFD_TRY(launch_sgemm(s, true, true, dY2, h.out, D1, h.hid, G[2], h.hid, h.out, h.hid, BN, 0.f, nullptr));
  DFD_TRY(colsum_f32(s, dY2, BN, h.out, G[3]));
  DFD_TRY(launch_sgemm(s, false, true, dY2, h.out, P[2], h.hid, dD1, h.hid, BN, h.hid, h.out, 0.f, nullptr));
  // dropout + ReLU, gcn.fc1, A_norm mixing
  DFD_TRY(launch_relu_drop_bwd(s, Y1, dD1, dY1, (int64_t)BN * h.hid, seed, ST_GCN, p));
  DFD_TRY(launch_sgemm(s, true, true, dY1, h.hid, H1, h.Dv, G[0], h.Dv, h.hid, h.Dv, BN, 0.f, nullptr));
  DFD_TRY(colsum_f32(s, dY1, BN, h.hid, G[1]));
  DFD_TRY(launch_sgemm(s, false, true, dY1, h.hid, P[0], h.Dv, dH1, h.Dv, BN, h.Dv, h.hid, 0.f, nullptr));
  return launch_gcn_mix(s, A, dH1, h.B, h.N, h.Dv, true, dfeats);
}

int head_check(const HeadDims& h) {
  if (h.B < 1 || h.N < 1 || h.Dv < 8 || h.hid < 1 || h.out < 1 || h.classes < 1) {
    set_error("gcn head: bad dimensions", __FILE__, __LINE__);
    return -1;
  }
  return 0;
}

}  // namespace

}  // namespace dfd

using dfd::VitDims;

#define VIT_GUARD_BEGIN try {
#define VIT_GUARD_END                                \
  }                                                  \
  catch (const std::exception& e) {                  \
    dfd::set_error(e.what(), __FILE__, __LINE__);    \
    return -1;                                       \
  }

extern "C" {

int dfd_vit_param_count(int depth) { return depth < 1 || depth > 12 ? -1 : dfd::vit_nparams(depth); }

int64_t dfd_vit_work_bytes(int dtype, int depth, int images, int height, int width) {
  const VitDims d{dtype, depth, images, height, width};
  if (dfd::vit_check(d)) return -1;
  return dfd::vit_layout(d).total;
}

int64_t dfd_vit_scratch_bytes(int dtype, int depth, int images, int height, int width) {
  const VitDims d{dtype, depth, images, height, width};
  if (dfd::vit_check(d)) return -1;
  return dfd::vit_layout(d).stotal;
}

int dfd_vit_forward(void* stream, int dtype, int depth, int images, int nodes, int height, int width, const float* x,
                    const int64_t* x_strides5, const float* const* params, void* work, float* feats) {
  return dfd_vit_forward_ex(stream, dtype, depth, images, nodes, height, width, x, x_strides5, params, work, feats, 1);
}

int dfd_vit_forward_ex(void* stream, int dtype, int depth, int images, int nodes, int height, int width, const float* x,
                       const int64_t* x_strides5, const float* const* params, void* work, float* feats,
                       int keep_backward) {
  VIT_GUARD_BEGIN
  const VitDims d{dtype, depth, images, height, width};
  if (dfd::vit_check(d)) return -1;
  if (!x || !x_strides5 || !params || !work || !feats || nodes < 1 || images % nodes) {
    dfd::set_error("vit forward: null argument or images not a multiple of nodes", __FILE__, __LINE__);
    return -1;
  }
  const dfd::VitImg im{nodes, height, width, x_strides5[0], x_strides5[1], x_strides5[2], x_strides5[3], x_strides5[4]};
  const auto L = dfd::vit_layout(d);
  if (dtype == 1)
    return dfd::vit_forward_t<dfd::bf16>((hipStream_t)stream, d, L, params, x, im, (char*)work, feats,
                                         keep_backward != 0);
  return dfd::vit_forward_t<float>((hipStream_t)stream, d, L, params, x, im, (char*)work, feats, keep_backward != 0);
  VIT_GUARD_END
}

int dfd_vit_backward(void* stream, int dtype, int depth, int images, int height, int width,
                     const float* const* params, void* work, void* scratch, const float* dfeats, float* const* grads) {
  VIT_GUARD_BEGIN
  const VitDims d{dtype, depth, images, height, width};
  if (dfd::vit_check(d)) return -1;
  if (!params || !work || !scratch || !dfeats || !grads) {
    dfd::set_error("vit backward: null argument", __FILE__, __LINE__);
    return -1;
  }
  const auto L = dfd::vit_layout(d);
  if (dtype == 1)
    return dfd::vit_backward_t<dfd::bf16>((hipStream_t)stream, d, L, params, (char*)work, (char*)scratch, dfeats, grads);
  return dfd::vit_backward_t<float>((hipStream_t)stream, d, L, params, (char*)work, (char*)scratch, dfeats, grads);
  VIT_GUARD_END
}

int64_t dfd_gcn_head_work_floats(int B, int N, int feat_dim, int hid, int out, int num_classes) {
  const dfd::HeadDims h{B, N, feat_dim, hid, out, num_classes};
  if (dfd::head_check(h)) return -1;
  return dfd::head_layout(h).total;
}

int64_t dfd_gcn_head_scratch_floats(int B, int N, int feat_dim, int hid, int out, int num_classes) {
  const dfd::HeadDims h{B, N, feat_dim, hid, out, num_classes};
  if (dfd::head_check(h)) return -1;
  return dfd::head_layout(h).stotal;
}

int dfd_gcn_head_forward(void* stream, int B, int N, int feat_dim, int hid, int out, int num_classes,
                         const float* feats, const float* a_norm, const float* const* params, float* work,
                         int training, uint64_t seed, float p, float* logits) {
  VIT_GUARD_BEGIN
  const dfd::HeadDims h{B, N, feat_dim, hid, out, num_classes};
  if (dfd::head_check(h)) return -1;
  if (!feats || !a_norm || !params || !work || !logits) {
    dfd::set_error("gcn head forward: null argument", __FILE__, __LINE__);
    return -1;
  }
  return dfd::head_forward((hipStream_t)stream, h, params, feats, a_norm, work, training != 0, seed, p, logits);
  VIT_GUARD_END
}

int dfd_gcn_head_backward(void* stream, int B, int N, int feat_dim, int hid, int out, int num_classes,
                          const float* a_norm, const float* const* params, const float* work, float* scratch,
                          int training, uint64_t seed, float p, const float* dlogits, float* const* grads,
                          float* dfeats) {
  VIT_GUARD_BEGIN
  const dfd::HeadDims h{B, N, feat_dim, hid, out, num_classes};
  if (dfd::head_check(h)) return -1;
  if (!a_norm || !params || !work || !scratch || !dlogits || !grads || !dfeats) {
    dfd::set_error("gcn head backward: null argument", __FILE__, __LINE__);
    return -1;
  }
  return dfd::head_backward((hipStream_t)stream, h, params, a_norm, work, scratch, seed, training ? p : 0.f, dlogits,
                            grads, dfeats);
  VIT_GUARD_END
}

}  // extern "C"
