// EfficientNet-B0 trunk plan: topology (timm efficientnet_b0), tensor table in
// timm state_dict order, per-shape workspace layout and the forward/backward launch sequences.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "kernels.h"

namespace dfd {

enum TensorKind { TK_PARAM = 0, TK_BNBUF = 1, TK_COUNTER = 2 };

struct TensorSpec {
  std::string name;  // relative to the trunk Sequential, e.g. "2.1.0.conv_dw.weight"
  int kind;
  std::vector<int64_t> shape;
};

struct BNL {        // one BatchNorm(+act) layer
  int C;
  int t_w, t_b, t_rm, t_rv;  // tensor indices
  int64_t o_mean, o_invstd, o_scale, o_shift;  // workspace byte offsets (fp32 [C] each)
};

struct PWL {        // one 1x1 conv
  int cin, cout, t_w;
  int64_t o_w, o_wt;  // workspace byte offsets of compute-dtype W [cout][cin] and W^T [cin][cout]
};

struct Block {
  int ds;           // 1 = DepthwiseSeparable (stage 0), 0 = InvertedResidual
  int stage, idx;
  int cin, cout, mid, rd, k, s;
  int hin, win, hout, wout;
  bool skip;
  PWL pw, pwl;      // ds: only pw (32->16) is used, stored in `pwl`
  BNL bn1, bn2, bn3;  // ds: bn1 after dw, bn3 after pw (bn2 unused)
  int t_dw, t_se_wr, t_se_br, t_se_we, t_se_be;
  // workspace byte offsets of saved tensors
  int64_t o_y1, o_y2, o_y3, o_x, o_sq, o_rpre, o_gate;
  int64_t o_s2;  // materialised silu(bn2(y2)) for the late stages (-1: conv_pwl recomputes it)
  int64_t o_de, o_dz;  // SE backward operands of the deferred SE weight gradients ([F][mid], [F][rd] fp32)
};

// Live timing of one launch site inside the plan (HIP events; created when armed, never on the
// launch path).  kind: see ProbeKind.
enum ProbeKind { PK_PW_FWD = 0, PK_DW_FWD = 1, PK_PWL_FWD = 2, PK_DW_DGRAD = 3, PK_DW_WGRAD = 4, PK_PW_DGRAD = 5,
                 PK_PW_WGRAD = 6, PK_PWL_DGRAD = 7, PK_PWL_WGRAD = 8, PK_SE_SQUEEZE = 9, PK_BN_APPLY = 10 };
struct Probe {
  int kind = -1, stage = -1, idx = -1, n = 0, count = 0;
  std::vector<hipEvent_t> b, e;
};

constexpr int kCtrSlots = 1024;
// counters [0, kCtrSe): last-arrival tails; [kCtrSe, kCtrAbort): SE slice barriers; kCtrAbort: the
// device abort word of the slice barriers (tail.h SyncAbort)
constexpr int kCtrSe = 64;
constexpr int kCtrAbort = kCtrSlots - 1;

struct Plan {
  int frames, H, W, dtype;
  int H1, W1, Hf, Wf;  // stem output, final feature map
  std::vector<TensorSpec> tensors;
  std::vector<int64_t> offs;  // bound offsets (params: into param flat, bnbufs: into bn flat)
  bool bound = false;
  int t_stem;
  BNL bn_stem, bn_head;
  PWL head;
  std::vector<Block> blocks;
  // workspace
  int64_t ws_bytes = 0;
  int64_t o_ystem, o_yh, o_stats, o_slab, o_part, o_coef, o_bc, o_de, o_dz, o_pf;
  int64_t o_gx[2], o_gs, o_ge1, o_ge2;
  int64_t o_w1t, o_q, o_bv, o_tg, o_gram, o_cs;  // conv_pw backward through its BN (bn_fold_pw)
  int64_t o_coef1, o_stats2;  // BN1 backward coefficients / col_sums partials read on the wgrad stream
  int64_t o_bar;  // grid-barrier counters + abort flag of the fused 7x7 MBConv launches (zeroed per forward)
  int64_t o_ctr;  // kCtrSlots last-arrival / SE slice-barrier counters (zeroed per forward)
  int64_t stats_cap, slab_cap, part_cap;
  // cast table (device copy)
  std::vector<CastSeg> cast_host;
  CastSeg* cast_dev = nullptr;
  int cast_max = 0;
  int device = 0;
  int pending_rows = 0;  // stat rows written by the stage-0 dw dgrad, consumed by the stem segment
  Probe probe;
  Tuning tune;  // per-plan kernel-selection overrides (dfd_b0_plan_set_tuning)
  // the backward's weight-gradient stream (created on first use, on the caller stream's device)
  // and the events that order it against the caller's stream
  hipStream_t aux = nullptr;
  int aux_dev = -1;
  hipEvent_t ev[6] = {};
  // sticky error word in coherent pinned host memory: a device-side software barrier that timed out
  // (its launch's outputs invalid) sets it; every later forward / backward of the plan then fails
  // (dfd_last_error) until dfd_b0_plan_clear_status -- loud, with no host synchronisation per call
  int* err_host = nullptr;
};
// the sticky status word (0: ok), read without synchronising (the caller synchronises first for a
// definitive answer)
int plan_status(const Plan& p);

int probe_arm(Plan& p, int kind, int stage, int idx, int n);
int probe_read(Plan& p, float* ms, int cap, int* count);
void probe_disarm(Plan& p);

int plan_build(Plan& p, int frames, int H, int W, int dtype);
int plan_bind(Plan& p, const int64_t* offs, int n);
void plan_free(Plan& p);
int plan_forward(Plan& p, hipStream_t s, const void* x, const int64_t* xs, const InputFmt& in, const float* params,
                 float* bnbuf, char* ws, float* feat, int training, float momentum);
int plan_backward_x(Plan& p, hipStream_t s, const void* x, const int64_t* xs, const InputFmt& in, const float* dfeat,
                    const float* params, char* ws, float* grads, int training, int seg_begin, int seg_end,
                    int accumulate);
// segments: 0 = conv_head+bn2, 1..7 = stage 6..0, 8 = stem.  Tensor index range [lo, hi) whose
// gradients are final once the segment has run.
void plan_segment_range(const Plan& p, int seg, int* lo, int* hi);
constexpr int kNumSegments = 9;
// number of blocks the bf16 forward runs through the fused 7x7 MBConv kernel (0: none)
int plan_fused7_blocks(const Plan& p);
// static topology (shape-independent)
const std::vector<TensorSpec>& b0_tensor_table();

}  // namespace dfd
