// EfficientNet-B0 trunk runtime: topology, workspace layout and launch sequences.
//
// Native replacement for the trunk the reference obtains from
// timm.create_model('efficientnet_b0') and runs as nn.Sequential(children()[:-1])
// (src/pretrained_detector.py:43-46, called at :116).  The tensor table reproduces timm's
// state_dict names/shapes/order, so checkpoints written by the reference load unchanged
// (app.py:1413-1528 strips prefixes and shape-filters by these names).
#include "plan.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace dfd {

namespace {

struct ArchRow {
  int ds, repeats, k, s, e, cout;
};
// timm efficientnet_b0 arch_def: ds_r1_k3_s1_e1_c16, ir_r2_k3_s2_e6_c24, ir_r2_k5_s2_e6_c40,
// ir_r3_k3_s2_e6_c80, ir_r3_k5_s1_e6_c112, ir_r4_k5_s2_e6_c192, ir_r1_k3_s1_e6_c320 (all se0.25)
const ArchRow kArch[7] = {{1, 1, 3, 1, 1, 16},  {0, 2, 3, 2, 6, 24},  {0, 2, 5, 2, 6, 40},  {0, 3, 3, 2, 6, 80},
                          {0, 3, 5, 1, 6, 112}, {0, 4, 5, 2, 6, 192}, {0, 1, 3, 1, 6, 320}};
constexpr int kStem = 32, kHead = 1280;
constexpr int64_t kMaterialiseRows = 20000;  // the 7x7 stages (see Block::o_s2)
// weight-gradient slab regions: a backward segment's wgrad partials each get their own region so
// their reductions can be deferred to one batched launch at the end of the segment (SlabDefer)
constexpr int kSlabRegions = 16;
// fused 7x7 MBConv launches: one 16-B slot (barrier counter) each, the abort flag in the last word
constexpr int kBarSlots = 15;
constexpr int64_t kBarBytes = 256;

struct Topo {
  std::vector<TensorSpec> t;
  int t_stem;
  BNL bn_stem, bn_head;
  PWL head;
  std::vector<Block> blocks;
  int stage_first[8];  // first tensor index of stage s (stage_first[7] = conv_head)

  int add(const std::string& n, int kind, std::vector<int64_t> shape) {
    t.push_back(TensorSpec{n, kind, std::move(shape)});
    return (int)t.size() - 1;
  }
  BNL bn(const std::string& pre, int C) {
    BNL b{};
    b.C = C;
    b.t_w = add(pre + ".weight", TK_PARAM, {C});
    b.t_b = add(pre + ".bias", TK_PARAM, {C});
    b.t_rm = add(pre + ".running_mean", TK_BNBUF, {C});
    b.t_rv = add(pre + ".running_var", TK_BNBUF, {C});
    add(pre + ".num_batches_tracked", TK_COUNTER, {});
    return b;
  }
  PWL pw(const std::string& n, int cin, int cout) {
    PWL p{};
    p.cin = cin;
    p.cout = cout;
    p.t_w = add(n, TK_PARAM, {cout, cin, 1, 1});
    return p;
  }
  Topo() {
    t_stem = add("0.weight", TK_PARAM, {kStem, 3, 3, 3});
    bn_stem = bn("1", kStem);
    int cin = kStem;
    for (int si = 0; si < 7; ++si) {
      stage_first[si] = (int)t.size();
      const ArchRow& a = kArch[si];
      for (int bi = 0; bi < a.repeats; ++bi) {
        Block b{};
        b.ds = a.ds;
        b.stage = si;
        b.idx = bi;
        b.cin = cin;
        b.cout = a.cout;
        b.k = a.k;
        b.s = bi == 0 ? a.s : 1;
        b.mid = cin * a.e;
        b.rd = (int)((double)cin * 0.25 + 0.5);  // round(0.25 * block_in_chs)
        b.skip = (b.s == 1 && cin == a.cout);
        const std::string pre = "2." + std::to_string(si) + "." + std::to_string(bi) + ".";
        if (b.ds) {
          b.t_dw = add(pre + "conv_dw.weight", TK_PARAM, {b.mid, 1, b.k, b.k});
          b.bn1 = bn(pre + "bn1", b.mid);
        } else {
          b.pw = pw(pre + "conv_pw.weight", cin, b.mid);
          b.bn1 = bn(pre + "bn1", b.mid);
          b.t_dw = add(pre + "conv_dw.weight", TK_PARAM, {b.mid, 1, b.k, b.k});
          b.bn2 = bn(pre + "bn2", b.mid);
        }
        b.t_se_wr = add(pre + "se.conv_reduce.weight", TK_PARAM, {b.rd, b.mid, 1, 1});
        b.t_se_br = add(pre + "se.conv_reduce.bias", TK_PARAM, {b.rd});
        b.t_se_we = add(pre + "se.conv_expand.weight", TK_PARAM, {b.mid, b.rd, 1, 1});
        b.t_se_be = add(pre + "se.conv_expand.bias", TK_PARAM, {b.mid});
        if (b.ds) {
          b.pwl = pw(pre + "conv_pw.weight", b.mid, b.cout);
          b.bn3 = bn(pre + "bn2", b.cout);
        } else {
          b.pwl = pw(pre + "conv_pwl.weight", b.mid, b.cout);
          b.bn3 = bn(pre + "bn3", b.cout);
        }
        blocks.push_back(b);
        cin = a.cout;
      }
    }
    stage_first[7] = (int)t.size();
    head = pw("3.weight", cin, kHead);
    bn_head = bn("4", kHead);
  }
};

const Topo& topo() {
  static const Topo tp;
  return tp;
}

int conv_out(int h, int k, int s) { return (h + 2 * (((s - 1) + (k - 1)) / 2) - k) / s + 1; }

}  // namespace

const std::vector<TensorSpec>& b0_tensor_table() { return topo().t; }

void plan_segment_range(const Plan& p, int seg, int* lo, int* hi) {
  const Topo& tp = topo();
  const int n = (int)tp.t.size();
  if (seg == 0) { *lo = tp.stage_first[7]; *hi = n; }
  else if (seg >= 1 && seg <= 7) { const int st = 7 - seg; *lo = tp.stage_first[st]; *hi = tp.stage_first[st + 1]; }
  else { *lo = 0; *hi = tp.stage_first[0]; }
  (void)p;
}

int plan_build(Plan& p, int frames, int H, int W, int dtype) {
  if (frames <= 0 || H < 8 || W < 8) { set_error("plan: bad shape", __FILE__, __LINE__); return -1; }
  if (dtype < 0 || dtype > 2) { set_error("plan: dtype must be 0 (fp32), 1 (bf16) or 2 (fp16)", __FILE__, __LINE__); return -1; }
  const Topo& tp = topo();
  p.frames = frames; p.H = H; p.W = W; p.dtype = dtype;
  p.tensors = tp.t;
  p.t_stem = tp.t_stem;
  p.bn_stem = tp.bn_stem;
  p.bn_head = tp.bn_head;
  p.head = tp.head;
  p.blocks = tp.blocks;
  p.H1 = conv_out(H, 3, 2);
  p.W1 = conv_out(W, 3, 2);
  const int64_t es = dtype ? 2 : 4;
  int64_t cur = 0;
  auto alloc = [&](int64_t bytes) { const int64_t o = cur; cur += (std::max<int64_t>(bytes, 1) + 255) & ~int64_t(255); return o; };
  auto alloc_bn = [&](BNL& b) {
    b.o_mean = alloc(b.C * 4); b.o_invstd = alloc(b.C * 4); b.o_scale = alloc(b.C * 4); b.o_shift = alloc(b.C * 4);
  };
  const int64_t F = frames;
  p.o_ystem = alloc(F * p.H1 * p.W1 * kStem * es);
  alloc_bn(p.bn_stem);
  int h = p.H1, w = p.W1;
  int64_t maxX = F * h * w * kStem, maxS = 0, maxE1 = F * h * w * kStem, maxE2 = 0, maxSE = 0, maxRD = 0;
  for (Block& b : p.blocks) {
    b.hin = h; b.win = w;
    b.hout = conv_out(h, b.k, b.s); b.wout = conv_out(w, b.k, b.s);
    const int64_t Min = F * b.hin * b.win, Mout = F * b.hout * b.wout;
    if (!b.ds) { b.o_y1 = alloc(Min * b.mid * es); alloc_bn(b.bn1); alloc_bn(b.bn2); }
    else { b.o_y1 = -1; alloc_bn(b.bn1); }
    b.o_y2 = alloc(Mout * b.mid * es);
    b.o_y3 = alloc(Mout * b.cout * es);
    b.o_x = alloc(Mout * b.cout * es);
    alloc_bn(b.bn3);
    b.o_sq = alloc(F * b.mid * 4);
    b.o_rpre = alloc(F * b.rd * 4);
    b.o_gate = alloc(F * b.mid * 4);
    b.o_de = alloc(F * b.mid * 4);
    b.o_dz = alloc(F * b.rd * 4);
    // below the streaming threshold conv_pwl runs on the tiled GEMMs, which would recompute the
    // BN+SiLU prologue once per N tile (forward) and per N tile of the weight gradient: the SE
    // squeeze writes the activation once instead (+1 write of the tensor)
    b.o_s2 = Mout < kMaterialiseRows ? alloc(Mout * b.mid * es) : -1;
    maxX = std::max({maxX, Min * b.cin, Mout * b.cout});
    maxS = std::max(maxS, Mout * b.cout);
    if (!b.ds) maxE1 = std::max(maxE1, Min * b.mid);
    maxE2 = std::max(maxE2, Mout * b.mid);
    maxSE = std::max<int64_t>(maxSE, b.mid);
    maxRD = std::max<int64_t>(maxRD, b.rd);
    h = b.hout; w = b.wout;
  }
  p.Hf = h; p.Wf = w;
  const int64_t Mf = F * h * w;
  p.o_yh = alloc(Mf * kHead * es);
  alloc_bn(p.bn_head);
  maxS = std::max(maxS, Mf * kHead);
  maxX = std::max(maxX, Mf * 320);
  // compute-dtype 1x1 weights (+ transposes for dgrad)
  p.cast_host.clear();
  p.cast_max = 0;
  auto alloc_pw = [&](PWL& q) {
    q.o_w = alloc((int64_t)q.cout * q.cin * es);
    q.o_wt = alloc((int64_t)q.cout * q.cin * es);
    p.cast_max = std::max(p.cast_max, q.cout * q.cin);
  };
  for (Block& b : p.blocks) { if (!b.ds) alloc_pw(b.pw); alloc_pw(b.pwl); }
  alloc_pw(p.head);
  // scratch
  p.stats_cap = (int64_t)2048 * 2 * kHead;
  p.slab_cap = (int64_t)4 << 20;  // floats per slab region; kSlabRegions regions (see backward_impl)
  p.part_cap = std::max<int64_t>((int64_t)4 << 20, 5 * F * std::max<int64_t>(kHead, maxSE));
  p.o_stats = alloc(p.stats_cap * 4);
  p.o_slab = alloc(kSlabRegions * p.slab_cap * 4);
  p.o_part = alloc(p.part_cap * 4);
  p.o_coef = alloc(3 * kHead * 4);
  p.o_coef1 = alloc(3 * kHead * 4);
  p.o_stats2 = alloc(p.stats_cap * 4);
  p.o_bc = alloc(F * maxSE * 4);
  p.o_pf = alloc(4 * F * maxSE * 4);  // per-frame SE/BN backward sums
  p.o_de = alloc(F * maxSE * 4);
  p.o_dz = alloc(F * maxRD * 4);
  p.o_gx[0] = alloc(maxX * es);
  p.o_gx[1] = alloc(maxX * es);
  p.o_gs = alloc(maxS * es);
  p.o_ge1 = alloc(maxE1 * es);
  p.o_ge2 = alloc(maxE2 * es);
  int64_t maxPW = 0, maxCin = 0;
  for (const Block& b : p.blocks)
    if (!b.ds) { maxPW = std::max<int64_t>(maxPW, (int64_t)b.mid * b.cin); maxCin = std::max<int64_t>(maxCin, b.cin); }
  p.o_w1t = alloc(maxPW * es);
  p.o_q = alloc(maxCin * maxCin * es);
  p.o_bv = alloc(maxCin * 4);
  p.o_tg = alloc(maxPW * 4);
  p.o_gram = alloc(maxCin * maxCin * 4);
  p.o_cs = alloc(maxCin * 4);
  p.o_bar = alloc(kBarBytes);
  // last-arrival / slice-barrier counters (tail.h, k_bn.hip se_chain): in the per-call workspace, so
  // concurrent calls of one plan on different streams (the app's worker threads) never share them;
  // zeroed at the start of every forward, and every use leaves them zero again
  p.o_ctr = alloc(kCtrSlots * sizeof(unsigned));
  p.ws_bytes = cur;
  p.offs.assign(p.tensors.size(), -1);
  p.bound = false;
  DFD_HIP_CHECK(hipGetDevice(&p.device));
  if (!p.err_host) {
    DFD_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p.err_host), sizeof(int), hipHostMallocCoherent));
    *reinterpret_cast<volatile int*>(p.err_host) = 0;
  }
  return 0;
}

int plan_status(const Plan& p) { return p.err_host ? *reinterpret_cast<volatile const int*>(p.err_host) : 0; }

// every plan entry refuses to run after a timed-out software barrier (plan_status)
static int check_status(const Plan& p) {
  if (plan_status(p) == 0) return 0;
  set_error("b0 plan: a software barrier (SE slice sync) timed out in an earlier call -- that call's outputs "
            "were invalid (another stream's kernels held the CUs the grid needed); clear the status "
            "(dfd_b0_plan_clear_status) to use this plan again", __FILE__, __LINE__);
  return -1;
}

int plan_bind(Plan& p, const int64_t* offs, int n) {
  if (n != (int)p.tensors.size()) { set_error("bind: tensor count mismatch", __FILE__, __LINE__); return -1; }
  p.offs.assign(offs, offs + n);
  const int64_t es = p.dtype ? 2 : 4;
  p.cast_host.clear();
  auto seg = [&](const PWL& q) {
    p.cast_host.push_back(CastSeg{p.offs[q.t_w], q.o_w / es, q.cout, q.cin, 0});
    p.cast_host.push_back(CastSeg{p.offs[q.t_w], q.o_wt / es, q.cout, q.cin, 1});
  };
  for (const Block& b : p.blocks) { if (!b.ds) seg(b.pw); seg(b.pwl); }
  seg(p.head);
  if (!p.cast_dev) DFD_HIP_CHECK(hipMalloc(&p.cast_dev, p.cast_host.size() * sizeof(CastSeg)));

  DFD_HIP_CHECK(hipMemcpy(p.cast_dev, p.cast_host.data(), p.cast_host.size() * sizeof(CastSeg), hipMemcpyHostToDevice));
  p.bound = true;
  return 0;
}

void probe_disarm(Plan& p) {
  for (auto ev : p.probe.b) (void)hipEventDestroy(ev);
  for (auto ev : p.probe.e) (void)hipEventDestroy(ev);
  p.probe = Probe{};
}

int probe_arm(Plan& p, int kind, int stage, int idx, int n) {
  probe_disarm(p);
  p.probe.b.resize(n);
  p.probe.e.resize(n);
  for (int i = 0; i < n; ++i) {
    DFD_HIP_CHECK(hipEventCreate(&p.probe.b[i]));
    DFD_HIP_CHECK(hipEventCreate(&p.probe.e[i]));
  }
  p.probe.kind = kind; p.probe.stage = stage; p.probe.idx = idx; p.probe.n = n; p.probe.count = 0;
  return 0;
}

int probe_read(Plan& p, float* ms, int cap, int* count) {
  const int c = std::min(p.probe.count, std::min(p.probe.n, cap));
  for (int i = 0; i < c; ++i) {
    DFD_HIP_CHECK(hipEventSynchronize(p.probe.e[i]));
    DFD_HIP_CHECK(hipEventElapsedTime(&ms[i], p.probe.b[i], p.probe.e[i]));
  }
  *count = c;
  return 0;
}

static void aux_free(Plan& p) {
  for (auto& e : p.ev)
    if (e) { (void)hipEventDestroy(e); e = nullptr; }
  if (p.aux) { (void)hipStreamDestroy(p.aux); p.aux = nullptr; }
  p.aux_dev = -1;
}

// the weight-gradient stream on the device of the caller's stream (plans are per device, but the
// stream of each call is the caller's)
static int aux_init(Plan& p, hipStream_t s) {
  int dev = 0;
  DFD_HIP_CHECK(hipStreamGetDevice(s, &dev));
  if (p.aux && p.aux_dev == dev) return 0;
  aux_free(p);
  int cur = 0;
  DFD_HIP_CHECK(hipGetDevice(&cur));
  if (cur != dev) DFD_HIP_CHECK(hipSetDevice(dev));
  hipError_t e = hipStreamCreateWithFlags(&p.aux, hipStreamNonBlocking);
  for (int i = 0; i < 6 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&p.ev[i], hipEventDisableTiming);
  if (cur != dev) (void)hipSetDevice(cur);
  if (e != hipSuccess) {
    aux_free(p);
    set_error((std::string("wgrad stream: ") + hipGetErrorString(e)).c_str(), __FILE__, __LINE__);
    return -1;
  }
  p.aux_dev = dev;
  return 0;
}

void plan_free(Plan& p) {
  probe_disarm(p);
  aux_free(p);
  if (p.cast_dev) { (void)hipFree(p.cast_dev); p.cast_dev = nullptr; }
  if (p.err_host) { (void)hipHostFree(p.err_host); p.err_host = nullptr; }
}

// ------------------------------------------------------------------ forward / backward
namespace {


// launch-site log for the PMC traffic attribution (tools/pmc_traffic_r06.py): with DFD_SITE_LOG=<path> every
// launch of the attributed classes appends "<kernel class> <site>" in dispatch order, so per-launch counters
// are matched to layers by the plan's own decisions (which BN takes the fused finalize + apply, ...)
static FILE* site_log_file() {
  static FILE* f = [] {
    const char* path = getenv("DFD_SITE_LOG");
    return path && *path ? fopen(path, "a") : nullptr;
  }();
  return f;
}
static void log_site(const char* cls, const char* what, const Block* b) {
  FILE* f = site_log_file();
  if (!f) return;
  if (b) fprintf(f, "%s %s %d.%d\n", cls, what, b->stage, b->idx);
  else fprintf(f, "%s %s\n", cls, what);
  fflush(f);
}

inline bool probe_hit(const Plan& p, int kind, const Block* b) {
  return p.probe.kind == kind && p.probe.count < p.probe.n && b && b->stage == p.probe.stage &&
         b->idx == p.probe.idx;
}
// Wrap one launch: PROBED(kind, block, launch-expression)
#define PROBED_ON(KIND, BLK, STREAM, EXPR)                                                 \
  do {                                                                                     \
    const bool _hit = probe_hit(p, KIND, BLK);                                             \
    if (_hit) (void)hipEventRecord(p.probe.b[p.probe.count], STREAM);                      \
    DFD_TRY(EXPR);                                                                         \
    if (_hit) { (void)hipEventRecord(p.probe.e[p.probe.count], STREAM); ++p.probe.count; } \
  } while (0)
#define PROBED(KIND, BLK, EXPR) PROBED_ON(KIND, BLK, s, EXPR)

// the fused 7x7-stage MBConv forward (k_mbconv7.hip) for the bf16 plan: knob mbconv7, 0 off (default),
// 1 on.  Off by default: measured 394 us per block (training) against ~135 us for the unfused launches
// (six grid barriers at ~14 us each, per-frame weight re-reads from L2).
// blocks of the 7x7 stages that run as one fused launch (k_mbconv7.hip) in the bf16 forward
static bool block_fused7(const Plan& p, const Block& b) {
  return !b.ds && b.o_s2 >= 0 && tune(TK_MBCONV7) != 0 &&
         mbconv7_supported(p.frames, b.hin, b.win, b.cin, b.mid, b.cout, b.rd, b.k, b.s);
}

template <typename T>
struct Run {
  Plan& p;
  hipStream_t s;
  char* ws;
  const float* P;
  int tr;
  float* f(int64_t o) const { return reinterpret_cast<float*>(ws + o); }
  T* a(int64_t o) const { return reinterpret_cast<T*>(ws + o); }
  const float* prm(int t) const { return P + p.offs[t]; }
  Pro pro_bn(const BNL& b, int rpf, const float* gate = nullptr) const {
    Pro q{};
    q.scale = f(b.o_scale); q.shift = f(b.o_shift); q.gate = gate; q.rows_per_frame = rpf; q.C = b.C;
    return q;
  }
};

// dense NHWC uint8 frames (channel stride 1, pixel stride 3, 4-B aligned rows) take the stem's
// dword-staged load (InputFmt.u8 = 2)
static InputFmt stem_fmt(const InputFmt& in, const void* x, const int64_t* xs) {
  InputFmt o = in;
  if (in.u8 && xs[1] == 1 && xs[3] == 3 && xs[2] % 4 == 0 && xs[0] % 4 == 0 && ((uintptr_t)x & 3) == 0) o.u8 = 2;
  return o;
}

template <typename T>
int forward_impl(Plan& p, hipStream_t s, const void* x, const int64_t* xs, const InputFmt& in, const float* P,
                 float* bnb, char* ws, float* feat, int tr, float mom) {
  Run<T> r{p, s, ws, P, tr};
  const float eps = 1e-5f;
  float* stats = tr ? r.f(p.o_stats) : nullptr;
  int rows = 0;
  // eval mode: every BN's scale / shift from its running statistics in one launch up front (the
  // per-layer finalize launches below are skipped), when the offsets fit the table's 32-bit fields
  bool eval_all = false;
  if (!tr) {
    EvalBnTable t{};
    bool ok = true;
    auto add = [&](const BNL& b) {
      const int64_t v[8] = {p.offs[b.t_w], p.offs[b.t_b], p.offs[b.t_rm], p.offs[b.t_rv],
                            b.o_mean / 4, b.o_invstd / 4, b.o_scale / 4, b.o_shift / 4};
      for (int64_t x : v) ok = ok && x >= 0 && x < INT32_MAX;
      ok = ok && t.n < kEvalBnMax && (b.o_mean | b.o_invstd | b.o_scale | b.o_shift) % 4 == 0;
      if (!ok) return;
      t.e[t.n++] = EvalBnEntry{b.C, (int)v[0], (int)v[1], (int)v[2], (int)v[3], (int)v[4], (int)v[5], (int)v[6], (int)v[7]};
    };
    add(p.bn_stem);
    for (const Block& b : p.blocks) {
      if (!b.ds) add(b.bn1);
      add(b.ds ? b.bn1 : b.bn2);
      add(b.bn3);
    }
    add(p.bn_head);
    if (ok) {
      DFD_TRY(launch_bn_eval_all(s, P, bnb, reinterpret_cast<float*>(ws), t, eps));
      eval_all = true;
    }
  }
  auto fin = [&](const BNL& b, int64_t count) {
    if (eval_all) return 0;
    return launch_bn_finalize(s, r.f(p.o_stats), rows, count, b.C, r.prm(b.t_w), r.prm(b.t_b), bnb + p.offs[b.t_rm],
                              bnb + p.offs[b.t_rv], mom, eps, tr != 0, r.f(b.o_mean), r.f(b.o_invstd), r.f(b.o_scale),
                              r.f(b.o_shift));
  };
  // training: the finalize handed to the BN's consumer (the depthwise forward, the SE squeeze, the
  // global average pool), which runs it inside its own launch where the stat rows are few (bnfin.h;
  // knob tail_fin bit 3) or launches it first; eval: nothing to finalize (fin() is a no-op too)
  const bool cfin = tr && (tune(TK_TAIL_FIN) & 8) != 0;
  auto fin_desc = [&](const BNL& b, int64_t count, float* rows_at) {
    return BnFwdFin{rows_at, rows, count, r.prm(b.t_w), r.prm(b.t_b), bnb + p.offs[b.t_rm],
                    bnb + p.offs[b.t_rv], mom, eps, r.f(b.o_mean), r.f(b.o_invstd), r.f(b.o_scale), r.f(b.o_shift)};
  };
  // the depthwise forward reduces BN1's stat rows (o_stats) in its prologue while its own workgroups
  // store BN2's partial rows in their epilogue: with the finalize inside that launch the BN2 rows go to
  // o_stats2, so no workgroup can overwrite a BN1 row another one has not read yet
  float* const dstats = cfin ? r.f(p.o_stats2) : stats;
  DFD_HIP_CHECK(hipMemsetAsync(ws + p.o_ctr, 0, kCtrSlots * sizeof(unsigned), s));
  unsigned* const ctr = reinterpret_cast<unsigned*>(ws + p.o_ctr);
  DFD_TRY(launch_cast_params<T>(s, P, reinterpret_cast<T*>(ws), p.cast_dev, (int)p.cast_host.size(), p.cast_max));
  const int64_t F = p.frames;
  StemGeom sg{p.frames, p.H, p.W, p.H1, p.W1, xs[0], xs[1], xs[2], xs[3], stem_fmt(in, x, xs)};
  DFD_TRY(launch_stem_fwd<T>(s, sg, x, r.prm(p.t_stem), r.a(p.o_ystem), stats, &rows));
  DFD_TRY(fin(p.bn_stem, F * p.H1 * p.W1));
  const T* xin = nullptr;
  // fused 7x7-stage blocks (bf16): which blocks take the one-launch path, and their barrier slots
  auto fused7 = [&](const Block& b) { return is_bf16<T> && block_fused7(p, b); };
  const int nfused = is_bf16<T> ? plan_fused7_blocks(p) : 0;
  if (nfused && tr) DFD_HIP_CHECK(hipMemsetAsync(ws + p.o_bar, 0, kBarBytes, s));
  int slot = 0;
  for (size_t i = 0; i < p.blocks.size(); ++i) {
    Block& b = p.blocks[i];
    const int64_t Min = F * b.hin * b.win, Mout = F * b.hout * b.wout;
    const int hwo = b.hout * b.wout;
    const BNL& bn_dw = b.ds ? b.bn1 : b.bn2;  // BN after the depthwise conv
    DwGeom g{p.frames, b.hin, b.win, b.mid, b.k, b.s, b.k / 2, b.hout, b.wout};
    if (nfused && fused7(b)) {
      if constexpr (is_bf16<T>) {
        auto bnp = [&](const BNL& q) {
          return Mb7Bn{r.prm(q.t_w), r.prm(q.t_b), bnb + p.offs[q.t_rm], bnb + p.offs[q.t_rv], r.f(q.o_mean),
                       r.f(q.o_invstd), r.f(q.o_scale), r.f(q.o_shift)};
        };
        Mb7Args a{};
        a.frames = p.frames; a.cin = b.cin; a.mid = b.mid; a.cout = b.cout; a.rd = b.rd; a.k = b.k;
        a.skip = b.skip ? 1 : 0; a.training = tr; a.momentum = mom; a.eps = eps;
        a.x = xin; a.w1 = r.a(b.pw.o_w); a.wdw = r.prm(b.t_dw);
        a.wr = r.prm(b.t_se_wr); a.br = r.prm(b.t_se_br); a.we = r.prm(b.t_se_we); a.be = r.prm(b.t_se_be);
        a.w3 = r.a(b.pwl.o_w);
        a.bn[0] = bnp(b.bn1); a.bn[1] = bnp(b.bn2); a.bn[2] = bnp(b.bn3);
        a.y1 = r.a(b.o_y1); a.y2 = r.a(b.o_y2); a.s2 = r.a(b.o_s2); a.y3 = r.a(b.o_y3); a.xo = r.a(b.o_x);
        a.sq = r.f(b.o_sq); a.rpre = r.f(b.o_rpre); a.gate = r.f(b.o_gate); a.part = r.f(p.o_stats);
        a.bar = reinterpret_cast<unsigned*>(ws + p.o_bar) + 4 * slot;
        a.abort = reinterpret_cast<int*>(ws + p.o_bar) + 63;
        ++slot;
        DFD_TRY(launch_mbconv7_fwd(s, a));
      }
      xin = r.a(b.o_x);
      continue;
    }
    if (b.ds) {
      DFD_TRY(launch_dw_fwd<T>(s, g, r.a(p.o_ystem), r.prm(b.t_dw), r.a(b.o_y2), r.pro_bn(p.bn_stem, b.hin * b.win),
                               PRO_BN_SILU, dstats, &rows));
    } else {
      PROBED(PK_PW_FWD, &b, (launch_pw_gemm<T>(s, xin, r.a(b.pw.o_w), r.a(b.o_y1), nullptr, Min, b.mid, b.cin,
                                               PRO_NONE, Pro{}, stats, &rows)));
      if (!cfin) DFD_TRY(fin(b.bn1, Min));
      const BnFwdFin f1 = fin_desc(b.bn1, Min, stats);
      PROBED(PK_DW_FWD, &b, (launch_dw_fwd<T>(s, g, r.a(b.o_y1), r.prm(b.t_dw), r.a(b.o_y2),
                                              r.pro_bn(b.bn1, b.hin * b.win), PRO_BN_SILU, dstats, &rows,
                                              cfin ? &f1 : nullptr)));
    }
    if (!cfin) DFD_TRY(fin(bn_dw, Mout));
    const BnFwdFin f2 = fin_desc(bn_dw, Mout, dstats);
    T* s2 = b.o_s2 >= 0 ? r.a(b.o_s2) : nullptr;
    int hs = 1;
    PROBED(PK_SE_SQUEEZE, &b, (launch_se_squeeze<T>(s, r.a(b.o_y2), r.pro_bn(bn_dw, hwo), p.frames, hwo, b.mid,
                                                    r.f(p.o_part), p.part_cap, &hs, s2, cfin ? &f2 : nullptr)));
    // the excitation's first product split over its channel slices (knob tail_fin bit 1); o_stats is free
    // between the BN2 finalize and the projection's BN3 statistics
    const SeScratch sesc{ctr + kCtrSe, kCtrAbort - kCtrSe, r.f(p.o_stats), p.stats_cap,
                         reinterpret_cast<int*>(ctr + kCtrAbort), p.err_host};
    DFD_TRY(launch_se_fc_fwd(s, r.f(p.o_part), hs, 1.0f / (float)hwo, r.f(b.o_sq), r.prm(b.t_se_wr),
                             r.prm(b.t_se_br), r.prm(b.t_se_we), r.prm(b.t_se_be), p.frames, b.mid, b.rd,
                             r.f(b.o_rpre), r.f(b.o_gate), (tune(TK_TAIL_FIN) & 2) ? &sesc : nullptr));
    PROBED(PK_PWL_FWD, &b, (launch_pw_gemm<T>(s, s2 ? s2 : r.a(b.o_y2), r.a(b.pwl.o_w), r.a(b.o_y3), nullptr, Mout,
                                              b.cout, b.mid, s2 ? PRO_GATE : PRO_BN_SILU_G,
                                              r.pro_bn(bn_dw, hwo, r.f(b.o_gate)), stats, &rows)));
    DFD_TRY(fin(b.bn3, Mout));
    DFD_TRY(launch_bn_apply<T>(s, r.a(b.o_y3), r.f(b.bn3.o_scale), r.f(b.bn3.o_shift), b.skip ? xin : nullptr,
                               r.a(b.o_x), Mout, b.cout));
    xin = r.a(b.o_x);
  }
  const int64_t Mf = F * p.Hf * p.Wf;
  DFD_TRY(launch_pw_gemm<T>(s, xin, r.a(p.head.o_w), r.a(p.o_yh), nullptr, Mf, kHead, p.head.cin, PRO_NONE, Pro{},
                            stats, &rows));
  if (!cfin) DFD_TRY(fin(p.bn_head, Mf));
  const BnFwdFin fh = fin_desc(p.bn_head, Mf, stats);
  DFD_TRY(launch_gap<T>(s, r.a(p.o_yh), r.pro_bn(p.bn_head, p.Hf * p.Wf), p.frames, p.Hf * p.Wf, kHead, feat,
                        cfin ? &fh : nullptr));
  return 0;
}

// Plan knobs (per plan, dfd_b0_plan_set_tuning; defaults in kTuneDefault):
// fold_min_rows: blocks with at least this many conv_pw rows take the BN-folded backward
//   (bn_fold_pw); below it the extra small passes over x cost more than the expanded-tensor passes
//   they save (tests force both paths);
// wgrad_stream: 1x1-conv weight gradients on the plan's second stream (0 off, 1 every block, N > 1
//   blocks with >= N gradient rows).  Off by default: measured 0.17-0.26 ms/step SLOWER at every
//   threshold (in-process A/B, tools/ab_bench.py) -- the persistent, occupancy-sized depthwise kernels
//   of the main chain lose resident workgroup slots to the concurrent gradients;
// pwl_fused: the projection backward of the bf16 plan as one fused launch (k_pwl_bwd.hip: data
//   gradient, weight gradient and the SE + BN2 backward sums; 0 runs the three unfused ones);
// fold_fused: the fold path's conv_pw backward of the bf16 plan as one fused launch
//   (k_pw_fold_bwd.hip: x . Q, the data gradient and the three weight-gradient products; 0: unfused).

template <typename T>
int backward_impl(Plan& p, hipStream_t s, const void* x, const int64_t* xs, const InputFmt& ifmt, const float* dfeat,
                  const float* P, char* ws, float* G, int tr, int seg_begin, int seg_end, int acc) {
  Run<T> r{p, s, ws, P, tr};
  int rows = 0;
  const int64_t F = p.frames;
  unsigned* const ctr = reinterpret_cast<unsigned*>(ws + p.o_ctr);  // zeroed by the forward (see plan_build)
  auto grad = [&](int t) { return G + p.offs[t]; };
  // BN backward finalize + apply: one launch (bn_bwd_apply_fin, knob tail_fin bit 2) when the stat rows are
  // few enough for every apply workgroup to reduce its channels' rows itself, else the two launches
  const bool apply_fin = (tune(TK_TAIL_FIN) & 4) != 0;
  auto fin_apply = [&](const BnBwdIn& in, const BNL& b, const T* Y, int64_t M, T* out, int nrows, const char* what,
                       const Block* blk) {
    int rc = 0;
    if (apply_fin)
      rc = launch_bn_bwd_apply_fin<T>(s, in, Y, M, b.C, r.f(p.o_stats), nrows, M, r.prm(b.t_w), r.f(b.o_mean),
                                      r.f(b.o_invstd), tr != 0, grad(b.t_w), grad(b.t_b), acc != 0, r.f(p.o_coef), out);
    if (rc < 0) return -1;
    log_site(rc == 1 ? "bn_bwd_apply_fin" : "bn_bwd_apply", what, blk);
    if (rc == 1) return 0;
    DFD_TRY(launch_bn_bwd_finalize(s, r.f(p.o_stats), nrows, M, b.C, r.prm(b.t_w), r.f(b.o_mean), r.f(b.o_invstd),
                                   tr != 0, grad(b.t_w), grad(b.t_b), acc != 0, r.f(p.o_coef)));
    DFD_TRY(launch_bn_bwd_apply<T>(s, in, Y, r.f(p.o_coef), out, M, b.C));
    return 0;
  };
  auto bwd_bn = [&](BnBwdIn in, const BNL& b, const T* Y, int64_t M, T* out, const char* what, const Block* blk) {
    in.mean = r.f(b.o_mean); in.invstd = r.f(b.o_invstd); in.scale = r.f(b.o_scale); in.shift = r.f(b.o_shift);
    // the fused finalize + apply reads <= 256 stat rows: the reduction takes that cap on the smaller
    // (late-stage) tensors, where its workgroups still cover the rows in a few passes
    const int cap = apply_fin && M <= 16384 ? 256 : 0;
    DFD_TRY(launch_bn_bwd_reduce<T>(s, in, Y, M, b.C, r.f(p.o_stats), &rows, cap));
    return fin_apply(in, b, Y, M, out, rows, what, blk);
  };
  // BN backward when the partials of g, g*xhat are already in o_stats (written by a fused producer)
  auto bwd_bn_from_stats = [&](BnBwdIn in, const BNL& b, const T* Y, int64_t M, T* out, int nrows, const char* what,
                               const Block* blk) {
    in.mean = r.f(b.o_mean); in.invstd = r.f(b.o_invstd); in.scale = r.f(b.o_scale); in.shift = r.f(b.o_shift);
    return fin_apply(in, b, Y, M, out, nrows, what, blk);
  };
  const int nb = (int)p.blocks.size();
  // the gradient buffer's extent: slab reductions into it are deferred (one launch per segment)
  int64_t gext = 0;
  for (size_t t = 0; t < p.tensors.size(); ++t) {
    if (p.tensors[t].kind != TK_PARAM) continue;
    int64_t nel = 1;
    for (int64_t d : p.tensors[t].shape) nel *= d;
    gext = std::max(gext, p.offs[t] + nel);
  }
  SlabDefer defer{};
  defer.stream = s;
  defer.lo = G;
  defer.hi = G + gext;
  struct DeferScope {
    SlabDefer* prev;
    ~DeferScope() { set_slab_defer(prev); }
  } scope{set_slab_defer(&defer)};
  // The 1x1-conv weight gradients run on the plan's second stream `w`, overlapping the main chain
  // on `s` (BN/SE backward, depthwise backward, data gradients).  Events order the two: w starts
  // a gradient once its operands are final on s (fork), and s waits for w (join) before it
  // overwrites a scratch buffer a queued gradient still reads: o_gs (g3, read by the conv_pwl
  // weight gradient) and o_ge1 / o_coef1 / o_stats2 (the conv_pw weight gradient).  Slab
  // reductions from both streams are batched on s (SlabDefer joins both ways at every flush).
  // knob: 0 off; 1 every block; N > 1 only blocks whose gradient rows reach N (the cross-stream
  // waits cost a few us each: small late-stage gradients are not worth them)
  const int64_t ws_min = tune(TK_WGRAD_STREAM);
  hipStream_t w_aux = s;
  if (ws_min != 0) {
    DFD_TRY(aux_init(p, s));
    w_aux = p.aux;
    defer.aux = w_aux;
    defer.ev_aux = p.ev[4];
    defer.ev_main = p.ev[5];
  }
  hipStream_t w = s;  // the stream of the current block's weight gradients
  bool gs_busy = false, ge1_busy = false;
  auto fork = [&](hipEvent_t ev) -> int {  // w waits for everything enqueued on s so far
    if (w == s) return 0;
    DFD_HIP_CHECK(hipEventRecord(ev, s));
    DFD_HIP_CHECK(hipStreamWaitEvent(w, ev, 0));
    return 0;
  };
  auto mark = [&](hipEvent_t ev, bool& busy) -> int {  // the buffers read on w so far stay busy until ev
    if (w == s) return 0;
    DFD_HIP_CHECK(hipEventRecord(ev, w));
    busy = true;
    return 0;
  };
  auto join = [&](hipEvent_t ev, bool& busy) -> int {  // s waits for the last mark(ev)
    if (busy) DFD_HIP_CHECK(hipStreamWaitEvent(s, ev, 0));
    busy = false;
    return 0;
  };
  MfmaGemm se_jobs[2 * kMfmaBatch];
  int n_se = 0;
  auto flush_se = [&]() -> int {
    const int n = n_se;
    n_se = 0;
    return n ? launch_mfma_small_gemm_batch(s, se_jobs, n) : 0;
  };
  int region = 0, slab_err = 0;
  auto slab = [&]() -> float* {
    if (region == kSlabRegions) {  // every region holds a pending slab: reduce them first
      slab_err |= defer.flush();
      region = 0;
    }
    return r.f(p.o_slab) + (int64_t)(region++) * p.slab_cap;
  };
  for (int seg = seg_begin; seg < seg_end; ++seg) {
    if (seg == 0) {
      const int64_t Mf = F * p.Hf * p.Wf;
      const Block& last = p.blocks[nb - 1];
      BnBwdIn in{};
      in.bc = dfeat; in.bc_scale = 1.0f / (float)(p.Hf * p.Wf); in.rows_per_frame = p.Hf * p.Wf; in.silu = true;
      DFD_TRY(bwd_bn(in, p.bn_head, r.a(p.o_yh), Mf, r.a(p.o_gs), "bn_head", nullptr));
      DFD_TRY(launch_pw_gemm<T>(s, r.a(p.o_gs), r.a(p.head.o_wt), r.a(p.o_gx[(nb - 1) & 1]), nullptr, Mf, p.head.cin,
                                kHead, PRO_NONE, Pro{}, nullptr, nullptr));
      DFD_TRY(launch_pw_wgrad<T>(s, r.a(p.o_gs), r.a(last.o_x), Mf, kHead, p.head.cin, PRO_NONE, Pro{},
                                 slab(), p.slab_cap, grad(p.head.t_w), acc != 0));
    } else if (seg <= 7) {
      const int st = 7 - seg;
      for (int i = nb - 1; i >= 0; --i) {
        const Block& b = p.blocks[i];
        if (b.stage != st) continue;
        const int64_t Min = F * b.hin * b.win, Mout = F * b.hout * b.wout;
        const int hwo = b.hout * b.wout;
        const BNL& bn_dw = b.ds ? b.bn1 : b.bn2;
        T* gout = r.a(p.o_gx[i & 1]);
        DwGeom g{p.frames, b.hin, b.win, b.mid, b.k, b.s, b.k / 2, b.hout, b.wout};
        w = (ws_min != 0 && Mout >= ws_min) ? w_aux : s;
        // BN after the 1x1 projection (no activation)
        BnBwdIn i3{};
        i3.dZ = gout; i3.rows_per_frame = hwo; i3.silu = false;
        DFD_TRY(join(p.ev[1], gs_busy));  // the previous conv_pwl weight gradient is done with o_gs
        int hs = 1, pf = 1;
        const bool fpwl = is16<T> && tune(TK_PWL_FUSED) != 0 &&
                          pwl_bwd_covers(p.frames, hwo, b.cout, b.mid);
        // the BN3 backward applied in the fused kernel's staging pays where the projection is 16 wide
        // (blocks.0.0: +12 us in the kernel against a 49 us apply pass); at 24 wide the kernel's
        // extra time exceeds the pass (+29 / +36 us against 18 us, tools/kbench fused)
        if (fpwl && b.cout <= 16) {
          // data gradient, weight gradient and the SE + BN2 sums in one pass (k_pwl_bwd.hip), the BN3
          // backward applied in its staging: only the BN3 reduction + finalize run here
          i3.mean = r.f(b.bn3.o_mean); i3.invstd = r.f(b.bn3.o_invstd);
          i3.scale = r.f(b.bn3.o_scale); i3.shift = r.f(b.bn3.o_shift);
          DFD_TRY(launch_bn_bwd_reduce<T>(s, i3, r.a(b.o_y3), Mout, b.cout, r.f(p.o_stats), &rows));
          DFD_TRY(launch_bn_bwd_finalize(s, r.f(p.o_stats), rows, Mout, b.cout, r.prm(b.bn3.t_w), r.f(b.bn3.o_mean),
                                         r.f(b.bn3.o_invstd), tr != 0, grad(b.bn3.t_w), grad(b.bn3.t_b), acc != 0,
                                         r.f(p.o_coef)));
          if constexpr (is16<T>) {
            PROBED(PK_PWL_DGRAD, &b, ((pf = launch_pwl_bwd<T>(s, gout, r.a(b.o_y3), r.f(p.o_coef), r.a(b.pwl.o_wt),
                                                           r.a(b.o_y2), r.f(bn_dw.o_scale), r.f(bn_dw.o_shift),
                                                           r.f(bn_dw.o_mean), r.f(bn_dw.o_invstd), r.f(b.o_gate),
                                                           p.frames, hwo, b.cout, b.mid, r.a(p.o_ge2), slab(),
                                                           p.slab_cap, grad(b.pwl.t_w), acc != 0, r.f(p.o_part),
                                                           p.part_cap, &hs)) < 0 ? -1 : 0));
          }
          if (pf != 0) {
            // declined (1: its partial-sum slab or part buffer would not hold this frame count)
            // or launched without the weight gradient (2): materialise gs with the apply pass for the
            // unfused launches below
            DFD_TRY(launch_bn_bwd_apply<T>(s, i3, r.a(b.o_y3), r.f(p.o_coef), r.a(p.o_gs), Mout, b.cout));
            log_site("bn_bwd_apply", "bn3", &b);
          }
        } else {
          DFD_TRY(bwd_bn(i3, b.bn3, r.a(b.o_y3), Mout, r.a(p.o_gs), "bn3", &b));
          if (fpwl) {
            if constexpr (is16<T>) {
              PROBED(PK_PWL_DGRAD, &b, ((pf = launch_pwl_bwd<T>(s, r.a(p.o_gs), nullptr, nullptr, r.a(b.pwl.o_wt),
                                                             r.a(b.o_y2), r.f(bn_dw.o_scale), r.f(bn_dw.o_shift),
                                                             r.f(bn_dw.o_mean), r.f(bn_dw.o_invstd), r.f(b.o_gate),
                                                             p.frames, hwo, b.cout, b.mid, r.a(p.o_ge2), slab(),
                                                             p.slab_cap, grad(b.pwl.t_w), acc != 0, r.f(p.o_part),
                                                             p.part_cap, &hs)) < 0 ? -1 : 0));
            }
          }
        }
        if (pf == 1) {
          PROBED(PK_PWL_DGRAD, &b, (launch_pw_gemm<T>(s, r.a(p.o_gs), r.a(b.pwl.o_wt), r.a(p.o_ge2), nullptr, Mout,
                                                      b.mid, b.cout, PRO_NONE, Pro{}, nullptr, nullptr)));
        }
        if (pf != 0) {  // the weight gradient as its own launch (unfused, or the fused kernel without it)
          const bool mat = b.o_s2 >= 0;
          DFD_TRY(fork(p.ev[0]));
          PROBED_ON(PK_PWL_WGRAD, &b, w,
                    (launch_pw_wgrad<T>(w, r.a(p.o_gs), mat ? r.a(b.o_s2) : r.a(b.o_y2), Mout, b.cout, b.mid,
                                        mat ? PRO_GATE : PRO_BN_SILU_G, r.pro_bn(bn_dw, hwo, r.f(b.o_gate)), slab(),
                                        p.slab_cap, grad(b.pwl.t_w), acc != 0)));
          DFD_TRY(mark(p.ev[1], gs_busy));
        }
        if (pf == 1) {
          // squeeze-excite + the BN+SiLU after the depthwise conv: one pass over (ge2, y2) gives the SE
          // gate gradient and the per-frame sums of the BN backward (input grad = gated + squeeze path)
          DFD_TRY(launch_se_bn_bwd_reduce<T>(s, r.a(p.o_ge2), r.a(b.o_y2), r.f(bn_dw.o_scale), r.f(bn_dw.o_shift),
                                             r.f(bn_dw.o_mean), r.f(bn_dw.o_invstd), p.frames, hwo, b.mid,
                                             r.f(p.o_part), p.part_cap, &hs));
        }
        // the SE weight gradients (two small products per block, off the critical chain) are
        // batched into one launch per segment: de / dz stay in per-block buffers until then
        if (n_se + 2 > (int)(sizeof(se_jobs) / sizeof(se_jobs[0]))) DFD_TRY(flush_se());
        // the BN2 backward finalize (dbeta, dgamma, k1..k3 from gate, bc and the frame sums) in the
        // excitation launch's last workgroups (knob tail_fin bit 0), o_stats free as row scratch here
        const bool sefin = (tune(TK_TAIL_FIN) & 1) != 0;
        // the split excitation's partial products behind the finalize rows in o_stats
        const SeScratch sesc{ctr + kCtrSe, kCtrAbort - kCtrSe, r.f(p.o_stats) + p.stats_cap / 2,
                             p.stats_cap / 2, reinterpret_cast<int*>(ctr + kCtrAbort), p.err_host};
        // (the finalize rows may use only the first half: the split's products sit in the second)
        const BnFramesFin bnf{reinterpret_cast<double*>(r.f(p.o_stats)), p.stats_cap / 2, ctr, kCtrSe, Mout,
                              r.prm(bn_dw.t_w), r.f(bn_dw.o_mean), r.f(bn_dw.o_invstd), tr != 0, acc != 0,
                              grad(bn_dw.t_w), grad(bn_dw.t_b), r.f(p.o_coef)};
        DFD_TRY(launch_se_fc_bwd(s, r.f(p.o_part), hs, r.f(b.o_gate), r.f(b.o_de), r.f(b.o_sq), r.f(b.o_rpre),
                                 r.prm(b.t_se_wr), r.prm(b.t_se_we), p.frames, b.mid, b.rd, 1.0f / (float)hwo,
                                 r.f(b.o_dz), r.f(p.o_bc), grad(b.t_se_wr), grad(b.t_se_br), grad(b.t_se_we),
                                 grad(b.t_se_be), acc != 0, se_jobs + n_se, sefin ? &bnf : nullptr,
                                 (tune(TK_TAIL_FIN) & 2) ? &sesc : nullptr));
        n_se += 2;
        if (!sefin)
          DFD_TRY(launch_bn_bwd_finalize_frames(s, r.f(p.o_part), hs, r.f(b.o_gate), r.f(p.o_bc), p.frames, b.mid,
                                                Mout, r.prm(bn_dw.t_w), r.f(bn_dw.o_mean), r.f(bn_dw.o_invstd),
                                                tr != 0, grad(bn_dw.t_w), grad(bn_dw.t_b), acc != 0, r.f(p.o_coef)));
        // depthwise conv
        // depthwise dgrad fused with the backward reduction of the producer's BN+SiLU
        // (stem BN for the stage-0 block, bn1 otherwise): ge1 = g, stats = partials of g, g*xhat
        const BNL& bn_in = b.ds ? p.bn_stem : b.bn1;
        const T* y_in = b.ds ? r.a(p.o_ystem) : r.a(b.o_y1);
        BnBwdIn fz{};
        fz.mean = r.f(bn_in.o_mean); fz.invstd = r.f(bn_in.o_invstd);
        fz.scale = r.f(bn_in.o_scale); fz.shift = r.f(bn_in.o_shift); fz.silu = true;
        DFD_TRY(join(p.ev[3], ge1_busy));  // the previous conv_pw weight gradient is done with o_ge1
        int fused = 1;
        // stride 1: one kernel also applies the BN2(+SiLU, gate) backward while staging dY
        // (k_dw_bwd1.hip); otherwise the apply pass materialises dY first
        if (dw_bwd2_covers(g)) {  // stride 2 (k_dw_bwd2.hip)
          PROBED(PK_DW_DGRAD, &b, (launch_dw_bwd2<T>(s, g, r.a(p.o_ge2), r.a(b.o_y2), r.f(b.o_gate), r.f(p.o_bc),
                                                     r.f(bn_dw.o_scale), r.f(bn_dw.o_shift), r.f(p.o_coef),
                                                     r.prm(b.t_dw), y_in, fz, r.a(p.o_ge1), r.f(p.o_stats), &rows,
                                                     slab(), p.slab_cap, grad(b.t_dw), acc != 0)));
          log_site("dw_bwd2", "dw", &b);
          fused = 0;
        } else if (dw_bwd1_covers(g)) {
          PROBED(PK_DW_DGRAD, &b, (launch_dw_bwd1<T>(s, g, r.a(p.o_ge2), r.a(b.o_y2), r.f(b.o_gate), r.f(p.o_bc),
                                                     r.f(bn_dw.o_scale), r.f(bn_dw.o_shift), r.f(p.o_coef),
                                                     r.prm(b.t_dw), y_in, fz, r.a(p.o_ge1), r.f(p.o_stats), &rows,
                                                     slab(), p.slab_cap, grad(b.t_dw), acc != 0)));
          log_site("dw_bwd1", "dw", &b);
          fused = 0;
        } else {
          BnBwdIn i2{};
          i2.dZ = r.a(p.o_ge2); i2.gate = r.f(b.o_gate); i2.bc = r.f(p.o_bc); i2.bc_scale = 1.f;
          i2.rows_per_frame = hwo; i2.silu = true;
          i2.mean = r.f(bn_dw.o_mean); i2.invstd = r.f(bn_dw.o_invstd);
          i2.scale = r.f(bn_dw.o_scale); i2.shift = r.f(bn_dw.o_shift);
          DFD_TRY(launch_bn_bwd_apply<T>(s, i2, r.a(b.o_y2), r.f(p.o_coef), r.a(p.o_ge2), Mout, b.mid));
          log_site("bn_bwd_apply", "bn2", &b);
          PROBED(PK_DW_DGRAD, &b, ((fused = launch_dw_bwd<T>(s, g, r.a(p.o_ge2), r.prm(b.t_dw), r.a(p.o_ge1), y_in,
                                                             &fz, r.f(p.o_stats), &rows, slab(), p.slab_cap,
                                                             grad(b.t_dw), acc != 0)) < 0 ? -1 : 0));
        }
        if (fused == 1) {
          PROBED(PK_DW_DGRAD, &b, (launch_dw_dgrad<T>(s, g, r.a(p.o_ge2), r.prm(b.t_dw), r.a(p.o_ge1), y_in, &fz,
                                                      r.f(p.o_stats), &rows)));
          p.pending_rows = rows;
          PROBED(PK_DW_WGRAD, &b, (launch_dw_wgrad<T>(s, g, r.a(p.o_ge2), y_in, r.pro_bn(bn_in, b.hin * b.win),
                                                      PRO_BN_SILU, slab(), p.slab_cap, grad(b.t_dw),
                                                      acc != 0)));
        }
        p.pending_rows = rows;
        if (!b.ds && Min < tune(TK_FOLD_MIN_ROWS)) {
          BnBwdIn i1{};
          i1.dZ = r.a(p.o_ge1); i1.rows_per_frame = b.hin * b.win; i1.silu = false;
          DFD_TRY(bwd_bn_from_stats(i1, b.bn1, r.a(b.o_y1), Min, r.a(p.o_ge1), p.pending_rows, "bn1", &b));
          const T* xin = r.a(p.blocks[i - 1].o_x);
          PROBED(PK_PW_DGRAD, &b, (launch_pw_gemm<T>(s, r.a(p.o_ge1), r.a(b.pw.o_wt), r.a(p.o_gx[(i - 1) & 1]),
                                                     b.skip ? gout : nullptr, Min, b.cin, b.mid, PRO_NONE, Pro{},
                                                     nullptr, nullptr)));
          DFD_TRY(fork(p.ev[2]));
          PROBED_ON(PK_PW_WGRAD, &b, w, (launch_pw_wgrad<T>(w, r.a(p.o_ge1), xin, Min, b.mid, b.cin, PRO_NONE, Pro{},
                                                            slab(), p.slab_cap, grad(b.pw.t_w), acc != 0)));
          DFD_TRY(mark(p.ev[3], ge1_busy));
        } else if (!b.ds) {
          // conv_pw + its BN (no activation): ge1 = k1*g + k2*y1 + k3 is never materialised; by
          // linearity (y1 = x . W^T) the gradients need only g (in ge1) and the block input x:
          //   dX = g . diag(k1)W + x . W^T diag(k2) W + W^T k3 (+ skip);  dW = diag(k1) g^T x +
          //   diag(k2) W x^T x + k3 1^T x   (bn_fold_pw, k_bn.hip)
          const T* xin = r.a(p.blocks[i - 1].o_x);
          T* gxo = r.a(p.o_gx[(i - 1) & 1]);
          DFD_TRY(launch_bn_bwd_finalize(s, r.f(p.o_stats), p.pending_rows, Min, b.mid, r.prm(b.bn1.t_w),
                                         r.f(b.bn1.o_mean), r.f(b.bn1.o_invstd), tr != 0, grad(b.bn1.t_w),
                                         grad(b.bn1.t_b), acc != 0, r.f(p.o_coef1)));
          DFD_TRY(launch_bn_fold_pw<T>(s, r.prm(b.pw.t_w), r.f(p.o_coef1), b.mid, b.cin, r.a(p.o_w1t), r.a(p.o_q),
                                       r.f(p.o_bv)));
          DFD_TRY(join(p.ev[1], gs_busy));  // the conv_pwl weight gradient is done with o_gs
          int ff = 1;
          if (is16<T> && tune(TK_FOLD_FUSED) != 0) {
            // x . Q, the data gradient and the partial products g^T x, x^T x, 1^T x in one pass
            // (k_pw_fold_bwd.hip); their three slab reductions as ONE batched launch
            if constexpr (is16<T>) {
              float* const parts[3] = {r.f(p.o_tg), r.f(p.o_gram), r.f(p.o_cs)};
              const int64_t extent[3] = {(int64_t)b.mid * b.cin, (int64_t)b.cin * b.cin, (int64_t)b.cin};
              SlabDefer loc{};
              loc.stream = s;
              loc.lo = parts[0];
              loc.hi = parts[0] + extent[0];
              for (int q = 1; q < 3; ++q) {
                loc.lo = std::min<const float*>(loc.lo, parts[q]);
                loc.hi = std::max<const float*>(loc.hi, parts[q] + extent[q]);
              }
              const DeferScope inner{set_slab_defer(&loc)};
              PROBED(PK_PW_DGRAD, &b, ((ff = launch_pw_fold_bwd(s, r.a(p.o_ge1), xin, b.skip ? gout : nullptr,
                                                                r.a(p.o_w1t), r.a(p.o_q), r.f(p.o_bv), gxo, Min,
                                                                b.mid, b.cin, slab(), p.slab_cap, parts[0], parts[1],
                                                                parts[2])) < 0 ? -1 : 0));
              if (ff == 0) DFD_TRY(loc.flush());
            }
          }
          if (ff == 0) {
            DFD_TRY(launch_pw_wgrad_bn_combine(s, r.f(p.o_tg), r.f(p.o_gram), r.f(p.o_cs), r.prm(b.pw.t_w),
                                               r.f(p.o_coef1), b.mid, b.cin, grad(b.pw.t_w), acc != 0));
            continue;
          }
          DFD_TRY(launch_tf_gemm<T>(s, xin, r.a(p.o_q), r.a(p.o_gs), b.skip ? gout : nullptr, r.f(p.o_bv), nullptr,
                                    Min, b.cin, b.cin, PRO_NONE, EPI_BIAS | (b.skip ? EPI_RESID : 0)));
          PROBED(PK_PW_DGRAD, &b, (launch_pw_gemm<T>(s, r.a(p.o_ge1), r.a(p.o_w1t), gxo, r.a(p.o_gs), Min, b.cin,
                                                     b.mid, PRO_NONE, Pro{}, nullptr, nullptr)));
          // the weight gradient through the BN on w: g (o_ge1), x, the BN1 coefficients (o_coef1)
          DFD_TRY(fork(p.ev[2]));
          {
            // the three partial products' slab reductions (into o_tg, o_gram, o_cs) run as ONE
            // batched launch before the combine reads them
            float* const parts[3] = {r.f(p.o_tg), r.f(p.o_gram), r.f(p.o_cs)};
            const int64_t extent[3] = {(int64_t)b.mid * b.cin, (int64_t)b.cin * b.cin, (int64_t)b.cin};
            SlabDefer loc{};
            loc.stream = w;
            loc.lo = parts[0];
            loc.hi = parts[0] + extent[0];
            for (int q = 1; q < 3; ++q) {
              loc.lo = std::min<const float*>(loc.lo, parts[q]);
              loc.hi = std::max<const float*>(loc.hi, parts[q] + extent[q]);
            }
            const DeferScope inner{set_slab_defer(&loc)};  // the segment's defer again on exit
            PROBED_ON(PK_PW_WGRAD, &b, w, (launch_pw_wgrad<T>(w, r.a(p.o_ge1), xin, Min, b.mid, b.cin, PRO_NONE, Pro{},
                                                              slab(), p.slab_cap, parts[0], false)));
            DFD_TRY(launch_pw_wgrad<T>(w, xin, xin, Min, b.cin, b.cin, PRO_NONE, Pro{}, slab(), p.slab_cap, parts[1],
                                       false));
            DFD_TRY(launch_col_sums<T>(w, xin, Min, b.cin, r.f(p.o_stats2), p.stats_cap, parts[2]));
            DFD_TRY(loc.flush());
          }
          DFD_TRY(launch_pw_wgrad_bn_combine(w, r.f(p.o_tg), r.f(p.o_gram), r.f(p.o_cs), r.prm(b.pw.t_w),
                                             r.f(p.o_coef1), b.mid, b.cin, grad(b.pw.t_w), acc != 0));
          DFD_TRY(mark(p.ev[3], ge1_busy));
        }
      }
    } else {
      const int64_t M = F * p.H1 * p.W1;
      // ge1 holds g (the stage-0 depthwise backward fused the BN+SiLU part and the stats); the BN's
      // dY = k1*g + k2*y + k3 is applied inside the stem weight gradient's tile staging
      const BNL& b = p.bn_stem;
      DFD_TRY(launch_bn_bwd_finalize(s, r.f(p.o_stats), p.pending_rows, M, b.C, r.prm(b.t_w), r.f(b.o_mean),
                                     r.f(b.o_invstd), tr != 0, grad(b.t_w), grad(b.t_b), acc != 0, r.f(p.o_coef)));
      StemGeom sg{p.frames, p.H, p.W, p.H1, p.W1, xs[0], xs[1], xs[2], xs[3], stem_fmt(ifmt, x, xs)};
      DFD_TRY(launch_stem_wgrad<T>(s, sg, x, r.a(p.o_ge1), r.a(p.o_ystem), r.f(p.o_coef), slab(), p.slab_cap,
                                   grad(p.t_stem), acc != 0));
    }
    // this segment's weight gradients are final when the call returns: flushed here unless the call
    // covers more segments (nobody waits for one; the batches then fill up across segments -- slab()
    // and the SE batch flush themselves when full)
    if (seg + 1 == seg_end) {
      DFD_TRY(flush_se());
      DFD_TRY(defer.flush());
      region = 0;
    }
    DFD_TRY(slab_err);
  }
  return 0;
}

}  // namespace

int plan_fused7_blocks(const Plan& p) {
  if (p.dtype != 1) return 0;  // bf16 plans only
  const TuningScope ts(&p.tune);
  int n = 0;
  for (const Block& b : p.blocks) n += block_fused7(p, b) ? 1 : 0;
  return n > kBarSlots ? 0 : n;
}


const char* const kTuneNames[TK_COUNT] = {"stream_min_rows", "fold_min_rows", "dw_bwd_fused", "gemm_tile", "dw_bwd1",
                                          "dw_fwd1", "wgrad_stream", "mbconv7", "pwl_fused", "fold_fused", "pw_sk", "dw_pf", "dw_rb", "stem_occ", "vg_xp",
                                          "tail_fin", "wg_pf"};
static thread_local const Tuning* t_tune = nullptr;
int64_t tune_override(TuneKey k) { return t_tune ? t_tune->v[k] : kTuneUnset; }
TuningScope::TuningScope(const Tuning* t) : prev(t_tune) { t_tune = t; }
TuningScope::~TuningScope() { t_tune = prev; }

int plan_forward(Plan& p, hipStream_t s, const void* x, const int64_t* xs, const InputFmt& in, const float* params,
                 float* bnbuf, char* ws, float* feat, int training, float momentum) {
  if (!p.bound) { set_error("plan not bound", __FILE__, __LINE__); return -1; }
  DFD_TRY(check_status(p));
  const TuningScope ts(&p.tune);
  if (p.dtype == 1) return forward_impl<bf16>(p, s, x, xs, in, params, bnbuf, ws, feat, training, momentum);
  if (p.dtype == 2) return forward_impl<f16>(p, s, x, xs, in, params, bnbuf, ws, feat, training, momentum);
  return forward_impl<float>(p, s, x, xs, in, params, bnbuf, ws, feat, training, momentum);
}

int plan_backward_x(Plan& p, hipStream_t s, const void* x, const int64_t* xs, const InputFmt& in, const float* dfeat,
                    const float* params, char* ws, float* grads, int training, int seg_begin, int seg_end,
                    int accumulate) {
  if (!p.bound) { set_error("plan not bound", __FILE__, __LINE__); return -1; }
  DFD_TRY(check_status(p));
  if (seg_begin < 0 || seg_end > kNumSegments || seg_begin > seg_end) {
    set_error("backward: bad segment range", __FILE__, __LINE__);
    return -1;
  }
  const TuningScope ts(&p.tune);
  if (p.dtype == 1)
    return backward_impl<bf16>(p, s, x, xs, in, dfeat, params, ws, grads, training, seg_begin, seg_end, accumulate);
  if (p.dtype == 2)
    return backward_impl<f16>(p, s, x, xs, in, dfeat, params, ws, grads, training, seg_begin, seg_end, accumulate);
  return backward_impl<float>(p, s, x, xs, in, dfeat, params, ws, grads, training, seg_begin, seg_end, accumulate);
}

}  // namespace dfd
