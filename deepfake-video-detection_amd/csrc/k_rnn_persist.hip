// Persistent recurrence of LogicRNNLSTM (src/RNNModel.py:81-133): the T x L (step, layer) cells of
// the forward, and of the backward-through-time, each run as ONE launch whose workgroups meet at
// grid-wide barriers (grid_sync.h) instead of two launches per cell (K-sliced product + cell
// kernel, k_rnn.hip: 64 launches per direction at T = 16, L = 2, ~13 + 10 us each).
//
// Forward.  Workgroup w owns hidden units j0 = 2w, 2w+1 of every layer.  The 14 packed weight rows
// of those units (the six u-gates' h-columns and the not-gate, rows g*H + j of P_l, see
// rnn_pack_kernel) stay in LDS for the whole launch.  Phase (t, l): every workgroup reads the
// layer's hidden input h_in[B][H] (written by all workgroups in the previous phase; 128 KB, L2),
// computes its 14 gate pre-activations per row with fp32 MFMA (v_mfma_f32_16x16x4f32: exact fp32
// products, 16 B per lane per load: lane (r, q) feeds k = 16s + 4q + i to MFMA i, the same k
// permutation on both operands), applies the cell (the operations of rnn_cell_fwd_kernel) and
// writes h' where the next phase reads it.  The cell state of unit j never leaves its workgroup's
// threads.  One barrier per phase.
//
// Backward.  Phase (t, l), t = T-1..0, l = L-1..0: the cell backward of the workgroup's units
// (as rnn_cell_bwd_kernel; dh from the previous phase's product slices, summed in slice order),
// a barrier, then the product dh_in = DZ_l(t) . P_l as a tiled GEMM over the whole grid:
// workgroup w owns output columns 16*(w % (H/16)) .. +15 and the K slice w / (H/16) of the 7H
// gate rows (8 slices), its P_l slice transposed in LDS for the launch; a barrier.
//
// Numerics: fp32 products and accumulation as the K-sliced path; only the summation order
// inside the products differs (covered by the rtol 1e-4 / 1e-3 bounds of tests/test_rnn.py).
#include "grid_sync.h"
#include "kernels.h"
#include "rnn.h"

namespace dfd {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int RP_UJ = 2;        // hidden units per workgroup
constexpr int RP_ROWS = 7 * RP_UJ;  // gate rows per workgroup (padded to 16 MFMA columns)
constexpr int RP_KS = 8;        // K slices of the backward product
constexpr int RP_LDS = 150 * 1024;

__device__ __forceinline__ float sig_p(float x) { return 1.f / (1.f + __expf(-x)); }

// same counter hash as k_rnn.hip's rnn_drop (identical masks on both paths)
__device__ __forceinline__ float drop_p(uint64_t seed, uint32_t st, int64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  uint64_t z = seed ^ ((uint64_t)st << 56) ^ (uint64_t)idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// acc(16 x 16) += A[16 rows][K] . Bt[16 cols][K]^T ; A rows from global (row pointer per lane,
// nullptr = zero row), Bt from LDS with row stride bs floats.  K % 16 == 0.
__device__ __forceinline__ void mfma_rows16(f32x4_t& acc, const float* __restrict__ arow, const float* bt, int bs,
                                            int K) {
  const int lane = threadIdx.x & 63, q = lane >> 4;
  const float* bp = bt + (lane & 15) * bs + 4 * q;
  const float* ap = arow ? arow + 4 * q : nullptr;
  int s = 0;
  for (; s + 4 <= K / 16; s += 4) {
    float4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = ap ? *reinterpret_cast<const float4*>(ap + 16 * (s + u)) : make_float4(0.f, 0.f, 0.f, 0.f);
      b[u] = *reinterpret_cast<const float4*>(bp + 16 * (s + u));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].x, b[u].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].y, b[u].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].z, b[u].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].w, b[u].w, acc, 0, 0, 0);
    }
  }
  for (; s < K / 16; ++s) {
    const float4 a = ap ? *reinterpret_cast<const float4*>(ap + 16 * s) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b = *reinterpret_cast<const float4*>(bp + 16 * s);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  }
}

}  // namespace


__global__ __launch_bounds__(256, 1) void rnn_fwd_persist_kernel(RnnPersist a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int B = a.B, T = a.T, H = a.H, L = a.L;
  const int PS = H + 4;  // LDS row stride of the weight rows (16 B skew: conflict-free 16-B reads)
  float* zt = lds + (size_t)L * 16 * PS;  // [64][17] gate pre-activations of one 64-row chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * RP_UJ;
  const int64_t ldr = (int64_t)T * H;
  // weight rows: column c = g * RP_UJ + u  <-  P_l row g*H + j0 + u ; columns 14, 15 zero
  for (int l = 0; l < L; ++l)
    for (int i = tid; i < 16 * (H / 4); i += 256) {
      const int c = i / (H / 4), k4 = (i - c * (H / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c < RP_ROWS) {
        const int g = c / RP_UJ, u = c - g * RP_UJ;
        v = *reinterpret_cast<const float4*>(a.P[l] + (int64_t)(g * H + j0 + u) * H + k4);
      }
      *reinterpret_cast<float4*>(lds + ((size_t)l * 16 + c) * PS + k4) = v;
    }
  __syncthreads();
  const unsigned G = gridDim.x;
  unsigned target = 0;
  int phase = 0;
  for (int t = 0; t < T; ++t)
    for (int l = 0; l < L; ++l, ++phase) {
      if (phase > 0 && !grid_sync(a.bar, target += G, a.abort)) return;
      const float* hin = a.UH[l] + (int64_t)t * H;
      const float* wl = lds + (size_t)l * 16 * PS;
      const bool last = l == L - 1;
      for (int b0 = 0; b0 < B; b0 += 64) {
        {
          const int b = b0 + wave * 16 + (lane & 15);
          f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
          mfma_rows16(acc, b < B ? hin + (int64_t)b * ldr : nullptr, wl, PS, H);
#pragma unroll
          for (int i = 0; i < 4; ++i) zt[(wave * 16 + 4 * (lane >> 4) + i) * 17 + (lane & 15)] = acc[i];
        }
        __syncthreads();
        for (int idx = tid; idx < 64 * RP_UJ; idx += 256) {
          const int bl = idx / RP_UJ, u = idx - bl * RP_UJ, b = b0 + bl;
          if (b >= B) continue;
          const int j = j0 + u;
          const int64_t row = (int64_t)b * T + t;
          float z[7];
#pragma unroll
          for (int g = 0; g < 7; ++g) {
            float v = zt[bl * 17 + g * RP_UJ + u] + a.bias7[l][g * H + j];
            if (l == 0 && g < 6) v += a.X0[row * 6 * H + g * H + j];
            z[g] = v;
          }
          const float ga = sig_p(z[0]), go = sig_p(z[1]), gf = sig_p(z[2]), gi = sig_p(z[3]), gg = tanhf(z[4]);
          const float gu = sig_p(z[5]), gn = tanhf(z[6]);
          const float c = a.CI[l][(int64_t)b * ldr + (int64_t)t * H + j];
          const float cn = gf * c + gi * gg;
          const float cl = ga * cn + go * gn;
          const float h = gu * tanhf(cl);
          float* act = a.ACT[l] + row * 7 * H;
          act[0 * H + j] = ga; act[1 * H + j] = go; act[2 * H + j] = gf; act[3 * H + j] = gi;
          act[4 * H + j] = gg; act[5 * H + j] = gu; act[6 * H + j] = gn;
          a.CN[l][row * H + j] = cn;
          a.CL[l][row * H + j] = cl;
          if (last) {
            a.O[row * H + j] = h;
            if (t + 1 < T) {
              a.UH[0][(int64_t)b * ldr + (int64_t)(t + 1) * H + j] = h;
              a.CI[0][(int64_t)b * ldr + (int64_t)(t + 1) * H + j] = cl;
            }
          } else {
            a.UH[l + 1][(int64_t)b * ldr + (int64_t)t * H + j] = h * drop_p(a.seed, (uint32_t)l, row * H + j, a.p);
            a.CI[l + 1][(int64_t)b * ldr + (int64_t)t * H + j] = cl;
          }
        }
        __syncthreads();  // zt is rewritten by the next chunk
      }
    }
}

__global__ __launch_bounds__(256, 1) void rnn_bwd_persist_kernel(RnnPersist a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int B = a.B, T = a.T, H = a.H, L = a.L;
  const int ct = H / 16, kc = 7 * H / RP_KS;
  const int KS_ = kc + 4;  // LDS row stride of the transposed weight slice
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * RP_UJ;
  const int n0 = (blockIdx.x % ct) * 16, ks = blockIdx.x / ct, k0 = ks * kc;
  const int64_t ldr = (int64_t)T * H;
  // this workgroup's product tile: Pt[l][n][k] = P_l[k0 + k][n0 + n]
  for (int l = 0; l < L; ++l)
    for (int i = tid; i < kc * 16; i += 256) {
      const int k = i / 16, n = i - k * 16;
      lds[((size_t)l * 16 + n) * KS_ + k] = a.P[l][(int64_t)(k0 + k) * H + n0 + n];
    }
  __syncthreads();
  const unsigned G = gridDim.x;
  unsigned target = 0;
  bool first_phase = true;
  for (int t = T - 1; t >= 0; --t)
    for (int l = L - 1; l >= 0; --l) {
      const bool last = l == L - 1;
      const bool tlast = t == T - 1;  // nothing flows back from step T
      // ---- cell backward of the workgroup's units (dh slices of the previous phase) ----
      if (!first_phase && !grid_sync(a.bar, target += G, a.abort)) return;
      first_phase = false;
      const bool has_b = !(last && tlast);
      for (int idx = tid; idx < B * RP_UJ; idx += 256) {
        const int b = idx / RP_UJ, u = idx - b * RP_UJ, j = j0 + u;
        const int64_t row = (int64_t)b * T + t;
        float dh = last ? a.dOm[(int64_t)b * ldr + (int64_t)t * H + j] : 0.f;
        if (has_b) {
          const float* pp = a.part + (int64_t)b * H + j;
          const int64_t st = (int64_t)B * H;
          float v = pp[0];
#pragma unroll
          for (int s = 1; s < RP_KS; ++s) v += pp[s * st];
          if (!last) v *= drop_p(a.seed, (uint32_t)l, row * H + j, a.p);
          dh += v;
        }
        float* dcv = last ? a.dc : a.dcl;
        const float dcl0 = (last && tlast) ? 0.f : dcv[(int64_t)b * H + j];
        const float* act = a.ACT[l] + row * 7 * H;
        const float ga = act[0 * H + j], go = act[1 * H + j], gf = act[2 * H + j], gi = act[3 * H + j];
        const float gg = act[4 * H + j], gu = act[5 * H + j], gn = act[6 * H + j];
        const float cn = a.CN[l][row * H + j], cl = a.CL[l][row * H + j];
        const float c = a.CI[l][(int64_t)b * ldr + (int64_t)t * H + j];
        const float tc = tanhf(cl);
        const float dou = dh * tc;
        const float dcl = dh * gu * (1.f - tc * tc) + dcl0;
        const float da = dcl * cn, dcn = dcl * ga, do_ = dcl * gn, dnn = dcl * go;
        const float df = dcn * c, di = dcn * gg, dg = dcn * gi;
        float* dz = a.DZ[l] + row * 7 * H;
        dz[0 * H + j] = da * ga * (1.f - ga);
        dz[1 * H + j] = do_ * go * (1.f - go);
        dz[2 * H + j] = df * gf * (1.f - gf);
        dz[3 * H + j] = di * gi * (1.f - gi);
        dz[4 * H + j] = dg * (1.f - gg * gg);
        dz[5 * H + j] = dou * gu * (1.f - gu);
        dz[6 * H + j] = dnn * (1.f - gn * gn);
        (l > 0 ? a.dcl : a.dc)[(int64_t)b * H + j] = dcn * gf;
      }
      if (l == 0 && t == 0) break;  // no gradient into step 0's h = 0
      // ---- product slice: part[ks][b][n0 + n] = sum_{k in slice} DZ_l[b*T+t][k] P_l[k][n0 + n] ----
      if (!grid_sync(a.bar, target += G, a.abort)) return;
      const float* pt = lds + (size_t)l * 16 * KS_;
      for (int b0 = wave * 16; b0 < B; b0 += 64) {
        const int b = b0 + (lane & 15);
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
        mfma_rows16(acc, b < B ? a.DZ[l] + ((int64_t)b * T + t) * 7 * H + k0 : nullptr, pt, KS_, kc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int bo = b0 + 4 * (lane >> 4) + i;
          if (bo < B) a.part[((int64_t)ks * B + bo) * H + n0 + (lane & 15)] = acc[i];
        }
      }
    }
}

static size_t fwd_lds(const RnnDims& d) { return ((size_t)d.L * 16 * (d.H + 4) + 64 * 17) * 4; }
static size_t bwd_lds(const RnnDims& d) { return (size_t)d.L * 16 * (7 * d.H / RP_KS + 4) * 4; }

bool rnn_persist_supported(const RnnDims& d) {
  if (d.H % 128 || d.H < 128 || d.L < 1 || d.L > 8 || d.B < 1 || d.T < 1) return false;
  if (fwd_lds(d) > RP_LDS || bwd_lds(d) > RP_LDS) return false;
  const int grid = d.H / RP_UJ;
  if (grid != (d.H / 16) * RP_KS) return false;
  static const int resident = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;  // one 256-thread workgroup per CU (the LDS footprint allows no more)
  }();
  return grid <= resident;
}

int64_t rnn_persist_scratch_floats(const RnnDims& d) { return (int64_t)RP_KS * d.B * d.H; }

static int launch_persist(hipStream_t s, bool fwd, const RnnDims& d, const RnnPersist& a) {
  DFD_HIP_CHECK(hipMemsetAsync(a.bar, 0, 64, s));  // counter + abort flag (the 64-B sync block)
  const size_t lds = fwd ? fwd_lds(d) : bwd_lds(d);
  auto k = fwd ? rnn_fwd_persist_kernel : rnn_bwd_persist_kernel;
  static bool attr_set[2] = {false, false};
  if (!attr_set[fwd]) {
    DFD_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      RP_LDS));
    attr_set[fwd] = true;
  }
  hipLaunchKernelGGL(k, dim3(d.H / RP_UJ), dim3(256), lds, s, a);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int launch_rnn_fwd_persist(hipStream_t s, const RnnDims& d, const RnnPersist& a) { return launch_persist(s, true, d, a); }
int launch_rnn_bwd_persist(hipStream_t s, const RnnDims& d, const RnnPersist& a) { return launch_persist(s, false, d, a); }

}  // namespace dfd
