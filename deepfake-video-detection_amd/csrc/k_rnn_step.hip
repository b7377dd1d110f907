// One launch per recurrent cell of LogicRNNLSTM (src/RNNModel.py:81-133), replacing the K-sliced
// product + cell kernel pair of k_rnn.hip (at T = 16, L = 2: 64 launches per direction of 13 + 10 us).
//
// Forward, cell (t, l): workgroup w owns hidden units j0 = 2w, 2w+1.  It stages the 14 packed
// weight rows of those units (the six u-gates' h-columns and the not-gate: rows g*H + j of P_l, see
// rnn_pack_kernel) in LDS, computes the 14 gate pre-activations of every row b from the layer's
// hidden input h_in[B][H] with fp32 MFMA (v_mfma_f32_16x16x4f32, exact fp32 products; lane (r, q)
// loads 16 B and feeds k = 16s + 4q + i to MFMA i -- the same k permutation on both operands), then
// applies the cell (the operations of rnn_cell_fwd_kernel) and writes h' / c' where the next cell
// reads them.  No partial products leave the workgroup.  Every A operand of the lane is loaded before
// the first MFMA (all of h_in's row slice in flight at once) and four accumulators break the MFMA
// dependency chain.
//
// Backward, the product dh_in = DZ_l(t) . P_l (7H -> H) that feeds the next cell backward: a
// (H/16) x 8 grid, workgroup (column tile, K slice) with its P_l slice transposed in LDS, writes
// part[slice][B][H]; rnn_cell_bwd_kernel adds the 8 slices in order.
//
// A persistent form (the whole recurrence in one launch, grid-wide barriers between cells) was
// built and measured first: 790 us forward / 1389 us backward at the bench shape, against 1.45-1.9 us
// per kernel boundary here -- each grid barrier (release + counter + acquire) cost more than the
// launch boundary it replaced, as MI355X_MICROARCH.md's price list says for latency-bound phases.
#include "kernels.h"
#include "rnn.h"

namespace dfd {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int UJ = 2;          // hidden units per workgroup (forward)
constexpr int ROWS = 7 * UJ;   // its gate rows (padded to 16 MFMA columns)
constexpr int KSL = 8;         // K slices of the backward product

__device__ __forceinline__ float sig_s(float x) { return 1.f / (1.f + __expf(-x)); }

// same counter hash as k_rnn.hip's rnn_drop (identical masks on both paths)
__device__ __forceinline__ float drop_s(uint64_t seed, uint32_t st, int64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  uint64_t z = seed ^ ((uint64_t)st << 56) ^ (uint64_t)idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// lane's A operand: NS float4 of row `arow` (nullptr: zeros) at k = 16s + 4q
template <int NS>
__device__ __forceinline__ void load_a(float4 (&av)[NS], const float* __restrict__ arow) {
  const int q = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    av[s] = arow ? *reinterpret_cast<const float4*>(arow + 16 * s + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
}
// D(16x16) = A . Bt^T over K = 16*NS; Bt in LDS [16][bs]
template <int NS>
__device__ __forceinline__ f32x4_t mma_rows(const float4 (&av)[NS], const float* bt, int bs) {
  const int lane = threadIdx.x & 63;
  const float* bp = bt + (lane & 15) * bs + 4 * (lane >> 4);
  f32x4_t acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const float4 b = *reinterpret_cast<const float4*>(bp + 16 * s);
    acc[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s].x, b.x, acc[s & 3], 0, 0, 0);
    acc[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s].y, b.y, acc[s & 3], 0, 0, 0);
    acc[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s].z, b.z, acc[s & 3], 0, 0, 0);
    acc[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s].w, b.w, acc[s & 3], 0, 0, 0);
  }
  return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

}  // namespace

#define RS_TS(i) \
  if (a.ts && threadIdx.x == 0) a.ts[blockIdx.x * 8 + (i)] = wall_clock64()

template <int NS>  // NS = H / 16
__global__ __launch_bounds__(256) void rnn_step_fwd_kernel(RnnStep a, int t, int l) {
  RS_TS(0);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int H = 16 * NS, PS = H + 4;  // weight row stride: 16-B skew, conflict-free 16-B reads
  float* wl = lds;                        // [16][PS]
  float* zt = lds + 16 * PS;              // [64][17]
  const int B = a.B, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * UJ;
  const int64_t ldr = (int64_t)T * H;
  const float* hin = a.UH[l] + (int64_t)t * H;
  const bool last = l == a.L - 1;
  float4 av[NS];
  {  // first chunk's A operands in flight before the weight rows
    const int b = wave * 16 + (lane & 15);
    load_a<NS>(av, b < B ? hin + (int64_t)b * ldr : nullptr);
  }
  // the cell operands that do not depend on the product (bias, x projection, c), loaded per chunk
  // ahead of the product: thread idx < 64*UJ owns (row b0 + idx/UJ, unit j0 + idx%UJ)
  float cz[7], cc = 0.f;
  auto cell_loads = [&](int b0) {
    const int bl = tid / UJ, u = tid - bl * UJ, b = b0 + bl, j = j0 + u;
    if (tid >= 64 * UJ || b >= B) return;
    const int64_t row = (int64_t)b * T + t;
#pragma unroll
    for (int g = 0; g < 7; ++g) {
      float v = a.bias7[l][g * H + j];
      if (l == 0 && g < 6) v += a.X0[row * 6 * H + g * H + j];
      cz[g] = v;
    }
    cc = a.CI[l][(int64_t)b * ldr + (int64_t)t * H + j];
  };
  cell_loads(0);
  // weight rows: column c = g * UJ + u  <-  P_l row g*H + j0 + u ; columns 14, 15 zero.  All of the
  // thread's loads are issued before the first LDS store (one round trip, not one per float4).
  constexpr int WV = 16 * (H / 4) / 256;  // float4 per thread
  float4 wv[WV];
#pragma unroll
  for (int r = 0; r < WV; ++r) {
    const int i = tid + 256 * r, c = i / (H / 4), k4 = (i - c * (H / 4)) * 4;
    const int g = c / UJ, u = c - g * UJ;
    wv[r] = c < ROWS ? *reinterpret_cast<const float4*>(a.P[l] + (int64_t)(g * H + j0 + u) * H + k4)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int r = 0; r < WV; ++r) {
    const int i = tid + 256 * r, c = i / (H / 4), k4 = (i - c * (H / 4)) * 4;
    *reinterpret_cast<float4*>(wl + c * PS + k4) = wv[r];
  }
  __syncthreads();
  RS_TS(1);
  for (int b0 = 0; b0 < B; b0 += 64) {
    if (b0 > 0) {
      const int b = b0 + wave * 16 + (lane & 15);
      load_a<NS>(av, b < B ? hin + (int64_t)b * ldr : nullptr);
      cell_loads(b0);
    }
    const f32x4_t d = mma_rows<NS>(av, wl, PS);
#pragma unroll
    for (int i = 0; i < 4; ++i) zt[(wave * 16 + 4 * (lane >> 4) + i) * 17 + (lane & 15)] = d[i];
    __syncthreads();
    RS_TS(2);
    {
      const int idx = tid;
      const int bl = idx / UJ, u = idx - bl * UJ, b = b0 + bl;
      if (idx >= 64 * UJ || b >= B) goto cell_done;
      const int j = j0 + u;
      const int64_t row = (int64_t)b * T + t;
      float z[7];
#pragma unroll
      for (int g = 0; g < 7; ++g) z[g] = zt[bl * 17 + g * UJ + u] + cz[g];
      const float ga = sig_s(z[0]), go = sig_s(z[1]), gf = sig_s(z[2]), gi = sig_s(z[3]), gg = tanhf(z[4]);
      const float gu = sig_s(z[5]), gn = tanhf(z[6]);
      const float c = cc;
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
        a.UH[l + 1][(int64_t)b * ldr + (int64_t)t * H + j] = h * drop_s(a.seed, (uint32_t)l, row * H + j, a.p);
        a.CI[l + 1][(int64_t)b * ldr + (int64_t)t * H + j] = cl;
      }
    }
  cell_done:
    __syncthreads();  // zt is rewritten by the next chunk
    RS_TS(3);
  }
}

// part[ks][b][n0 + n] = sum_{k < kc} DZ[b*ldz + k0 + k] * P[(k0 + k) * H + n0 + n],  kc = 7H / 8 = 16 * NS
template <int NS>
__global__ __launch_bounds__(256) void rnn_dh_kernel(const float* __restrict__ DZ, int64_t ldz,
                                                     const float* __restrict__ P, int B, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float pt[];  // [16][kc + 4]
  constexpr int kc = 16 * NS, KS_ = kc + 4, H = kc * KSL / 7;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = H / 16;
  const int n0 = (blockIdx.x % ct) * 16, ks = blockIdx.x / ct, k0 = ks * kc;
  float4 av[NS];
  {
    const int b = wave * 16 + (lane & 15);
    load_a<NS>(av, b < B ? DZ + (int64_t)b * ldz + k0 : nullptr);
  }
  // one float4 = 4 columns of one k row; all loads issued before the transposing LDS stores
  constexpr int PV = (kc * 4 + 255) / 256;
  float4 pv[PV];
#pragma unroll
  for (int r = 0; r < PV; ++r) {
    const int i = tid + 256 * r, k = i >> 2, n4 = (i & 3) * 4;
    pv[r] = i < kc * 4 ? *reinterpret_cast<const float4*>(P + (int64_t)(k0 + k) * H + n0 + n4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int r = 0; r < PV; ++r) {
    const int i = tid + 256 * r, k = i >> 2, n4 = (i & 3) * 4;
    if (i < kc * 4) {
      pt[(n4 + 0) * KS_ + k] = pv[r].x;
      pt[(n4 + 1) * KS_ + k] = pv[r].y;
      pt[(n4 + 2) * KS_ + k] = pv[r].z;
      pt[(n4 + 3) * KS_ + k] = pv[r].w;
    }
  }
  __syncthreads();
  for (int b0 = wave * 16; b0 < B; b0 += 64) {
    if (b0 != wave * 16) {
      const int b = b0 + (lane & 15);
      load_a<NS>(av, b < B ? DZ + (int64_t)b * ldz + k0 : nullptr);
    }
    const f32x4_t d = mma_rows<NS>(av, pt, KS_);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int bo = b0 + 4 * (lane >> 4) + i;
      if (bo < B) part[((int64_t)ks * B + bo) * H + n0 + (lane & 15)] = d[i];
    }
  }
}

bool rnn_step_supported(const RnnDims& d) {
  return (d.H == 128 || d.H == 256 || d.H == 384 || d.H == 512) && d.L >= 1 && d.L <= 8 && d.B >= 1 && d.T >= 1;
}
int rnn_step_slices() { return KSL; }

int launch_rnn_step_fwd(hipStream_t s, const RnnStep& a, int t, int l) {
  const size_t lds = (16 * (a.H + 4) + 64 * 17) * sizeof(float);
  const dim3 grid(a.H / UJ);
  switch (a.H) {
    case 128: hipLaunchKernelGGL(rnn_step_fwd_kernel<8>, grid, dim3(256), lds, s, a, t, l); break;
    case 256: hipLaunchKernelGGL(rnn_step_fwd_kernel<16>, grid, dim3(256), lds, s, a, t, l); break;
    case 384: hipLaunchKernelGGL(rnn_step_fwd_kernel<24>, grid, dim3(256), lds, s, a, t, l); break;
    case 512: hipLaunchKernelGGL(rnn_step_fwd_kernel<32>, grid, dim3(256), lds, s, a, t, l); break;
    default: set_error("rnn step: unsupported hidden size", __FILE__, __LINE__); return -1;
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

int launch_rnn_dh(hipStream_t s, const float* DZ, int64_t ldz, const float* P, int B, int H, float* part) {
  const int kc = 7 * H / KSL;
  const size_t lds = (size_t)16 * (kc + 4) * sizeof(float);
  const dim3 grid((H / 16) * KSL);
  switch (H) {
    case 128: hipLaunchKernelGGL(rnn_dh_kernel<7>, grid, dim3(256), lds, s, DZ, ldz, P, B, part); break;
    case 256: hipLaunchKernelGGL(rnn_dh_kernel<14>, grid, dim3(256), lds, s, DZ, ldz, P, B, part); break;
    case 384: hipLaunchKernelGGL(rnn_dh_kernel<21>, grid, dim3(256), lds, s, DZ, ldz, P, B, part); break;
    case 512: hipLaunchKernelGGL(rnn_dh_kernel<28>, grid, dim3(256), lds, s, DZ, ldz, P, B, part); break;
    default: set_error("rnn step: unsupported hidden size", __FILE__, __LINE__); return -1;
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
