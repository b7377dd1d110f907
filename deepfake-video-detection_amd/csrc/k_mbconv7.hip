// Fused MBConv FORWARD for the 7x7 stages of EfficientNet-B0 (timm InvertedResidual blocks.5.1-5.3
// and 6.0, run by self.backbone(x_flat) at src/pretrained_detector.py:116), bf16 storage:
//
//     y1 = x . W1^T            (conv_pw, MFMA)         -> BN1 + SiLU
//     y2 = dwconv_k(a1)        (conv_dw, packed fp32)  -> BN2 + SiLU -> a2
//     gate = sigmoid(We silu(Wr mean_hw(a2) + br) + be)              (SqueezeExcite, per frame)
//     y3 = (a2 * gate) . W3^T  (conv_pwl, MFMA)        -> BN3 (+ x)  -> x_out
//
// ONE workgroup per frame keeps the frame's whole 49 x mid expanded tensor (113 KB bf16) in LDS
// from the expansion GEMM through the depthwise conv, the SE squeeze/excite and the projection GEMM,
// so the expanded activations never make an HBM round trip between those steps (the unfused plan
// runs 9 launches with 6 passes over it).  Weights stream from L2 straight into MFMA fragments.
//
// Training mode: BatchNorm uses batch statistics over all frames.  After each BN-producing step
// every workgroup publishes its frame's per-channel sums; a grid barrier; each workgroup
// finalises its own channel slice (mean, invstd, scale, shift, running-statistics update -- the
// plan's BN buffers, which the backward reads); a second barrier; everyone reads scale/shift.
// That is 6 grid barriers per block (monotonic counter, agent-scope release/acquire, bounded spin
// with an abort flag so a non-resident grid can never hang the device).  The saved tensors of the
// unfused path (y1, y2, s2 = bf16(a2), y3, the SE squeeze/pre-activation/gate vectors and the block
// output) are written for the backward.  Eval mode: running statistics, no barriers, no saved tensors.
// Requires frames <= the co-resident grid (one 156 KB workgroup per CU); the plan checks that and
// otherwise keeps the unfused launches.
#include "kernels.h"
#include "grid_sync.h"

namespace dfd {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int HW7 = 49;
constexpr int MID_MAX = 1152, CIN_MAX = 192, COUT_MAX = 320, RD_MAX = 48;
constexpr int YS = MID_MAX + 8;   // LDS row stride (elements) of the expanded tensor: +16 B per row
constexpr int CC = 64;            // depthwise channel chunk (32 channel pairs)
constexpr int WORK_BYTES = 33024; // union: x tile / padded activation chunk / y3 tile

__device__ __forceinline__ float bfv(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ v2f bf2v(uint32_t w) { return v2f{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)}; }

// D[m][n] = sum_k A[m][k] B[n][k] for m < 49 (A rows 49..63 read as zero), n < N; A: bf16 in LDS
// with row stride AS, B: bf16 [N][K] in global memory (L2-resident weights).  Each wave owns a
// contiguous range of 16-column blocks, NCB at a time (4 x NCB accumulator tiles), with the B
// fragments of the next PF k-steps in flight.  epi(m, n, v) receives the fp32 result.
template <int NCB, int PF, class Epi>
__device__ __forceinline__ void gemm49(const bf16* __restrict__ A, int AS, int K, const bf16* __restrict__ B, int N,
                                       Epi&& epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ncb = N >> 4, per = (ncb + 3) >> 2;
  const int cb0 = wave * per, cb1 = min(ncb, cb0 + per);
  const int nk = K >> 5;
  const int lr = lane & 15, lk = 8 * (lane >> 4);
  for (int g0 = cb0; g0 < cb1; g0 += NCB) {
    f32x4_t acc[4][NCB];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int j = 0; j < NCB; ++j) acc[rb][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    bf16x8_t ring[PF][NCB];
    auto loadb = [&](auto pc, int ks) {
      constexpr int p = decltype(pc)::value;
#pragma unroll
      for (int j = 0; j < NCB; ++j) {
        const int cb = g0 + j;
        const bool ok = cb < cb1;
        const bf16* src = B + (int64_t)((ok ? cb : cb0) * 16 + lr) * K + ks * 32 + lk;
        const uint4 v = *reinterpret_cast<const uint4*>(src);
        ring[p][j] = __builtin_bit_cast(bf16x8_t, v);
      }
    };
    static_for<PF>([&](auto pc) {
      if (decltype(pc)::value < nk) loadb(pc, decltype(pc)::value);
    });
    for (int ks0 = 0; ks0 < nk; ks0 += PF) {
      static_for<PF>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        const int ks = ks0 + p;
        if (ks >= nk) return;
        bf16x8_t af[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int row = rb * 16 + lr;
          const uint4 v = row < HW7 ? *reinterpret_cast<const uint4*>(A + row * AS + ks * 32 + lk) : make_uint4(0, 0, 0, 0);
          af[rb] = __builtin_bit_cast(bf16x8_t, v);
        }
#pragma unroll
        for (int j = 0; j < NCB; ++j)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
            acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rb], ring[p][j], acc[rb][j], 0, 0, 0);
        if (ks + PF < nk) loadb(pc, ks + PF);
      });
    }
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
      if (g0 + j >= cb1) continue;
      const int n = (g0 + j) * 16 + lr;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rb * 16 + 4 * (lane >> 4) + r;
          if (m < HW7) epi(m, n, acc[rb][j][r]);
        }
    }
  }
}

// fixed-order block sum of a double (4 waves x 64 lanes), valid in thread 0
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) r = ((sh[0] + sh[1]) + sh[2]) + sh[3];
  __syncthreads();
  return r;
}

}  // namespace

// BN finalisation of this workgroup's channel slice from the per-frame partial rows
// part[F][2][C] (training): the plan's BN buffers (mean, invstd, scale, shift) and running stats
__device__ void mb7_bn_finalize(const Mb7Bn& bn, const float* __restrict__ part, int F, int C, float momentum,
                                float eps, double* sh) {
  const int G = gridDim.x, per = (C + G - 1) / G;
  const int c0 = blockIdx.x * per, c1 = min(C, c0 + per);
  const int64_t count = (int64_t)F * HW7;
  for (int c = c0; c < c1; ++c) {
    double s = 0.0, q = 0.0;
    for (int r = threadIdx.x; r < F; r += 256) {
      s += (double)part[((int64_t)r * 2 + 0) * C + c];
      q += (double)part[((int64_t)r * 2 + 1) * C + c];
    }
    s = block_sum_d(s, sh);
    q = block_sum_d(q, sh);
    if (threadIdx.x == 0) {
      const double m = s / (double)count;
      double var = q / (double)count - m * m;
      if (var < 0.0) var = 0.0;
      const float is = (float)(1.0 / sqrt(var + (double)eps));
      const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      bn.run_mean[c] = (float)((1.0 - momentum) * bn.run_mean[c] + momentum * m);
      bn.run_var[c] = (float)((1.0 - momentum) * bn.run_var[c] + momentum * unb);
      const float sc = bn.gamma[c] * is;
      bn.mean[c] = (float)m;
      bn.invstd[c] = is;
      bn.scale[c] = sc;
      bn.shift[c] = bn.beta[c] - (float)m * sc;
    }
  }
}

// scale / shift of channel c: the finalised buffers (training) or the running statistics (eval,
// the operations of bn_finalize_kernel's eval branch)
__device__ __forceinline__ void mb7_ss(const Mb7Bn& bn, int training, float eps, int c, float& sc, float& sh) {
  if (training) {
    sc = bn.scale[c];
    sh = bn.shift[c];
  } else {
    const float is = 1.0f / sqrtf(bn.run_var[c] + eps);
    sc = bn.gamma[c] * is;
    sh = bn.beta[c] - bn.run_mean[c] * sc;
  }
}

// development timing (tools/kbench mb7): wall-clock stamp of phase i of this workgroup
#define MB7_TS(i) \
  if (a.ts && threadIdx.x == 0) a.ts[blockIdx.x * 24 + (i)] = wall_clock64()

template <int K>
__global__ __launch_bounds__(256, 1) void mbconv7_fwd_kernel(Mb7Args a) {
  constexpr int PAD = K / 2, PW = 7 + K - 1;
  __shared__ __attribute__((aligned(16))) bf16 ybuf[HW7 * YS];
  __shared__ __attribute__((aligned(16))) char work[WORK_BYTES];
  __shared__ __attribute__((aligned(16))) float sqs[MID_MAX];
  __shared__ __attribute__((aligned(16))) float gts[MID_MAX];
  __shared__ float zs[RD_MAX];
  __shared__ float stp[8][2][CC];
  __shared__ double dsh[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int f = blockIdx.x, F = a.frames;
  const int mid = a.mid, cin = a.cin, cout = a.cout, rd = a.rd;
  const int training = a.training;
  unsigned bar_target = 0;
  const unsigned G = gridDim.x;
  uint16_t* yb = reinterpret_cast<uint16_t*>(ybuf);
  const int64_t row0 = (int64_t)f * HW7;
  MB7_TS(0);

  // ---- x tile -> LDS (bf16 [49][cin + 8]) ----
  const int XS = cin + 8;
  bf16* xbuf = reinterpret_cast<bf16*>(work);
  for (int v = tid; v < HW7 * (cin / 8); v += 256) {
    const int r = v / (cin / 8), c8 = (v - r * (cin / 8)) * 8;
    *reinterpret_cast<uint4*>(xbuf + r * XS + c8) = *reinterpret_cast<const uint4*>(a.x + (row0 + r) * cin + c8);
  }
  __syncthreads();
  MB7_TS(1);

  // ---- conv_pw: y1 = x . W1^T (rounded to bf16) -> ybuf ----
  gemm49<3, 3>(xbuf, XS, cin, a.w1, mid, [&](int m, int n, float v) { ybuf[m * YS + n] = Tr<bf16>::from_f(v); });
  __syncthreads();
  MB7_TS(2);
  // BN1 per-frame sums (of the rounded values, as the GEMM epilogues of the unfused path) and the
  // saved y1 (training)
  if (training) {
    for (int c2 = tid; c2 < mid / 2; c2 += 256) {
      v2f s = {0.f, 0.f}, q = {0.f, 0.f};
      for (int p = 0; p < HW7; ++p) {
        const v2f v = bf2v(*reinterpret_cast<const uint32_t*>(yb + p * YS + 2 * c2));
        s += v;
        q += v * v;
      }
      float* pr = a.part + (int64_t)f * 2 * mid;
      pr[2 * c2] = s.x; pr[2 * c2 + 1] = s.y;
      pr[mid + 2 * c2] = q.x; pr[mid + 2 * c2 + 1] = q.y;
    }
    for (int v = tid; v < HW7 * (mid / 8); v += 256) {
      const int r = v / (mid / 8), c8 = (v - r * (mid / 8)) * 8;
      *reinterpret_cast<uint4*>(a.y1 + (row0 + r) * mid + c8) = *reinterpret_cast<const uint4*>(yb + r * YS + c8);
    }
    MB7_TS(3);
    if (!grid_sync(a.bar, bar_target += G, a.abort)) return;
    MB7_TS(4);
    mb7_bn_finalize(a.bn[0], a.part, F, mid, a.momentum, a.eps, dsh);
    MB7_TS(5);
    if (!grid_sync(a.bar, bar_target += G, a.abort)) return;
    MB7_TS(6);
  }

  // ---- conv_dw on BN1+SiLU(y1), 64-channel chunks; y2 (bf16) replaces y1 in ybuf ----
  float* act = reinterpret_cast<float*>(work);  // [PW*PW][CC]
  {
    const int cp = tid & 31, slot = tid >> 5;
    for (int c0 = 0; c0 < mid; c0 += CC) {
      for (int i = tid; i < PW * PW * (CC / 2); i += 256) {
        const int pix = i / (CC / 2), q2 = i - pix * (CC / 2);
        const int py = pix / PW - PAD, px = pix % PW - PAD;
        v2f o = {0.f, 0.f};
        if (py >= 0 && py < 7 && px >= 0 && px < 7) {
          const int c = c0 + 2 * q2;
          float s0, h0, s1, h1;
          mb7_ss(a.bn[0], training, a.eps, c, s0, h0);
          mb7_ss(a.bn[0], training, a.eps, c + 1, s1, h1);
          const v2f y = bf2v(*reinterpret_cast<const uint32_t*>(yb + (py * 7 + px) * YS + c));
          const float z0 = y.x * s0 + h0, z1 = y.y * s1 + h1;
          o = v2f{siluf_(z0), siluf_(z1)};
        }
        *reinterpret_cast<v2f*>(act + pix * CC + 2 * q2) = o;
      }
      __syncthreads();
      const int c = c0 + 2 * cp;
      v2f wk[K * K];
#pragma unroll
      for (int t = 0; t < K * K; ++t) wk[t] = v2f{a.wdw[(int64_t)c * K * K + t], a.wdw[(int64_t)(c + 1) * K * K + t]};
      v2f s = {0.f, 0.f}, q = {0.f, 0.f};
      for (int p = slot; p < HW7; p += 8) {
        const int oy = p / 7, ox = p - oy * 7;
        v2f acc = {0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int kw = 0; kw < K; ++kw)
            acc = __builtin_elementwise_fma(*reinterpret_cast<const v2f*>(act + ((oy + kh) * PW + ox + kw) * CC + 2 * cp),
                                            wk[kh * K + kw], acc);
        const uint32_t w2 = pack2bf(acc.x, acc.y);
        *reinterpret_cast<uint32_t*>(yb + p * YS + c) = w2;
        const v2f v = bf2v(w2);
        s += v;
        q += v * v;
      }
      stp[slot][0][2 * cp] = s.x; stp[slot][0][2 * cp + 1] = s.y;
      stp[slot][1][2 * cp] = q.x; stp[slot][1][2 * cp + 1] = q.y;
      __syncthreads();  // act is rebuilt by the next chunk; stp complete
      if (training && tid < 2 * CC) {
        const int w = tid / CC, cl = tid - w * CC;
        float v = 0.f;
#pragma unroll
        for (int sl = 0; sl < 8; ++sl) v += stp[sl][w][cl];
        a.part[((int64_t)f * 2 + w) * mid + c0 + cl] = v;
      }
    }
  }
  __syncthreads();
  MB7_TS(7);
  if (training) {
    for (int v = tid; v < HW7 * (mid / 8); v += 256) {
      const int r = v / (mid / 8), c8 = (v - r * (mid / 8)) * 8;
      *reinterpret_cast<uint4*>(a.y2 + (row0 + r) * mid + c8) = *reinterpret_cast<const uint4*>(yb + r * YS + c8);
    }
    MB7_TS(8);
    if (!grid_sync(a.bar, bar_target += G, a.abort)) return;
    MB7_TS(9);
    mb7_bn_finalize(a.bn[1], a.part, F, mid, a.momentum, a.eps, dsh);
    MB7_TS(10);
    if (!grid_sync(a.bar, bar_target += G, a.abort)) return;
    MB7_TS(11);
  }

  // ---- BN2 + SiLU: a2 (fp32) -> squeeze sums; s2 = bf16(a2) in place (and saved) ----
  for (int c2 = tid; c2 < mid / 2; c2 += 256) {
    const int c = 2 * c2;
    float s0, h0, s1, h1;
    mb7_ss(a.bn[1], training, a.eps, c, s0, h0);
    mb7_ss(a.bn[1], training, a.eps, c + 1, s1, h1);
    v2f sum = {0.f, 0.f};
    for (int p = 0; p < HW7; ++p) {
      uint32_t* cell = reinterpret_cast<uint32_t*>(yb + p * YS + c);
      const v2f y = bf2v(*cell);
      const float a0 = siluf_(y.x * s0 + h0), a1 = siluf_(y.y * s1 + h1);
      sum += v2f{a0, a1};
      const uint32_t w2 = pack2bf(a0, a1);
      *cell = w2;
      if (training) *reinterpret_cast<uint32_t*>(a.s2 + (row0 + p) * mid + c) = w2;
    }
    sqs[c] = sum.x * (1.0f / HW7);
    sqs[c + 1] = sum.y * (1.0f / HW7);
  }
  __syncthreads();
  MB7_TS(12);
  // ---- SE: rpre = Wr sq + br ; z = silu(rpre) ; gate = sigmoid(We z + be) ----
  for (int j = wave; j < rd; j += 4) {
    float v = 0.f;
    for (int c = lane; c < mid; c += 64) v += a.wr[(int64_t)j * mid + c] * sqs[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    v += a.br[j];
    if (lane == 0) {
      zs[j] = siluf_(v);
      if (training) a.rpre[(int64_t)f * rd + j] = v;
    }
  }
  __syncthreads();
  for (int c = tid; c < mid; c += 256) {
    float v = a.be[c];
    for (int j = 0; j < rd; ++j) v += a.we[(int64_t)c * rd + j] * zs[j];
    const float g = sigmoidf_(v);
    gts[c] = g;
    if (training) {
      a.gate[(int64_t)f * mid + c] = g;
      a.sq[(int64_t)f * mid + c] = sqs[c];
    }
  }
  __syncthreads();
  MB7_TS(13);
  // ---- a2g = bf16(s2 * gate) in place (the PRO_GATE operand of the unfused projection) ----
  for (int v = tid; v < HW7 * (mid / 2); v += 256) {
    const int p = v / (mid / 2), c = (v - p * (mid / 2)) * 2;
    uint32_t* cell = reinterpret_cast<uint32_t*>(yb + p * YS + c);
    const v2f x2 = bf2v(*cell);
    *cell = pack2bf(x2.x * gts[c], x2.y * gts[c + 1]);
  }
  __syncthreads();
  MB7_TS(14);

  // ---- conv_pwl: y3 = a2g . W3^T -> LDS tile (bf16 [49][cout + 8]) ----
  const int TS = cout + 8;
  bf16* ytile = reinterpret_cast<bf16*>(work);
  gemm49<3, 6>(ybuf, YS, mid, a.w3, cout, [&](int m, int n, float v) { ytile[m * TS + n] = Tr<bf16>::from_f(v); });
  __syncthreads();
  MB7_TS(15);
  const uint16_t* yt = reinterpret_cast<const uint16_t*>(ytile);
  if (training) {
    for (int c = tid; c < cout; c += 256) {
      float s = 0.f, q = 0.f;
      for (int p = 0; p < HW7; ++p) {
        const float v = bfv(yt[p * TS + c]);
        s += v;
        q += v * v;
      }
      a.part[((int64_t)f * 2 + 0) * cout + c] = s;
      a.part[((int64_t)f * 2 + 1) * cout + c] = q;
    }
    for (int v = tid; v < HW7 * (cout / 8); v += 256) {
      const int r = v / (cout / 8), c8 = (v - r * (cout / 8)) * 8;
      *reinterpret_cast<uint4*>(a.y3 + (row0 + r) * cout + c8) = *reinterpret_cast<const uint4*>(yt + r * TS + c8);
    }
    MB7_TS(16);
    if (!grid_sync(a.bar, bar_target += G, a.abort)) return;
    MB7_TS(17);
    mb7_bn_finalize(a.bn[2], a.part, F, cout, a.momentum, a.eps, dsh);
    MB7_TS(18);
    if (!grid_sync(a.bar, bar_target += G, a.abort)) return;
    MB7_TS(19);
  }
  // ---- BN3 (+ skip) -> block output ----
  for (int v = tid; v < HW7 * (cout / 8); v += 256) {
    const int r = v / (cout / 8), c8 = (v - r * (cout / 8)) * 8;
    float y[8], o[8];
    ld8(reinterpret_cast<const bf16*>(yt + r * TS + c8), y);
    float xr[8];
    if (a.skip) ld8(a.x + (row0 + r) * cin + c8, xr);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sc, sh;
      mb7_ss(a.bn[2], training, a.eps, c8 + j, sc, sh);
      o[j] = a.skip ? y[j] * sc + sh + xr[j] : y[j] * sc + sh;
    }
    st8(a.xo + (row0 + r) * cout + c8, o);
  }
  MB7_TS(20);
}

bool mbconv7_supported(int frames, int H, int W, int cin, int mid, int cout, int rd, int k, int s) {
  if (H != 7 || W != 7 || s != 1 || (k != 3 && k != 5)) return false;
  if (cin > CIN_MAX || mid > MID_MAX || cout > COUT_MAX || rd > RD_MAX || rd < 1) return false;
  if (cin % 32 || mid % CC || cout % 16) return false;
  if ((cin + 8) * HW7 * 2 > WORK_BYTES || (cout + 8) * HW7 * 2 > WORK_BYTES ||
      (7 + k - 1) * (7 + k - 1) * CC * 4 > WORK_BYTES)
    return false;
  static const int resident = [] {
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int p3 = 0, p5 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&p3, mbconv7_fwd_kernel<3>, 256, 0) != hipSuccess) p3 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&p5, mbconv7_fwd_kernel<5>, 256, 0) != hipSuccess) p5 = 0;
    per = std::min(p3, p5);
    return per * cus;
  }();
  return frames >= 1 && frames <= resident;
}

int launch_mbconv7_fwd(hipStream_t s, const Mb7Args& a) {
  if (a.k == 3) hipLaunchKernelGGL(mbconv7_fwd_kernel<3>, dim3(a.frames), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(mbconv7_fwd_kernel<5>, dim3(a.frames), dim3(256), 0, s, a);
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
