// Train-mode BatchNorm finalize inside a CONSUMER's workgroup (no launch of its own).
//
// The producers of a BN's input write per-workgroup partial rows stats[rows][2][C] (sum, sum of
// squares, fixed order).  bn_finalize_kernel (k_bn.hip) turned them into mean / invstd / scale /
// shift in a ~5 us launch of its own.  Where the producer wrote few rows (the late stages: the
// small-K 1x1 GEMM writes one row per workgroup, ~12-51 rows; the depthwise forward ~14-50), every
// workgroup of the consumer -- which owns a channel slice anyway -- reduces the rows of its own
// channels itself: rows / (256 / (nc / 4)) x 2 loads per thread, fp64, in a fixed order, so every
// workgroup of a channel slice gets bit-identical constants.  One designated workgroup per slice
// also stores mean / invstd / scale / shift (read by the backward and by later consumers) and
// updates the running statistics (momentum), exactly once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfd {

struct BnFwdFin {
  const float* stats;  // [rows][2][C] partial rows of the producer; rows == 0: not in use
  int rows;
  int64_t count;       // elements per channel (frames x H x W)
  const float *gamma, *beta;
  float *run_mean, *run_var;  // null: no running statistics
  float momentum, eps;
  float *mean, *invstd, *scale, *shift;
};

// rows the consumer-side finalize is used for (larger row counts keep bn_finalize_kernel)
#ifndef DFD_BNFIN_ROWS
#define DFD_BNFIN_ROWS 128  // 64 -> 128: 9.379-9.386 vs 9.384-9.405 ms/step (profiles/r05 ab_bnfin_rows_r05n.txt)
#endif
constexpr int kBnFinRowsMax = DFD_BNFIN_ROWS;
// LDS scratch of bn_fin_wg in doubles (2 x 256 threads x 4 channels)
constexpr int kBnFinScratch = 2 * 256 * 4;

// 256-thread workgroup; channels [c0, c0 + nc), nc <= 128 and a multiple of 4, C % 4 == 0.  Leaves
// scale / shift of the slice in sc[0..nc) / sh[0..nc) (LDS) -- valid after the final __syncthreads.
__device__ __forceinline__ void bn_fin_wg(const BnFwdFin& f, int C, int c0, int nc, bool writer, float* sc, float* sh,
                                          double* scratch) {
  const int tid = threadIdx.x;
  const int cols = nc >> 2;              // float4 columns (<= 32)
  const int RL = 256 / cols;             // row lanes
  const int col = tid % cols, rl = tid / cols;
  double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
  if (rl < RL) {
    const float* base = f.stats + c0 + 4 * col;
    int r = rl;
    for (; r + 3 * RL < f.rows; r += 4 * RL) {  // 8 loads in flight, added in row order
      float4 vs[4], vq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        vs[u] = *reinterpret_cast<const float4*>(base + (int64_t)(r + u * RL) * 2 * C);
        vq[u] = *reinterpret_cast<const float4*>(base + ((int64_t)(r + u * RL) * 2 + 1) * C);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s[0] += vs[u].x; s[1] += vs[u].y; s[2] += vs[u].z; s[3] += vs[u].w;
        q[0] += vq[u].x; q[1] += vq[u].y; q[2] += vq[u].z; q[3] += vq[u].w;
      }
    }
    for (; r < f.rows; r += RL) {
      const float4 vs = *reinterpret_cast<const float4*>(base + (int64_t)r * 2 * C);
      const float4 vq = *reinterpret_cast<const float4*>(base + ((int64_t)r * 2 + 1) * C);
      s[0] += vs.x; s[1] += vs.y; s[2] += vs.z; s[3] += vs.w;
      q[0] += vq.x; q[1] += vq.y; q[2] += vq.z; q[3] += vq.w;
    }
  }
  __syncthreads();  // the caller may alias scratch with LDS it used before
  if (rl < RL) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      scratch[tid * 4 + j] = s[j];  // tid = rl * cols + col
      scratch[1024 + tid * 4 + j] = q[j];
    }
  }
  __syncthreads();
  if (tid < nc) {
    const int cc = tid >> 2, j = tid & 3;
    double ts = 0.0, tq = 0.0;
    for (int l = 0; l < RL; ++l) {  // row lanes in order
      ts += scratch[(l * cols + cc) * 4 + j];
      tq += scratch[1024 + (l * cols + cc) * 4 + j];
    }
    // bn_finalize_kernel's arithmetic (plain sum / sum-of-squares rows)
    const int c = c0 + tid;
    const double cnt = (double)f.count;
    const double m = ts / cnt;
    double var = tq / cnt - m * m;
    if (var < 0.0) var = 0.0;
    const float mu = (float)m, is = (float)(1.0 / sqrt(var + (double)f.eps));
    const float g = f.gamma[c];
    const float scv = g * is, shv = f.beta[c] - mu * scv;
    sc[tid] = scv;
    sh[tid] = shv;
    if (writer) {
      f.mean[c] = mu;
      f.invstd[c] = is;
      f.scale[c] = scv;
      f.shift[c] = shv;
      if (f.run_mean) {
        const double unb = f.count > 1 ? var * cnt / (cnt - 1.0) : var;
        f.run_mean[c] = (float)((1.0 - f.momentum) * f.run_mean[c] + f.momentum * m);
        f.run_var[c] = (float)((1.0 - f.momentum) * f.run_var[c] + f.momentum * unb);
      }
    }
  }
  __syncthreads();
}

}  // namespace dfd
