// Device-side clip collate: the frame gather of collate_batch_cnn_lstm /
// collate_batch (src/train.py:38-61, 62-100) on uint8 face crops already resident in HBM.
//   out[s] = src[sel[s]]          (sel[s] < 0: an all-zero frame -- a clip with no faces)
// as uint8 (the stem normalises it, k_stem.hip) or as fp32 v / 255 (the reference's
// `.float() / 255.0`, correctly rounded division -> bit-identical).  The frame index table (the
// linspace / last-frame-pad rule) is host index math; the bytes never touch the host again.
// HBM-bound byte work: 16 B per lane in, 16 B (uint8) or 64 B (fp32) per lane out, one frame
// per blockIdx.y so consecutive workgroups stream consecutive bytes of one frame.
#include "kernels.h"

namespace dfd {

template <bool F32>
__global__ __launch_bounds__(256) void collate_gather_vec_kernel(const uint8_t* __restrict__ src,
                                                                 const int64_t* __restrict__ sel, int64_t frame_bytes,
                                                                 void* __restrict__ out) {
  const int64_t s = blockIdx.y;
  const int64_t f = sel[s];
  const int64_t nv = frame_bytes / 16;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256) {
    uint4 q = make_uint4(0u, 0u, 0u, 0u);
    if (f >= 0) q = reinterpret_cast<const uint4*>(src + f * frame_bytes)[v];
    if constexpr (F32) {
      float4* o = reinterpret_cast<float4*>(static_cast<float*>(out) + s * frame_bytes) + v * 4;
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = make_float4((float)(w[j] & 0xffu) / 255.0f, (float)((w[j] >> 8) & 0xffu) / 255.0f,
                           (float)((w[j] >> 16) & 0xffu) / 255.0f, (float)(w[j] >> 24) / 255.0f);
    } else {
      reinterpret_cast<uint4*>(static_cast<uint8_t*>(out) + s * frame_bytes)[v] = q;
    }
  }
}

// any frame size / alignment: one byte per lane
template <bool F32>
__global__ __launch_bounds__(256) void collate_gather_byte_kernel(const uint8_t* __restrict__ src,
                                                                  const int64_t* __restrict__ sel, int64_t frame_bytes,
                                                                  void* __restrict__ out) {
  const int64_t s = blockIdx.y;
  const int64_t f = sel[s];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < frame_bytes; i += (int64_t)gridDim.x * 256) {
    const uint8_t v = f >= 0 ? src[f * frame_bytes + i] : (uint8_t)0;
    if constexpr (F32)
      static_cast<float*>(out)[s * frame_bytes + i] = (float)v / 255.0f;
    else
      static_cast<uint8_t*>(out)[s * frame_bytes + i] = v;
  }
}

int launch_collate_gather(hipStream_t s, const uint8_t* src, const int64_t* sel, int64_t nsel, int64_t frame_bytes,
                          bool f32, void* out) {
  if (nsel <= 0 || frame_bytes <= 0) return 0;
  if (nsel > 65535) { set_error("collate: at most 65535 frames per call", __FILE__, __LINE__); return -1; }
  const bool vec = (frame_bytes % 16) == 0 && ((uintptr_t)src % 16) == 0 && ((uintptr_t)out % 16) == 0;
  const int64_t units = vec ? frame_bytes / 16 : frame_bytes;
  const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv64(units, 256), 64));
  const dim3 grid(gx, (unsigned)nsel);
  if (vec) {
    if (f32) hipLaunchKernelGGL(collate_gather_vec_kernel<true>, grid, dim3(256), 0, s, src, sel, frame_bytes, out);
    else hipLaunchKernelGGL(collate_gather_vec_kernel<false>, grid, dim3(256), 0, s, src, sel, frame_bytes, out);
  } else {
    if (f32) hipLaunchKernelGGL(collate_gather_byte_kernel<true>, grid, dim3(256), 0, s, src, sel, frame_bytes, out);
    else hipLaunchKernelGGL(collate_gather_byte_kernel<false>, grid, dim3(256), 0, s, src, sel, frame_bytes, out);
  }
  DFD_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace dfd
