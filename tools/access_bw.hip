// Access-pattern bandwidth probe (development tool): how fast does the chip move an NHWC bf16
// activation with the per-lane access shapes of the depthwise kernels?
//   copy16   16 B per lane, contiguous 1 KiB per wave-instruction (the reference stream)
//   pix16    16 B per lane, 4 lanes = one pixel's 64-B channel slice, pixels C*2 B apart
//   pair4    4 B per lane (a bf16 channel pair), 16 lanes = one pixel's 64-B slice, the wave's 4
//            lane groups on 4 different rows (the channel-pair strips of k_dw_bwd1 / k_dw_bwd2)
// Each kernel reads one buffer and writes another of the same shape (the dw backward reads y1 and
// writes the data gradient with these shapes).  build: hipcc -O3 --offload-arch=gfx950 -o access_bw access_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ void copy16(const uint4* __restrict__ a, uint4* __restrict__ b, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) b[i] = a[i];
}

// map [F][H][W][C] bf16, 32-channel groups; one workgroup = one group x 8 rows x 56 px tile
__global__ void pix16(const char* __restrict__ a, char* __restrict__ b, int F, int H, int W, int C, int tiles) {
  const int groups = C / 32, tid = threadIdx.x;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int grp = t % groups, tt = t / groups;
    const int tx = tt % (W / 56), ty = (tt / (W / 56)) % (H / 8), f = tt / ((W / 56) * (H / 8));
    for (int p = tid >> 2; p < 8 * 56; p += 64) {
      const int y = ty * 8 + p / 56, x = tx * 56 + p % 56;
      const long o = ((((long)f * H + y) * W + x) * C + grp * 32) * 2 + (tid & 3) * 16;
      *reinterpret_cast<uint4*>(b + o) = *reinterpret_cast<const uint4*>(a + o);
    }
  }
}

__global__ void pair4(const char* __restrict__ a, char* __restrict__ b, int F, int H, int W, int C, int tiles) {
  const int groups = C / 32, tid = threadIdx.x, cp = tid & 15, slot = tid >> 4;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int grp = t % groups, tt = t / groups;
    const int tx = tt % (W / 56), ty = (tt / (W / 56)) % (H / 8), f = tt / ((W / 56) * (H / 8));
    // 32 strips of 14 px (8 rows x 4 strips), 16 slots, 2 passes
    for (int s = slot; s < 32; s += 16) {
      const int y = ty * 8 + (s & 7), x0 = tx * 56 + (s >> 3) * 14;
      uint32_t v[14];
#pragma unroll
      for (int px = 0; px < 14; ++px)
        v[px] = *reinterpret_cast<const uint32_t*>(a + ((((long)f * H + y) * W + x0 + px) * C + grp * 32 + 2 * cp) * 2);
#pragma unroll
      for (int px = 0; px < 14; ++px)
        *reinterpret_cast<uint32_t*>(b + ((((long)f * H + y) * W + x0 + px) * C + grp * 32 + 2 * cp) * 2) = v[px] + 1;
    }
  }
}


// as pix16, but one workgroup walks every channel group of its tile in turn (group-minor order)
__global__ void pix16g(const char* __restrict__ a, char* __restrict__ b, int F, int H, int W, int C, int tiles) {
  const int groups = C / 32, tid = threadIdx.x;
  for (int tt = blockIdx.x; tt < tiles / groups; tt += gridDim.x) {
    const int tx = tt % (W / 56), ty = (tt / (W / 56)) % (H / 8), f = tt / ((W / 56) * (H / 8));
    for (int grp = 0; grp < groups; ++grp)
      for (int p = tid >> 2; p < 8 * 56; p += 64) {
        const int y = ty * 8 + p / 56, x = tx * 56 + p % 56;
        const long o = ((((long)f * H + y) * W + x) * C + grp * 32) * 2 + (tid & 3) * 16;
        *reinterpret_cast<uint4*>(b + o) = *reinterpret_cast<const uint4*>(a + o);
      }
  }
}

// whole pixels: the tile's rows are contiguous runs of 56 * C * 2 bytes
__global__ void pixall(const char* __restrict__ a, char* __restrict__ b, int F, int H, int W, int C, int tiles) {
  const int groups = C / 32, tid = threadIdx.x;
  const int rowv = 56 * C * 2 / 16;  // 16-B vectors per tile row
  for (int tt = blockIdx.x; tt < tiles / groups; tt += gridDim.x) {
    const int tx = tt % (W / 56), ty = (tt / (W / 56)) % (H / 8), f = tt / ((W / 56) * (H / 8));
    for (int v = tid; v < 8 * rowv; v += 256) {
      const int y = ty * 8 + v / rowv, q = v % rowv;
      const long o = ((((long)f * H + y) * W + tx * 56) * C) * 2 + (long)q * 16;
      *reinterpret_cast<uint4*>(b + o) = *reinterpret_cast<const uint4*>(a + o);
    }
  }
}

__device__ __forceinline__ int xswz(int b, int n) {
  const int full = n & ~7;
  if (b >= full) return b;
  return (b & 7) * (full >> 3) + (b >> 3);
}
// pix16 with the XCD-aware block order of the depthwise kernels (groups of a tile on one XCD)
__global__ void pix16x(const char* __restrict__ a, char* __restrict__ b, int F, int H, int W, int C, int tiles) {
  const int groups = C / 32, tid = threadIdx.x;
  const int bid = xswz(blockIdx.x, gridDim.x);
  for (int t = bid; t < tiles; t += gridDim.x) {
    const int grp = t % groups, tt = t / groups;
    const int tx = tt % (W / 56), ty = (tt / (W / 56)) % (H / 8), f = tt / ((W / 56) * (H / 8));
    for (int p = tid >> 2; p < 8 * 56; p += 64) {
      const int y = ty * 8 + p / 56, x = tx * 56 + p % 56;
      const long o = ((((long)f * H + y) * W + x) * C + grp * 32) * 2 + (tid & 3) * 16;
      *reinterpret_cast<uint4*>(b + o) = *reinterpret_cast<const uint4*>(a + o);
    }
  }
}

int main() {
  const int F = 256, H = 112, W = 112, C = 96;
  const long bytes = (long)F * H * W * C * 2;
  char *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int tiles = F * (H / 8) * (W / 56) * (C / 32);
  for (int k = 0; k < 6; ++k) {
    for (int grid : {1024, 2048, 4096}) {
      float best = 1e9;
      for (int it = 0; it < 6; ++it) {
        CK(hipEventRecord(e0));
        if (k == 0) hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
        if (k == 1) hipLaunchKernelGGL(pix16, dim3(grid), dim3(256), 0, 0, a, b, F, H, W, C, tiles);
        if (k == 2) hipLaunchKernelGGL(pair4, dim3(grid), dim3(256), 0, 0, a, b, F, H, W, C, tiles);
        if (k == 3) hipLaunchKernelGGL(pix16g, dim3(grid), dim3(256), 0, 0, a, b, F, H, W, C, tiles);
        if (k == 5) hipLaunchKernelGGL(pix16x, dim3(grid), dim3(256), 0, 0, a, b, F, H, W, C, tiles);
        if (k == 4) hipLaunchKernelGGL(pixall, dim3(grid), dim3(256), 0, 0, a, b, F, H, W, C, tiles);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0 && ms < best) best = ms;
      }
      printf("%-7s grid %5d  %8.1f us  %6.2f TB/s (read+write)\n", k == 0 ? "copy16" : k == 1 ? "pix16" : k == 2 ? "pair4" : k == 3 ? "pix16g" : k == 4 ? "pixall" : "pix16x", grid,
             best * 1e3, 2.0 * bytes / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
