// FETCH_SIZE / WRITE_SIZE calibration on known byte counts (MI355X_MICROARCH.md, HBM section:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Each kernel touches exactly BYTES bytes of a buffer larger than the 256 MiB
// Infinity Cache, with one access pattern per kernel:
//   wr16      16-byte stores, lane-contiguous (streaming)
//   wr16_row  the halo epilogue's pattern: 8-channel groups of pixel rows of C = 206 bf16
//             channels at a 208-channel pixel stride (25 x 16-byte + 6 x 2-byte stores a row)
//   wr2       2-byte stores, lane-contiguous
//   rd16      16-byte loads, lane-contiguous
//   rd16_lds  16-byte loads staged through LDS (the halo kernels' ring)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
// Run:   rocprofv3 --kernel-trace --pmc WRITE_SIZE -d DIR -o run -- tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void wr16(u32x4* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

__global__ void wr2(unsigned short* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (unsigned short)i;
}

// rows of 206 bf16 at a stride of 208: 26 groups of 8 channels, the last one 6 wide
__global__ void wr16_row(unsigned short* __restrict__ p, int64_t rows) {
  const int64_t groups = rows * 26;
  for (int64_t it = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; it < groups; it += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = it / 26;
    const int c0 = (int)(it - row * 26) * 8;
    unsigned short* dst = p + row * 208 + c0;
    if (c0 + 8 <= 206) {
      *reinterpret_cast<u32x4*>(dst) = u32x4{(unsigned)it, 1u, 2u, 3u};
    } else {
      for (int e = 0; e < 206 - c0; ++e) dst[e] = (unsigned short)e;
    }
  }
}

__global__ void rd16(const u32x4* __restrict__ p, int64_t n, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads live; practically never stores
}

__global__ void rd16_lds(const u32x4* __restrict__ p, int64_t n, unsigned* out) {
  __shared__ u32x4 s[256];
  unsigned acc = 0;
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = b + threadIdx.x;
    s[threadIdx.x] = i < n ? p[i] : u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    const u32x4 v = s[(threadIdx.x + 1) & 255];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
    __syncthreads();
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

int main() {
  const int64_t BYTES = 512ll << 20;  // 2x the Infinity Cache
  void* buf;
  unsigned* out;
  CHECK(hipMalloc(&buf, BYTES + 4096));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(buf, 0, BYTES));
  const int grid = 256 * 16, block = 256;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(wr16, dim3(grid), dim3(block), 0, 0, (u32x4*)buf, BYTES / 16);
    hipLaunchKernelGGL(wr2, dim3(grid), dim3(block), 0, 0, (unsigned short*)buf, BYTES / 2);
    hipLaunchKernelGGL(wr16_row, dim3(grid), dim3(block), 0, 0, (unsigned short*)buf, BYTES / 416);
    hipLaunchKernelGGL(rd16, dim3(grid), dim3(block), 0, 0, (const u32x4*)buf, BYTES / 16, out);
    hipLaunchKernelGGL(rd16_lds, dim3(grid), dim3(block), 0, 0, (const u32x4*)buf, BYTES / 16, out);
  }
  CHECK(hipDeviceSynchronize());
  printf("bytes per kernel: wr16 %lld wr2 %lld wr16_row %lld (of %lld touched) rd16 %lld rd16_lds %lld\n",
         (long long)BYTES, (long long)BYTES, (long long)(BYTES / 416 * 412), (long long)(BYTES / 416 * 416),
         (long long)BYTES, (long long)BYTES);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
