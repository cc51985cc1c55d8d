// Dev: does kernarg preloading shorten a short dependent launch?  A 4096^2-int4-sized streaming
// read (8.4 MB: 256 blocks x 8 waves, each wave 4 KB of 16-B nt loads, reduced to one word)
// whose operands arrive (a) in a by-value struct (s_load from the kernarg segment), (b) as
// scalar arguments preloaded into SGPRs (built with -mllvm -amdgpu-kernarg-preload-count=16).
// tools/dev/kp_lab.py times 64 dependent launches over a ring of distinct buffers in one graph.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct SArgs {
  const u32x4* src;
  uint32_t* out;
  int64_t per_block;  // u32x4 per block
  int n;
};

__device__ __forceinline__ void body(const u32x4* __restrict__ src, uint32_t* out,
                                     int64_t per_block, int n) {
  const u32x4* b = src + blockIdx.x * per_block;
  uint32_t acc = 0;
  u32x4 r[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) r[u] = __builtin_nontemporal_load(b + u * blockDim.x + threadIdx.x);
#pragma unroll
  for (int u = 0; u < 4; ++u) acc ^= r[u].x + r[u].y + r[u].z + r[u].w;
  if (acc == 0x12345678u + (uint32_t)n) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(512) void k_struct(const SArgs a) {
  body(a.src, a.out, a.per_block, a.n);
}
__global__ __launch_bounds__(512) void k_scalar(const u32x4* src, uint32_t* out,
                                                int64_t per_block, int n) {
  body(src, out, per_block, n);
}

extern "C" int kp_launch(int variant, const void* src, void* out, int64_t bytes, void* stream) {
  const int blocks = 256, threads = 512;
  const int64_t per = bytes / 16 / blocks;  // 4 x 512 u32x4 per block for 8 MB
  hipStream_t st = (hipStream_t)stream;
  if (variant == 0) {
    SArgs a{(const u32x4*)src, (uint32_t*)out, per, 0};
    hipLaunchKernelGGL(k_struct, dim3(blocks), dim3(threads), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_scalar, dim3(blocks), dim3(threads), 0, st, (const u32x4*)src,
                       (uint32_t*)out, per, 0);
  }
  return (int)hipGetLastError();
}
