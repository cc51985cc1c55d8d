// Dev lab (round 6): does a decode GEMV run faster when the previous launch has just read its
// packed weights on the SAME XCD (L2-warm), not merely somewhere on the chip (MALL-warm)?
// Every M = 1 route (fast, rows, work queue) computes tile row r on block r % nb, i.e. on XCD
// r % 8 (round-robin dispatch of a grid no larger than the resident capacity).  touch_rows: block
// b (XCD b % 8) reads whole tile rows r with r % 8 == (b + shift) % 8 — shift 0 puts each row in
// the L2 of the XCD that will compute it, shift 1 in another XCD's.  Loaded values are folded
// into a register stored only when `flag` (always 0) is set, so the loads stay.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void touch_rows(const uint4* __restrict__ qw, int64_t qrow16,
                                                 const uint4* __restrict__ sz, int64_t srow16,
                                                 int Nt, int shift, int flag, uint4* sink) {
  const int b = blockIdx.x, nb = gridDim.x;
  const int x = (b + shift) & 7;          // the XCD whose rows this block reads
  const int per = nb / 8;                 // blocks per XCD
  uint4 acc = make_uint4(0u, 0u, 0u, 0u);
  for (int r = x + 8 * (b >> 3); r < Nt; r += 8 * per) {
    const uint4* p = qw + (int64_t)r * qrow16;
    for (int64_t i = threadIdx.x; i < qrow16; i += 256 * 4) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t j = i + 256 * u;
        v[u] = j < qrow16 ? p[j] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x ^= v[u].x; acc.y ^= v[u].y; acc.z ^= v[u].z; acc.w ^= v[u].w;
      }
    }
    const uint4* s = sz + (int64_t)r * srow16;
    for (int64_t i = threadIdx.x; i < srow16; i += 256) {
      const uint4 v = s[i];
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
  }
  if (flag) sink[b * 256 + threadIdx.x] = acc;
}

extern "C" int lab_touch_rows(const void* qw, int64_t qrow16, const void* sz, int64_t srow16,
                              int Nt, int nblocks, int shift, void* sink, void* stream) {
  hipLaunchKernelGGL(touch_rows, dim3(nblocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)qw, qrow16, (const uint4*)sz, srow16, Nt, shift, 0,
                     (uint4*)sink);
  return (int)hipGetLastError();
}
