// Dev: what caps the batched sub-byte stream?  Persistent waves each stream their own contiguous
// region (like gemv_stream_kernel's tile rows) with PF loads of W bytes per lane in flight (rolling,
// nt), and C VALU ops per load standing in for the dequant; grid = CUs x waves per CU.  Prints GB/s
// of one launch over a 480 MB buffer (best of 5, after a 1 GiB flush each).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

template <int W> struct Ld;
template <> struct Ld<8> {
  typedef u2 T;
  static __device__ uint32_t fold(T v) { return v.x ^ v.y; }
};
template <> struct Ld<16> {
  typedef u4 T;
  static __device__ uint32_t fold(T v) { return v.x ^ v.y ^ v.z ^ v.w; }
};

template <int W, int PF, int C>
__global__ __launch_bounds__(256) void rd(const char* __restrict__ src, int64_t per_wave,
                                          int64_t waves, uint32_t* out) {
  typedef typename Ld<W>::T T;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= waves) return;
  const int lane = threadIdx.x & 63;
  const T* p = reinterpret_cast<const T*>(src + w * per_wave) + lane;
  const int64_t n = per_wave / (64 * W);  // loads per wave
  T r[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) r[u] = __builtin_nontemporal_load(p + u * 64);
  float a0 = 0.f, a1 = 1.f, a2 = 2.f, a3 = 3.f;
  uint32_t acc = 0;
  for (int64_t i = PF; i < n + PF; i += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const uint32_t v = Ld<W>::fold(r[u]);
      acc ^= v;
      float f = __uint_as_float((v & 0x007fffffu) | 0x3f800000u);
#pragma unroll
      for (int c = 0; c < C / 4; ++c) {
        a0 = __builtin_fmaf(a0, f, 1.f);
        a1 = __builtin_fmaf(a1, f, 1.f);
        a2 = __builtin_fmaf(a2, f, 1.f);
        a3 = __builtin_fmaf(a3, f, 1.f);
      }
      if (i + u < n) r[u] = __builtin_nontemporal_load(p + (i + u) * 64);
    }
  }
  if (acc == 0x12345678u || a0 + a1 + a2 + a3 == 1234.5f) out[0] = acc;
}

template <int W, int PF, int C>
void run(const char* src, int64_t total, char* fl, uint32_t* out, int cus, int wpcu) {
  const int64_t waves = (int64_t)cus * wpcu;
  int64_t per = total / waves;
  per -= per % (64 * W * PF);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 5; ++rep) {
    hipMemsetAsync(fl, rep, 1ull << 30);
    hipEventRecord(e0);
    hipLaunchKernelGGL((rd<W, PF, C>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, src,
                       per, waves, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  printf("W=%2d PF=%2d C=%3d waves/CU=%2d per-wave=%6lld KB: %7.1f us  %6.0f GB/s\n", W, PF, C,
         wpcu, (long long)(per >> 10), best * 1e3, (double)per * waves / (best * 1e-3) / 1e9);
  fflush(stdout);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  const int64_t total = 480ll << 20;
  char *src, *fl;
  uint32_t* out;
  hipMalloc(&src, total);
  hipMalloc(&fl, 1ull << 30);
  hipMalloc(&out, 64);
  hipMemset(src, 1, total);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int wpcus[] = {8, 16, 20, 32};
  for (int wp : wpcus) {
    run<16, 8, 0>(src, total, fl, out, cus, wp);
    run<8, 8, 0>(src, total, fl, out, cus, wp);
    run<8, 16, 0>(src, total, fl, out, cus, wp);
    run<16, 4, 0>(src, total, fl, out, cus, wp);
  }
  for (int wp : wpcus) {
    run<16, 8, 64>(src, total, fl, out, cus, wp);
    run<8, 8, 64>(src, total, fl, out, cus, wp);
    run<8, 8, 32>(src, total, fl, out, cus, wp);
    run<8, 16, 32>(src, total, fl, out, cus, wp);
  }
  return 0;
}
