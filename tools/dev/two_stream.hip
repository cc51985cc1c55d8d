// Dev: when do two 16-KB streams issued back to back by one block land? Each of G blocks of 256
// threads issues 16 KB from stream A (4 x dwordx4 per lane) then 16 KB from stream B (16 x dword
// per lane, the decode attention's V pattern), waits for A, stamps, waits for B, stamps.
// Cases: B in another allocation; B in the same allocation at +1 MiB; B = A's next 16 KB.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__global__ void two(const u4* __restrict__ a, const uint32_t* __restrict__ b, int64_t stride_u4,
                    uint64_t* st, uint32_t* out) {
  const u4* pa = a + blockIdx.x * stride_u4;
  const uint32_t* pb = b + blockIdx.x * stride_u4 * 4;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  u4 ra[4];
  uint32_t rb[16];
#pragma unroll
  for (int u = 0; u < 4; ++u) ra[u] = __builtin_nontemporal_load(pa + u * 256 + threadIdx.x);
  asm volatile("" ::: "memory");
#pragma unroll
  for (int u = 0; u < 16; ++u) rb[u] = __builtin_nontemporal_load(pb + u * 256 + threadIdx.x);
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) acc += ra[u].x ^ ra[u].y ^ ra[u].z ^ ra[u].w;
  __syncthreads();
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int u = 0; u < 16; ++u) acc += rb[u];
  __syncthreads();
  const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    st[blockIdx.x * 3 + 0] = t0;
    st[blockIdx.x * 3 + 1] = t1;
    st[blockIdx.x * 3 + 2] = t2;
  }
  if (acc == 0x9u) out[0] = acc;
}

int main() {
  const int G = 72;
  const int64_t stride = 64 * 1024 / 16;  // blocks 64 KB apart
  char *A, *B, *fl;
  uint64_t* st;
  uint32_t* out;
  hipMalloc(&A, 64ull << 20);
  hipMalloc(&B, 64ull << 20);
  hipMalloc(&fl, 1ull << 30);
  hipMalloc(&st, G * 3 * 8);
  hipMalloc(&out, 64);
  hipMemset(A, 1, 64ull << 20);
  hipMemset(B, 1, 64ull << 20);
  struct Case { const char* name; const void* a; const void* b; };
  Case cases[] = {{"B other alloc", A, B}, {"B same alloc +1MiB", A, A + (1 << 20)},
                  {"B = A + 16KB", A, A + 16384}, {"B other alloc +32MiB", A, B + (32 << 20)}};
  std::vector<uint64_t> h(G * 3);
  for (auto& c : cases) {
    std::vector<double> da, db;
    for (int rep = 0; rep < 5; ++rep) {
      hipMemset(fl, rep, 1ull << 30);
      hipLaunchKernelGGL(two, dim3(G), dim3(256), 0, 0, (const u4*)c.a, (const uint32_t*)c.b,
                         stride, st, out);
      hipDeviceSynchronize();
      hipMemcpy(h.data(), st, G * 3 * 8, hipMemcpyDeviceToHost);
      uint64_t t0 = ~0ull;
      for (int i = 0; i < G; ++i) t0 = std::min(t0, h[i * 3]);
      for (int i = 0; i < G; ++i) {
        da.push_back((h[i * 3 + 1] - t0) / 100.0);
        db.push_back((h[i * 3 + 2] - t0) / 100.0);
      }
    }
    std::sort(da.begin(), da.end());
    std::sort(db.begin(), db.end());
    printf("%-24s A landed med %.2f us  B landed med %.2f us (max %.2f / %.2f)\n", c.name,
           da[da.size() / 2], db[db.size() / 2], da.back(), db.back());
  }
  return 0;
}
