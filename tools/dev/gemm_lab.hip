// Development-only GEMM ablations: the product GEMM kernel with its ABL template bit set.
#include "../../llama3-quantization_amd/csrc/qlin_gemm.hip"

extern "C" int lab_gemm(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                        int64_t M, int N, int K, int abl, void* stream) {
  // abl bit 2: the wide (128 x 512) tile
  const bool wn = abl & 4;
  const int tiles_n = (N + (wn ? 512 : 256) - 1) / (wn ? 512 : 256);
  const int tiles_m = (int)((M + BM - 1) / BM);
  const dim3 grid(tiles_m * tiles_n);
#define L(W, A)                                                                                 \
  hipLaunchKernelGGL((gemm_kernel<4, W, 1, false, true, A>), grid, dim3(kThreads), 0,                 \
                     (hipStream_t)stream, qw, qsz, (const _Float16*)x, nullptr, (_Float16*)y, M, \
                     N, K, 128, group_magic(128), tiles_m, tiles_n)
  const int a = abl & 3;
  if (wn) { if (a == 0) L(true, 0); else if (a == 1) L(true, 1); else if (a == 2) L(true, 2); else L(true, 3); }
  else { if (a == 0) L(false, 0); else if (a == 1) L(false, 1); else if (a == 2) L(false, 2); else L(false, 3); }
#undef L
  return (int)hipGetLastError();
}

// the lab library does not link the GEMV: qlin_linear_f16's skinny branch is never taken here
extern "C" int qlin_gemv_f16(const uint32_t*, const uint32_t*, int, const uint16_t*,
                             const uint16_t*, uint16_t*, int64_t, int64_t, int64_t, int, int,
                             void*) {
  return QLIN_EINVAL;
}
