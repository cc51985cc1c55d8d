// Development-only GEMM ablations: the product GEMM kernel with its ABL template bit set.
#include "../../llama3-quantization_amd/csrc/qlin_gemm.hip"

// 64-row blocks at width bn (256 / 384 / 512), 8 waves: two blocks per CU for one-round grids
extern "C" int lab_gemm_half(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                             int64_t M, int N, int K, int bn, void* stream) {
  const int tn = (N + bn - 1) / bn, tm = (int)((M + 63) / 64);
#define L(B) hipLaunchKernelGGL((gemm_kernel<4, B, 1, kZNarrow, true, 0, 8, true>), dim3(tm * tn), dim3(512), \
                                0, (hipStream_t)stream, qw, qsz, (const _Float16*)x, nullptr,           \
                                (_Float16*)y, M, N, K, 128, group_magic(128), tm, tn, nullptr, 0)
  if (bn == 512) L(512);
  else if (bn == 384) L(384);
  else L(256);
#undef L
  return (int)hipGetLastError();
}

extern "C" int lab_gemm(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                        int64_t M, int N, int K, int abl, void* stream) {
  // abl bit 2: the wide (128 x 512) tile; bit 3: 8 waves per block (else 4)
  const bool wn = abl & 4;
  const bool w8 = abl & 8;
  if (abl & 32) {  // bit 5: the 64 x 128 tile, 8 waves, no ablation
    const int tn = (N + 127) / 128, tm = (int)((M + 63) / 64);
    hipLaunchKernelGGL((gemm_kernel<4, 128, 1, kZNarrow, true, 0, 8>), dim3(tm * tn), dim3(512), 0,
                       (hipStream_t)stream, qw, qsz, (const _Float16*)x, nullptr, (_Float16*)y, M,
                       N, K, 128, group_magic(128), tm, tn, nullptr, 0);
    return (int)hipGetLastError();
  }
  if (abl & 16) {  // bit 4: the 128 x 384 tile, 8 waves, no ablation
    const int tn = (N + 383) / 384, tm = (int)((M + 127) / 128);
    hipLaunchKernelGGL((gemm_kernel<4, 384, 1, kZNarrow, true, 0, 8>), dim3(tm * tn), dim3(512), 0,
                       (hipStream_t)stream, qw, qsz, (const _Float16*)x, nullptr, (_Float16*)y, M,
                       N, K, 128, group_magic(128), tm, tn, nullptr, 0);
    return (int)hipGetLastError();
  }
  const int tiles_n = (N + (wn ? 512 : 256) - 1) / (wn ? 512 : 256);
  const int tiles_m = (int)((M + 127) / 128);
  const dim3 grid(tiles_m * tiles_n);
#define L(W, A, NW)                                                                             \
  hipLaunchKernelGGL((gemm_kernel<4, W, 1, kZNarrow, true, A, NW>), grid, dim3(64 * NW), 0,     \
                     (hipStream_t)stream, qw, qsz, (const _Float16*)x, nullptr, (_Float16*)y, M, \
                     N, K, 128, group_magic(128), tiles_m, tiles_n, nullptr, 0)
#define LA(W, NW) \
  { if (a == 0) L(W, 0, NW); else if (a == 1) L(W, 1, NW); else if (a == 2) L(W, 2, NW); else L(W, 3, NW); }
  const int a = abl & 3;
  if (w8) { if (wn) LA(512, 8) else LA(256, 8) }
  else { if (wn) LA(512, 4) else LA(256, 4) }
#undef LA
#undef L
  return (int)hipGetLastError();
}

// the product's 8-wave 128 x BN block with the dequant VALU skipped (ABL bit 2) or not
extern "C" int lab_gemm_nodq(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                             int64_t M, int N, int K, int bn, int nodq, void* stream) {
  const int tn = (N + bn - 1) / bn, tm = (int)((M + 127) / 128);
#define L(B, A) hipLaunchKernelGGL((gemm_kernel<4, B, 1, kZNarrow, true, A, 8>), dim3(tm * tn), dim3(512), \
                                   0, (hipStream_t)stream, qw, qsz, (const _Float16*)x, nullptr,         \
                                   (_Float16*)y, M, N, K, 128, group_magic(128), tm, tn, nullptr, 0)
  if (bn == 512) { if (nodq) L(512, 4); else L(512, 0); }
  else { if (nodq) L(256, 4); else L(256, 0); }
#undef L
  return (int)hipGetLastError();
}

// the lab library does not link the GEMV or the quantizer: the skinny / act-quant branches of
// qlin_linear_*_f16 are never taken here
int qlin::gemv_ep(const uint32_t*, const uint32_t*, int, const uint16_t*, const uint16_t*,
                  const uint16_t*, uint16_t*, int64_t, int64_t, int64_t, int, int, int, int, int,
                  void*) {
  return QLIN_EINVAL;
}
extern "C" int qlin_gemv_f16(const uint32_t*, const uint32_t*, int, const uint16_t*,
                             const uint16_t*, uint16_t*, int64_t, int64_t, int64_t, int, int,
                             void*) {
  return QLIN_EINVAL;
}
extern "C" int qlin_quantize(const void*, int, int64_t, int64_t, int, int, int, const void*,
                             const void*, void*, void*, void*, uint32_t*, uint32_t*, void*) {
  return QLIN_EINVAL;
}
