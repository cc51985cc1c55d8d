// Development-only: the product GEMV kernel (int4, M = 1, g128, narrow zeros) launched with an
// explicit waves-per-block / prefetch-depth geometry, for tools/dev/gemv_geo.py.
#include "../../llama3-quantization_amd/csrc/qlin_gemv.hip"

extern "C" int geo_gemv(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                        int N, int K, int W, int PF, void* stream) {
  const int Nt = (N + kTileN - 1) / kTileN;
  const int Kt = (K + kTileK - 1) / kTileK;
  const int tpw = (Kt + W - 1) / W;
  const int Wn = (Kt + tpw - 1) / tpw;
  const uint32_t gs = group_magic(128);
#define G(P)                                                                                   \
  hipLaunchKernelGGL((gemv_kernel<4, 1, 1, kZNarrow, P>), dim3(Nt), dim3(64 * Wn), 0,          \
                     (hipStream_t)stream, qw, qsz, (const _Float16*)x, (const _Float16*)nullptr, \
                     (_Float16*)y, 1, N, K, 128, gs, tpw, (const _Float16*)nullptr, 0)
  if (PF == 2) G(2);
  else if (PF == 4) G(4);
  else G(8);
#undef G
  return (int)hipGetLastError();
}
