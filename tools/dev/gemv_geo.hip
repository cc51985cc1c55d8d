// Development-only: the product GEMV kernel (int4, g128, narrow zeros) launched with an explicit
// waves-per-block / prefetch-depth / row-tiles-per-block geometry, for tools/dev/gemv_geo.py.
#include "../../llama3-quantization_amd/csrc/qlin_gemv.hip"

extern "C" int geo_gemv(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                        int M, int N, int K, int W, int PF, int NTB, void* stream) {
  const int Nt = (N + kTileN - 1) / kTileN;
  const int Kt = (K + kTileK - 1) / kTileK;
  const int tpw = (Kt + W - 1) / W;
  const int Wn = (Kt + tpw - 1) / tpw;
  const uint32_t gs = group_magic(128);
  const dim3 grid((Nt + NTB - 1) / NTB);
#define G(MT, P, T)                                                                             \
  hipLaunchKernelGGL((gemv_kernel<4, MT, 1, kZNarrow, P, T>), grid, dim3(64 * Wn), 0,          \
                     (hipStream_t)stream, qw, qsz, (const _Float16*)x, (const _Float16*)nullptr, \
                     (_Float16*)y, M, N, K, 128, gs, tpw, (const _Float16*)nullptr, 0, ActQ{})
#define GT(MT, P) \
  { if (NTB == 1) G(MT, P, 1); else G(MT, P, 2); }
  if (M == 1) { if (PF == 2) GT(1, 2) else if (PF == 4) GT(1, 4) else GT(1, 8) }
  else if (M <= 8) { if (PF == 2) GT(8, 2) else GT(8, 4) }
  else { if (PF == 2) GT(16, 2) else GT(16, 4) }
#undef GT
#undef G
  return (int)hipGetLastError();
}

// the decode fast path (gemv_fast_kernel) with an explicit geometry: W waves (power of two),
// PF tiles in flight (every wave's tiles: ceil(Kt / W) <= PF); LOOP must be 0
extern "C" int geo_fast(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                        int N, int K, int W, int PF, int LOOP, void* stream) {
  const int Nt = (N + kTileN - 1) / kTileN;
  FastArgs a;
  a.qw = qw; a.qsz = qsz; a.x = (const _Float16*)x; a.bias = nullptr; a.res = nullptr;
  a.y = (_Float16*)y; a.M = 1; a.N = N; a.K = K; a.Kt = K / kTileK; a.G = K / 128;
  int lw = 0;
  while ((2 << lw) <= W) ++lw;
  a.W = 1 << lw; a.lw = lw; a.cmagic = 1u << 31;
  if ((a.Kt + a.W - 1) / a.W > PF && !LOOP) return 1;
#define F(P) hipLaunchKernelGGL((gemv_fast_kernel<4, 1, 1, kZNarrow, kEpNone, P>), dim3(Nt), \
                                dim3(64 * a.W), 0, (hipStream_t)stream, a)
  if (LOOP) return 1;  // the product fast path has no refill loop (round 2)
  if (PF == 2) F(2);
  else F(4);
#undef F
  return (int)hipGetLastError();
}
