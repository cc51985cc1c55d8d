// Dev: ablations of the batched streaming GEMV (csrc/qlin_gemv_batched.hip gemv_stream_kernel,
// M = 1, narrow zeros, 8 tiles in flight, round-wide (scale, zero) words with per-round group
// constants) to find what bounds the 2/3-bit rings.  ABL bits (wrong results unless 0):
//   1  no dequant: the raw extracted pairs go to the MFMA (no zero subtraction / scale multiply)
//   2  no MFMA: the dequantized words are xor-folded into one accumulator instead
//   4  no x loads: the A operand is a register constant (no LDS park either)
//   8  no (scale, zero) loads: the round's words are constants (still parked)
//  16  no LDS reads of the group constants: constants from registers
//  32  (exact) the group constants of tile u + 1 read from LDS while tile u computes
//  64  (exact) the x fragments of tile u + 1 parked and read while tile u computes
// 128  (exact) two tile rows per wave side by side (lab2_kernel)
// Variant 0 must match the product bit for bit.
#include "../../llama3-quantization_amd/csrc/qlin_common.h"
#include "../../llama3-quantization_amd/csrc/qlin_gemv_tile.h"

#include <algorithm>
#include <type_traits>

namespace {

struct LA {
  const uint32_t* qw;
  const uint32_t* qsz;
  const _Float16* x;
  _Float16* y;
  int64_t bs_qw, bs_sz, bs_x, bs_y;
  int N, K, Kt, G, Nt;
  int64_t T, Wt;
  int xcd_chunk;
};

constexpr int kW = 4, PF = 8;

template <int BITS, int GPT, int ABL, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void lab_kernel(const LA a) {
  __shared__ __attribute__((aligned(16))) uint32_t xs[kW][64];
  constexpr int SW = PF * GPT * kTileN;
  constexpr int NC = SW >= 256 ? SW / 256 : 1;
  constexpr int NPL = BITS < 4 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) uint32_t szs[kW][NPL * SW];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  int blk = blockIdx.x;
  if (a.xcd_chunk > 0) blk = (blk & 7) * a.xcd_chunk + (blk >> 3);
  const int64_t w = (int64_t)blk * kW + wave;
  if (w >= a.Wt) return;
  const int64_t r0 = w * a.T / a.Wt;
  const int64_t nrows = (w + 1) * a.T / a.Wt - r0;
  if (nrows <= 0) return;
  const int xlane = 2 * lane;
  int64_t lr = r0;
  int lkt = 0;
  const uint32_t *lqw, *lsz;
  const _Float16* lx;
  auto set_row = [&](int64_t r) {
    const int64_t b = r / a.Nt;
    const int nt = (int)(r - b * a.Nt);
    lqw = a.qw + b * a.bs_qw + (int64_t)nt * a.Kt * (64 * BITS) + lane * BITS;
    lsz = a.qsz + b * a.bs_sz + (int64_t)nt * a.G * kTileN;
    lx = a.x + b * a.bs_x + xlane;
  };
  set_row(lr);
  Piece<BITS> pc[PF];
  uint32_t xq[PF];
  uint4 szr[NC];
  auto load_szr = [&](int kt0) {
    const uint32_t* p = lsz + kt0 * GPT * kTileN;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (ABL & 8) szr[c] = make_uint4(0x3c00u + kt0, 0x3c00u + c, 0x3c01u, 0x3c02u);
      else szr[c] = *reinterpret_cast<const uint4*>(p + 256 * c + (4 * lane) % (SW < 256 ? SW : 256));
    }
  };
  uint32_t* sslot = &szs[wave][0];
  auto park_sz = [&] {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const uint32_t ws[4] = {szr[c].x, szr[c].y, szr[c].z, szr[c].w};
      uint32_t pl[3][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const _Float16 s = sz_scale(ws[e]);
        const _Float16 z = (_Float16)(int16_t)(ws[e] >> 16);
        pl[0][e] = as_u32(h2{s, s});
        pl[1][e] = as_u32(h2{z, z} + h2{(_Float16)pair_off<BITS>(0), (_Float16)pair_off<BITS>(1)});
        pl[2][e] = as_u32(h2{z, z} + h2{(_Float16)pair_off<BITS>(2), (_Float16)pair_off<BITS>(3)});
      }
      const int o = 256 * c + (4 * lane) % (SW < 256 ? SW : 256);
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        *reinterpret_cast<uint4*>(sslot + p * SW + o) = make_uint4(pl[p][0], pl[p][1], pl[p][2], pl[p][3]);
    }
  };
  auto load = [&](int u, int kt) {
    pc[u] = load_piece_nt<BITS>(lqw + kt * (64 * BITS));
    if (!(ABL & 4)) xq[u] = *reinterpret_cast<const uint32_t*>(lx + kt * kTileK);
  };
  const Magics mg = make_magics<BITS>();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  uint32_t fold = 0;
  uint32_t* slot = &xs[wave][0];
  const uint32_t xconst = 0x3c003c00u + (uint32_t)lane;
  uint32_t rc[GPT][3], rn[GPT][3];
  auto read_rec = [&](int u, uint32_t (&r)[GPT][3]) {
#pragma unroll
    for (int g = 0; g < GPT; ++g) {
      const int si = (u * GPT + g) * kTileN + n_in;
      r[g][0] = sslot[si];
      r[g][1] = sslot[SW + si];
      r[g][2] = NPL > 2 ? sslot[2 * SW + si] : 0u;
    }
  };
  h8 xc[4], xn[4];
  auto read_x = [&](int u, h8 (&xa)[4]) {
    XRaw<1> r;
    r.w[0] = xq[u];
    park_x<1>(xa, r, slot, lane, n_in);
  };
  auto tile = [&](int u) {
    h8 xa[4];
    if (ABL & 4) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        xa[c] = __builtin_bit_cast(h8, make_uint4(xconst, xconst + c, xconst, xconst));
    } else if (ABL & 64) {
      if (u == 0) read_x(0, xc);
      if (u + 1 < PF) read_x(u + 1, xn);
#pragma unroll
      for (int c = 0; c < 4; ++c) xa[c] = xc[c];
    } else {
      read_x(u, xa);
    }
    if (ABL & 32) {
      if (u == 0) read_rec(0, rc);
      if (u + 1 < PF) read_rec(u + 1, rn);
    }
    auto step = [&](auto S_) {
#pragma clang fp contract(off)
      constexpr int S = decltype(S_)::value;
      uint32_t v[4];
      const int si = (u * GPT + S * GPT / 4) * kTileN + n_in;
      if constexpr (ABL & 1) {
        step_pairs<BITS, S>(pc[u], mg, v);
      } else {
        uint32_t s0, s1, s2;
        if (ABL & 16) {
          s0 = 0x3c003c00u; s1 = 0x64006400u + u; s2 = 0x5c005c00u + S;
        } else if (ABL & 32) {
          s0 = rc[S * GPT / 4][0]; s1 = rc[S * GPT / 4][1]; s2 = rc[S * GPT / 4][2];
        } else {
          s0 = sslot[si]; s1 = sslot[SW + si]; s2 = NPL > 2 ? sslot[2 * SW + si] : 0u;
        }
        uint32_t vv[4];
        step_pairs<BITS, S>(pc[u], mg, vv);
        const h2 ss = as_h2(s0), ha = as_h2(s1), hb = as_h2(s2);
#pragma unroll
        for (int P = 0; P < 4; ++P) {
          const h2 zs = (BITS >= 4 || P < 2) ? ha : hb;
          const _Float16 z = (BITS == 8 || (P & 1) == 0) ? zs.x : zs.y;
          v[P] = as_u32((as_h2(vv[P]) - h2{z, z}) * ss);
        }
      }
      if constexpr (ABL & 2) {
        fold ^= v[0] ^ v[1] ^ v[2] ^ v[3];
      } else {
        const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
      }
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    if (ABL & 32) {
#pragma unroll
      for (int g = 0; g < GPT; ++g)
#pragma unroll
        for (int j = 0; j < 3; ++j) rc[g][j] = rn[g][j];
    }
    if (ABL & 64) {
#pragma unroll
      for (int c = 0; c < 4; ++c) xc[c] = xn[c];
    }
  };
  auto store = [&](int64_t r) {
    const int64_t b = r / a.Nt;
    const int64_t row = (r - b * a.Nt) * kTileN + n_in;
    if (ABL & 2) acc[0] += (float)(fold & 0xFFu);
    if (lane < 16 && row < a.N) a.y[b * a.bs_y + row] = (_Float16)acc[0];
    acc = f4{0.f, 0.f, 0.f, 0.f};
  };
  load_szr(0);
#pragma unroll
  for (int u = 0; u < PF; ++u) load(u, u);
  int64_t cr = r0;
  int ckt = 0;
  const int64_t rounds = nrows * (a.Kt / PF);
  for (int64_t q = 0; q + 1 < rounds; ++q) {
    park_sz();
    lkt += PF;
    if (lkt == a.Kt) {
      lkt = 0;
      ++lr;
      set_row(lr);
    }
    load_szr(lkt);
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      tile(u);
      load(u, lkt + u);
    }
    ckt += PF;
    if (ckt == a.Kt) {
      store(cr);
      ckt = 0;
      ++cr;
    }
  }
  park_sz();
#pragma unroll
  for (int u = 0; u < PF; ++u) tile(u);
  store(cr);
}

template <int BITS, int GPT, int ABL, int WPE>
int launch(LA a, hipStream_t st) {
  auto k = lab_kernel<BITS, GPT, ABL, WPE>;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0) != hipSuccess || nb < 1) nb = 1;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  a.Wt = std::min<int64_t>(a.T, (int64_t)cus * nb * kW);
  const int64_t blocks = (a.Wt + kW - 1) / kW;
  a.xcd_chunk = blocks % 8 == 0 ? (int)(blocks / 8) : 0;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError() ? -2 : nb;
}


// two tile rows side by side (rows 2p, 2p + 1 of one problem): each x fragment is parked and read
// once per k-tile for both rows; 4 k-tiles x 2 rows in flight per wave
template <int BITS, int GPT, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void lab2_kernel(const LA a) {
  constexpr int PF2 = 4;
  __shared__ __attribute__((aligned(16))) uint32_t xs[kW][64];
  constexpr int SW2 = PF2 * GPT * kTileN;          // words per row and round
  constexpr int SWT = 2 * SW2;                      // both rows
  constexpr int NC = SWT >= 256 ? SWT / 256 : 1;
  constexpr int NPL = BITS < 4 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) uint32_t szs[kW][NPL * SWT];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  int blk = blockIdx.x;
  if (a.xcd_chunk > 0) blk = (blk & 7) * a.xcd_chunk + (blk >> 3);
  const int64_t w = (int64_t)blk * kW + wave;
  if (w >= a.Wt) return;
  const int64_t T2 = a.T / 2;
  const int64_t p0 = w * T2 / a.Wt;
  const int64_t npairs = (w + 1) * T2 / a.Wt - p0;
  if (npairs <= 0) return;
  int64_t lp = p0;
  int lkt = 0;
  const uint32_t *lqw, *lsz;
  const _Float16* lx;
  const int64_t rw = (int64_t)a.Kt * (64 * BITS), rs = (int64_t)a.G * kTileN;
  auto set_pair = [&](int64_t pp) {
    const int64_t r = 2 * pp;
    const int64_t b = r / a.Nt;
    const int nt = (int)(r - b * a.Nt);
    lqw = a.qw + b * a.bs_qw + (int64_t)nt * rw + lane * BITS;
    lsz = a.qsz + b * a.bs_sz + (int64_t)nt * rs;
    lx = a.x + b * a.bs_x + 2 * lane;
  };
  set_pair(lp);
  Piece<BITS> pc[2][PF2];
  uint32_t xq[PF2];
  uint4 szr[NC];
  auto load_szr = [&](int kt0) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int o = 256 * c + (4 * lane) % (SWT < 256 ? SWT : 256);
      const int row = o / SW2, within = o - row * SW2;
      szr[c] = *reinterpret_cast<const uint4*>(lsz + row * rs + kt0 * GPT * kTileN + within);
    }
  };
  uint32_t* sslot = &szs[wave][0];
  auto park_sz = [&] {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const uint32_t ws[4] = {szr[c].x, szr[c].y, szr[c].z, szr[c].w};
      uint32_t pl[3][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const _Float16 s = sz_scale(ws[e]);
        const _Float16 z = (_Float16)(int16_t)(ws[e] >> 16);
        pl[0][e] = as_u32(h2{s, s});
        pl[1][e] = as_u32(h2{z, z} + h2{(_Float16)pair_off<BITS>(0), (_Float16)pair_off<BITS>(1)});
        pl[2][e] = as_u32(h2{z, z} + h2{(_Float16)pair_off<BITS>(2), (_Float16)pair_off<BITS>(3)});
      }
      const int o = 256 * c + (4 * lane) % (SWT < 256 ? SWT : 256);
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        *reinterpret_cast<uint4*>(sslot + p * SWT + o) = make_uint4(pl[p][0], pl[p][1], pl[p][2], pl[p][3]);
    }
  };
  auto load = [&](int u, int kt) {
    pc[0][u] = load_piece_nt<BITS>(lqw + kt * (64 * BITS));
    pc[1][u] = load_piece_nt<BITS>(lqw + rw + kt * (64 * BITS));
    xq[u] = *reinterpret_cast<const uint32_t*>(lx + kt * kTileK);
  };
  const Magics mg = make_magics<BITS>();
  f4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  uint32_t* slot = &xs[wave][0];
  auto tile = [&](int u) {
    h8 xa[4];
    XRaw<1> xr;
    xr.w[0] = xq[u];
    park_x<1>(xa, xr, slot, lane, n_in);
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      auto step = [&](auto S_) {
#pragma clang fp contract(off)
        constexpr int S = decltype(S_)::value;
        const int si = rr * SW2 + (u * GPT + S * GPT / 4) * kTileN + n_in;
        uint32_t vv[4], v[4];
        step_pairs<BITS, S>(pc[rr][u], mg, vv);
        const h2 ss = as_h2(sslot[si]), ha = as_h2(sslot[SWT + si]),
                 hb = as_h2(NPL > 2 ? sslot[2 * SWT + si] : 0u);
#pragma unroll
        for (int P = 0; P < 4; ++P) {
          const h2 zs = (BITS >= 4 || P < 2) ? ha : hb;
          const _Float16 z = (BITS == 8 || (P & 1) == 0) ? zs.x : zs.y;
          v[P] = as_u32((as_h2(vv[P]) - h2{z, z}) * ss);
        }
        const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        acc[rr] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc[rr], 0, 0, 0);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
    }
  };
  auto store = [&](int64_t pp) {
    const int64_t r = 2 * pp;
    const int64_t b = r / a.Nt;
    const int64_t row = (r - b * a.Nt) * kTileN + n_in;
    if (lane < 16) {
      a.y[b * a.bs_y + row] = (_Float16)acc[0][0];
      a.y[b * a.bs_y + row + kTileN] = (_Float16)acc[1][0];
    }
    acc[0] = f4{0.f, 0.f, 0.f, 0.f};
    acc[1] = f4{0.f, 0.f, 0.f, 0.f};
  };
  load_szr(0);
#pragma unroll
  for (int u = 0; u < PF2; ++u) load(u, u);
  int64_t cp = p0;
  int ckt = 0;
  const int64_t rounds = npairs * (a.Kt / PF2);
  for (int64_t q = 0; q + 1 < rounds; ++q) {
    park_sz();
    lkt += PF2;
    if (lkt == a.Kt) {
      lkt = 0;
      ++lp;
      set_pair(lp);
    }
    load_szr(lkt);
#pragma unroll
    for (int u = 0; u < PF2; ++u) {
      tile(u);
      load(u, lkt + u);
    }
    ckt += PF2;
    if (ckt == a.Kt) {
      store(cp);
      ckt = 0;
      ++cp;
    }
  }
  park_sz();
#pragma unroll
  for (int u = 0; u < PF2; ++u) tile(u);
  store(cp);
}

template <int BITS, int GPT, int WPE>
int launch2(LA a, hipStream_t st) {
  auto k = lab2_kernel<BITS, GPT, WPE>;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0) != hipSuccess || nb < 1) nb = 1;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  a.Wt = std::min<int64_t>(a.T / 2, (int64_t)cus * nb * kW);
  const int64_t blocks = (a.Wt + kW - 1) / kW;
  a.xcd_chunk = blocks % 8 == 0 ? (int)(blocks / 8) : 0;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError() ? -2 : nb;
}

template <int BITS, int GPT, int WPE>
int by_abl(int abl, const LA& a, hipStream_t st) {
  switch (abl) {
    case 0: return launch<BITS, GPT, 0, WPE>(a, st);
    case 1: return launch<BITS, GPT, 1, WPE>(a, st);
    case 2: return launch<BITS, GPT, 2, WPE>(a, st);
    case 3: return launch<BITS, GPT, 3, WPE>(a, st);
    case 4: return launch<BITS, GPT, 4, WPE>(a, st);
    case 8: return launch<BITS, GPT, 8, WPE>(a, st);
    case 12: return launch<BITS, GPT, 12, WPE>(a, st);
    case 16: return launch<BITS, GPT, 16, WPE>(a, st);
    case 7: return launch<BITS, GPT, 7, WPE>(a, st);
    case 32: return launch<BITS, GPT, 32, WPE>(a, st);
    case 64: return launch<BITS, GPT, 64, WPE>(a, st);
    case 96: return launch<BITS, GPT, 96, WPE>(a, st);
    case 128: return launch2<BITS, GPT, WPE>(a, st);
    case 15: return launch<BITS, GPT, 15, WPE>(a, st);
    default: return -1;
  }
}

}  // namespace

// returns resident blocks per CU (> 0) or < 0 on error; wpe 0 = compiler's choice (1)
extern "C" int lab_stream(int abl, int wpe, const uint32_t* qw, const uint32_t* qsz,
                          const uint16_t* x, uint16_t* y, int64_t batch, int64_t N, int64_t K,
                          int bits, int group, void* stream) {
  LA a;
  a.qw = qw; a.qsz = qsz; a.x = (const _Float16*)x; a.y = (_Float16*)y;
  const int64_t Nt = N / kTileN, Kt = K / kTileK;
  a.bs_qw = Nt * Kt * 64 * bits; a.bs_sz = Nt * (K / group) * kTileN; a.bs_x = K; a.bs_y = N;
  a.N = (int)N; a.K = (int)K; a.Kt = (int)Kt; a.G = (int)(K / group); a.Nt = (int)Nt;
  a.T = Nt * batch;
  hipStream_t st = (hipStream_t)stream;
  if (N % kTileN || K % (PF * kTileK)) return -3;
#define LB(B, G)                                                             \
  if (bits == B && group == 128 / G) {                                       \
    if (wpe == 0) return by_abl<B, G, 1>(abl, a, st);                        \
    if (wpe == 4) return by_abl<B, G, 4>(abl, a, st);                        \
    if (wpe == 5) return by_abl<B, G, 5>(abl, a, st);                        \
    if (wpe == 6) return by_abl<B, G, 6>(abl, a, st);                        \
    return -4;                                                               \
  }
  LB(2, 2)
  LB(3, 2)
  LB(4, 1)
#undef LB
  return -5;
}
