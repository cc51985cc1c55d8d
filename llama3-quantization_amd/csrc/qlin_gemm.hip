// qlin_gemm.hip — fused dequant + MFMA GEMM for batched tokens (M > 64 via qlin_linear_f16),
// gfx950.
//
// y[M, N] = x[M, K] @ W_dq[N, K]^T (+ bias): replaces F.linear at quant/int_linear.py:62 for the
// prefill / PPL-window shapes (M = 2048 per window, main.py:127-136; M = 65,536 for batch 32).
//
// Structure (512-thread block = 8 waves side by side in N, block tile 128 x 256 / 384 / 512, or
// 64 x 128 for grids that would leave most CUs idle (pick_bn; int8: 128 x 256), wave tile
// 128 x 32 / 48 / 64 (64 x 16), BK = 128 = one packed k-tile, two LDS stages; wide-in-N waves
// because B is read packed, 4x cheaper per LDS byte than A):
//   - every operand reaches LDS by LDS-DMA (global_load_lds, 16 B per lane): the x tile (BM rows x
//     256 B, XOR-swizzled per 16-B chunk by (row & 15) through the per-lane SOURCE address, so the
//     LDS image stays lane-linear per instruction), the packed codes of the 8 row tiles (already
//     lane-linear in the qlin tiled layout) and their (scale, zero) words;
//   - B stays PACKED in LDS (bits/16 of the fp16 bytes): each wave reads the lane pieces of its 8
//     row tiles once per k-tile and dequantizes them bit-exactly in registers (qlin_common.h) into
//     the B operand of v_mfma_f32_16x16x32_f16 — the piece layout IS that operand, so no shuffle
//     and no fp16 B image exist;
//   - A fragments: ds_read_b128 of row (lane & 15), chunk (4s + q) ^ (row & 15): conflict-free,
//     the next k-step's fragments read while this step's MFMAs run;
//   - the next k-tile's DMA is issued right after the barrier and runs under this tile's MFMAs;
//   - blocks are remapped so each XCD owns a contiguous band of M tiles (x re-use in its L2).
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

#include <atomic>
#include <type_traits>

using namespace qlin;

namespace {

// 8 waves per block, side by side in N (2 per SIMD: one wave's dequant VALU and LDS reads run
// under the other's MFMAs).  Measured against 4 waves (tools/dev/gemm_lab.py, int4 g128
// N = K = 4096): M = 2048 narrow 923 -> 1010, M = 16384 wide 1021 -> 1135, M = 65536 wide
// 1049 -> 1112 TFLOP/s.
constexpr int kWaves = 8;
constexpr int BK = kTileK;  // one packed k-tile per stage
constexpr int64_t kSkinnyMaxM = 64;   // qlin_linear_f16: M <= this runs the GEMV kernel
constexpr int64_t kActFuseMaxN = 16384;  // act fake-quant fused into the GEMV up to this N

typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(1))) void* gbl_ptr;

// Wave tiles are 128 rows x BN / 8 columns: each B fragment dequantized per k-step feeds 8 MFMAs
// (one per 16-row block), so its 13 VALU fit the issue slots the MFMAs leave free, and the waves
// sit side by side in N, so every B element is dequantized once per block.
// BN_: block 128 x 256, 128 x 384 or 128 x 512 columns (int8: 256 only, twice the code bytes),
// chosen per launch by pick_bn (whole rounds of blocks over the CUs).
// BN_ = 128: the 64 x 128 block for grids that leave most CUs idle at 128 x 256 (fewer rows
// and columns per block, the same k order per output).
// HALF: 64-row blocks at width 256 (two fit a CU; pick_bn)
template <int BITS, int BN_, int NW = 4, bool HALF = false> struct Cfg {
  static constexpr int BN = BN_;
  static constexpr int BM = (BN_ == 128 || HALF) ? 64 : 128;  // block rows
  static constexpr int THREADS = 64 * NW;
  static constexpr int WGN = NW, WGM = 1;  // the waves side by side in N: B dequantized once
  static constexpr int WM = BM / WGM, WN = BN / WGN;
  static constexpr int MB = WM / 16, NB = WN / kTileN;  // 16 x 16 MFMA blocks per wave
  static constexpr int RT = BN / kTileN;                // packed row tiles per block
  static constexpr int A_BYTES = BM * BK * 2;           // 32 KB
  static constexpr int B_BYTES = RT * 256 * BITS;       // packed codes
  static constexpr int SZ_BYTES = RT * 4 * 64;          // up to 4 group slots per k-tile
  static constexpr int STAGE = A_BYTES + B_BYTES + SZ_BYTES;
};

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_ptr)g, (lds_ptr)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_ptr)g, (lds_ptr)lds, 4, 0, 0);
}

struct GemmEp {  // output epilogue (qlin_common.h kEp*)
  const uint16_t* res;
  int ep;
};

struct GemmGeo {
  int64_t M;
  int N, K, Kt, G, group, wave, lane;
  uint32_t gmagic;
  int64_t m0, nt0, ntl;
};

// k / group, branch-free (see qlin_gemv.hip group_of)
__device__ __forceinline__ int gemm_group_of(const GemmGeo& g, int k) {
  const int gi = (int)(((uint64_t)(uint32_t)(k >> 5) * g.gmagic) >> 31);
  return min(gi, g.G - 1);
}

// one k-tile's DMA into stage buffer `st`: x tile, packed codes, (scale, zero) words
template <int BITS, int WN_, int GPT, int NW, bool HALF = false>
__device__ __forceinline__ void load_stage(unsigned char* st, const GemmGeo& g, int kt,
                                           const _Float16* __restrict__ x,
                                           const uint32_t* __restrict__ qw,
                                           const uint32_t* __restrict__ qsz) {
  using C = Cfg<BITS, WN_, NW, HALF>;
  // x: BM rows x 16 chunks; one instruction = 4 rows (1 KB); wave w owns rows [BM/NW w, +BM/NW).
  // Rows >= M re-read row M-1 and k >= K re-reads the row's last chunk: those C rows are never
  // stored and those k-steps are skipped.
  {
    const int sub = g.lane >> 4, p = g.lane & 15;
#pragma unroll
    for (int j = 0; j < C::BM / (4 * NW); ++j) {
      const int r = (C::BM / NW) * g.wave + 4 * j + sub;  // LDS row
      const int c = p ^ (r & 15);                      // logical chunk held at physical p
      const int64_t m = min(g.m0 + r, g.M - 1);
      const int k = min(kt * BK + 8 * c, g.K - 8);
      glds16(x + m * g.K + k, st + ((C::BM / NW) * g.wave + 4 * j) * 256);
    }
  }
  // packed codes: RT row tiles x 256*BITS bytes, lane-linear 16-B chunks
  {
    constexpr int CH = C::RT * 16 * BITS;  // chunks per stage
    unsigned char* bs = st + C::A_BYTES;
#pragma unroll
    for (int j = g.wave; j < CH / 64; j += NW) {
      const int c = 64 * j + g.lane;
      const int rt = c / (16 * BITS), o = c % (16 * BITS);
      const int64_t nt = min(g.nt0 + rt, g.ntl);
      glds16(qw + ((nt * g.Kt + kt) * 64 * BITS + 4 * o), bs + 1024 * j);
    }
  }
  // (scale, zero) words: [row tile][slot][16], 4 B per lane
  {
    unsigned char* ss = st + C::A_BYTES + C::B_BYTES;
    constexpr int WORDS = C::RT * GPT * 16;
#pragma unroll
    for (int j = g.wave; j < WORDS / 64; j += NW) {
      const int w = 64 * j + g.lane;
      const int rt = w / (16 * GPT), i = (w / 16) % GPT, n = w & 15;
      const int64_t nt = min(g.nt0 + rt, g.ntl);
      const int gi = gemm_group_of(g, kt * BK + 32 * (i * 4 / GPT));
      glds4(qsz + sz_index(nt, gi, g.G, n), ss + 256 * j);
    }
  }
}

// KFULL (every k-tile inside K, the sources within 2 GB of their bases): the per-lane byte
// offsets of a stage's DMA sources are formed once, and a k-tile only moves three uniform base
// pointers — scalar adds; the checked form above spends ~39 VALU per k-tile and wave on 64-bit
// addresses and clamps (M = 65,536 main loop: 259 VALU per 128 MFMAs)
template <int BITS, int WN_, int GPT, int NW, bool HALF>
struct StageOff {
  using C = Cfg<BITS, WN_, NW, HALF>;
  static constexpr int NX = C::BM / (4 * NW);
  static constexpr int CH = C::RT * 16 * BITS / 64, NCH = (CH + NW - 1) / NW;
  static constexpr int SW = C::RT * GPT * 16 / 64, NSZ = (SW + NW - 1) / NW;
  uint32_t x[NX], c[NCH], s[NSZ > 0 ? NSZ : 1];
};

template <int BITS, int WN_, int GPT, int NW, bool HALF>
__device__ __forceinline__ void stage_offsets(StageOff<BITS, WN_, GPT, NW, HALF>& so,
                                              const GemmGeo& g) {
  using C = Cfg<BITS, WN_, NW, HALF>;
  using O = StageOff<BITS, WN_, GPT, NW, HALF>;
  const int sub = g.lane >> 4, p = g.lane & 15;
#pragma unroll
  for (int j = 0; j < O::NX; ++j) {
    const int r = (C::BM / NW) * g.wave + 4 * j + sub;
    const int c = p ^ (r & 15);
    const int64_t m = min(g.m0 + r, g.M - 1);
    so.x[j] = (uint32_t)((m * g.K + 8 * c) * 2);
  }
#pragma unroll
  for (int jj = 0; jj < O::NCH; ++jj) {
    const int c = 64 * (g.wave + jj * NW) + g.lane;
    const int rt = c / (16 * BITS), o = c % (16 * BITS);
    const int64_t nt = min(g.nt0 + rt, g.ntl);
    so.c[jj] = (uint32_t)((nt * g.Kt * 64 * BITS + 4 * o) * 4);
  }
#pragma unroll
  for (int jj = 0; jj < O::NSZ; ++jj) {
    const int w = 64 * (g.wave + jj * NW) + g.lane;
    const int rt = w / (16 * GPT), i = (w / 16) % GPT, n = w & 15;
    const int64_t nt = min(g.nt0 + rt, g.ntl);
    so.s[jj] = (uint32_t)(((nt * g.G + i) * kTileN + n) * 4);
  }
}

// a buffer descriptor over [p, p + 2 GB) from readfirstlane'd inputs (provably wave-uniform)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gemm_srd(const void* p) {
  const uint64_t ad = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ad);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(ad >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0x7fffffff,
                                           0x00020000);
}

struct StageSrd {
  __amdgpu_buffer_rsrc_t x, qw, sz;
};

// the same sources as load_stage (x chunk k = kt BK + 8 c, the codes of k-tile kt, the group
// slots of the k-tile's first group + i: a k-tile's groups are consecutive) as buffer_load ... lds
// with the per-lane byte offset in voffset and kt's part in soffset: no VALU per k-tile
template <int BITS, int WN_, int GPT, int NW, bool HALF>
__device__ __forceinline__ void load_stage_kf(unsigned char* st, const GemmGeo& g, int kt,
                                              const StageOff<BITS, WN_, GPT, NW, HALF>& so,
                                              const StageSrd& r) {
  using C = Cfg<BITS, WN_, NW, HALF>;
  using O = StageOff<BITS, WN_, GPT, NW, HALF>;
  const int xs = kt * (BK * 2), qs = kt * (64 * BITS * 4);
  const int gs = gemm_group_of(g, kt * BK) * (kTileN * 4);
#pragma unroll
  for (int j = 0; j < O::NX; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r.x, (lds_ptr)(st + ((C::BM / NW) * g.wave + 4 * j) * 256), 16, (int)so.x[j], xs, 0, 0);
  unsigned char* bs = st + C::A_BYTES;
#pragma unroll
  for (int jj = 0; jj < O::NCH; ++jj) {
    const int j = g.wave + jj * NW;  // wave-uniform
    if (O::NCH * NW == O::CH || j < O::CH)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r.qw, (lds_ptr)(bs + 1024 * j), 16, (int)so.c[jj],
                                               qs, 0, 0);
  }
  unsigned char* ss = st + C::A_BYTES + C::B_BYTES;
#pragma unroll
  for (int jj = 0; jj < O::NSZ; ++jj) {
    const int j = g.wave + jj * NW;
    if (O::NSZ * NW == O::SW || j < O::SW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r.sz, (lds_ptr)(ss + 256 * j), 4, (int)so.s[jj], gs,
                                               0, 0);
  }
}

// A fragments of k-step S for the wave's MB row blocks: row (lane & 15), chunk (4S + q) ^ (row & 15)
template <int S, int MB, int WM>
__device__ __forceinline__ void read_a(h8 (&a)[MB], const unsigned char* as, int wm, int n_in,
                                       int q) {
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int r = wm * WM + mb * 16 + n_in;
    const int c = (4 * S + q) ^ (r & 15);
    a[mb] = *reinterpret_cast<const h8*>(as + r * 256 + c * 16);
  }
}

// FULL: every k-tile lies inside K (K % 128 == 0, chosen per launch): straight-line k-steps
// (ABL bit 2, lab only: the raw packed words stand in for the dequantized B fragment)
template <int BITS, int WN_, int GPT, int ZM, bool FULL, int NW, int ABL = 0, bool HALF = false>
__device__ __forceinline__ void compute_stage(
    const unsigned char* st, const GemmGeo& g, int kt,
    f4 (&acc)[Cfg<BITS, WN_, NW, HALF>::MB][Cfg<BITS, WN_, NW, HALF>::NB]) {
  using C = Cfg<BITS, WN_, NW, HALF>;
  constexpr int MB = C::MB, NB = C::NB, WM = C::WM;
  const int wm = g.wave / C::WGN, wn = g.wave % C::WGN;
  const int lane = g.lane, n_in = lane & 15, q = lane >> 4;
  const unsigned char* as = st;
  const uint32_t* bs = reinterpret_cast<const uint32_t*>(st + C::A_BYTES);
  const uint32_t* ss = reinterpret_cast<const uint32_t*>(st + C::A_BYTES + C::B_BYTES);
  const Magics mg = make_magics<BITS>();
  // the wave's 8 lane pieces; int8 pieces (32 B) are read per half (steps 0-1, then 2-3)
  constexpr int PW = BITS == 8 ? 4 : BITS;  // words held per piece at a time
  Piece<BITS> pc[NB];
  auto read_pieces = [&](int half) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const uint32_t* p = bs + (wn * NB + nb) * 64 * BITS + lane * BITS + half * PW;
      if constexpr (BITS == 8) {
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        pc[nb].w[4 * half] = v.x; pc[nb].w[4 * half + 1] = v.y;
        pc[nb].w[4 * half + 2] = v.z; pc[nb].w[4 * half + 3] = v.w;
      } else {
        pc[nb] = load_piece<BITS>(p);
      }
    }
  };
  GroupQ gq[NB];
  auto read_groups = [&](int slot) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const uint32_t sw = ss[((wn * NB + nb) * GPT + slot) * 16 + n_in];
      gq[nb] = make_group_w<BITS, ZM>(sw);
    }
  };

  h8 a[2][MB];
  read_pieces(0);
  read_a<0, MB, WM>(a[0], as, wm, n_in, q);
  auto step = [&](auto S_) {
    constexpr int S = decltype(S_)::value;
    if constexpr (S * GPT / 4 != (S - 1) * GPT / 4 || S == 0) read_groups(S * GPT / 4);
    if constexpr (BITS == 8 && S == 2) read_pieces(1);
    if constexpr (S < 3) read_a<S + 1, MB, WM>(a[(S + 1) & 1], as, wm, n_in, q);  // next A in flight
    if (!FULL && kt * BK + 32 * S >= g.K) return;  // wave-uniform
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      uint32_t v[4];
      if constexpr (ABL & 4) {
        v[0] = pc[nb].w[0]; v[1] = pc[nb].w[1 % BITS]; v[2] = pc[nb].w[2 % BITS]; v[3] = pc[nb].w[3 % BITS];
      } else {
        dequant_step<BITS, ZM, S>(pc[nb], mg, gq[nb], v);
      }
      const h8 b = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[S & 1][mb], b, acc[mb][nb], 0, 0, 0);
    }
  };
  step(std::integral_constant<int, 0>{});
  step(std::integral_constant<int, 1>{});
  step(std::integral_constant<int, 2>{});
  step(std::integral_constant<int, 3>{});
}

// epilogue of a wave's MB x NB blocks of 16 x 16: lane (n, q) holds C[4q + i][n] of each block;
// the wave's rows start at wrow0, its columns at 16-column tile ct0 (the block's rows at m0, BM
// of them)
template <int MB, int NB, int BM>
__device__ __forceinline__ void store_tile(const f4 (&acc)[MB][NB], int64_t M, int N, int64_t m0,
                                           int64_t wrow0, int64_t ct0, int lane,
                                           const _Float16* __restrict__ bias,
                                           _Float16* __restrict__ y,
                                           const _Float16* __restrict__ res, int ep) {
  const int n_in = lane & 15, q = lane >> 4;
  if (ep == kEpSiluMul) {  // N % 16 == 0: gate column n_in < 8 pairs with up column n_in + 8
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int64_t j = ct0 + nb;  // interleaved tile = output columns 8j..8j+7
      const int64_t n = j * kTileN + n_in;
      const bool in_n = n < N;     // wave-uniform
      const float bv = (bias && in_n) ? (float)bias[n] : 0.f;
      // lane n_in < 8 holds gate column c = n_in, lane n_in + 8 the up column c, rows 4q + i:
      // the pair splits the rows — the low lane forms rows 4q, 4q + 1, the high lane 4q + 2,
      // 4q + 3 — so each SiLU is evaluated once (row_ror:8 swaps the halves of a 16-lane row)
      const bool lo = n_in < 8;
      const int c = n_in & 7;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        float t[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) t[i] = (float)(_Float16)(acc[mb][nb][i] + bv);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          // what the partner lane needs: the low lane's gate of row 2 + h, the high lane's up
          // of row h
          const float r = dpp_f<0x128>(lo ? t[2 + h] : t[h]);
          const float gv = lo ? t[h] : r, uv = lo ? r : t[2 + h];
          const int64_t m = wrow0 + mb * 16 + 4 * q + (lo ? h : 2 + h);
          if (in_n && m < M) y[m * (N >> 1) + j * 8 + c] = (_Float16)(silu_rn16(gv) * uv);
        }
      }
    }
    return;
  }
  if (m0 + BM <= M && (int64_t)BM * N < (1ll << 31)) {
    // whole row tile inside M: a uniform row base and 32-bit per-lane offsets, no row checks
    // (M = 65,536: 1151 -> 1206 TFLOP/s against the per-element checked stores below)
    const int64_t base = wrow0 * (int64_t)N;
    _Float16* __restrict__ yb = y + base;
    const _Float16* __restrict__ rb = res + base;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int n = (int)((ct0 + nb) * kTileN) + n_in;
      if (n >= N) continue;
      const float bv = bias ? (float)bias[n] : 0.f;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t o = (uint32_t)((mb * 16 + 4 * q + i) * N + n);
          if (ep == kEpResidual)
            yb[o] = (_Float16)((float)(_Float16)(acc[mb][nb][i] + bv) + (float)rb[o]);
          else
            yb[o] = (_Float16)(acc[mb][nb][i] + bv);
        }
    }
    return;
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int64_t n = (ct0 + nb) * kTileN + n_in;
    if (n >= N) continue;
    const float bv = bias ? (float)bias[n] : 0.f;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = wrow0 + mb * 16 + 4 * q + i;
        if (m >= M) continue;
        if (ep == kEpResidual)
          y[m * N + n] = (_Float16)((float)(_Float16)(acc[mb][nb][i] + bv) + (float)res[m * N + n]);
        else
          y[m * N + n] = (_Float16)(acc[mb][nb][i] + bv);
      }
    }
  }
}

// ABL: development ablations (tools/dev/gemm_lab.hip): bit 0 skips the MFMA/dequant work, bit 1
// the DMA after the first k-tile, bit 2 the dequant VALU; the library instantiates ABL = 0 only.
// HALF: 64-row blocks (Cfg).  SPLIT: split-K — S blocks per output tile each run k-tiles
// [s kts, (s + 1) kts) and write their fp32 accumulators, thread-linear, to `part`
// ([tile][s][thread][MB NB 4]); gemm_splitk_reduce sums them in s order (deterministic) and
// applies the epilogue
template <int BITS, int WN_, int GPT, int ZM, bool KFULL, int ABL = 0, int NW = 4, bool HALF = false,
          bool SPLIT = false>
__global__ __launch_bounds__(64 * NW) void gemm_kernel(
    const uint32_t* __restrict__ qw, const uint32_t* __restrict__ qsz,
    const _Float16* __restrict__ x, const _Float16* __restrict__ bias, _Float16* __restrict__ y,
    int64_t M, int N, int K, int group, uint32_t gmagic, int tiles_m, int tiles_n,
    const _Float16* __restrict__ res, int ep, int S = 1, float* __restrict__ part = nullptr) {
  using C = Cfg<BITS, WN_, NW, HALF>;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * C::STAGE];
  GemmGeo g;
  g.M = M;
  g.N = N;
  g.K = K;
  g.Kt = (K + BK - 1) / BK;
  g.G = K / group;
  g.group = group;
  g.gmagic = gmagic;
  g.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  g.lane = threadIdx.x & 63;
  // XCD-aware order: dispatch puts block b on XCD b % 8; give each XCD a contiguous run of
  // (tile_m, tile_n) with n fastest so its blocks share x tiles in that XCD's L2
  const int nblk = tiles_m * tiles_n * (SPLIT ? S : 1);
  const int b = blockIdx.x;
  int lb = b;
  if ((nblk & 7) == 0) lb = (b & 7) * (nblk >> 3) + (b >> 3);
  int split = 0;
  if constexpr (SPLIT) {  // the S splits of a tile are adjacent: same XCD, shared x tile
    split = lb % S;
    lb /= S;
  }
  const int tile_m = lb / tiles_n, tile_n = lb - tile_m * tiles_n;
  g.m0 = (int64_t)tile_m * C::BM;
  g.nt0 = (int64_t)tile_n * C::RT;
  g.ntl = (N + kTileN - 1) / kTileN - 1;

  f4 acc[C::MB][C::NB];
#pragma unroll
  for (int i = 0; i < C::MB; ++i)
#pragma unroll
    for (int j = 0; j < C::NB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  int kt_beg = 0, kt_end = g.Kt;
  if constexpr (SPLIT) {
    const int kts = (g.Kt + S - 1) / S;
    kt_beg = min(split * kts, g.Kt);
    kt_end = min(kt_beg + kts, g.Kt);
  }
  StageOff<BITS, WN_, GPT, NW, HALF> so;
  StageSrd srd;
  if constexpr (KFULL) {
    stage_offsets(so, g);
    srd = StageSrd{gemm_srd(x), gemm_srd(qw), gemm_srd(qsz)};
  }
  auto stage = [&](unsigned char* st, int kt) {
    if constexpr (KFULL) load_stage_kf<BITS, WN_, GPT, NW, HALF>(st, g, kt, so, srd);
    else load_stage<BITS, WN_, GPT, NW, HALF>(st, g, kt, x, qw, qsz);
  };
  if (kt_beg < kt_end) stage(smem, kt_beg);
  // the younger wave of each SIMD pair (waves NW/2 .. NW - 1) loses every VALU arbitration to its
  // partner at equal priority; one static raise before the loop (MI355X_MICROARCH.md, two waves
  // per SIMD, item 4)
  if (NW == 8 && g.wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  for (int kt = kt_beg; kt < kt_end; ++kt) {
    // stage kt has landed for every wave, and every wave is done reading stage kt - 1
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    __syncthreads();
    if (!(ABL & 2) && kt + 1 < kt_end) stage(smem + ((kt - kt_beg + 1) & 1) * C::STAGE, kt + 1);
    if (!(ABL & 1))
      compute_stage<BITS, WN_, GPT, ZM, KFULL, NW, ABL, HALF>(smem + ((kt - kt_beg) & 1) * C::STAGE,
                                                               g, kt, acc);
  }

  if constexpr (SPLIT) {
    f4* pp = reinterpret_cast<f4*>(part) +
             (((int64_t)lb * S + split) * C::THREADS + threadIdx.x) * (C::MB * C::NB);
#pragma unroll
    for (int i = 0; i < C::MB; ++i)
#pragma unroll
      for (int j = 0; j < C::NB; ++j) pp[i * C::NB + j] = acc[i][j];
    return;
  }
  const int wm = g.wave / C::WGN, wn = g.wave % C::WGN;
  store_tile<C::MB, C::NB, C::BM>(acc, M, N, g.m0, g.m0 + wm * C::WM, g.nt0 + wn * C::NB, g.lane,
                                  bias, y, res, ep);
}

// split-K second pass: one block per output tile, each thread sums its S partial accumulators in
// s order and stores them through the GEMM's own epilogue
template <int BITS, int WN_, int NW>
__global__ __launch_bounds__(64 * NW) void gemm_splitk_reduce(
    const float* __restrict__ part, int S, int64_t M, int N, int tiles_n,
    const _Float16* __restrict__ bias, _Float16* __restrict__ y,
    const _Float16* __restrict__ res, int ep) {
  using C = Cfg<BITS, WN_, NW>;
  const int tile = blockIdx.x;
  const int tile_m = tile / tiles_n, tile_n = tile - tile_m * tiles_n;
  f4 acc[C::MB][C::NB];
#pragma unroll
  for (int i = 0; i < C::MB; ++i)
#pragma unroll
    for (int j = 0; j < C::NB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < S; ++sp) {
    const f4* pp = reinterpret_cast<const f4*>(part) +
                   (((int64_t)tile * S + sp) * C::THREADS + threadIdx.x) * (C::MB * C::NB);
#pragma unroll
    for (int i = 0; i < C::MB; ++i)
#pragma unroll
      for (int j = 0; j < C::NB; ++j) acc[i][j] += pp[i * C::NB + j];
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  const int64_t m0 = (int64_t)tile_m * C::BM;
  const int64_t nt0 = (int64_t)tile_n * C::RT;
  store_tile<C::MB, C::NB, C::BM>(acc, M, N, m0, m0 + wm * C::WM, nt0 + wn * C::NB, lane, bias, y,
                                  res, ep);
}

uint32_t group_magic(int group) {
  const uint64_t d = (uint64_t)(group / 32);
  return (uint32_t)(((1ull << 31) + d - 1) / d);
}

// KFULL launches address their DMA sources by 32-bit per-lane byte offsets (load_stage_kf)
static inline bool kf_offsets_fit(int64_t M, int N, int K, int bits) {
  const int64_t lim = (int64_t)1 << 31;
  return M * K * 2 < lim && (int64_t)(N + 15) * K * bits / 8 < lim;
}

template <int BITS, int WN_, int GPT, int ZM, bool HALF = false>
int launch_gemm_t(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int64_t M, int N, int K, int group, hipStream_t st, const GemmEp& e) {
  using C = Cfg<BITS, WN_, kWaves, HALF>;
  const int tiles_n = (N + C::BN - 1) / C::BN;
  const int64_t tiles_m = (M + C::BM - 1) / C::BM;
  const int64_t blocks = tiles_m * tiles_n;
  if (blocks > 0x7fffffff) return QLIN_EINVAL;
#define QLIN_GL(KF)                                                                           \
  hipLaunchKernelGGL((gemm_kernel<BITS, WN_, GPT, ZM, KF, 0, kWaves, HALF>),                  \
                     dim3((unsigned)blocks),                                                   \
                     dim3(64 * kWaves), 0, st, qw, qsz, (const _Float16*)x, (const _Float16*)bias, \
                     (_Float16*)y, M, N, K, group, group_magic(group), (int)tiles_m, tiles_n, \
                     (const _Float16*)e.res, e.ep)
  // straight-line k-steps need K % 128 == 0; the wider tiles with 2-4 group slots per k-tile then
  // spill (the per-step checks bound the scheduler), so they keep the checked form
  if (K % BK == 0 && !(WN_ > 256 && GPT > 1) && kf_offsets_fit(M, N, K, BITS)) QLIN_GL(true);
  else QLIN_GL(false);
#undef QLIN_GL
  return (int)hipGetLastError();
}

int cu_count() { return qlin::device_cu_count(); }

// Block width.  The 128 x 256 / 384 / 512 blocks use 2 x 48-72 KB of LDS stages, so one block
// fits a CU and a launch runs in rounds of `CUs` blocks.  Cost model fitted on int4 g128
// (tools/dev/gemm_bn.py, MI355X): a full round of 128 x 256 / 384 / 512 blocks takes 1 / 1.42 /
// 1.84 units (wider blocks dequantize each B fragment for more MFMAs), and a partial round with a
// fraction f of the CUs busy takes (0.5 + 0.5 f) of a full one (less contention for L2 / HBM).
// M = 2048: N = 4096 -> 256 (one round), N = 6144 -> 384 (one round instead of 1.5: 121 -> 97
// us), N = 14336 / 28672 -> 512; M >= 8192 -> 512.
// Grids of 128 x 256 blocks that leave half the CUs or more idle take 64 x 128 blocks, four
// times as many (2 x 13-16 KB stages: three blocks fit a CU, so the round model above does not
// apply to them; tools/dev/gemm_bn.py, int4 g128 K = 4096): the GQA k / v projection N = 1024 at
// M = 2048 53 -> 29 us; N = 4096 at M = 128-512 50 -> 24-32 us, M = 1024 57 -> 52 us.
// Grids that small take 64-row blocks: 64 x 128 (three fit a CU) while that grid stays within
// ~a round of blocks, 64 x 256 (two fit a CU, each B fragment feeding 4 MFMAs instead of 2) once
// it would not (tools/dev/gemm_half.py: N = 4096 M = 768 / 1024 43.6 / 46.6 -> 40.7 / 43.0 us,
// 4096 x 14336 M = 1024 146 -> 135 us, N = 6144 M = 512 42.6 -> 39.8 us, N = 28672 M = 128 42.7
// -> 38.9 us; bit-identical); returned as kHalf256.
constexpr int kHalf256 = 255;
int pick_bn(int64_t M, int N, int bits) {
  if (bits == 8) return 256;
  const int64_t tm = (M + 127) / 128, cus = cu_count();
  const int64_t n256 = (N + 255) / 256;
  if (tm * n256 * 2 <= cus) return tm * n256 * 4 > cus ? kHalf256 : 128;
  static const int bn[3] = {256, 384, 512};
  static const double rel[3] = {1.0, 1.42, 1.84};
  int best = 256;
  double best_cost = 0;
  for (int i = 0; i < 3; ++i) {
    const int64_t blocks = tm * ((N + bn[i] - 1) / bn[i]);
    const int64_t full = blocks / cus;
    const double f = (double)(blocks - full * cus) / (double)cus;
    const double cost = rel[i] * ((double)full + (f > 0 ? 0.5 + 0.5 * f : 0.0));
    if (i == 0 || cost < best_cost) best = bn[i], best_cost = cost;
  }
  return best;
}

// split-K launch of the 64 x 128 block (S splits, `part` = the caller's workspace)
template <int BITS, int GPT, int ZM>
int launch_gemm_split(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x,
                      const uint16_t* bias, uint16_t* y, int64_t M, int N, int K, int group,
                      hipStream_t st, const GemmEp& e, int S, float* part) {
  using C = Cfg<BITS, 128, kWaves>;
  const int tiles_n = (N + C::BN - 1) / C::BN;
  const int tiles_m = (int)((M + C::BM - 1) / C::BM);
  const int tiles = tiles_m * tiles_n;
#define QLIN_GS(KF)                                                                            \
  hipLaunchKernelGGL((gemm_kernel<BITS, 128, GPT, ZM, KF, 0, kWaves, false, true>),           \
                     dim3((unsigned)(tiles * S)), dim3(64 * kWaves), 0, st, qw, qsz,           \
                     (const _Float16*)x, nullptr, nullptr, M, N, K, group, group_magic(group), \
                     tiles_m, tiles_n, nullptr, 0, S, part)
  if (K % BK == 0 && kf_offsets_fit(M, N, K, BITS)) QLIN_GS(true);
  else QLIN_GS(false);
#undef QLIN_GS
  hipLaunchKernelGGL((gemm_splitk_reduce<BITS, 128, kWaves>), dim3((unsigned)tiles),
                     dim3(64 * kWaves), 0, st, part, S, M, N, tiles_n, (const _Float16*)bias,
                     (_Float16*)y, (const _Float16*)e.res, e.ep);
  return (int)hipGetLastError();
}

template <int BITS, int GPT, int ZM>
int launch_gemm(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                uint16_t* y, int64_t M, int N, int K, int group, hipStream_t st, const GemmEp& e,
                int S = 1, float* part = nullptr) {
  if constexpr (BITS != 8) {
    if (S > 1) return launch_gemm_split<BITS, GPT, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e,
                                                       S, part);
    const int bn = pick_bn(M, N, BITS);
    if (bn == 512)
      return launch_gemm_t<BITS, 512, GPT, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
    if (bn == 384)
      return launch_gemm_t<BITS, 384, GPT, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
    if (bn == 128)
      return launch_gemm_t<BITS, 128, GPT, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
    if (bn == kHalf256)
      return launch_gemm_t<BITS, 256, GPT, ZM, true>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  }
  return launch_gemm_t<BITS, 256, GPT, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
}

template <int BITS, int ZM>
int launch_gemm_g(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int64_t M, int N, int K, int group, hipStream_t st, const GemmEp& e,
                  int S, float* part) {
  if (group % 128 == 0)
    return launch_gemm<BITS, 1, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e, S, part);
  if (group % 64 == 0)
    return launch_gemm<BITS, 2, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e, S, part);
  return launch_gemm<BITS, 4, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e, S, part);
}

// split-K parts for an M x N x K launch: grids of 64 x 128 blocks that leave most CUs idle (the
// lone block is issue-bound at 24-50 us whatever M is) split K into up to 8 parts
// of >= 4 k-tiles while the grid stays within one block per CU
int splitk_parts(int64_t M, int64_t N, int64_t K, int bits) {
  if (bits == 8 || M <= kSkinnyMaxM || pick_bn(M, (int)N, bits) != 128) return 1;
  const int64_t tiles = ((M + 63) / 64) * ((N + 127) / 128), cus = cu_count();
  const int64_t kt = (K + BK - 1) / BK;
  int S = 1;
  while (S < 8 && tiles * S * 2 <= cus && kt / (S * 2) >= 4) S *= 2;
  return S;
}
int64_t splitk_bytes(int64_t M, int64_t N, int S) {
  if (S <= 1) return 0;
  const int64_t tiles = ((M + 63) / 64) * ((N + 127) / 128);
  return tiles * S * (64 * kWaves) * 16 * 4;  // 64 x 128 block: MB NB 4 = 16 floats per thread
}

bool valid(int64_t M, int64_t N, int64_t K, int bits, int group) {
  return M >= 0 && M <= (1ll << 40) && N >= 0 && N <= (1 << 30) && K > 0 && K % 32 == 0 &&
         K <= (1 << 20) && group > 0 && group % 32 == 0 && K % group == 0 &&
         (bits == 2 || bits == 3 || bits == 4 || bits == 8);
}

}  // namespace

namespace {
// splitk_ws: the caller's split-K workspace (splitk_bytes of the launch) or nullptr (no split)
int gemm_ep(const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
            const uint16_t* bias, const uint16_t* residual, uint16_t* y, int64_t M, int64_t N,
            int64_t K, int bits, int group, int epilogue, void* stream, void* splitk_ws = nullptr) {
  if (!qweight || !qsz || !x || !y || !valid(M, N, K, bits, group)) return QLIN_EINVAL;
  if (M == 0 || N == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const GemmEp e{residual, epilogue};
  const int zm = zero_mode(flags);
  const int n = (int)N, k = (int)K;
  const int S = splitk_ws ? splitk_parts(M, N, K, bits) : 1;
  float* part = (float*)splitk_ws;
#define QLIN_M(B)                                                                              \
  return zm == kZFloat                                                                         \
             ? launch_gemm_g<B, kZFloat>(qweight, qsz, x, bias, y, M, n, k, group, st, e, S, part) \
         : zm == kZWide                                                                        \
             ? launch_gemm_g<B, kZWide>(qweight, qsz, x, bias, y, M, n, k, group, st, e, S, part)  \
             : launch_gemm_g<B, kZNarrow>(qweight, qsz, x, bias, y, M, n, k, group, st, e, S, part)
  switch (bits) {
    case 2: QLIN_M(2);
    case 3: QLIN_M(3);
    case 4: QLIN_M(4);
    default: QLIN_M(8);
  }
#undef QLIN_M
}
}  // namespace

// block columns pick_bn takes for this launch (255: the 64-row block of width 256)
extern "C" int qlin_gemm_block_cols(int64_t M, int64_t N, int bits) {
  if (M < 1 || N < 1 || N > (1 << 30) || !(bits == 2 || bits == 3 || bits == 4 || bits == 8))
    return -QLIN_EINVAL;
  return pick_bn(M, (int)N, bits);
}

namespace {
// act fake-quant x_dq region of qlin_linear_ep_f16's workspace (fp16 [M, K], 256-B aligned) when
// that launch needs one, else 0
int64_t act_ws_bytes(int64_t M, int64_t N, int64_t K, int act_bits) {
  const bool fuse_act = M <= kSkinnyMaxM && N <= kActFuseMaxN;
  return (act_bits && !fuse_act) ? (M * K * 2 + 255) / 256 * 256 : 0;
}
}  // namespace

extern "C" int64_t qlin_linear_workspace_bytes(int64_t M, int64_t N, int64_t K, int bits,
                                               int group, int act_bits) {
  if (!valid(M < 1 ? 1 : M, N, K, bits, group) || M < 0 || act_bits < 0 || act_bits > 8) return -1;
  return act_ws_bytes(M, N, K, act_bits) + splitk_bytes(M, N, splitk_parts(M, N, K, bits));
}

// the split-K workspace when the caller's buffer holds this launch's partials, else nullptr
// (the launch then runs unsplit: a short buffer is never written past its end)
void* splitk_ws_of(void* ws, int64_t ws_bytes, int64_t M, int64_t N, int64_t K, int bits) {
  if (!ws || ws_bytes <= 0 || M < 1 || N < 1 || N > (1 << 30) || K < 1) return nullptr;
  const int S = splitk_parts(M, N, K, bits);
  return S > 1 && ws_bytes >= splitk_bytes(M, N, S) ? ws : nullptr;
}

extern "C" int qlin_gemm_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                             const uint16_t* x, const uint16_t* bias, uint16_t* y, int64_t M,
                             int64_t N, int64_t K, int bits, int group, void* workspace,
                             int64_t workspace_bytes, void* stream) {
  if (workspace_bytes < 0) return QLIN_EINVAL;
  return gemm_ep(qweight, qsz, flags, x, bias, nullptr, y, M, N, K, bits, group, kEpNone, stream,
                 splitk_ws_of(workspace, workspace_bytes, M, N, K, bits));
}

extern "C" int qlin_linear_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                               const uint16_t* x, const uint16_t* bias, uint16_t* y, int64_t M,
                               int64_t N, int64_t K, int bits, int group, void* stream) {
  if (M == 0) return QLIN_OK;
  if (M <= kSkinnyMaxM) {
    // skinny batches: the GEMV kernel in 16-row chunks (weights re-streamed per chunk; a 64-row
    // GEMM block alone on its CU is issue-bound at ~24 us for K = 4096)
    for (int64_t m0 = 0; m0 < M; m0 += 16) {
      const int64_t mc = M - m0 < 16 ? M - m0 : 16;
      const int rc = qlin_gemv_f16(qweight, qsz, flags, x + m0 * K, bias, y + m0 * N, mc, N, K,
                                   bits, group, stream);
      if (rc) return rc;
    }
    return QLIN_OK;
  }
  return qlin_gemm_f16(qweight, qsz, flags, x, bias, y, M, N, K, bits, group, nullptr, 0, stream);
}

extern "C" int qlin_linear_ep_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                                  const uint16_t* x, const uint16_t* bias,
                                  const uint16_t* residual, uint16_t* y, int64_t M, int64_t N,
                                  int64_t K, int bits, int group, int epilogue, int act_bits,
                                  int act_flags, uint16_t* workspace, int64_t workspace_bytes,
                                  void* stream) {
  if (workspace_bytes < 0 || (workspace_bytes > 0 && !workspace)) return QLIN_EINVAL;
  if (epilogue < kEpNone || epilogue > kEpSiluMul) return QLIN_EINVAL;
  if (epilogue == kEpResidual && !residual) return QLIN_EINVAL;
  if (epilogue == kEpSiluMul && N % kTileN) return QLIN_EINVAL;
  if (act_bits && (act_bits < 2 || act_bits > 8)) return QLIN_EINVAL;
  if (M < 0) return QLIN_EINVAL;
  if (M == 0) return QLIN_OK;
  const int64_t ny = epilogue == kEpSiluMul ? N / 2 : N;  // columns of y (and residual)
  // the fused activation statistics are recomputed by every GEMV block: past ~1024 row tiles
  // the quantizer launch + plain GEMV is cheaper (tools/dev/act_ab.py: 28672 x 4096 fused
  // 24.0 us vs 22.6 us; 4096 x 4096 fused 7.0 us vs 12.8 us)
  const bool fuse_act = act_bits && M <= kSkinnyMaxM && N <= kActFuseMaxN;
  const int64_t act_bytes = act_ws_bytes(M, N, K, act_bits);
  if (act_bits && !fuse_act) {
    if (!workspace || workspace_bytes < act_bytes) return QLIN_EINVAL;
    const int rc = qlin_quantize(x, QLIN_F16, M, K, act_bits, (int)K,
                                 act_flags & (QLIN_SYMMETRIC | QLIN_DISABLE_ZERO_POINT), nullptr,
                                 nullptr, workspace, nullptr, nullptr, nullptr, nullptr, stream);
    if (rc) return rc;
    x = workspace;
    act_bits = 0;
  }
  if (M <= kSkinnyMaxM) {
    for (int64_t m0 = 0; m0 < M; m0 += 16) {
      const int64_t mc = M - m0 < 16 ? M - m0 : 16;
      const int rc = qlin::gemv_ep(qweight, qsz, flags, x + m0 * K, bias,
                                   residual ? residual + m0 * ny : nullptr, y + m0 * ny, mc, N, K,
                                   bits, group, epilogue, act_bits, act_flags, stream);
      if (rc) return rc;
    }
    return QLIN_OK;
  }
  return gemm_ep(qweight, qsz, flags, x, bias, residual, y, M, N, K, bits, group, epilogue,
                 stream,
                 workspace ? splitk_ws_of((char*)workspace + act_bytes, workspace_bytes - act_bytes,
                                          M, N, K, bits)
                           : nullptr);
}

// CUs of the current device, cached per device id (the first call per device queries it; racing
// first calls store the same value)
int qlin::device_cu_count() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
  int n = dev < kMaxDev ? cache[dev].load(std::memory_order_relaxed) : 0;
  if (n > 0) return n;
  int c = 0;
  n = (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
       c > 0) ? c : 256;
  if (dev < kMaxDev) cache[dev].store(n, std::memory_order_relaxed);
  return n;
}
