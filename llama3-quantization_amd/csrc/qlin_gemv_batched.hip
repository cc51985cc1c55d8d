// qlin_gemv_batched.hip — strided batch of independent decode GEMVs in one launch (gfx950).
//
// qlin_gemv_batched_f16: y[b] = x[b] @ W_dq[b]^T (+ bias[b]) for b < batch, the same
// QuantLinear.forward -> F.linear(input, W_dq, bias) (quant/int_linear.py:62) as qlin_gemv_f16,
// for many same-shaped packed matrices at once.  The single-launch GEMV is latency-bound (a
// dependent 4096^2 launch pays a ~1.5 us kernel boundary and a ~1 us wave ramp for 8.8 MB,
// DESIGN.md §4); a batch pays them once and is bound by HBM bandwidth instead.
#include "qlin_common.h"
#include "qlin_gemv_tile.h"

#include <algorithm>
#include <type_traits>

using namespace qlin;

namespace {

// ---------------------------------------------------------------------------------------------
// Batched streaming GEMV: a launch over a batch is throughput-, not latency-bound, so the
// decomposition differs from the single-launch fast path (qlin_gemv.hip):
//   - ONE wave owns whole 16-row tile rows and streams all of their K (int4, K = 4096: a
//     contiguous 32 KB region per tile row) with PF tiles in flight, accumulating each tile row in
//     a single MFMA chain in k order: no cross-wave reduction, no LDS barrier, no block phases (a
//     block is 4 independent waves).  Each output is one v_mfma_f32_16x16x32_f16 chain over
//     k = 0, 32, 64, ... -- the order of qlin_gemm_f16 (bit-identical to it without split-K);
//   - the grid is sized to the resident capacity (CUs x blocks per CU from the occupancy query)
//     and wave w takes the contiguous tile rows [w T / Wt, (w + 1) T / Wt) of the batch's T, so
//     every wave streams from start to end (one-tile-row-per-wave grids ran in ~2.3 rounds and the
//     last, partial round streamed with a third of the chip's loads in flight);
//   - the prefetch runs across tile-row boundaries (rounds of PF tiles never straddle one:
//     Kt % PF == 0), so a wave's loads never drain between its rows;
//   - blocks are remapped so that each XCD takes a contiguous run of tile rows (a problem's x stays
//     in one L2).
// ---------------------------------------------------------------------------------------------
struct StreamArgs {
  const uint32_t* qw;
  const uint32_t* qsz;
  const _Float16* x;
  const _Float16* bias;
  _Float16* y;
  int64_t bs_qw, bs_sz, bs_x, bs_b, bs_y;  // per-problem element strides
  int M, N, K, Kt, G, Nt;
  int64_t T;         // tile rows over the batch (batch x Nt)
  int64_t Wt;        // waves of the launch (<= T); wave w streams tile rows [wT/Wt, (w+1)T/Wt)
  uint32_t cmagic;   // GPT == 1: kt / (group / 128) = (kt * cmagic) >> 31
  int xcd_chunk;     // > 0: blocks per XCD of the remapped order (grid % 8 == 0)
  int64_t* plan;     // host only: non-NULL = report {blocks, dyn LDS, static LDS, blocks per CU}
                     // of the launch into plan[0..3] instead of launching (qlin_gemv_batched_plan)
};

constexpr int kStreamWaves = 4;
constexpr int kStreamPF = 8;  // tiles in flight per wave (16 for the 2/3-bit tiles,
                              // 6 or 8 waves per SIMD forced, measured slower)

// SZR (group = 128 / GPT, i.e. 32, 64 or 128): the (scale, zero) words of a whole round of PF
// tiles -- PF * GPT groups x 16 rows, contiguous in the qsz layout -- arrive as ONE 16-B-per-lane
// load per 1 KB (one round ahead, like the codes) and are parked in the wave's LDS slot, from
// where each k-step reads its lane's word, instead of GPT 64-byte loads per tile: fewer vector
// memory instructions per tile (int2 g64: 4 -> 2 + 1/round).  tools/dev/batch_geo.py, one box,
// best of 3: int2 g64 131 -> 125 us, int3 g64 116 -> 115, int4 g128 97.9 -> 96.7 (bit-identical).
// PRE (SZR with narrow int16 zeros): the group constants are formed once per round, when the
// round's (scale, zero) words are parked, instead of once per tile and group in every lane: the
// parked slot holds three planes of SW words -- (s, s), (z + off_0, z + off_1), (z + off_2,
// z + off_3) in fp16 (off_P = pair_off<BITS>(P); the sums are exact, |z| <= 1024) -- and a k-step
// reads its lane's words and subtracts the half its pair needs (op_sel), so the per-pair work is
// the extract, the zero subtraction and the scale multiply alone: the same fp16 operations on the
// same values as dequant_step (bit-identical): 62.5 -> 52.4 VALU per int2 g64 tile (int3: 99 ->
// 65 with step_pairs' v_bfi_b32 extract).  tools/dev/batch_geo.py, one box, best of 3: int2 g64
// 129.9 -> 126.0 us per 96-matrix ring, int3 g64 120.2 -> 108.8 us per 64 (the two-v_and_or_b32
// int3 extract of that build); int4 g128 +-1 %.
template <int BITS, int S>
__device__ __forceinline__ void dequant_step_pre(const Piece<BITS>& c, const Magics& mg,
                                                 uint32_t ssw, uint32_t za, uint32_t zb,
                                                 uint32_t (&out)[4]) {
#pragma clang fp contract(off)
  uint32_t v[4];
  step_pairs<BITS, S>(c, mg, v);
  const h2 ss = as_h2(ssw), ha = as_h2(za), hb = as_h2(zb);
#pragma unroll
  for (int P = 0; P < 4; ++P) {
    const h2 zs = (BITS >= 4 || P < 2) ? ha : hb;
    const _Float16 z = (BITS == 8 || (P & 1) == 0) ? zs.x : zs.y;
    out[P] = as_u32((as_h2(v[P]) - h2{z, z}) * ss);
  }
}

// NR tile rows side by side (NR = 2: rows 2p, 2p + 1 of one problem; M = 1 with the per-round
// group constants): every x fragment is parked and read once per k-tile for both rows and each
// round covers PF / NR k-tiles of both rows, so PF tiles stay in flight.  Each row keeps its own
// MFMA chain in k order (bit-identical).  tools/dev/stream_lab.hip (`lab2_kernel`), same box:
// int2 g64 119.3 -> 115.0 us per 96-matrix ring, int3 g64 107.8 -> 105.4, int4 g128 97.6 -> 96.2,
// at 4 waves per SIMD (see pad_lds_to).
template <int BITS, int MT, int GPT, int ZM, int PF, bool SZR, int NR>
__global__ __launch_bounds__(64 * kStreamWaves) void gemv_stream_kernel(const StreamArgs a) {
  static_assert(NR == 1 || (MT == 1 && SZR && ZM == kZNarrow), "two rows: M = 1, narrow zeros");
  constexpr int PFK = PF / NR;                   // k-tiles per round
  __shared__ __attribute__((aligned(16))) uint32_t xs[kStreamWaves][64 * MT];
  constexpr int SWR = PFK * GPT * kTileN;       // SZR: (scale, zero) words per row and round
  constexpr int SW = NR * SWR;                  // ... of all NR rows
  constexpr int NC = SW >= 256 ? SW / 256 : 1;  // 16-B loads per lane per round
  constexpr bool PRE = SZR && ZM == kZNarrow;
  constexpr int NPL = PRE ? (BITS < 4 ? 3 : 2) : 1;  // parked planes
  __shared__ __attribute__((aligned(16))) uint32_t szs[SZR ? kStreamWaves : 1][SZR ? NPL * SW : 4];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  int blk = blockIdx.x;
  if (a.xcd_chunk > 0) blk = (blk & 7) * a.xcd_chunk + (blk >> 3);  // XCD j: a contiguous run
  const int64_t w = (int64_t)blk * kStreamWaves + wave;
  if (w >= a.Wt) return;  // wave-uniform; no barriers below
  // row units (NR tile rows each) of this wave: contiguous [wU/Wt, (w+1)U/Wt) (an interleaved
  // w, w + Wt, ... measured within noise, round 3)
  const int64_t U = a.T / NR;
  const int64_t r0 = w * U / a.Wt;
  const int64_t nrows = (w + 1) * U / a.Wt - r0;
  if (nrows <= 0) return;
  constexpr int LPR = 64 / MT;
  const int xlane = min(lane / LPR, a.M - 1) * a.K + 2 * MT * (lane % LPR);

  // load stream: row unit lr, round start lkt, its operand bases
  int64_t lr = r0;
  int lkt = 0;
  const uint32_t* lqw;
  const uint32_t* lsz;   // SZR: the unit's first row tile's qsz base; else + n_in
  const _Float16* lx;
  const int64_t rw = (int64_t)a.Kt * (64 * BITS), rs = (int64_t)a.G * kTileN;  // per tile row
  auto set_row = [&](int64_t u) {
    const int64_t r = u * NR;
    const int64_t b = r / a.Nt;
    const int nt = (int)(r - b * a.Nt);
    lqw = a.qw + b * a.bs_qw + (int64_t)nt * rw + lane * BITS;
    lsz = a.qsz + b * a.bs_sz + (int64_t)nt * rs + (SZR ? 0 : n_in);
    lx = a.x + b * a.bs_x + xlane;
  };
  set_row(lr);
  auto group_of_tile = [&](int kt) {
    return GPT == 1 ? (int)(((uint64_t)(uint32_t)kt * a.cmagic) >> 31) : kt * GPT;
  };
  WTile<BITS, GPT> wt[NR][PFK];
  XRaw<MT> xq[PFK];
  uint4 szr[NC];  // SZR: the next round's (scale, zero) words, lane l: words 4l .. 4l + 3
  auto load_szr = [&](int kt0) {  // round starting at tile kt0: groups kt0 * GPT .. of each row
    if constexpr (SZR) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int o = 256 * c + (4 * lane) % (SW < 256 ? SW : 256);
        const int rr = o / SWR;
        szr[c] = *reinterpret_cast<const uint4*>(lsz + rr * rs + kt0 * GPT * kTileN + (o - rr * SWR));
      }
    }
  };
  uint32_t* sslot = &szs[SZR ? wave : 0][0];
  auto park_sz = [&] {
    if constexpr (PRE) {
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
    } else if constexpr (SZR) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        *reinterpret_cast<uint4*>(sslot + 256 * c + (4 * lane) % (SW < 256 ? SW : 256)) = szr[c];
    }
  };
  auto load = [&](int u, int kt) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      wt[rr][u].pc = load_piece_nt<BITS>(lqw + rr * rw + kt * (64 * BITS));
      if constexpr (!SZR) {
        const int g0 = group_of_tile(kt);
#pragma unroll
        for (int s = 0; s < GPT; ++s) wt[rr][u].sz[s] = lsz[rr * rs + (g0 + s) * kTileN];
      }
    }
    const _Float16* p = lx + kt * kTileK;
    if constexpr (MT == 1) {
      xq[u].w[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (MT == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(p);
      xq[u].w[0] = v.x; xq[u].w[1] = v.y;
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(p);
      xq[u].w[0] = v.x; xq[u].w[1] = v.y; xq[u].w[2] = v.z; xq[u].w[3] = v.w;
    }
  };
  const Magics mg = make_magics<BITS>();
  f4 acc[NR];
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) acc[rr] = f4{0.f, 0.f, 0.f, 0.f};
  uint32_t* slot = &xs[wave][0];
  auto tile = [&](int u) {
    h8 xa[4];
    park_x<MT>(xa, xq[u], slot, lane, n_in);
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      auto step = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        const int si = rr * SWR + (u * GPT + S * GPT / 4) * kTileN + n_in;
        if constexpr (PRE) {
          dequant_step_pre<BITS, S>(wt[rr][u].pc, mg, sslot[si], sslot[SW + si],
                                    NPL > 2 ? sslot[(NPL - 1) * SW + si] : 0u, v);
        } else {
          const uint32_t szw = SZR ? sslot[si] : wt[rr][u].sz[S * GPT / 4];
          const GroupQ gq = make_group_w<BITS, ZM>(szw);
          dequant_step<BITS, ZM, S>(wt[rr][u].pc, mg, gq, v);
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
  // C row m = 4q + e sits in lane n + 16q, element e: lanes 0..15 hold rows 0..3
  auto store = [&](int64_t u) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int64_t r = u * NR + rr;
      const int64_t b = r / a.Nt;
      const int64_t row = (r - b * a.Nt) * kTileN + n_in;
      if (lane < 16 && row < a.N) {
        const float bv = a.bias ? (float)a.bias[b * a.bs_b + row] : 0.f;
#pragma unroll
        for (int e = 0; e < MT && e < 4; ++e) {
          if (e < a.M) {
            float t = acc[rr][e];
            if (a.bias) t += bv;
            a.y[b * a.bs_y + (int64_t)e * a.N + row] = (_Float16)t;
          }
        }
      }
      acc[rr] = f4{0.f, 0.f, 0.f, 0.f};
    }
  };

  // rounds of PFK k-tiles (Kt % PFK == 0: a round never straddles two row units); every round but
  // the last refills each slot right after computing it with the next round's tile
  load_szr(0);
#pragma unroll
  for (int u = 0; u < PFK; ++u) load(u, u);
  int64_t cr = r0;  // compute stream: row unit, round start
  int ckt = 0;
  const int64_t rounds = nrows * (a.Kt / PFK);
  for (int64_t q = 0; q + 1 < rounds; ++q) {
    park_sz();  // this round's (scale, zero) words into the wave's LDS slot
    lkt += PFK;
    if (lkt == a.Kt) {  // wave-uniform
      lkt = 0;
      ++lr;
      set_row(lr);
    }
    load_szr(lkt);
#pragma unroll
    for (int u = 0; u < PFK; ++u) {
      tile(u);
      load(u, lkt + u);
    }
    ckt += PFK;
    if (ckt == a.Kt) {  // wave-uniform: the row unit is complete
      store(cr);
      ckt = 0;
      ++cr;
    }
  }
  park_sz();
#pragma unroll
  for (int u = 0; u < PFK; ++u) tile(u);
  store(cr);
}

// resident blocks per CU of a stream-kernel instance with `dyn` bytes of dynamic LDS (occupancy
// query; the caller caches it per instance)
template <typename Kern>
int blocks_per_cu(Kern k, size_t dyn) {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 64 * kStreamWaves, dyn) ==
                     hipSuccess && n > 0
             ? n : 1;
}

template <typename Kern>
size_t static_lds(Kern k) {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k)) == hipSuccess
             ? fa.sharedSizeBytes : 0;
}

// The two-row instances fit 5 waves per SIMD in registers, but measured fastest at 4 (lab2_kernel
// int2 g64 at 5: 127.4 us, at 4: 114.9): their launches pad each block's LDS to a quarter of the
// CU's 160 KB so that 4 blocks are resident per CU.  Each instance has its own static LDS size,
// so the padding is computed from that instance's own sharedSizeBytes.
constexpr size_t kCuLds = 160 * 1024;
inline size_t pad_lds_to(size_t static_bytes, int blocks_per_cu_wanted) {
  const size_t want = kCuLds / blocks_per_cu_wanted - 64;
  return static_bytes < want ? want - static_bytes : (size_t)0;
}

// Geometry of one stream-kernel instance, computed once per template instance (a function-local
// static of the instance's own launcher: every gemv_stream_kernel<...> has the same C++ type, so
// a cache keyed on the kernel's type would be shared by all of them).
struct StreamGeo {
  size_t dyn, stat;
  int per_cu;
};

template <int BITS, int MT, int GPT, int ZM, int PF, bool SZR, int NR>
int launch_stream_nr(StreamArgs a, hipStream_t st) {
  auto k = gemv_stream_kernel<BITS, MT, GPT, ZM, PF, SZR, NR>;
  static const StreamGeo geo = [&] {
    StreamGeo g;
    g.stat = static_lds(k);
    g.dyn = NR == 2 ? pad_lds_to(g.stat, 4) : 0;
    g.per_cu = blocks_per_cu(k, g.dyn);
    return g;
  }();
  // persistent: the grid is the resident capacity (one tile row per wave, a grid of T waves, ran
  // its last round with a third of the loads in flight)
  const int64_t Wt = std::min<int64_t>(
      a.T / NR, (int64_t)device_cu_count() * geo.per_cu * kStreamWaves);
  a.Wt = Wt;
  const int64_t blocks = (Wt + kStreamWaves - 1) / kStreamWaves;
  if (a.plan) {
    a.plan[0] = blocks;
    a.plan[1] = (int64_t)geo.dyn;
    a.plan[2] = (int64_t)geo.stat;
    a.plan[3] = geo.per_cu;
    a.plan[4] = NR;
    return 0;
  }
  a.xcd_chunk = blocks % 8 == 0 ? (int)(blocks / 8) : 0;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(64 * kStreamWaves), geo.dyn, st, a);
  return (int)hipGetLastError();
}

// two tile rows per wave for one-row products with narrow zeros and an even tile-row count
template <int BITS, int MT, int GPT, int ZM, int PF, bool SZR>
int launch_stream_pf(const StreamArgs& a, hipStream_t st) {
  if constexpr (MT == 1 && SZR && ZM == kZNarrow && PF == kStreamPF) {
    if (a.Nt % 2 == 0) return launch_stream_nr<BITS, MT, GPT, ZM, PF, SZR, 2>(a, st);
  }
  return launch_stream_nr<BITS, MT, GPT, ZM, PF, SZR, 1>(a, st);
}

// kStreamPF tiles in flight per wave, 4 when K is not a multiple of 8 tiles (Kt % 4 == 0: host)
template <int BITS, int MT, int GPT, int ZM, bool SZR>
int launch_stream_s(const StreamArgs& a, hipStream_t st) {
  if (a.Kt % kStreamPF == 0) return launch_stream_pf<BITS, MT, GPT, ZM, kStreamPF, SZR>(a, st);
  return launch_stream_pf<BITS, MT, GPT, ZM, 4, SZR>(a, st);
}

// group = 128 / GPT: round-wide (scale, zero) loads; GPT == 1 with group > 128 (a multiple of
// 128, per-channel included): per-tile loads (one group covers several tiles)
template <int BITS, int MT, int GPT, int ZM>
int launch_stream_t(const StreamArgs& a, hipStream_t st) {
  if (GPT > 1 || a.K / a.G == kTileK) return launch_stream_s<BITS, MT, GPT, ZM, true>(a, st);
  return launch_stream_s<BITS, MT, GPT, ZM, false>(a, st);
}

}  // namespace

// Strided batch of independent products y_b = x_b @ W_dq,b^T (+ bias_b), b < batch, in ONE launch
// (grid Nt x batch): the per-launch floor of a dependent 4096^2 GEMV (kernel boundary + wave ramp,
// DESIGN.md §4) is paid once per batch instead of once per matrix.  Problems the decode fast path
// does not take (M > 4, K % 128, tiles per wave > 4) run as one gemv launch each.
namespace {
int gemv_batched(const uint32_t* qweight, int64_t qweight_stride, const uint32_t* qsz,
                 int64_t qsz_stride, int flags, const uint16_t* x, int64_t x_stride,
                 const uint16_t* bias, int64_t bias_stride, uint16_t* y, int64_t y_stride,
                 int64_t batch, int64_t M, int64_t N, int64_t K, int bits, int group,
                 void* stream, int64_t* plan) {
  if (!qweight || !qsz || !x || !y || batch < 0 || batch > 65535 || M < 1 || M > kGemvMaxM ||
      !valid_layout(N, K, bits, group))
    return QLIN_EINVAL;
  const int64_t Nt = (N + kTileN - 1) / kTileN, Kt = (K + kTileK - 1) / kTileK;
  // strides must not let two problems' packed operands or outputs overlap; x and bias may be
  // shared (stride 0: several matrices applied to one activation)
  if (qweight_stride < Nt * Kt * 64 * bits || qsz_stride < Nt * (K / group) * kTileN ||
      (x_stride != 0 && x_stride < M * K) || y_stride < M * N ||
      (bias && bias_stride != 0 && bias_stride < N))
    return QLIN_EINVAL;
  if (batch == 0 || N == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  // the streaming kernel: M <= 4, whole tiles (a multiple of 4 per row), group a multiple of 128
  // or 32 / 64, and every problem's operands 16-B aligned (it issues 16-B loads of the codes, of a
  // round's (scale, zero) words and of x rows): qweight / qsz / x bases 16-B aligned, strides whole
  // 16-B units (qweight / qsz words % 4, x halfs % 8); anything else takes the per-problem path
  const bool aligned = ((uintptr_t)qweight & 15) == 0 && ((uintptr_t)qsz & 15) == 0 &&
                       ((uintptr_t)x & 15) == 0 && qweight_stride % 4 == 0 &&
                       qsz_stride % 4 == 0 && x_stride % 8 == 0 && (M == 1 || K % 8 == 0);
  if (aligned && M <= 4 && K % kTileK == 0 &&
      (group % kTileK == 0 || group == 32 || group == 64) && Kt % 4 == 0) {
    StreamArgs a;
    a.qw = qweight; a.qsz = qsz; a.x = (const _Float16*)x; a.bias = (const _Float16*)bias;
    a.y = (_Float16*)y;
    a.bs_qw = qweight_stride; a.bs_sz = qsz_stride; a.bs_x = x_stride;
    a.bs_b = bias ? bias_stride : 0; a.bs_y = y_stride;
    a.M = (int)M; a.N = (int)N; a.K = (int)K; a.Kt = (int)(K / kTileK); a.G = (int)(K / group);
    a.Nt = (int)Nt;
    a.T = Nt * batch;
    const uint64_t c = group % kTileK == 0 ? (uint64_t)(group / kTileK) : 1;
    a.cmagic = (uint32_t)(((1ull << 31) + c - 1) / c);
    a.xcd_chunk = 0;
    a.plan = plan;
    const int zm = zero_mode(flags), m = (int)M;
#define QLIN_SM(B, Z, G)                                                                       \
  return m == 1 ? launch_stream_t<B, 1, G, Z>(a, st)                                   \
         : m == 2 ? launch_stream_t<B, 2, G, Z>(a, st)                                 \
                  : launch_stream_t<B, 4, G, Z>(a, st)
#define QLIN_SG(B, Z)                                                                          \
  if (group % kTileK == 0) QLIN_SM(B, Z, 1);                                                   \
  if (group == 64) QLIN_SM(B, Z, 2);                                                           \
  QLIN_SM(B, Z, 4)
#define QLIN_SB(B)                                                                             \
  if (zm == kZFloat) { QLIN_SG(B, kZFloat); }                                                  \
  if (zm == kZWide) { QLIN_SG(B, kZWide); }                                                    \
  QLIN_SG(B, kZNarrow)
    switch (bits) {
      case 2: QLIN_SB(2);
      case 3: QLIN_SB(3);
      case 4: QLIN_SB(4);
      default: QLIN_SB(8);
    }
#undef QLIN_SB
#undef QLIN_SG
#undef QLIN_SM
  }
  // anything else: one launch per problem
  if (plan) {
    plan[0] = plan[1] = plan[2] = plan[3] = plan[4] = 0;  // not the streaming kernel
    return QLIN_OK;
  }
  for (int64_t b = 0; b < batch; ++b) {
    const int rc = qlin::gemv_ep(qweight + b * qweight_stride, qsz + b * qsz_stride, flags,
                                 x + b * x_stride, bias ? bias + b * bias_stride : nullptr,
                                 nullptr, y + b * y_stride, M, N, K, bits, group, kEpNone, 0, 0,
                                 stream);
    if (rc) return rc;
  }
  return QLIN_OK;
}

}  // namespace

extern "C" int qlin_gemv_batched_f16(const uint32_t* qweight, int64_t qweight_stride,
                                     const uint32_t* qsz, int64_t qsz_stride, int flags,
                                     const uint16_t* x, int64_t x_stride, const uint16_t* bias,
                                     int64_t bias_stride, uint16_t* y, int64_t y_stride,
                                     int64_t batch, int64_t M, int64_t N, int64_t K, int bits,
                                     int group, void* stream) {
  return gemv_batched(qweight, qweight_stride, qsz, qsz_stride, flags, x, x_stride, bias,
                      bias_stride, y, y_stride, batch, M, N, K, bits, group, stream, nullptr);
}

// The launch geometry qlin_gemv_batched_f16 would use for these arguments (nothing launched);
// operands are checked for alignment only, never dereferenced.
extern "C" int qlin_gemv_batched_plan(const uint32_t* qweight, int64_t qweight_stride,
                                      const uint32_t* qsz, int64_t qsz_stride, int flags,
                                      const uint16_t* x, int64_t x_stride, int64_t batch,
                                      int64_t M, int64_t N, int64_t K, int bits, int group,
                                      int64_t* plan) {
  if (!plan) return QLIN_EINVAL;
  for (int i = 0; i < 5; ++i) plan[i] = 0;
  uint16_t* y_dummy = reinterpret_cast<uint16_t*>(16);
  return gemv_batched(qweight, qweight_stride, qsz, qsz_stride, flags, x, x_stride, nullptr, 0,
                      y_dummy, M * N, batch, M, N, K, bits, group, nullptr, plan);
}
