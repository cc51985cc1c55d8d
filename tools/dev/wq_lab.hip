// Dev lab (not product): one-token-row GEMV for wide matrices with the block's tiles handed out
// by a per-block work queue (an LDS counter), int4 g128 only.  Question: does dynamic chunk
// assignment remove the whole-row kernel's tail (the second wave of each SIMD finishing ~3 us
// after the first: profiles/r4_gemv_wide_ab.txt)?
//
// Block b owns tile rows b, b + nb, ...; their tiles form chunks of C consecutive k-tiles of one
// row; waves take chunks from the counter (the first two statically), keep two chunks of loads in
// flight, and store each chunk's 16 partial sums in LDS; after one barrier the chunks of every row
// are added in k order (deterministic) and the epilogue applied.
#include "../../llama3-quantization_amd/csrc/qlin_common.h"
#include "../../llama3-quantization_amd/csrc/qlin_gemv_tile.h"

#include <type_traits>

using namespace qlin;

namespace {

constexpr int kMaxW = 8;       // waves per block (at most)
constexpr int kMaxRows = 8;    // tile rows per block
constexpr int kNwF16 = 2;

struct LabArgs {
  const uint32_t* qw;
  const uint32_t* qsz;
  const _Float16* x;
  const _Float16* nw;  // fp16 RMSNorm weight or null
  float eps;
  _Float16* y;
  int N, K, Kt, G, Nt, nb, ep;
  uint32_t cmagic;
  uint64_t* stamps;
};

#define LAB_STAMP(k)                                                                        \
  if (a.stamps && lane == 0)                                                                \
  a.stamps[((int64_t)blockIdx.x * kMaxW + wave) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()

// W waves, chunks of C k-tiles, XI 16-B x chunks per thread, SZC: one (scale, zero) load per
// chunk (lane l: word l of the chunk's C x 16, spread to the tiles by ds_bpermute) instead of one
// per tile
template <int W, int C, int NRM, int XI, bool SZC, int D = 2>
__global__ __launch_bounds__(64 * W) void wq_kernel(const LabArgs a) {
  constexpr int kW = W, kXIter = XI;
  constexpr int BITS = 4, GPT = 1, ZM = kZNarrow;
  extern __shared__ __attribute__((aligned(16))) uint4 xs4[];
  __shared__ float part[kMaxRows * 32][kTileN];  // [row * CPR + kc][n]
  __shared__ float nss[kMaxW];
  __shared__ int ctr;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15, q = lane >> 4;
  const int nthr = blockDim.x;
  const int b = blockIdx.x;
  LAB_STAMP(0);
  const int nrows = b < a.Nt ? (a.Nt - 1 - b) / a.nb + 1 : 0;
  const int CPR = a.Kt / C;
  const int NC = nrows * CPR;
  auto group_of_tile = [&](int kt) { return (int)(((uint64_t)(uint32_t)kt * a.cmagic) >> 31); };

  const int nch = a.K >> 3;
  uint4 xc[kXIter];
  uint4 nc[NRM ? kXIter : 1];
#pragma unroll
  for (int i = 0; i < kXIter; ++i) {
    const int c = min(tid + i * nthr, nch - 1);
    xc[i] = reinterpret_cast<const uint4*>(a.x)[c];
    if constexpr (NRM) nc[i] = reinterpret_cast<const uint4*>(a.nw)[c];
  }
  asm volatile("" ::: "memory");

  const int64_t wrow = (int64_t)a.Kt * (64 * BITS), srow = (int64_t)a.G * kTileN;
  WTile<BITS, GPT> wt[D * C];
  constexpr int SZW = C * kTileN / 64;  // chunk (scale, zero) words per lane (SZC)
  uint32_t szc[D][SZC ? SZW : 1];
  // chunk c -> (row j, first k-tile); clamped into the block's chunks (a clamped load is a
  // repeat that is never computed)
  auto load_chunk = [&](int set, int c) {
    c = min(c, max(NC - 1, 0));
    const int j = c / CPR, kt0 = (c - j * CPR) * C;
    const int64_t r = min((int64_t)b + (int64_t)j * a.nb, (int64_t)a.Nt - 1);
    const uint32_t* qp = a.qw + r * wrow + lane * BITS;
    if constexpr (SZC) {
      const uint32_t* sp = a.qsz + r * srow + kt0 * kTileN + lane * SZW;
      if constexpr (SZW == 1) szc[set][0] = sp[0];
      else {
        const uint2 v = *reinterpret_cast<const uint2*>(sp);
        szc[set][0] = v.x; szc[set][1] = v.y;
      }
    }
#pragma unroll
    for (int u = 0; u < C; ++u) {
      wt[set * C + u].pc = load_piece_nt<BITS>(qp + (kt0 + u) * (64 * BITS));
      if constexpr (!SZC)
        wt[set * C + u].sz[0] = a.qsz[r * srow + n_in + group_of_tile(kt0 + u) * kTileN];
    }
  };
  // the (scale, zero) word of tile u of a chunk for this lane (SZC): word 16u + n_in of the chunk
  auto chunk_sz = [&](int set, int u) -> uint32_t {
    const int wi = 16 * u + n_in;
    if constexpr (SZW == 1) {
      return (uint32_t)__builtin_amdgcn_ds_bpermute(wi * 4, (int)szc[set][0]);
    } else {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((wi >> 1) * 4, (int)szc[set][0]);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((wi >> 1) * 4, (int)szc[set][1]);
      return (wi & 1) ? hi : lo;
    }
  };
  int cs[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    cs[d] = wave + kW * d;
    load_chunk(d, cs[d]);
  }
#pragma unroll
  for (int i = 0; i < kXIter; ++i) {
    asm volatile("" : "+v"(xc[i].x), "+v"(xc[i].y), "+v"(xc[i].z), "+v"(xc[i].w)::"memory");
    if constexpr (NRM)
      asm volatile("" : "+v"(nc[i].x), "+v"(nc[i].y), "+v"(nc[i].z), "+v"(nc[i].w)::"memory");
  }
  LAB_STAMP(1);
  if (tid == 0) ctr = D * kW;
  if constexpr (NRM) {
#pragma clang fp contract(off)
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < kXIter; ++i) {
      const h8 v = __builtin_bit_cast(h8, xc[i]);
      float s8 = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s8 = s8 + (float)v[j] * (float)v[j];
      ss = ss + (tid + i * nthr < nch ? s8 : 0.f);
    }
    ss = wave_sum(ss);
    if (lane == 0) nss[wave] = ss;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float tot = 0.f;
    for (int w = 0; w < kW; ++w) tot += nss[w];
    const float rn = rsqrtf(tot / (float)a.K + a.eps);
#pragma unroll
    for (int i = 0; i < kXIter; ++i) {
      const h8 v = __builtin_bit_cast(h8, xc[i]);
      const h8 h = __builtin_bit_cast(h8, nc[i]);
      h8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (_Float16)((float)h[j] * ((float)v[j] * rn));
      xc[i] = __builtin_bit_cast(uint4, o);
    }
  }
#pragma unroll
  for (int i = 0; i < kXIter; ++i)
    if (tid + i * nthr < nch) xs4[tid + i * nthr] = xc[i];
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  LAB_STAMP(2);

  const Magics mg = make_magics<BITS>();
  auto grab = [&]() {
    int v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(&ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(v);
  };
  auto body = [&](auto SET_, int c, int cn) {
    constexpr int SET = decltype(SET_)::value;
    const int j = c / CPR, kc = c - j * CPR;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    const int cl = min(cn, max(NC - 1, 0));
    const int jn = cl / CPR, ktn = (cl - jn * CPR) * C;
    const int64_t rn_ = min((int64_t)b + (int64_t)jn * a.nb, (int64_t)a.Nt - 1);
    const uint32_t* qp = a.qw + rn_ * wrow + lane * BITS;
    const uint32_t* sp = a.qsz + rn_ * srow + n_in;
    uint32_t szt[C];
    if constexpr (SZC) {
#pragma unroll
      for (int u = 0; u < C; ++u) szt[u] = chunk_sz(SET, u);
      const uint32_t* spc = a.qsz + rn_ * srow + ktn * kTileN + lane * SZW;
      if constexpr (SZW == 1) szc[SET][0] = spc[0];
      else {
        const uint2 v = *reinterpret_cast<const uint2*>(spc);
        szc[SET][0] = v.x; szc[SET][1] = v.y;
      }
    }
#pragma unroll
    for (int u = 0; u < C; ++u) {
      const int kt = kc * C + u;
      h8 xa[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, xs4[kt * 16 + 4 * s + q]);
      WTile<BITS, GPT>& t = wt[SET * C + u];
      auto step = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        const GroupQ gq = make_group_w<BITS, ZM>(SZC ? szt[u] : t.sz[0]);
        dequant_step<BITS, ZM, S>(t.pc, mg, gq, v);
        const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
      t.pc = load_piece_nt<BITS>(qp + (ktn + u) * (64 * BITS));
      if constexpr (!SZC) t.sz[0] = sp[group_of_tile(ktn + u) * kTileN];
    }
    if (lane < kTileN) part[j * CPR + kc][lane] = acc[0];
  };
  auto run = [&](auto SET_) {
    constexpr int d = decltype(SET_)::value;
    if (cs[d] >= NC) return false;
    const int cn = grab();
    body(SET_, cs[d], cn);
    cs[d] = cn;
    return true;
  };
  for (;;) {
    if (!run(std::integral_constant<int, 0>{})) break;
    if (!run(std::integral_constant<int, 1>{})) break;
    if constexpr (D > 2) {
      if (!run(std::integral_constant<int, 2>{})) break;
    }
  }
  LAB_STAMP(4);
  __syncthreads();
  if (tid < nrows * kTileN) {
    const int j = tid >> 4, n = tid & 15;
    float t = 0.f;
    for (int kc = 0; kc < CPR; ++kc) t += part[j * CPR + kc][n];
    t = (float)(_Float16)t;
    const float up = __shfl(t, (lane & ~15) + ((n + 8) & 15));
    const int64_t r = (int64_t)b + (int64_t)j * a.nb;
    if (a.ep == kEpSiluMul) {
      if (n < 8 && r * kTileN + n + 8 < a.N) a.y[r * 8 + n] = (_Float16)(silu_rn16(t) * up);
    } else if (r * kTileN + n < a.N) {
      a.y[r * kTileN + n] = (_Float16)t;
    }
  }
  LAB_STAMP(5);
}

}  // namespace

extern "C" int lab_wq(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* nw,
                      float eps, uint16_t* y, int N, int K, int ep, int variant, int nb,
                      uint64_t* stamps, void* stream) {
  // variant = D * 1000 + W * 100 + C * 10 + SZC (D = 2 when absent)
  const int C = variant / 10 % 10;
  if (K % 1024 || N % 16) return -1;
  LabArgs a;
  a.qw = qw;
  a.qsz = qsz;
  a.x = (const _Float16*)x;
  a.nw = (const _Float16*)nw;
  a.eps = eps;
  a.y = (_Float16*)y;
  a.N = N;
  a.K = K;
  a.Kt = K / 128;
  a.G = K / 128;
  a.Nt = N / 16;
  a.nb = nb;
  a.ep = ep;
  a.cmagic = (uint32_t)((1ull << 31));
  a.stamps = stamps;
  if ((a.Nt + nb - 1) / nb > kMaxRows || a.Kt / C > 32) return -2;
  const size_t lds = (size_t)K * 2;
  hipStream_t st = (hipStream_t)stream;
  const bool n = nw != nullptr;
#define L3(D_, W_, C_, S_)                                                                     \
  if (n) hipLaunchKernelGGL((wq_kernel<W_, C_, kNwF16, (4096 / 8 + 64 * W_ - 1) / (64 * W_), S_, D_>), \
                            dim3(nb), dim3(64 * W_), lds, st, a);                          \
  else hipLaunchKernelGGL((wq_kernel<W_, C_, 0, (4096 / 8 + 64 * W_ - 1) / (64 * W_), S_, D_>),        \
                          dim3(nb), dim3(64 * W_), lds, st, a)
#define L(W_, C_, S_) L3(2, W_, C_, S_)
  if (K != 4096) return -3;
  (void)hipGetLastError();  // clear anything sticky from earlier runtime calls
  switch (variant) {
    case 840: L(8, 4, false); break;
    case 841: L(8, 4, true); break;
    case 820: L(8, 2, false); break;
    case 480: L(4, 8, false); break;
    case 481: L(4, 8, true); break;
    case 440: L(4, 4, false); break;
    case 441: L(4, 4, true); break;
    case 3841: L3(3, 8, 4, true); break;
    case 3821: L3(3, 8, 2, true); break;
    case 3441: L3(3, 4, 4, true); break;
    default: return -4;
  }
#undef L
  return (int)hipGetLastError();
}

// ---- variant D: the same work queue, the tiles' codes staged by LDS-DMA into a per-wave ring of
// D chunks (no VGPRs for tiles in flight), one (scale, zero) load per chunk
namespace {
template <int D, int NRM>
__global__ __launch_bounds__(512) void wqd_kernel(const LabArgs a) {
  constexpr int BITS = 4, ZM = kZNarrow, C = 4, kW = 8;
  extern __shared__ __attribute__((aligned(16))) uint4 xs4[];             // x: K / 8 chunks
  __shared__ __attribute__((aligned(16))) uint4 ring[kW][D][C][64];       // codes: 1 KB per tile
  __shared__ float part[kMaxRows * 8][kTileN];
  __shared__ float nss[kW];
  __shared__ int ctr;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15, q = lane >> 4;
  const int nthr = 512;
  const int b = blockIdx.x;
  LAB_STAMP(0);
  const int nrows = b < a.Nt ? (a.Nt - 1 - b) / a.nb + 1 : 0;
  const int CPR = a.Kt / C;
  const int NC = nrows * CPR;
  const int64_t wrow = (int64_t)a.Kt * (64 * BITS), srow = (int64_t)a.G * kTileN;

  const int nch = a.K >> 3;
  const int xcI = min(tid, nch - 1);
  uint4 xc = reinterpret_cast<const uint4*>(a.x)[xcI];
  uint4 nc = NRM ? reinterpret_cast<const uint4*>(a.nw)[xcI] : uint4{0, 0, 0, 0};
  asm volatile("" ::: "memory");

  uint32_t szc[D];
  auto issue = [&](int slot, int c) {  // chunk c's codes into ring slot `slot`, its sz word
    c = min(c, max(NC - 1, 0));
    const int j = c / CPR, kt0 = (c - j * CPR) * C;
    const int64_t r = min((int64_t)b + (int64_t)j * a.nb, (int64_t)a.Nt - 1);
    szc[slot] = a.qsz[r * srow + kt0 * kTileN + lane];
    const uint32_t* qp = a.qw + r * wrow + (int64_t)kt0 * (64 * BITS) + lane * BITS;
#pragma unroll
    for (int u = 0; u < C; ++u)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(qp + u * 64 * BITS),
                                       (__attribute__((address_space(3))) void*)&ring[wave][slot][u][0],
                                       16, 0, 2 /* nt */);
  };
  int cs[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    cs[d] = wave + kW * d;
    issue(d, cs[d]);
  }
  asm volatile("" : "+v"(xc.x), "+v"(xc.y), "+v"(xc.z), "+v"(xc.w)::"memory");
  asm volatile("" : "+v"(nc.x), "+v"(nc.y), "+v"(nc.z), "+v"(nc.w)::"memory");
  LAB_STAMP(1);
  if (tid == 0) ctr = D * kW;
  if constexpr (NRM) {
#pragma clang fp contract(off)
    float ss = 0.f;
    {
      const h8 v = __builtin_bit_cast(h8, xc);
      float s8 = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s8 = s8 + (float)v[j] * (float)v[j];
      ss = tid < nch ? s8 : 0.f;
    }
    ss = wave_sum(ss);
    if (lane == 0) nss[wave] = ss;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float tot = 0.f;
    for (int w = 0; w < kW; ++w) tot += nss[w];
    const float rn = rsqrtf(tot / (float)a.K + a.eps);
    const h8 v = __builtin_bit_cast(h8, xc);
    const h8 h = __builtin_bit_cast(h8, nc);
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)((float)h[j] * ((float)v[j] * rn));
    xc = __builtin_bit_cast(uint4, o);
  }
  if (tid < nch) xs4[tid] = xc;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  LAB_STAMP(2);

  const Magics mg = make_magics<BITS>();
  auto grab = [&]() {
    int v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(&ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(v);
  };
  // chunk in slot d: wait until only the D - 1 younger chunks' ops (5 each) are outstanding
  auto body = [&](auto DS_) {
    constexpr int d = decltype(DS_)::value;
    const int c = cs[d];
    const int cn = grab();
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * (C + 1)) : "memory");
    const int j = c / CPR, kc = c - j * CPR;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    uint4 pc4[C];
#pragma unroll
    for (int u = 0; u < C; ++u) pc4[u] = ring[wave][d][u][lane];
    uint32_t szt[C];
#pragma unroll
    for (int u = 0; u < C; ++u)
      szt[u] = (uint32_t)__builtin_amdgcn_ds_bpermute((16 * u + n_in) * 4, (int)szc[d]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    issue(d, cn);  // the slot is free: its codes are in registers
    cs[d] = cn;
#pragma unroll
    for (int u = 0; u < C; ++u) {
      const int kt = kc * C + u;
      h8 xa[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, xs4[kt * 16 + 4 * s + q]);
      Piece<BITS> pc;
      pc.w[0] = pc4[u].x; pc.w[1] = pc4[u].y; pc.w[2] = pc4[u].z; pc.w[3] = pc4[u].w;
      auto step = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        const GroupQ gq = make_group_w<BITS, ZM>(szt[u]);
        dequant_step<BITS, ZM, S>(pc, mg, gq, v);
        const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
    }
    if (lane < kTileN) part[j * CPR + kc][lane] = acc[0];
    return c;
  };
  for (;;) {
    if (cs[0] >= NC) break;
    body(std::integral_constant<int, 0>{});
    if (cs[1] >= NC) break;
    body(std::integral_constant<int, 1>{});
    if constexpr (D > 2) {
      if (cs[2] >= NC) break;
      body(std::integral_constant<int, 2>{});
    }
    if constexpr (D > 3) {
      if (cs[3] >= NC) break;
      body(std::integral_constant<int, 3>{});
    }
  }
  LAB_STAMP(4);
  __syncthreads();
  if (tid < nrows * kTileN) {
    const int j = tid >> 4, n = tid & 15;
    float t = 0.f;
    for (int kc = 0; kc < CPR; ++kc) t += part[j * CPR + kc][n];
    t = (float)(_Float16)t;
    const float up = __shfl(t, (lane & ~15) + ((n + 8) & 15));
    const int64_t r = (int64_t)b + (int64_t)j * a.nb;
    if (a.ep == kEpSiluMul) {
      if (n < 8 && r * kTileN + n + 8 < a.N) a.y[r * 8 + n] = (_Float16)(silu_rn16(t) * up);
    } else if (r * kTileN + n < a.N) {
      a.y[r * kTileN + n] = (_Float16)t;
    }
  }
  LAB_STAMP(5);
}
}  // namespace

extern "C" int lab_wqd(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* nw,
                       float eps, uint16_t* y, int N, int K, int ep, int depth, int nb,
                       uint64_t* stamps, void* stream) {
  if (K != 4096 || N % 16) return -1;
  LabArgs a;
  a.qw = qw;
  a.qsz = qsz;
  a.x = (const _Float16*)x;
  a.nw = (const _Float16*)nw;
  a.eps = eps;
  a.y = (_Float16*)y;
  a.N = N;
  a.K = K;
  a.Kt = K / 128;
  a.G = K / 128;
  a.Nt = N / 16;
  a.nb = nb;
  a.ep = ep;
  a.cmagic = (uint32_t)((1ull << 31));
  a.stamps = stamps;
  if ((a.Nt + nb - 1) / nb > kMaxRows) return -2;
  (void)hipGetLastError();
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = (size_t)K * 2;
  if (depth == 2) hipLaunchKernelGGL((wqd_kernel<2, kNwF16>), dim3(nb), dim3(512), lds, st, a);
  else if (depth == 3) hipLaunchKernelGGL((wqd_kernel<3, kNwF16>), dim3(nb), dim3(512), lds, st, a);
  else if (depth == 4) hipLaunchKernelGGL((wqd_kernel<4, kNwF16>), dim3(nb), dim3(512), lds, st, a);
  else return -3;
  return (int)hipGetLastError();
}
