// qlin_decode.hip — persistent decode engine: ONE launch runs one decode step (batch 1, one new
// token over a KV cache) through n consecutive quantized LLaMA decoder layers, gfx950.
//
// Replaces, per layer, QuantLlamaDecoderLayer.forward at q_len == 1 (models/int_llama_layer.py:
// 213-267 of the reference): RMSNorm -> q/k/v QuantLinear -> RoPE + KV append -> attention ->
// o_proj + residual -> RMSNorm -> gate/up QuantLinear, SiLU * up -> down_proj + residual, every
// QuantLinear.forward being F.linear(x, W_dq) (quant/int_linear.py:62) on packed weights.
//
// Why one launch: a batch-1 decode layer is a chain of five dependent weight streams (q/k/v 25 MB,
// o 8.4 MB, gate/up 59 MB, down 29 MB for LLaMA3-8B int4 g128).  As five launches each stream
// starts only after the previous kernel's boundary, ramp and drain (45 us per layer,
// 2.5 TB/s).  The weights do not depend on the activations, so here every wave streams its share
// of ALL the layers' weights continuously, PF tiles ahead, and only the arithmetic waits for the
// activation hand-offs between the phases: the boundary and ramp costs overlap the stream.
//
// Workgroup roles (one 512-thread workgroup per CU, all resident; grid = CUs):
//   waves 1..7 ("stream waves")  a static share of every GEMV phase's 16-row x 128-k tiles:
//       CU c owns tile rows r = c, c + G, ... of each phase, its tiles (row-major) are cut into 7
//       contiguous runs, one per stream wave (16 tiles in flight each); a wave computes each tile as soon as the phase's
//       input vector is in LDS (xready), K-split partial rows meet in LDS and the last-arriving
//       wave sums them in k order (deterministic) and applies the epilogue (residual add, SiLU*up);
//   wave 0 ("IO wave")  everything that waits on other CUs: polls the phase counters, stages each
//       phase's input vector into LDS (the RMSNorm applied there: same fixed-order sum on every
//       CU), publishes the CU's finished output rows, runs this CU's attention units (RoPE,
//       KV append, split-L attention over a 64/128-row chunk prefetched into LDS by LDS-DMA,
//       partial merge by the last unit of the head).
// Keeping every inter-CU wait and every global store on the IO wave lets the stream waves keep
// their weight loads in flight across phase boundaries (a stream wave never drains vmcnt).
//
// Hand-offs (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md visibility table row 1):
// payload stored write-through (sc1 atomic stores) by the one storing wave -> s_waitcnt vmcnt(0)
// -> one agent-scope atomic add; consumers poll with sc1 loads and read the payload with sc1
// loads.  Phase counters are sharded by blockIdx % 8 (one arrival per CU per phase and layer).
// Every wait is bounded: a timeout sets the workspace's error word and every wave exits.
//
// Arithmetic: the GEMV tiles are exactly qlin_gemv's (exact W_dq, one MFMA per k-step, fp32
// accumulation, F.linear's fp16 output rounding, then the fp16 epilogues); a row split over waves
// is summed in k-run order.  RMSNorm and attention follow qlin_rmsnorm_linear_ep / qlin_attn_decode
// _rope's fp32 formulas (other summation orders: equal to the reference path to fp32 rounding).
#include "qlin_common.h"
#include "qlin_gemv_tile.h"

#include <type_traits>

using namespace qlin;

namespace {

typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(1))) void* gbl_ptr;

constexpr int kD = 128;            // head_dim
constexpr int kWaves = 8;          // wave 0: IO, waves 1..7: stream
constexpr int kStream = kWaves - 1;
constexpr int kShards = 8;         // phase counters sharded by blockIdx % 8
constexpr int kMaxRows = 8;        // tile rows per CU and phase
constexpr int kMaxX = 16384;       // longest phase input (halfs): intermediate size
constexpr int kMaxH = 8192;        // hidden size
constexpr int kMaxGrp = 8;         // query heads per KV head
constexpr int kMaxC = 128;         // attention chunk rows
constexpr int kMaxL = 4096;        // attention rows
constexpr int kPhases = 4;         // GEMV phases: q/k/v, o, gate/up, down
constexpr int kQKV = 0, kO = 1, kGU = 2, kDN = 3;
#ifndef DECODE_PF                  // tiles in flight per stream wave (dev knob)
#define DECODE_PF 16
#endif
#ifndef DECODE_TRACE               // dev build: IO-wave event timestamps after the partials
#define DECODE_TRACE 0
#endif
constexpr int kEv = 28;            // trace events per layer
#ifndef DECODE_POLL_SLEEP          // s_sleep between polls of a cross-CU counter (x 64 clocks):
#define DECODE_POLL_SLEEP 8        // 256 pollers re-reading counters steal HBM bandwidth
#endif
#ifndef DECODE_IO_PRIO             // issue priority of the IO wave over its SIMD's stream wave
#define DECODE_IO_PRIO 3
#endif
#ifndef DECODE_STREAM_ONLY         // dev ablation (wrong results): every phase input "ready" at
#define DECODE_STREAM_ONLY 0       // once, no IO work: the stream waves' weight throughput alone
#endif
#ifndef DECODE_SPIN_LIMIT          // polls before a wait gives up (each ~0.1-1 us)
#define DECODE_SPIN_LIMIT (1 << 22)
#endif

struct Layer {  // == qlin_decode_layer (include/qlin_gfx950.h)
  const uint32_t* qw[kPhases];
  const uint32_t* sz[kPhases];
  const float* w_in;
  const float* w_post;
  _Float16* kc;
  _Float16* vc;
};
static_assert(sizeof(Layer) == 12 * sizeof(void*), "qlin_decode_layer layout");
static_assert(kMaxGrp * kMaxC >= 1024, "the merge keeps 2 x 512 floats in Smem::pb");
// the layer table is read-only for the launch: through the constant address space its pointers
// come by scalar loads (a vector load would make every weight load behind it wait vmcnt(0))
typedef __attribute__((address_space(4))) const Layer CLayer;

struct Args {
  const Layer* layers;
  int nl, H, I, Hq, Hkv, grp, Nqkv, ncu;
  int R[kPhases], Kt[kPhases], Gs[kPhases];  // tile rows, k tiles, groups per row of each phase
  uint32_t cmagic;                          // GPT == 1: kt / (group / 128) = (kt * cmagic) >> 31
  float eps, scale_div;
  const _Float16* x;
  _Float16* y;
  const float* cosc;
  const float* sinc;
  int64_t cache_rows;
  const int64_t* pos;
  int L0;          // cache rows before this step (the new row is L0)
  int64_t kv_hs;   // cache head stride (elements)
  const _Float16* mask;  // [L0 + 1] additive, or null
  int C, S;        // attention chunk rows, chunks per KV head
  int* cnt;        // counters (zeroed before the launch): [0] error, then per layer (cnt_stride)
  int cnt_stride;
  _Float16* qkv;
  _Float16* abuf;
  _Float16* h2;
  _Float16* gu;
  _Float16* hb;
  float* part;     // attention partials [Hkv][S][grp][kD + 2]
  unsigned long long* trace;  // DECODE_TRACE: [nl][kEv][ncu] wall_clock64 stamps
};

// DECODE_TRACE: the IO wave stamps event e of layer l (100 MHz wall clock); the first stream
// wave stamps events 20 + 2 ph (its first tile of phase ph computed) and 21 + 2 ph (its last)
__device__ __forceinline__ void stamp(const Args& a, int l, int e) {
  if (DECODE_TRACE && (threadIdx.x & 63) == 0)
    a.trace[((int64_t)l * kEv + e) * a.ncu + blockIdx.x] = wall_clock64();
}

__device__ __forceinline__ const CLayer& layer_at(const Args& a, int l) {
  return ((const CLayer*)(uintptr_t)a.layers)[l];
}

__device__ __forceinline__ int* cnt_phase(const Args& a, int l, int ph) {
  return a.cnt + 1 + l * a.cnt_stride + ph * kShards;
}
__device__ __forceinline__ int* cnt_attn(const Args& a, int l) {
  return a.cnt + 1 + l * a.cnt_stride + kPhases * kShards;
}
__device__ __forceinline__ int* cnt_head(const Args& a, int l, int g) {
  return a.cnt + 1 + l * a.cnt_stride + kPhases * kShards + 1 + g;
}

__device__ __forceinline__ uint32_t ld_sc1(const void* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1_64(const void* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(void* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int add_agent(int* p, int v) {
  return __hip_atomic_fetch_add((gu32*)p, (uint32_t)v, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// rows of phase ph owned by CU c (rows c, c + G, ...)
__device__ __forceinline__ int rows_of(int R, int c, int G) { return c < R ? (R - c + G - 1) / G : 0; }

// ---------------------------------------------------------------------------------------------
// LDS (static; 16-B aligned pieces, total < 160 KB)
// ---------------------------------------------------------------------------------------------
struct Smem {
  _Float16 xbuf[kMaxX];                 // this phase's input vector (normed for q/k/v, gate/up)
  _Float16 hres[kMaxH];                 // layer input h (o_proj residual)
  _Float16 h2res[kMaxH];                // h2 = h + o (down_proj residual)
  _Float16 kvs[2][kMaxC * kD];          // attention chunk K, V rows (16-B segments swizzled)
  float part[kMaxRows][kStream][kTileN];  // K-split partial rows
  float qs[kMaxGrp][kD];                // roped q (fp32)
  float pb[kMaxGrp][kMaxC];             // probabilities of the chunk
  _Float16 ostage[kMaxRows][kTileN];    // finished output rows of the phase
  _Float16 knew[kD];
  _Float16 vnew[kD];
  int rowcnt[kMaxRows];
  int ndone;                            // finished rows, cumulative over the launch
  int xready;                           // sequence number of the phase whose input is staged
  int abort_;
  int pad_;
};

// ---------------------------------------------------------------------------------------------
// waits
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void set_error(const Args& a, Smem& sm, int code) {
  if ((threadIdx.x & 63) == 0) {
    st_sc1(a.cnt, (uint32_t)code);
    __hip_atomic_store(&sm.abort_, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// IO wave: every shard j of a phase counter reached the number of CUs with blockIdx % 8 == j
__device__ __forceinline__ bool wait_phase(const Args& a, Smem& sm, int l, int ph) {
  const int lane = threadIdx.x & 63;
  const int* c = cnt_phase(a, l, ph);
  const int want = lane < kShards ? (a.ncu - lane + kShards - 1) / kShards : 0;
  for (int spin = 0; spin < DECODE_SPIN_LIMIT; ++spin) {
    int v = lane < kShards ? (int)ld_sc1(c + lane) : 0;
    if (lane == kShards) v = (int)ld_sc1(a.cnt);  // error word: another CU gave up
    if (__builtin_amdgcn_readlane(v, kShards) != 0) {
      set_error(a, sm, 2);
      return false;
    }
    if (__all(lane >= kShards || v >= want)) return true;
    __builtin_amdgcn_s_sleep(DECODE_POLL_SLEEP);
  }
  set_error(a, sm, 3);
  return false;
}

// IO wave: a plain counter reached `want`
__device__ __forceinline__ bool wait_count(const Args& a, Smem& sm, const int* c, int want) {
  const int lane = threadIdx.x & 63;
  for (int spin = 0; spin < DECODE_SPIN_LIMIT; ++spin) {
    const int v = lane == 0 ? (int)ld_sc1(c) : lane == 1 ? (int)ld_sc1(a.cnt) : 0;
    if (__builtin_amdgcn_readlane(v, 1) != 0) {
      set_error(a, sm, 2);
      return false;
    }
    if (__builtin_amdgcn_readlane(v, 0) >= want) return true;
    __builtin_amdgcn_s_sleep(DECODE_POLL_SLEEP);
  }
  set_error(a, sm, 4);
  return false;
}

// IO wave: the CU's stream waves finished `want` rows (cumulative)
__device__ __forceinline__ bool wait_done(const Args& a, Smem& sm, int want) {
  for (int spin = 0; spin < DECODE_SPIN_LIMIT; ++spin) {
    if (__hip_atomic_load(&sm.ndone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= want)
      return true;
    __builtin_amdgcn_s_sleep(1);
  }
  set_error(a, sm, 5);
  return false;
}

// stream wave: the phase with sequence number `seq` has its input staged.  The bounded spin is ONE
// inline-asm block: a loop in the compiler's CFG inside the unrolled tile body makes hipcc's
// waitcnt pass give up its per-slot counts and drain the whole prefetch (vmcnt(0)) every tile
__device__ __forceinline__ bool wait_ready(Smem& sm, int seq) {
  typedef __attribute__((address_space(3))) int lds_int;
  const uint32_t xa = (uint32_t)(uintptr_t)(lds_int*)&sm.xready;
  const uint32_t aa = (uint32_t)(uintptr_t)(lds_int*)&sm.abort_;
  int ok, sv, cnt, v, w;
  seq = __builtin_amdgcn_readfirstlane(seq);  // uniform: keep it in an SGPR for s_cmp
  asm volatile(
      "s_mov_b32 %[cnt], %[lim]\n"
      "1:\n\t"
      "ds_read_b32 %[v], %[xa]\n\t"
      "ds_read_b32 %[w], %[aa]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %[sv], %[v]\n\t"
      "s_cmp_ge_i32 %[sv], %[seq]\n\t"
      "s_cbranch_scc1 2f\n\t"
      "v_readfirstlane_b32 %[sv], %[w]\n\t"
      "s_cmp_lg_u32 %[sv], 0\n\t"
      "s_cbranch_scc1 3f\n\t"
      "s_sleep 2\n\t"
      "s_sub_u32 %[cnt], %[cnt], 1\n\t"
      "s_cmp_lg_u32 %[cnt], 0\n\t"
      "s_cbranch_scc1 1b\n"
      "3:\n\t"
      "s_mov_b32 %[ok], 0\n\t"
      "s_branch 4f\n"
      "2:\n\t"
      "s_mov_b32 %[ok], 1\n"
      "4:"
      : [ok] "=s"(ok), [sv] "=&s"(sv), [cnt] "=&s"(cnt), [v] "=&v"(v), [w] "=&v"(w)
      : [xa] "v"(xa), [aa] "v"(aa), [seq] "s"(seq), [lim] "s"(DECODE_SPIN_LIMIT)
      : "memory", "scc");
  return ok != 0;
}

__device__ __forceinline__ int seq_of(int l, int ph) { return l * kPhases + ph + 1; }

// ---------------------------------------------------------------------------------------------
// IO wave helpers
// ---------------------------------------------------------------------------------------------
// n halfs from global into LDS by LDS-DMA: every 1-KB piece in flight at once, one wait (the
// IO wave otherwise pays one memory round trip per batch of loads).  SC1: the vector was written
// earlier in this launch by other CUs (write-through) — the loads bypass this CU's L1.  The last
// piece may run past n: its lanes re-read the vector's last 16 B into the buffer's padding (every
// LDS vector buffer is a multiple of 1 KB)
template <bool SC1>
__device__ __forceinline__ void stage(_Float16* dst, const _Float16* src, int n) {
  const int lane = threadIdx.x & 63;
  const int nb = n * 2;
  const unsigned char* s = reinterpret_cast<const unsigned char*>(src);
  unsigned char* d = reinterpret_cast<unsigned char*>(dst);
  for (int i = 0; i * 1024 < nb; ++i) {
    const int off = min(i * 1024 + lane * 16, nb - 16);
    __builtin_amdgcn_global_load_lds((gbl_ptr)(s + off), (lds_ptr)(d + i * 1024), 16, 0,
                                     SC1 ? 16 : 0);
  }
  drain();
}

// RMSNorm (OmniLlamaRMSNorm, quant/omni_norm.py:52-63 of the reference; the fused norm of
// qlin_rmsnorm_linear_ep), fused with the staging of its input: x (H halfs) arrives in `res` by
// LDS-DMA while the norm weights come into registers (32 per lane per round: one memory round
// trip for H <= 4096 instead of one per element group), then dst = RN16(w * (x * rsqrt(mean(x^2)
// + eps))) with the sum of squares in a fixed lane-strided + butterfly order, so every CU forms
// the same normed vector
template <bool SC1>
__device__ __forceinline__ void stage_norm(_Float16* res, _Float16* dst, const _Float16* src,
                                           const float* w, int H, float eps) {
#pragma clang fp contract(off)
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(1))) const f2v gf2;
  const int lane = threadIdx.x & 63;
  const int nb = H * 2;
  const unsigned char* s = reinterpret_cast<const unsigned char*>(src);
  unsigned char* d = reinterpret_cast<unsigned char*>(res);
  for (int i = 0; i * 1024 < nb; ++i) {
    const int off = min(i * 1024 + lane * 16, nb - 16);
    __builtin_amdgcn_global_load_lds((gbl_ptr)(s + off), (lds_ptr)(d + i * 1024), 16, 0,
                                     SC1 ? 16 : 0);
  }
  constexpr int R = 32;  // float2 weight loads per lane per round
  f2v ww[R];
  auto load_w = [&](int k0) {
#pragma unroll
    for (int c = 0; c < R; ++c) ww[c] = *((gf2*)(w + min(k0 + 128 * c + 2 * lane, H - 2)));
  };
  load_w(0);
  drain();
  float ss = 0.f;
  for (int k = 2 * lane; k < H; k += 128) {
    const h2 v = *reinterpret_cast<const h2*>(res + k);
    const float f0 = (float)v.x, f1 = (float)v.y;
    ss = ss + f0 * f0;
    ss = ss + f1 * f1;
  }
  ss = wave_sum(ss);
  const float rn = rsqrtf(ss / (float)H + eps);
  for (int k0 = 0; k0 < H; k0 += 128 * R) {
    if (k0) load_w(k0);
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const int k = k0 + 128 * c + 2 * lane;
      if (k < H) {
        const h2 v = *reinterpret_cast<const h2*>(res + k);
        const float n0 = ww[c].x * ((float)v.x * rn), n1 = ww[c].y * ((float)v.y * rn);
        *reinterpret_cast<h2*>(dst + k) = h2{(_Float16)n0, (_Float16)n1};
      }
    }
  }
}

// publish this CU's finished rows of phase ph (layer l): wait for the stream waves, store the rows
// write-through, drain, count in
__device__ __forceinline__ bool publish(const Args& a, Smem& sm, int l, int ph, int& done_total) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x;
  const int n = rows_of(a.R[ph], c, a.ncu);
  done_total += n;
  if (!wait_done(a, sm, done_total)) return false;
  const int per = ph == kGU ? 4 : 8;  // u32 words per row (8 or 16 halfs)
  _Float16* dst = ph == kQKV ? a.qkv
                  : ph == kO  ? a.h2
                  : ph == kGU ? a.gu
                  : (l == a.nl - 1 ? a.y : a.hb);
  for (int i = lane; i < n * per; i += 64) {
    const int row = i / per, w = i - row * per;
    const int r = c + row * a.ncu;
    const uint32_t v = reinterpret_cast<const uint32_t*>(&sm.ostage[row][0])[w];
    st_sc1(reinterpret_cast<uint32_t*>(dst + (int64_t)r * (2 * per)) + w, v);
  }
  drain();
  if (lane == 0) add_agent(cnt_phase(a, l, ph) + (c & (kShards - 1)), 1);
  return true;
}

// attention unit u = (kv head g, chunk ch): rows [ch * C, min(ch * C + C, L))
__device__ __forceinline__ int unit_cu(int u, int U, int G) { return (int)(((int64_t)u * G) / U); }

// 16-B segment s of cache row t sits at LDS segment s ^ (t & 15) (conflict-free row-per-lane reads)
__device__ __forceinline__ int kv_off(int t, int seg) { return t * kD + ((seg ^ (t & 15)) << 3); }

// LDS-DMA the chunk's cached rows (rows < L0) of layer l, head g
__device__ __forceinline__ void prefetch_kv(const Args& a, Smem& sm, const CLayer& ly, int g, int ch) {
  const int lane = threadIdx.x & 63;
  const int t0 = ch * a.C;
  const int n = min(a.C, a.L0 - t0);  // cached rows in the chunk (the new row comes later)
  if (n <= 0) return;
  // one instruction = 1 KB = 4 rows; lane l -> row 4i + l / 16, LDS segment l % 16, which holds
  // source segment (l % 16) ^ (row & 15)
  for (int kv = 0; kv < 2; ++kv) {
    const _Float16* src = (kv ? ly.vc : ly.kc) + (int64_t)g * a.kv_hs + (int64_t)t0 * kD;
    unsigned char* dst = reinterpret_cast<unsigned char*>(&sm.kvs[kv][0]);
    for (int i = 0; i < (n + 3) / 4; ++i) {
      const int t = min(4 * i + (lane >> 4), n - 1);
      const int seg = (lane & 15) ^ (t & 15);
      const _Float16* gp = src + (int64_t)t * kD + seg * 8;
      __builtin_amdgcn_global_load_lds((gbl_ptr)gp, (lds_ptr)(dst + i * 1024), 16, 0, 0);
    }
  }
}

__device__ __forceinline__ float h2f_lo(uint32_t w) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xFFFFu));
}
__device__ __forceinline__ float h2f_hi(uint32_t w) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
}

// one attention unit on the IO wave (its K / V rows already in LDS when `prefetched`); GRP query
// heads per KV head at compile time, so every loop below is branch-free and its LDS reads are
// issued in batches (a runtime head count left each read waiting for the previous one)
template <int GRP>
__device__ __forceinline__ bool attn_unit(const Args& a, Smem& sm, int l, int u, bool prefetched) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const CLayer& ly = layer_at(a, l);
  const int S = a.S, C = a.C;
  const int g = u / S, ch = u - g * S;
  const int L = a.L0 + 1;
  const int t0 = ch * C;
  const int n = min(C, L - t0);
  if (!prefetched) prefetch_kv(a, sm, ly, g, ch);
  // q heads g*GRP.., the new k / v row of head g (the q/k/v phase's output, other CUs' stores):
  // every word issued at once (one round trip), then RoPE
  const int64_t p = min(max(a.pos[0], (int64_t)0), a.cache_rows - 1);
  const float* cr = a.cosc + p * kD;
  const float* sr = a.sinc + p * kD;
  uint32_t qw0[GRP], qw1[GRP];
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    const _Float16* q = a.qkv + (int64_t)(g * GRP + h) * kD;
    qw0[h] = ld_sc1(q + (lane & ~1));
    qw1[h] = ld_sc1(q + 64 + (lane & ~1));
  }
  const _Float16* kp = a.qkv + a.H + (int64_t)g * kD;
  const _Float16* vp = a.qkv + a.H + a.Hkv * kD + (int64_t)g * kD;
  const uint32_t k0w = ld_sc1(kp + (lane & ~1)), k1w = ld_sc1(kp + 64 + (lane & ~1));
  const uint32_t v0w = ld_sc1(vp + (lane & ~1)), v1w = ld_sc1(vp + 64 + (lane & ~1));
  const float c0 = (float)(_Float16)cr[lane], c1 = (float)(_Float16)cr[lane + 64];
  const float s0 = (float)(_Float16)sr[lane], s1 = (float)(_Float16)sr[lane + 64];
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    const float x0 = (lane & 1) ? h2f_hi(qw0[h]) : h2f_lo(qw0[h]);
    const float x1 = (lane & 1) ? h2f_hi(qw1[h]) : h2f_lo(qw1[h]);
    // rotate_half: out[d] = x[d] c[d] - x[d + 64] s[d]; out[d + 64] = x[d + 64] c[d + 64] + x[d] s[d + 64]
    sm.qs[h][lane] = x0 * c0 + (-x1) * s0;
    sm.qs[h][lane + 64] = x1 * c1 + x0 * s1;
  }
  stamp(a, l, 14);
  const bool has_new = t0 + n == L;  // this chunk holds the new row L0
  if (has_new) {
    const float x0 = (lane & 1) ? h2f_hi(k0w) : h2f_lo(k0w);
    const float x1 = (lane & 1) ? h2f_hi(k1w) : h2f_lo(k1w);
    // fp16 ops, as the reference's k path (fp16 cos / sin)
    const _Float16 kn0 = (_Float16)((float)(_Float16)(x0 * c0) + (float)(_Float16)((-x1) * s0));
    const _Float16 kn1 = (_Float16)((float)(_Float16)(x1 * c1) + (float)(_Float16)(x0 * s1));
    const _Float16 vn0 = __builtin_bit_cast(_Float16, (uint16_t)((lane & 1) ? (v0w >> 16) : (v0w & 0xFFFFu)));
    const _Float16 vn1 = __builtin_bit_cast(_Float16, (uint16_t)((lane & 1) ? (v1w >> 16) : (v1w & 0xFFFFu)));
    sm.knew[lane] = kn0;
    sm.knew[lane + 64] = kn1;
    sm.vnew[lane] = vn0;
    sm.vnew[lane + 64] = vn1;
    // the cache row L0 for later steps (read by later launches only)
    const int64_t row = (int64_t)g * a.kv_hs + (int64_t)a.L0 * kD;
    ly.kc[row + lane] = kn0;
    ly.kc[row + lane + 64] = kn1;
    ly.vc[row + lane] = vn0;
    ly.vc[row + lane + 64] = vn1;
  }
  // the LDS-DMA rows have landed (vmcnt) and the new row joins them (swizzled like the DMA rows)
  drain();
  if (has_new) {
    const int t = n - 1;
    if (lane < 32) {
      const int kv = lane >> 4, sg = lane & 15;
      const _Float16* src = kv ? sm.vnew : sm.knew;
      *reinterpret_cast<uint4*>(&sm.kvs[kv][kv_off(t, sg)]) =
          *reinterpret_cast<const uint4*>(src + sg * 8);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes visible to this wave's reads
  stamp(a, l, 15);
  // scores: lane = row t (and t + 64 for 128-row chunks); fp32 dot products over the 128 dims
  float mloc[GRP];
#pragma unroll
  for (int h = 0; h < GRP; ++h) mloc[h] = -INFINITY;
  for (int tb = 0; tb < C; tb += 64) {
    const int t = tb + lane;
    const int tr = min(t, n - 1);  // rows past the chunk read its last row, then are masked
    float acc[GRP];
#pragma unroll
    for (int h = 0; h < GRP; ++h) acc[h] = 0.f;
    // 2 segments per step: a full unroll lets the scheduler hoist every q read (16 x GRP x 2
    // float4) and spill
#pragma unroll 2
    for (int seg = 0; seg < 16; ++seg) {
      const h8 kk = *reinterpret_cast<const h8*>(&sm.kvs[0][kv_off(tr, seg)]);
#pragma unroll
      for (int h = 0; h < GRP; ++h) {
        const float4 qa = *reinterpret_cast<const float4*>(&sm.qs[h][seg * 8]);
        const float4 qb = *reinterpret_cast<const float4*>(&sm.qs[h][seg * 8 + 4]);
        float s_ = acc[h];
        s_ = fmaf(qa.x, (float)kk[0], s_);
        s_ = fmaf(qa.y, (float)kk[1], s_);
        s_ = fmaf(qa.z, (float)kk[2], s_);
        s_ = fmaf(qa.w, (float)kk[3], s_);
        s_ = fmaf(qb.x, (float)kk[4], s_);
        s_ = fmaf(qb.y, (float)kk[5], s_);
        s_ = fmaf(qb.z, (float)kk[6], s_);
        s_ = fmaf(qb.w, (float)kk[7], s_);
        acc[h] = s_;
      }
    }
    const float mk = a.mask ? (float)a.mask[t0 + tr] : 0.f;
#pragma unroll
    for (int h = 0; h < GRP; ++h) {
      float s_ = acc[h] / a.scale_div + mk;
      s_ = (s_ != s_) ? s_ : fmaxf(s_, -3.402823466e38f);  // torch.max(w, finfo(fp32).min)
      if (t >= n) s_ = -INFINITY;
      sm.pb[h][t] = s_;
      mloc[h] = fmaxf(mloc[h], s_);
    }
  }
  stamp(a, l, 16);
  float m[GRP], lsum[GRP];
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    float v = mloc[h];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    m[h] = v;
  }
#pragma unroll
  for (int h = 0; h < GRP; ++h) lsum[h] = 0.f;
  for (int tb = 0; tb < C; tb += 64) {
    const int t = tb + lane;
#pragma unroll
    for (int h = 0; h < GRP; ++h) {
      const float e = t < n ? expf(sm.pb[h][t] - m[h]) : 0.f;  // rows past n: p = 0
      sm.pb[h][t] = e;
      lsum[h] += e;
    }
  }
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    float v = lsum[h];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    lsum[h] = v;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  stamp(a, l, 17);
  // P V: lane owns dims 2 * lane, 2 * lane + 1 (segment lane / 4 of each row), 8 rows per step
  // (rows past n: p = 0 times the chunk's last row)
  float o0[GRP], o1[GRP];
#pragma unroll
  for (int h = 0; h < GRP; ++h) o0[h] = o1[h] = 0.f;
  for (int tb = 0; tb < n; tb += 8) {
    uint32_t vw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      vw[j] = *reinterpret_cast<const uint32_t*>(
          &sm.kvs[1][kv_off(min(tb + j, n - 1), lane >> 2) + 2 * (lane & 3)]);
    float4 pa[GRP], pq[GRP];
#pragma unroll
    for (int h = 0; h < GRP; ++h) {
      pa[h] = *reinterpret_cast<const float4*>(&sm.pb[h][tb]);
      pq[h] = *reinterpret_cast<const float4*>(&sm.pb[h][tb + 4]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v0 = h2f_lo(vw[j]), v1 = h2f_hi(vw[j]);
#pragma unroll
      for (int h = 0; h < GRP; ++h) {
        const float4& pv = j < 4 ? pa[h] : pq[h];
        const float pp = (j & 3) == 0 ? pv.x : (j & 3) == 1 ? pv.y : (j & 3) == 2 ? pv.z : pv.w;
        o0[h] = fmaf(pp, v0, o0[h]);
        o1[h] = fmaf(pp, v1, o1[h]);
      }
    }
  }
  stamp(a, l, 18);
  const int64_t qh0 = (int64_t)g * GRP;  // first query head of the group
  if (S == 1) {
#pragma unroll
    for (int h = 0; h < GRP; ++h) {
      const _Float16 r0 = (_Float16)(o0[h] / lsum[h]), r1 = (_Float16)(o1[h] / lsum[h]);
      st_sc1(a.abuf + (qh0 + h) * kD + 2 * lane,
             (uint32_t)__builtin_bit_cast(uint16_t, r0) |
                 ((uint32_t)__builtin_bit_cast(uint16_t, r1) << 16));
    }
    drain();
    if (lane == 0) add_agent(cnt_attn(a, l), 1);
    return true;
  }
  // partials (sc1), count in; the last unit of the head merges
  float* pp = a.part + ((int64_t)(g * S + ch) * GRP) * (kD + 2);
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    float* ph = pp + h * (kD + 2);
    const unsigned long long ov = (unsigned long long)__builtin_bit_cast(uint32_t, o0[h]) |
                                  ((unsigned long long)__builtin_bit_cast(uint32_t, o1[h]) << 32);
    __hip_atomic_store((gu64*)(ph + 2 * lane), ov, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
      const unsigned long long mlv = (unsigned long long)__builtin_bit_cast(uint32_t, m[h]) |
                                     ((unsigned long long)__builtin_bit_cast(uint32_t, lsum[h]) << 32);
      __hip_atomic_store((gu64*)(ph + kD), mlv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  drain();
  int old = 0;
  if (lane == 0) old = add_agent(cnt_head(a, l, g), 1);
  old = __builtin_amdgcn_readfirstlane(old);
  stamp(a, l, 19);
  if (old != S - 1) return true;
  // merge (qlin_attn_decode's): weights w_j = exp(m_j - M_h), denominators sum_j w_j l_j over the
  // S partials j = s * GRP + h of each head.  Lane j of a 64-partial round holds partial j's (m, l)
  // (one round of 8-B loads; its head is lane % GRP), the head maxima / sums reduce over the lanes
  // of one head (xor butterflies over strides >= GRP), the weights go to LDS, then the partial
  // rows arrive in rounds of 32 8-B loads per lane
  const float* pg = a.part + (int64_t)g * S * GRP * (kD + 2);
  const int np = S * GRP;  // <= 512
  float* pbf = &sm.pb[0][0];
  float Ml = -INFINITY;
  for (int j0 = 0; j0 < np; j0 += 64) {
    const int j = min(j0 + lane, np - 1);
    const unsigned long long ml = ld_sc1_64(pg + (int64_t)j * (kD + 2) + kD);
    const float mj = j0 + lane < np ? __builtin_bit_cast(float, (uint32_t)ml) : -INFINITY;
    pbf[j0 + lane] = mj;
    pbf[512 + j0 + lane] = __builtin_bit_cast(float, (uint32_t)(ml >> 32));
    Ml = fmaxf(Ml, mj);
  }
#pragma unroll
  for (int o = 32; o >= GRP; o >>= 1) Ml = fmaxf(Ml, __shfl_xor(Ml, o));
  __builtin_amdgcn_s_waitcnt(0xc07f);
  float dl = 0.f;
  for (int j0 = 0; j0 < np; j0 += 64) {
    const float w = j0 + lane < np ? expf(pbf[j0 + lane] - Ml) : 0.f;
    dl += w * (j0 + lane < np ? pbf[512 + j0 + lane] : 0.f);
    pbf[j0 + lane] = w;
  }
#pragma unroll
  for (int o = 32; o >= GRP; o >>= 1) dl += __shfl_xor(dl, o);
  float den[GRP], acc0[GRP], acc1[GRP];
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    den[h] = __shfl(dl, h);
    acc0[h] = acc1[h] = 0.f;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  constexpr int SR = 32 / GRP;  // partial rows (s values) per round: 32 8-B loads per lane
  for (int s0 = 0; s0 < S; s0 += SR) {
    unsigned long long ov[SR][GRP];
#pragma unroll
    for (int k = 0; k < SR; ++k)
#pragma unroll
      for (int h = 0; h < GRP; ++h)
        ov[k][h] = ld_sc1_64(pg + ((int64_t)min(s0 + k, S - 1) * GRP + h) * (kD + 2) + 2 * lane);
#pragma unroll
    for (int k = 0; k < SR; ++k) {
#pragma unroll
      for (int h = 0; h < GRP; ++h) {
        const float w = s0 + k < S ? pbf[(s0 + k) * GRP + h] : 0.f;
        acc0[h] = fmaf(w, __builtin_bit_cast(float, (uint32_t)ov[k][h]), acc0[h]);
        acc1[h] = fmaf(w, __builtin_bit_cast(float, (uint32_t)(ov[k][h] >> 32)), acc1[h]);
      }
    }
  }
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    const _Float16 r0 = (_Float16)(acc0[h] / den[h]), r1 = (_Float16)(acc1[h] / den[h]);
    st_sc1(a.abuf + (qh0 + h) * kD + 2 * lane,
           (uint32_t)__builtin_bit_cast(uint16_t, r0) |
               ((uint32_t)__builtin_bit_cast(uint16_t, r1) << 16));
  }
  drain();
  if (lane == 0) add_agent(cnt_attn(a, l), 1);
  return true;
}

__device__ __forceinline__ bool attn_unit_g(const Args& a, Smem& sm, int l, int u, bool pre) {
  switch (a.grp) {
    case 1: return attn_unit<1>(a, sm, l, u, pre);
    case 2: return attn_unit<2>(a, sm, l, u, pre);
    case 4: return attn_unit<4>(a, sm, l, u, pre);
    default: return attn_unit<8>(a, sm, l, u, pre);
  }
}

__device__ __forceinline__ void io_wave(const Args& a, Smem& sm) {
  const int c = blockIdx.x;
  const int U = a.Hkv * a.S;
  int done_total = 0;
  for (int l = 0; l < a.nl; ++l) {
    const CLayer& ly = layer_at(a, l);
    stamp(a, l, 0);
    // --- q/k/v: the layer input h (launch input, or the previous layer's down output) + norm
    if (l == 0) {
      stage_norm<false>(sm.hres, sm.xbuf, a.x, ly.w_in, a.H, a.eps);
    } else {
      if (!wait_phase(a, sm, l - 1, kDN)) return;
      stage_norm<true>(sm.hres, sm.xbuf, a.hb, ly.w_in, a.H, a.eps);
    }
    __hip_atomic_store(&sm.xready, seq_of(l, kQKV), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    stamp(a, l, 1);
    // this CU's first attention unit of the layer: its cached K / V rows, early
    int u0 = -1;
    for (int u = 0; u < U; ++u)
      if (unit_cu(u, U, a.ncu) == c) { u0 = u; break; }
    if (u0 >= 0) prefetch_kv(a, sm, ly, u0 / a.S, u0 % a.S);
    if (!publish(a, sm, l, kQKV, done_total)) return;
    stamp(a, l, 2);
    // --- attention units of this CU
    if (u0 >= 0) {
      if (!wait_phase(a, sm, l, kQKV)) return;
      stamp(a, l, 3);
      for (int u = u0; u < U; ++u) {
        if (unit_cu(u, U, a.ncu) != c) continue;
        if (!attn_unit_g(a, sm, l, u, u == u0)) return;
      }
      stamp(a, l, 4);
    }
    // --- o_proj (+ residual h)
    if (!wait_count(a, sm, cnt_attn(a, l), a.Hkv)) return;
    stamp(a, l, 5);
    stage<true>(sm.xbuf, a.abuf, a.H);
    __hip_atomic_store(&sm.xready, seq_of(l, kO), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    stamp(a, l, 6);
    if (!publish(a, sm, l, kO, done_total)) return;
    stamp(a, l, 7);
    // --- gate/up (+ norm, SiLU * up)
    if (!wait_phase(a, sm, l, kO)) return;
    stamp(a, l, 8);
    stage_norm<true>(sm.h2res, sm.xbuf, a.h2, ly.w_post, a.H, a.eps);
    __hip_atomic_store(&sm.xready, seq_of(l, kGU), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    stamp(a, l, 9);
    if (!publish(a, sm, l, kGU, done_total)) return;
    stamp(a, l, 10);
    // --- down (+ residual h2)
    if (!wait_phase(a, sm, l, kGU)) return;
    stamp(a, l, 11);
    stage<true>(sm.xbuf, a.gu, a.I);
    __hip_atomic_store(&sm.xready, seq_of(l, kDN), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    stamp(a, l, 12);
    if (!publish(a, sm, l, kDN, done_total)) return;
    stamp(a, l, 13);
  }
}

// ---------------------------------------------------------------------------------------------
// stream waves
// ---------------------------------------------------------------------------------------------
// a wave's position in its tile sequence: layer, phase, flat index t of the CU's phase tiles
// (row-major over its rows), end of the wave's run in this phase
__device__ __forceinline__ void run_of(const Args& a, int ph, int wave, int& t, int& tend, int& T) {
  const int n = rows_of(a.R[ph], blockIdx.x, a.ncu);
  T = n * a.Kt[ph];
  t = (int)(((int64_t)wave * T) / kStream);
  tend = (int)(((int64_t)(wave + 1) * T) / kStream);
}

// the next non-empty run after (l, ph) of this wave; false at the end of the launch
__device__ __forceinline__ bool next_run(const Args& a, int wave, int& l, int& ph, int& t,
                                         int& tend, int& T) {
  for (;;) {
    if (++ph == kPhases) {
      ph = 0;
      if (++l == a.nl) return false;
    }
    run_of(a, ph, wave, t, tend, T);
    if (t < tend) return true;
  }
}

// load cursor: the tile whose lane pieces the next load() fetches.  Per tile only kt and, at a
// row end, two row pointers move; a run's operands come from the layer table through the
// constant address space (scalar loads: no vmcnt wait in the stream).  Past the wave's last tile
// (done) it cycles through that row's tiles: valid addresses that differ from load to load (a load
// the compiler can prove equal to the previous one becomes a copy of its result: a vmcnt(0) wait)
struct LoadCur {
  int l, ph, t, tend, T, kt, Kt, left;
  int64_t rstep_qw, rstep_sz;  // words between the CU's consecutive rows of this phase
  const gu32* row_qw;          // tile 0 of the current row (uniform; + lane * BITS at the load)
  const gu32* row_sz;          // (scale, zero) words of the current row (uniform; + n_in)
  bool done;
};

template <int BITS>
__device__ __forceinline__ void enter_run(const Args& a, LoadCur& c) {
  c.Kt = a.Kt[c.ph];
  const int Gs = a.Gs[c.ph];
  const int i = c.t / c.Kt;
  c.kt = c.t - i * c.Kt;
  const int64_t r = blockIdx.x + (int64_t)i * a.ncu;
  const CLayer& ly = layer_at(a, c.l);
  c.row_qw = (const gu32*)ly.qw[c.ph] + r * c.Kt * (64 * BITS);
  c.row_sz = (const gu32*)ly.sz[c.ph] + r * Gs * kTileN;
  c.rstep_qw = (int64_t)a.ncu * c.Kt * (64 * BITS);
  c.rstep_sz = (int64_t)a.ncu * Gs * kTileN;
}

template <int BITS>
__device__ __forceinline__ void advance_load(const Args& a, LoadCur& c, int wave) {
  if (c.done || --c.left == 0) {
    c.done = true;
    c.kt = c.kt + 1 == c.Kt ? 0 : c.kt + 1;
    return;
  }
  ++c.t;
  if (++c.kt == c.Kt) {
    c.kt = 0;
    c.row_qw += c.rstep_qw;
    c.row_sz += c.rstep_sz;
  }
  if (c.t == c.tend) {
    next_run(a, wave, c.l, c.ph, c.t, c.tend, c.T);  // left > 0: a run follows
    enter_run<BITS>(a, c);
  }
}

// compute cursor: the tile the next compute() multiplies, and where its item (a row's share of
// this wave) ends
struct CompCur {
  int l, ph, t, tend, T, kt, Kt, i;
};

__device__ __forceinline__ void enter_run(const Args& a, CompCur& c) {
  c.Kt = a.Kt[c.ph];
  c.i = c.t / c.Kt;
  c.kt = c.t - c.i * c.Kt;
}

// one tile on; true when the tile just passed ended an item (its row, or the wave's run)
__device__ __forceinline__ bool advance_comp(const Args& a, CompCur& c, int wave) {
  ++c.t;
  bool end = false;
  if (++c.kt == c.Kt) {
    c.kt = 0;
    ++c.i;
    end = true;
  }
  if (c.t == c.tend) {
    end = true;
    if (next_run(a, wave, c.l, c.ph, c.t, c.tend, c.T)) enter_run(a, c);
  }
  return end;
}

template <int BITS>
__device__ __forceinline__ Piece<BITS> load_piece_g(const gu32* p) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
  typedef __attribute__((address_space(1))) const u32x4 g4;
  typedef __attribute__((address_space(1))) const u32x2 g2;
  typedef __attribute__((address_space(1))) const u32x3 g3;
  Piece<BITS> c;
  if constexpr (BITS == 4) {
    const u32x4 v = __builtin_nontemporal_load((g4*)p);
    c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z; c.w[3] = v.w;
  } else if constexpr (BITS == 8) {
    const u32x4 v0 = __builtin_nontemporal_load((g4*)p);
    const u32x4 v1 = __builtin_nontemporal_load((g4*)(p + 4));
    c.w[0] = v0.x; c.w[1] = v0.y; c.w[2] = v0.z; c.w[3] = v0.w;
    c.w[4] = v1.x; c.w[5] = v1.y; c.w[6] = v1.z; c.w[7] = v1.w;
  } else if constexpr (BITS == 2) {
    const u32x2 v = __builtin_nontemporal_load((g2*)p);
    c.w[0] = v.x; c.w[1] = v.y;
  } else {
    const u32x3 v = __builtin_nontemporal_load((g3*)p);
    c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z;
  }
  return c;
}

template <int BITS, int GPT, int ZM, int PF>
__device__ __forceinline__ void stream_wave(const Args& a, Smem& sm, int wave) {
  const int lane = threadIdx.x & 63, n_in = lane & 15, q = lane >> 4;
  const int cu = blockIdx.x;
  int total = 0;  // this wave's tiles over the launch
  for (int ph = 0; ph < kPhases; ++ph) {
    int t, te, T;
    run_of(a, ph, wave, t, te, T);
    total += te - t;
  }
  total *= a.nl;
  if (total == 0) return;

  LoadCur lc;
  lc.l = 0;
  lc.ph = -1;
  lc.done = false;
  lc.left = total;
  next_run(a, wave, lc.l, lc.ph, lc.t, lc.tend, lc.T);  // total > 0: a run exists
  enter_run<BITS>(a, lc);
  CompCur cc;
  cc.l = lc.l;
  cc.ph = lc.ph;
  cc.t = lc.t;
  cc.tend = lc.tend;
  cc.T = lc.T;
  enter_run(a, cc);
  auto group_of_tile = [&](int kt) {
    return GPT == 1 ? (int)(((uint64_t)(uint32_t)kt * a.cmagic) >> 31) : kt * GPT;
  };
  WTile<BITS, GPT> wt[PF];
  auto load = [&](int u) {
    wt[u].pc = load_piece_g<BITS>(lc.row_qw + lc.kt * (64 * BITS) + lane * BITS);
    const gu32* sz = lc.row_sz + group_of_tile(lc.kt) * kTileN + n_in;
#pragma unroll
    for (int s = 0; s < GPT; ++s) wt[u].sz[s] = sz[s * kTileN];
    advance_load<BITS>(a, lc, wave);
  };

  const Magics mg = make_magics<BITS>();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int ready = 0;  // highest phase sequence known staged

  // flush the item the compute cursor just finished (row i of phase ph): lanes 0..15 hold the
  // row's 16 (partial) outputs in acc[0]
  auto flush = [&](int ph, int i, int T, int Kt) {
    const int lo = i * Kt, hi = lo + Kt;
    int nsplit = 0, j = 0;
#pragma unroll
    for (int w = 0; w < kStream; ++w) {
      const int b0 = (int)(((int64_t)w * T) / kStream), b1 = (int)(((int64_t)(w + 1) * T) / kStream);
      if (max(b0, lo) < min(b1, hi)) {
        if (w == wave) j = nsplit;
        ++nsplit;
      }
    }
    float v = acc[0];
    if (nsplit > 1) {
      if (lane < kTileN) sm.part[i][j][lane] = v;
      int old = 0;
      if (lane == 0)
        old = __hip_atomic_fetch_add(&sm.rowcnt[i], 1, __ATOMIC_ACQ_REL,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
      old = __builtin_amdgcn_readfirstlane(old);
      if (old != nsplit - 1) return;
      // the last piece: sum the pieces in k order
      float s_ = lane < kTileN ? sm.part[i][0][lane] : 0.f;
      for (int jj = 1; jj < nsplit; ++jj) s_ += lane < kTileN ? sm.part[i][jj][lane] : 0.f;
      v = s_;
      if (lane == 0) sm.rowcnt[i] = 0;
    }
    const int r = cu + i * a.ncu;
    const float t16 = (float)(_Float16)v;  // F.linear's fp16 output
    if (ph == kGU) {
      // interleaved gate rows (lanes 0-7) and up rows (lanes 8-15): silu(gate) * up
      const float up = __shfl(t16, (lane & 7) + 8);
      if (lane < 8) sm.ostage[i][lane] = (_Float16)(silu_rn16(t16) * up);
    } else if (lane < kTileN) {
      float o = t16;
      if (ph == kO) o = (float)sm.hres[r * kTileN + lane] + t16;
      if (ph == kDN) o = (float)sm.h2res[r * kTileN + lane] + t16;
      sm.ostage[i][lane] = (_Float16)o;
    }
    if (lane == 0)
      __hip_atomic_fetch_add(&sm.ndone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };

  // compute slot u (the compute cursor's tile).  After an abort (a timed-out wait anywhere) the
  // waits return at once and the wave runs out its (valid, bounded) tile sequence on garbage: an
  // early exit from this loop makes hipcc drain vmcnt at every tile
  auto compute = [&](int u) {
    const int seq = seq_of(cc.l, cc.ph);
    if (__builtin_expect(seq > ready, 0)) {
      wait_ready(sm, seq);
      ready = seq;
    }
    const _Float16* xb = sm.xbuf + cc.kt * kTileK + 8 * q;
    h8 xa[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) xa[s] = *reinterpret_cast<const h8*>(xb + 32 * s);
    auto step = [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      uint32_t v[4];
      const GroupQ gq = make_group_w<BITS, ZM>(wt[u].sz[S * GPT / 4]);
      dequant_step<BITS, ZM, S>(wt[u].pc, mg, gq, v);
      const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    const int ph = cc.ph, i = cc.i, T = cc.T, Kt = cc.Kt;
    if (DECODE_TRACE && wave == 0) {
      if (cc.t == (int)(((int64_t)wave * T) / kStream)) stamp(a, cc.l, 20 + 2 * ph);
      if (cc.t + 1 == cc.tend) stamp(a, cc.l, 21 + 2 * ph);
    }
    if (__builtin_expect(advance_comp(a, cc, wave), 0)) {
      flush(ph, i, T, Kt);
      acc = f4{0.f, 0.f, 0.f, 0.f};
    }
  };

  // every slot is loaded unconditionally (the load cursor cycles through the wave's last row once
  // it is past its last tile), so hipcc counts the loads with vmcnt(N) instead of draining at
  // each branch
#pragma unroll
  for (int u = 0; u < PF; ++u) load(u);
  for (int base = 0; base < total; base += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (base + u < total) compute(u);
      load(u);
    }
  }
}

template <int BITS, int GPT, int ZM>
__global__ __launch_bounds__(64 * kWaves) void decode_kernel(const Args a) {
  __shared__ Smem sm;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x == 0) {
    sm.ndone = 0;
    sm.xready = 0;
    sm.abort_ = 0;
  }
  if (threadIdx.x < kMaxRows) sm.rowcnt[threadIdx.x] = 0;
  __syncthreads();
  if (DECODE_STREAM_ONLY && wave == 0) {
    __hip_atomic_store(&sm.xready, 1 << 30, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return;
  }
  if (wave == 0) {
    // the IO wave's serial work (staging, norms, attention, publishing) is every CU's critical
    // path; the stream wave sharing its SIMD yields issue slots to it
    __builtin_amdgcn_s_setprio(DECODE_IO_PRIO);
    io_wave(a, sm);
  }
  else stream_wave<BITS, GPT, ZM, DECODE_PF>(a, sm, wave - 1);
}

int cu_count_cached() { return qlin::device_cu_count(); }

struct Dims {
  int64_t H, I;
  int Hq, Hkv, D, nl;
};

int64_t cnt_stride_of(const Dims& d) { return kPhases * kShards + 1 + d.Hkv; }

struct WsLayout {
  int64_t cnt_bytes, qkv, abuf, h2, gu, hb, part, trace, total;
};

int64_t up256(int64_t v) { return (v + 255) / 256 * 256; }

WsLayout ws_layout(const Dims& d, int64_t max_L) {
  WsLayout w;
  const int grp = d.Hq / d.Hkv;
  const int64_t Smax = (max_L + 63) / 64;
  w.cnt_bytes = up256((1 + d.nl * cnt_stride_of(d)) * 4);
  w.qkv = w.cnt_bytes;
  w.abuf = w.qkv + up256((d.H + 2 * d.Hkv * d.D) * 2);
  w.h2 = w.abuf + up256(d.H * 2);
  w.gu = w.h2 + up256(d.H * 2);
  w.hb = w.gu + up256(d.I * 2);
  w.part = w.hb + up256(d.H * 2);
  w.trace = w.part + up256((int64_t)d.Hkv * Smax * grp * (kD + 2) * 4);
  w.total = w.trace + (DECODE_TRACE ? up256((int64_t)d.nl * kEv * cu_count_cached() * 8) : 0);
  return w;
}

bool dims_ok(const Dims& d) {
  return d.nl >= 1 && d.nl <= 4096 && d.D == kD && d.Hq > 0 && d.Hkv > 0 && d.Hq % d.Hkv == 0 &&
         d.Hq / d.Hkv <= kMaxGrp && d.H == (int64_t)d.Hq * kD && d.H <= kMaxH &&
         d.H % kTileK == 0 && d.I > 0 && d.I <= kMaxX && d.I % kTileK == 0;
}

}  // namespace

extern "C" int64_t qlin_decode_workspace_bytes(int n_layers, int64_t H, int64_t I, int Hq,
                                               int Hkv, int D, int64_t max_L) {
  const Dims d{H, I, Hq, Hkv, D, n_layers};
  if (!dims_ok(d) || max_L < 1 || max_L > kMaxL) return -1;
  return ws_layout(d, max_L).total;
}

extern "C" int qlin_decode_supported(int n_layers, int64_t H, int64_t I, int Hq, int Hkv, int D,
                                     int bits, int group, int flags) {
  const Dims d{H, I, Hq, Hkv, D, n_layers};
  if (!dims_ok(d)) return 0;
  if (!(bits == 2 || bits == 3 || bits == 4 || bits == 8)) return 0;
  if (!(group % kTileK == 0 || group == 64)) return 0;
  if (H % group || I % group) return 0;
  if (flags & QLIN_WIDE_ZERO) return 0;
  const int G = cu_count_cached();
  const int64_t R[kPhases] = {(H + 2 * Hkv * D) / kTileN, H / kTileN, 2 * I / kTileN, H / kTileN};
  for (int p = 0; p < kPhases; ++p)
    if ((R[p] + G - 1) / G > kMaxRows) return 0;
  return 1;
}

extern "C" int qlin_decode_llama_f16(const void* layers, int n_layers, int64_t H, int64_t I,
                                     int Hq, int Hkv, int D, int bits, int group, int flags,
                                     float eps, const uint16_t* x, uint16_t* y,
                                     const float* cos_cache, const float* sin_cache,
                                     int64_t cache_rows, const int64_t* position, int64_t L0,
                                     int64_t kv_rows, const uint16_t* mask, float scale_div,
                                     void* workspace, int64_t workspace_bytes, void* stream) {
  const Dims d{H, I, Hq, Hkv, D, n_layers};
  if (!layers || !x || !y || !cos_cache || !sin_cache || !position || !workspace ||
      !qlin_decode_supported(n_layers, H, I, Hq, Hkv, D, bits, group, flags) || L0 < 0 ||
      L0 + 1 > kMaxL || kv_rows < L0 + 1 || cache_rows < 1 || !(eps >= 0.f) ||
      !(scale_div > 0.f) || ((uintptr_t)x & 15) || ((uintptr_t)y & 3))
    return QLIN_EINVAL;
  const WsLayout w = ws_layout(d, L0 + 1);
  if (workspace_bytes < w.total || ((uintptr_t)workspace & 255)) return QLIN_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int G = cu_count_cached();
  Args a;
  a.layers = (const Layer*)layers;
  a.nl = n_layers;
  a.H = (int)H;
  a.I = (int)I;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.grp = Hq / Hkv;
  a.Nqkv = (int)(H + 2 * Hkv * D);
  a.ncu = G;
  a.R[kQKV] = a.Nqkv / kTileN;
  a.R[kO] = (int)(H / kTileN);
  a.R[kGU] = (int)(2 * I / kTileN);
  a.R[kDN] = (int)(H / kTileN);
  a.Kt[kQKV] = a.Kt[kO] = a.Kt[kGU] = (int)(H / kTileK);
  a.Kt[kDN] = (int)(I / kTileK);
  a.Gs[kQKV] = a.Gs[kO] = a.Gs[kGU] = (int)(H / group);
  a.Gs[kDN] = (int)(I / group);
  const uint64_t cg = group % kTileK == 0 ? (uint64_t)(group / kTileK) : 1;
  a.cmagic = (uint32_t)(((1ull << 31) + cg - 1) / cg);
  a.eps = eps;
  a.scale_div = scale_div;
  a.x = (const _Float16*)x;
  a.y = (_Float16*)y;
  a.cosc = cos_cache;
  a.sinc = sin_cache;
  a.cache_rows = cache_rows;
  a.pos = position;
  a.L0 = (int)L0;
  a.kv_hs = kv_rows * D;
  a.mask = (const _Float16*)mask;
  const int64_t L = L0 + 1;
  a.C = (int64_t)Hkv * ((L + 63) / 64) <= G ? 64 : 128;
  a.S = (int)((L + a.C - 1) / a.C);
  unsigned char* ws = (unsigned char*)workspace;
  a.cnt = (int*)ws;
  a.cnt_stride = (int)cnt_stride_of(d);
  a.qkv = (_Float16*)(ws + w.qkv);
  a.abuf = (_Float16*)(ws + w.abuf);
  a.h2 = (_Float16*)(ws + w.h2);
  a.gu = (_Float16*)(ws + w.gu);
  a.hb = (_Float16*)(ws + w.hb);
  a.part = (float*)(ws + w.part);
  a.trace = (unsigned long long*)(ws + w.trace);
  hipError_t e = hipMemsetAsync(ws, 0, (size_t)w.cnt_bytes, st);
  if (e != hipSuccess) return (int)e;
  const int zm = zero_mode(flags);
#define QLIN_DK(B, GP, Z) \
  hipLaunchKernelGGL((decode_kernel<B, GP, Z>), dim3(G), dim3(64 * kWaves), 0, st, a)
#define QLIN_DG(B, Z)                  \
  if (group % kTileK == 0) QLIN_DK(B, 1, Z); \
  else QLIN_DK(B, 2, Z)
#define QLIN_DB(B)                                   \
  if (zm == kZFloat) { QLIN_DG(B, kZFloat); }        \
  else { QLIN_DG(B, kZNarrow); }                     \
  break
  switch (bits) {
    case 2: QLIN_DB(2);
    case 3: QLIN_DB(3);
    case 4: QLIN_DB(4);
    default: QLIN_DB(8);
  }
#undef QLIN_DB
#undef QLIN_DG
#undef QLIN_DK
  return (int)hipGetLastError();
}
