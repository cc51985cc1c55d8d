// qlin_decode_fused.hip — the decoder layer's input RMSNorm + fused q/k/v projection AND its decode
// attention (RoPE, KV-cache append, split-L attention) as ONE launch for one token row, gfx950.
//
// Replaces, for q_len == 1, models/int_llama_layer.py:113-165 of the reference (input_layernorm ->
// q_proj / k_proj / v_proj -> rotary_emb + apply_rotary_pos_emb -> torch.cat of the cache ->
// repeat_kv -> QK^T / sqrt(d) + mask -> softmax -> PV): the same arithmetic as the two launches
// qlin_rmsnorm_linear_ep_f16 (q/k/v) and qlin_attn_decode_rope (attention), which it runs as two
// kinds of blocks of one grid.
//
// Why one launch: the attention of KV head h needs only its own 48 of q/k/v's 384 row tiles (4
// query heads, its k and v rows: LLaMA3-8B), and ~2.1 MB of cached K / V rows that do not depend on
// this step at all.  Two launches serialise the cache reads behind the whole projection and pay a
// kernel boundary; here the attention blocks issue their cache-row loads at once and wait only for
// their head's row tiles (a head-local hand-off, never a grid barrier):
//   * blocks [0, 384): the fast GEMV body (qlin_gemv_fast.h) for row tile qkv_tile(b) — the tiles
//     ordered head by head, so head 0's rows are first — which stores its 16 outputs with
//     agent-scope (sc1) 4-byte stores, drains them (vmcnt) and adds 1 to the head's ready count
//     (agent-scope atomic);
//   * blocks [384, 384 + Hkv * S): the split-L attention body (qlin_attn_decode.h, HO) on 4 of the
//     block's 8 waves (the other 4 end; s_barrier waits for the surviving waves only), which
//     issues its K / V rows, then polls the head's count with agent-scope loads (one lane, s_sleep
//     between polls), then reads its q / k / v rows with agent-scope loads — MI355X_MICROARCH.md
//     hand-off table, row 1.  The head's merging block (or its only block) zeroes the count for
//     the next launch (graph replays).
// Producers come first in the grid and never wait, so every consumer's producers are dispatched
// before it (no dependency on co-residency); the poll is bounded regardless (a launch whose
// producers never ran ends with wrong output instead of a hang).
#include <stdlib.h>

#include "qlin_gemv_fast.h"
#include "qlin_attn_decode.h"
#include "../../include/qlin_gfx950.h"

using namespace qlin_gv;

namespace {

struct QkvMap {
  int per_head;  // row tiles a KV head's attention needs: GRP q heads + its k and v rows
  int qT, kT;    // q row tiles per KV head (GRP * D / 16), k (= v) row tiles per KV head (D / 16)
  int q_tiles, k_tiles;  // row tiles of all q rows, of all k rows
  int dbg;  // DEV ablation (QLIN_QKV_ATTN_DBG): 1 consumers exit, 2 consumers skip the wait, 4
            // producers exit -- wrong results, timing only
};

__device__ __forceinline__ int qkv_tile(int b, const QkvMap& m) {
  const int h = b / m.per_head, j = b - h * m.per_head;
  if (j < m.qT) return h * m.qT + j;
  if (j < m.qT + m.kT) return m.q_tiles + h * m.kT + (j - m.qT);
  return m.q_tiles + m.k_tiles + h * m.kT + (j - m.qT - m.kT);
}

constexpr int kFusedGrp = 4;   // query heads per KV head (LLaMA3-8B); other groups: two launches
constexpr int kFusedWaves = 8; // the fast GEMV's waves at q/k/v's shape (fast_geometry)

// two 8-wave blocks per CU (4 waves per SIMD: <= 128 VGPRs), so the 384 GEMV blocks and the
// attention blocks are resident at once (the attention body alone takes 148 VGPRs: its PV batch
// is smaller here, RB = 4)
template <int BITS, int GPT, int ZM, int PF>
__global__ __launch_bounds__(64 * kFusedWaves) __attribute__((amdgpu_waves_per_eu(4)))
void qkv_attn_kernel(const FastArgs f,
                                                                     const AttnArgs A,
                                                                     const QkvMap m, int nprod) {
  const int b = blockIdx.x;
  if (b < nprod) {
    if (m.dbg & 4) return;
    gemv_fast_body<BITS, 1, GPT, ZM, kEpNone, PF, kNwF16, true>(f, qkv_tile(b, m),
                                                                A.ready + b / m.per_head);
    return;
  }
  if (threadIdx.x >= kThreads) return;  // wave-uniform: the attention body runs on 4 waves
  if (m.dbg & 1) return;
  const int c = b - nprod;
  if (m.dbg & 2) {
    AttnArgs A2 = A;
    A2.ready_need = 0;
    attn_decode_body<kFusedGrp, true, true>(A2, c % A.Hkv, c / A.Hkv);
    return;
  }
  attn_decode_body<kFusedGrp, true, true>(A, c % A.Hkv, c / A.Hkv);
}

struct FusedPlan {
  int W, lw, tpw, PF;
  Split sp;
  QkvMap map;
  int nprod;
};

// the shapes the fused launch takes (else QLIN_EINVAL: the caller runs the two launches)
bool fused_plan(int Hq, int Hkv, int D, int64_t K, int bits, int group, int64_t L, FusedPlan& p) {
  if (D != kD || Hkv < 1 || Hq != kFusedGrp * Hkv || L < 1 || L > kMaxL || K < kTileK ||
      K % kTileK || K > (1 << 20) || !valid_layout((int64_t)(Hq + 2 * Hkv) * D, K, bits, group) ||
      !group_fast((int)K, group))
    return false;
  const int64_t N = (int64_t)(Hq + 2 * Hkv) * D;
  const int Nt = (int)(N / kTileN), Kt = (int)(K / kTileK);
  if (!fast_geometry(Nt, Kt, p.W, p.lw, p.tpw) || p.W != kFusedWaves || p.tpw > 4 || p.tpw < 3)
    return false;
  p.PF = 4;
  // one pass of kSub rows per attention block (its K / V stage in LDS holds one pass)
  p.sp = Split{kSub, (int)((L + kSub - 1) / kSub)};
  if (p.sp.S > kMaxSplit) return false;
  p.map.qT = kFusedGrp * D / kTileN;
  p.map.kT = D / kTileN;
  p.map.per_head = p.map.qT + 2 * p.map.kT;
  p.map.q_tiles = Hq * D / kTileN;
  p.map.k_tiles = Hkv * D / kTileN;
  p.nprod = Nt;
  const char* dbg = getenv("QLIN_QKV_ATTN_DBG");
  p.map.dbg = dbg ? atoi(dbg) : 0;
  return true;
}

}  // namespace

extern "C" int qlin_qkv_attn_supported(int Hq, int Hkv, int D, int64_t K, int bits, int group,
                                       int flags, int64_t L) {
  FusedPlan p;
  return (flags & QLIN_NORM_W16) && fused_plan(Hq, Hkv, D, K, bits, group, L, p) ? 1 : 0;
}

extern "C" int64_t qlin_qkv_attn_partials_bytes(int Hq, int Hkv, int64_t L) {
  if (Hkv < 1 || Hq != kFusedGrp * Hkv || L < 1 || L > kMaxL) return -1;
  const int64_t S = (L + kSub - 1) / kSub;
  return S > 1 ? (int64_t)Hkv * S * kFusedGrp * (kD + 2) * 4 : 0;
}

extern "C" int qlin_qkv_attn_decode_f16(
    const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
    const uint16_t* norm_weight, float eps, uint16_t* qkv_out, const float* cos_cache,
    const float* sin_cache, int64_t cache_rows, const int64_t* position_ids, uint16_t* k_cache,
    uint16_t* v_cache, int64_t kv_head_stride, const uint16_t* mask, void* out, int out_dtype,
    int Hq, int Hkv, int64_t L, int D, int64_t K, int bits, int group, float scale_div,
    float* partials, int32_t* counters, const int32_t* len, void* stream) {
  FusedPlan p;
  if (!qweight || !qsz || !x || !norm_weight || !qkv_out || !cos_cache || !sin_cache ||
      !k_cache || !v_cache || !out || !counters || !(flags & QLIN_NORM_W16) ||
      (out_dtype != QLIN_F32 && out_dtype != QLIN_F16) || cache_rows <= 0 || !(eps >= 0.f) ||
      !(scale_div > 0.f) || ((uintptr_t)norm_weight & 3) || ((uintptr_t)x & 3) ||
      ((uintptr_t)qkv_out & 3) || (len && (!position_ids || mask)) ||
      !fused_plan(Hq, Hkv, D, K, bits, group, L, p) || kv_head_stride < L * D ||
      kv_head_stride % 8 || (p.sp.S > 1 && !partials))
    return QLIN_EINVAL;
  const int64_t N = (int64_t)(Hq + 2 * Hkv) * D;
  FastArgs f;
  f.qw = qweight;
  f.qsz = qsz;
  f.x = (const _Float16*)x;
  f.bias = nullptr;
  f.res = nullptr;
  f.y = (_Float16*)qkv_out;
  f.M = 1;
  f.N = (int)N;
  f.K = (int)K;
  f.Kt = (int)(K / kTileK);
  f.G = (int)(K / group);
  f.W = p.W;
  f.lw = p.lw;
  f.cmagic = tile_group_magic(group);
  f.nw = norm_weight;
  f.eps = eps;
  const _Float16* qkv = (const _Float16*)qkv_out;
  const RopeIn ri{qkv, N, qkv + (int64_t)Hq * D, N, qkv + (int64_t)(Hq + Hkv) * D, N, cos_cache,
                  sin_cache, cache_rows, position_ids, 0, (_Float16*)k_cache, (_Float16*)v_cache};
  float* part_o = p.sp.S > 1 ? partials : nullptr;
  float* part_ml = p.sp.S > 1 ? part_o + (int64_t)Hkv * p.sp.S * kFusedGrp * kD : nullptr;
  const AttnArgs A{nullptr, (const _Float16*)k_cache, (const _Float16*)v_cache,
                   (const _Float16*)mask, out, out_dtype == QLIN_F16, Hq, Hkv, (int)L,
                   kv_head_stride, p.sp.chunk, p.sp.S, scale_div, (int*)counters, part_o,
                   part_ml, ri, len, (int*)counters + Hkv, p.map.per_head};
  {
    const char* ps = getenv("QLIN_QKV_POLL_SLEEPS");  // DEV
    const char* pr = getenv("QLIN_QKV_POLL_RMW");
    AttnArgs& Am = const_cast<AttnArgs&>(A);
    Am.poll_sleeps = ps ? atoi(ps) : 1;
    Am.poll_rmw = pr ? atoi(pr) : 0;
  }
  const dim3 grid((unsigned)(p.nprod + Hkv * p.sp.S));
  hipStream_t st = (hipStream_t)stream;
  const int zm = zero_mode(flags);
#define QLIN_FK(B, G, Z) \
  hipLaunchKernelGGL((qkv_attn_kernel<B, G, Z, 4>), grid, dim3(64 * kFusedWaves), 0, st, f, A, \
                     p.map, p.nprod)
#define QLIN_FZ(B, G)                        \
  if (zm == kZFloat) QLIN_FK(B, G, kZFloat); \
  else if (zm == kZWide) QLIN_FK(B, G, kZWide); \
  else QLIN_FK(B, G, kZNarrow)
#define QLIN_FG(B)                                 \
  if (group % kTileK == 0) { QLIN_FZ(B, 1); }      \
  else if (group == 64) { QLIN_FZ(B, 2); }         \
  else { QLIN_FZ(B, 4); }                          \
  break
  switch (bits) {
    case 2: QLIN_FG(2);
    case 3: QLIN_FG(3);
    case 4: QLIN_FG(4);
    default: QLIN_FG(8);
  }
#undef QLIN_FG
#undef QLIN_FZ
#undef QLIN_FK
  return (int)hipGetLastError();
}
