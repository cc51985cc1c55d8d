// qlin_attn.hip — fused decode attention (one query token) for the quantized LLaMA layer, gfx950.
//
// Replaces, for q_len == 1, the attention core of QuantLlamaAttention.forward
// (models/int_llama_layer.py:137-165 of the reference): repeat_kv of the fp16 K/V cache, the fp32
// QK^T bmm, the division by sqrt(head_dim), the additive mask with the finfo.min clamp, the fp32
// softmax and the fp32 PV bmm — six PyTorch kernels plus two K/V expansions and two fp16 -> fp32
// copies of the whole cache per layer and token — with one kernel that reads each K/V row once
// for all the query heads of its group (GQA).
//
// Split-L ("flash-decoding"): the grid is (B * Hkv) x S blocks, each over a chunk of `chunk`
// cache positions (a multiple of 64, chosen on the host for ~kTargetBlocks blocks: one sequence
// at batch 1 has only Hkv = 8 KV heads, far too few blocks to pull the cache at HBM rate).  A
// block writes its chunk's (max, sum, unnormalised P V) to `partials`; the last block of a
// (b, kv head) to count in merges the S partials and resets the counter, so the kernel is
// graph-replayable with no memset.
//
// Latency: decode attention at batch 1 is a chain of dependent memory round trips, not a bandwidth
// problem.  A block issues the q side first (ROPE: the q / k / v rows of the step and the cos /
// sin rows at the guessed position L - 1, the new token's cache row; a padded sequence whose
// position id differs redoes RoPE on its own path), then the K rows, V rows and mask of its first
// 64 positions, so its first wait covers the q side only and no load waits on another one (the
// position id -> cos / sin chain cost 1 us: profiles/r4_attn_decode.txt); mask values are loaded
// unconditionally (a load under a branch gets its own full wait).  The merge reads the partials
// with all 256 threads (one coalesced 256-B row per wave and load).
// One 1024-thread block per (b, kv head) streaming all 513 rows (no merge) and 256-row blocks
// were both slower: one CU takes ~4-6 us to land 256 KB of cold K / V, more than the merge chain
// (tools/dev/cu_bw.hip; profiles/r4_attn_decode.txt).
//
// Cross-block hand-off: the partials are written and read with agent-scope (sc1) accesses and the
// writer drains its stores (vmcnt) before the block barrier and the counter atomic.  A device-scope
// __threadfence() would do the same with an L2 writeback + invalidate per wave (buffer_wbl2 /
// buffer_inv), which costs 2-5x the kernel at batch 1 on the 8-XCD part (tools/dev/attn_ab.py).
//
// Arithmetic: fp32 throughout, as the reference (q is fp32, K/V are upcast exactly); dot products
// and sums run in a different order than hipBLASLt's bmm and the softmax is merged across chunks
// (exp(m_c - M) rescaling), so results agree with the reference to fp32 rounding, not bit for bit.
#include "qlin_common.h"  // QLIN_OK / QLIN_EINVAL
#include "qlin_attn_decode.h"

#include "../../include/qlin_gfx950.h"

namespace {

template <int GRP, bool ROPE = false>
__global__ __launch_bounds__(kThreads) void attn_decode_kernel(const AttnArgs A) {
  attn_decode_body<GRP, ROPE>(A, blockIdx.x, blockIdx.y);
}

int launch_decode(const float* q, const uint16_t* k, const uint16_t* v, const uint16_t* mask,
                  void* out, int out_dtype, int64_t B, int Hq, int Hkv, int64_t L, int64_t kv_hs,
                  float scale_div, float* part_o, float* part_ml, int32_t* counters,
                  const Split& sp, hipStream_t st, const RopeIn& ri, const int* len = nullptr) {
  const dim3 grid((unsigned)(B * Hkv), (unsigned)sp.S);
  const int grp = Hq / Hkv;
  AttnArgs A{q, (const _Float16*)k, (const _Float16*)v, (const _Float16*)mask, out,
                   out_dtype == QLIN_F16, Hq, Hkv, (int)L, kv_hs, sp.chunk, sp.S, scale_div,
                   (int*)counters, part_o, part_ml, ri, len, nullptr, 0};
#define QLIN_A(G, R) \
  hipLaunchKernelGGL((attn_decode_kernel<G, R>), grid, dim3(kThreads), 0, st, A)
#define QLIN_AR(G)                \
  if (ri.q16) QLIN_A(G, true);    \
  else QLIN_A(G, false);          \
  break
  switch (grp) {
    case 1: QLIN_AR(1);
    case 2: QLIN_AR(2);
    case 4: QLIN_AR(4);
    case 8: QLIN_AR(8);
    default: return QLIN_EINVAL;
  }
#undef QLIN_AR
#undef QLIN_A
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int64_t qlin_attn_decode_partials_bytes(int64_t B, int Hq, int Hkv, int64_t L) {
  if (B < 0 || Hq <= 0 || Hkv <= 0 || Hq % Hkv || L <= 0 || L > kMaxL) return -1;
  if (B == 0) return 0;
  const Split sp = choose_split(B, Hkv, L);
  const int64_t heads = B * Hkv, grp = Hq / Hkv;
  if (sp.S == 1) return 0;
  return heads * sp.S * grp * (kD + 2) * 4;
}

extern "C" int qlin_attn_decode(const float* q, const uint16_t* k, const uint16_t* v,
                                const uint16_t* mask, void* out, int out_dtype, int64_t B,
                                int Hq, int Hkv,
                                int64_t L, int D, int64_t kv_head_stride, float scale_div,
                                float* partials, int32_t* counters, void* stream) {
  if (!q || !k || !v || !out || (out_dtype != QLIN_F32 && out_dtype != QLIN_F16) || B < 0 ||
      Hq <= 0 || Hkv <= 0 || Hq % Hkv || L <= 0 ||
      L > kMaxL || D != kD || B * Hkv > 0x7fffffff ||
      (kv_head_stride != 0 && (kv_head_stride < L * kD || kv_head_stride % 8)))
    return QLIN_EINVAL;
  const int64_t kv_hs = kv_head_stride ? kv_head_stride : L * kD;
  const int grp = Hq / Hkv;
  if (grp > kMaxGroup) return QLIN_EINVAL;
  if (B == 0) return QLIN_OK;
  const Split sp = choose_split(B, Hkv, L);
  if (sp.S > kMaxSplit || sp.S > 65535) return QLIN_EINVAL;
  const int64_t heads = B * Hkv;
  float *part_o = nullptr, *part_ml = nullptr;
  if (sp.S > 1) {
    if (!partials || !counters) return QLIN_EINVAL;
    part_o = partials;
    part_ml = part_o + heads * sp.S * grp * kD;
  }
  return launch_decode(q, k, v, mask, out, out_dtype, B, Hq, Hkv, L, kv_hs, scale_div, part_o,
                       part_ml, counters, sp, (hipStream_t)stream, RopeIn{});
}

static int attn_decode_rope_impl(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                                     int64_t k_row_stride, const uint16_t* v,
                                     int64_t v_row_stride, const float* cos_cache,
                                     const float* sin_cache, int64_t cache_rows,
                                     const int64_t* position_ids, int64_t pos_batch_stride,
                                     uint16_t* k_cache, uint16_t* v_cache, int64_t kv_head_stride,
                                     const uint16_t* mask, void* out, int out_dtype, int64_t B,
                                     int Hq, int Hkv, int64_t L, int D, float scale_div,
                                     float* partials, int32_t* counters, void* stream,
                                     const int32_t* len = nullptr) {
  // position_ids NULL: cos_cache / sin_cache are the rows of the step's position (B == 1)
  if (!position_ids && B > 1) return QLIN_EINVAL;
  if (!q || !k || !v || !cos_cache || !sin_cache || !k_cache || !v_cache ||
      !out || (out_dtype != QLIN_F32 && out_dtype != QLIN_F16) || B < 0 || Hq <= 0 ||
      Hkv <= 0 || Hq % Hkv || L <= 0 || L > kMaxL || D != kD || B * Hkv > 0x7fffffff ||
      q_row_stride < (int64_t)Hq * kD || k_row_stride < (int64_t)Hkv * kD ||
      v_row_stride < (int64_t)Hkv * kD || cache_rows <= 0 || pos_batch_stride < 0 ||
      kv_head_stride < L * kD || kv_head_stride % 8)
    return QLIN_EINVAL;
  const int grp = Hq / Hkv;
  if (grp > kMaxGroup) return QLIN_EINVAL;
  if (B == 0) return QLIN_OK;
  const Split sp = choose_split(B, Hkv, L);
  if (sp.S > kMaxSplit || sp.S > 65535) return QLIN_EINVAL;
  const int64_t heads = B * Hkv;
  float *part_o = nullptr, *part_ml = nullptr;
  if (sp.S > 1) {
    if (!partials || !counters) return QLIN_EINVAL;
    part_o = partials;
    part_ml = part_o + heads * sp.S * grp * kD;
  }
  const RopeIn ri{(const _Float16*)q, q_row_stride, (const _Float16*)k, k_row_stride,
                  (const _Float16*)v, v_row_stride, cos_cache, sin_cache, cache_rows,
                  position_ids, pos_batch_stride, (_Float16*)k_cache, (_Float16*)v_cache};
  return launch_decode(nullptr, k_cache, v_cache, mask, out, out_dtype, B, Hq, Hkv, L,
                       kv_head_stride, scale_div, part_o, part_ml, counters, sp,
                       (hipStream_t)stream, ri, len);
}

extern "C" int qlin_attn_decode_rope(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                                     int64_t k_row_stride, const uint16_t* v,
                                     int64_t v_row_stride, const float* cos_cache,
                                     const float* sin_cache, int64_t cache_rows,
                                     const int64_t* position_ids, int64_t pos_batch_stride,
                                     uint16_t* k_cache, uint16_t* v_cache, int64_t kv_head_stride,
                                     const uint16_t* mask, void* out, int out_dtype, int64_t B,
                                     int Hq, int Hkv, int64_t L, int D, float scale_div,
                                     float* partials, int32_t* counters, void* stream) {
  return attn_decode_rope_impl(q, q_row_stride, k, k_row_stride, v, v_row_stride, cos_cache,
                               sin_cache, cache_rows, position_ids, pos_batch_stride, k_cache,
                               v_cache, kv_head_stride, mask, out, out_dtype, B, Hq, Hkv, L, D,
                               scale_div, partials, counters, stream);
}

extern "C" int qlin_attn_decode_rope_len(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                                         int64_t k_row_stride, const uint16_t* v,
                                         int64_t v_row_stride, const float* cos_cache,
                                         const float* sin_cache, int64_t cache_rows,
                                         const int64_t* position_ids, int64_t pos_batch_stride,
                                         uint16_t* k_cache, uint16_t* v_cache,
                                         int64_t kv_head_stride, void* out, int out_dtype,
                                         int64_t B, int Hq, int Hkv, int64_t L_cap, int D,
                                         float scale_div, float* partials, int32_t* counters,
                                         const int32_t* len, void* stream) {
  if (!len || !position_ids) return QLIN_EINVAL;
  return attn_decode_rope_impl(q, q_row_stride, k, k_row_stride, v, v_row_stride, cos_cache,
                               sin_cache, cache_rows, position_ids, pos_batch_stride, k_cache,
                               v_cache, kv_head_stride, nullptr, out, out_dtype, B, Hq, Hkv,
                               L_cap, D, scale_div, partials, counters, stream, len);
}

extern "C" int qlin_attn_decode_splits(int64_t B, int Hkv, int64_t L) {
  if (B < 1 || Hkv < 1 || L < 1 || L > kMaxL) return -1;
  return choose_split(B, Hkv, L).S;
}

