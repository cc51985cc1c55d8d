/*
 * qlin_gfx950_prefetch.h — weight prefetch for the decode layer (libqlin_gfx950.so; same
 * conventions as qlin_gfx950.h).
 *
 * qlin_prefetch: reads `bytes` bytes at `p` (16-B aligned) with plain loads and discards them, so
 * the lines sit in the memory-side cache (MALL) when the launch that needs them runs.  Meant for a
 * second stream beside a latency-bound launch (the decode attention leaves most CUs and most of
 * the HBM bandwidth idle): the packed weights of the next linears of the same layer step.  No
 * counterpart in the reference (its eval path reads fp16 weights through F.linear,
 * quant/int_linear.py:62); it changes no result.  blocks: grid size (0: one per CU).
 */
#ifndef QLIN_GFX950_PREFETCH_H
#define QLIN_GFX950_PREFETCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int qlin_prefetch(const void* p, int64_t bytes, int blocks, void* stream);

/*
 * qlin_attn_decode_rope (qlin_gfx950.h) whose launch also carries ~pf_blocks extra blocks that
 * read `pf_bytes` at `pf` (16-B aligned; e.g. o_proj's packed weights) while the attention blocks
 * wait on their K / V round trips: same attention result, bit for bit, and one launch (no second
 * stream).  pf_blocks in [1, 4096], rounded up to a multiple of B * Hkv.
 */
int qlin_attn_decode_rope_pf(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                             int64_t k_row_stride, const uint16_t* v, int64_t v_row_stride,
                             const float* cos_cache, const float* sin_cache, int64_t cache_rows,
                             const int64_t* position_ids, int64_t pos_batch_stride,
                             uint16_t* k_cache, uint16_t* v_cache, int64_t kv_head_stride,
                             const uint16_t* mask, void* out, int out_dtype, int64_t B, int Hq,
                             int Hkv, int64_t L, int D, float scale_div, float* partials,
                             int32_t* counters, void* stream, const void* pf, int64_t pf_bytes,
                             int pf_blocks);

#ifdef __cplusplus
}
#endif

#endif
