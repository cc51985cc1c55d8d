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

#ifdef __cplusplus
}
#endif

#endif
