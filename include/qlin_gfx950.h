/*
 * qlin_gfx950.h — C ABI of libqlin_gfx950.so, the MI355X (gfx950) quantized-linear hot path.
 *
 * Drop-in boundary for SilviaUvA/LLaMA3-Quantization's quantized-linear path.  The reference has no
 * native code (its arithmetic is PyTorch ops in quant/quantizer.py and F.linear in
 * quant/int_linear.py); each entry point below replaces the reference interface named in its
 * comment.  The Python host mirror (llama3-quantization_amd/quant/) binds these through ctypes —
 * see INTEGRATION.md for the binding a maintainer would add.
 *
 * Conventions (all entry points):
 *   - return 0 on success, otherwise a hipError_t code (1 = hipErrorInvalidValue for bad args);
 *     no C++ exception crosses the ABI; nothing is printed.
 *   - the caller owns every buffer (device pointers); the library allocates nothing, never
 *     synchronises, and enqueues all work on `stream` (a hipStream_t, NULL = legacy default).
 *   - stateless and reentrant; safe to call from any host thread and inside stream capture.
 *   - fp16 tensors are passed as uint16_t* (IEEE binary16 bit patterns).
 *
 * Canonical packed weight layout ("qlin tiled" layout):
 *   qweight  uint32 [ceil(N/16), ceil(K/128), 64, bits]: 16-row x 128-k tiles of 64 lane pieces;
 *            lane l = n + 16q of a tile holds the 32 codes of tile row n at k = 32s + 8q + j
 *            (s < 4, j < 8) — the B operand of v_mfma_f32_16x16x32_f16 k-step s.  bits in
 *            {2,3,4,8}; bit positions inside a piece: oracle/quant_oracle.py pack_qweight and
 *            llama3-quantization_amd/csrc/qlin_common.h.  Codes of rows >= N / k >= K are
 *            ignored (the packers write k >= K as 0; rows >= N are never written).
 *   qsz      uint32 [ceil(N/16), K/group, 16]: the (scale, zero) of row 16*nt + n, group g at
 *            [nt][g][n] — fp16 scale in bits 0..15 (== reference scales.view(N, -1),
 *            quant/omniquant.py:322-325), int16 integral zero point in bits 16..31 (== reference
 *            zeros.view(N, -1); disable_zero_point is stored as zero = 2^(bits-1)).  One 64-byte
 *            coalesced load gives a tile's 16 rows their group parameters.
 *   flags    QLIN_WIDE_ZERO when some |zero| > 1024 (possible only for degenerate groups: the
 *            reference clamps zero points to +-1e4), selecting the fp32 (u - zero) path.
 *            QLIN_FLOAT_ZERO: bits 16..31 of qsz hold an fp16 zero instead (HQQ checkpoints,
 *            whose zero points are not integral); W = RN16(RN16(u - zero) * scale), hqq's
 *            ((W_q - zero) * scale) in fp16.
 *   group    multiple of 32 dividing K (group = K for per-channel); K % 32 == 0.
 * Both arrays must be allocated padded (ceil(N/16)*16 rows, ceil(K/128)*128 codes) and zeroed
 * before packing; the packers write rows < N only.
 */
#ifndef QLIN_GFX950_H
#define QLIN_GFX950_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QLIN_ABI_VERSION 13

/* quantizer flags (UniformAffineQuantizer options, quant/quantizer.py:24-36) */
#define QLIN_SYMMETRIC          1
#define QLIN_DISABLE_ZERO_POINT 2
#define QLIN_LWC                4
/* packed-layout flags (dequant / GEMV / GEMM entry points) */
#define QLIN_WIDE_ZERO          8
#define QLIN_FLOAT_ZERO        16
/* qlin_rmsnorm_linear_ep_f16: the norm weight is fp16 (the module's own), not fp32 */
#define QLIN_NORM_W16          32

/* return codes (hipError_t values; anything else is a HIP error passed through) */
#define QLIN_OK     0
#define QLIN_EINVAL 1 /* hipErrorInvalidValue: bad argument, nothing launched */

/* element dtypes */
#define QLIN_F16 0
#define QLIN_F32 1

/* ABI version (QLIN_ABI_VERSION); lets a binding check it loaded the library it was written for. */
int qlin_abi_version(void);

/* Human-readable text for a return code. */
const char* qlin_error_string(int code);

/*
 * Fused RTN quantizer: per-group min/max calibration + fake-quant (+ optional packing), one pass.
 * Replaces UniformAffineQuantizer.forward -> per_token_dynamic_calibration -> fake_quant
 * (quant/quantizer.py:118-159, :94-115), bit-exact in the input dtype (fp16 or fp32).
 *   x          [rows, K] dtype;  group divides K (group = K: per-channel / per-token); K and
 *              group multiples of 32, except one group per row (group == K) without packing,
 *              which takes any K (QuantMatMul's per-token operands: K = the key count).
 *   lwc_up_sig, lwc_low_sig  [rows*K/group] dtype: sigmoid(upbound/lowbound_factor) (QLIN_LWC).
 *   x_dq       [rows, K] dtype or NULL;  scale_out / zp_out [rows*K/group] dtype or NULL
 *              (zp_out unused with QLIN_DISABLE_ZERO_POINT) — the reference's scale /
 *              round_zero_point tensors.
 *   qweight, qsz: canonical packed outputs (dtype must be QLIN_F16), or both NULL.
 */
int qlin_quantize(const void* x, int dtype, int64_t rows, int64_t K, int bits, int group,
                  int flags, const void* lwc_up_sig, const void* lwc_low_sig,
                  void* x_dq, void* scale_out, void* zp_out,
                  uint32_t* qweight, uint32_t* qsz, void* stream);

/*
 * fake_quant with given parameters (quant/quantizer.py:94-115): x_dq = RN(RN(clamp(round_ste(
 * RN(x / s)) + zp) - zp) * s), optionally also packing the integer codes (dtype QLIN_F16 only).
 *   scale, zp [rows*K/group] dtype (zp NULL iff QLIN_DISABLE_ZERO_POINT); outputs as in
 *   qlin_quantize; x_dq may be NULL.
 */
int qlin_fake_quant(const void* x, int dtype, const void* scale, const void* zp, int64_t rows,
                    int64_t K, int bits, int group, int flags, void* x_dq, uint32_t* qweight,
                    uint32_t* qsz, void* stream);

/*
 * Real-quant packer: canonical layout from (W_dq, scales, zeros) as registered by
 * register_scales_and_zeros (quant/quantizer.py:161-165).  Replaces the AutoGPTQ
 * QuantLinear.pack(module, scales, zeros) call of quant/omniquant.py:315-335.  Integer codes are
 * recovered with the quantizer's own fp16 arithmetic, so qlin_dequant_f16 of the result
 * reproduces W_dq bit-exactly.
 *   w_dq [N, K] fp16; scales_ref, zeros_ref [N*K/group] fp16 (zeros_ref NULL iff
 *   QLIN_DISABLE_ZERO_POINT).  Outputs as in qlin_quantize.
 */
int qlin_pack_f16(const uint16_t* w_dq, const uint16_t* scales_ref, const uint16_t* zeros_ref,
                  int64_t N, int64_t K, int bits, int group, int flags,
                  uint32_t* qweight, uint32_t* qsz, void* stream);

/*
 * Integer codes -> canonical qweight, for converters whose zero points are not integral (HQQ):
 *   codes uint8 [N, K] row-major, each < 2^bits (higher bits are ignored); qweight allocated and
 *   zeroed as above.  The matching qsz is plain data (scale | zero << 16) built by the caller.
 * Replaces the packing half of hqq's BaseQuantizeConfig / HQQLinear path (reference
 * quantizehqq.py:40-49; hqq.core.bitpack pack_4bit_u8 / pack_3bit_32 / pack_2bit_u8).
 */
int qlin_pack_codes(const uint8_t* codes, int64_t N, int64_t K, int bits, uint32_t* qweight,
                    void* stream);

/*
 * Dequantize the canonical layout: w[n,k] = RN16(RN16(q - zp) * s), bit-exact with the reference
 * fake_quant's x_dequant.sub(zp).mul(scale) (quant/quantizer.py:107-110).  Debug / parity and
 * the fake-quant eval mode (module.weight = W_dq, quant/utils.py:133-136).
 */
int qlin_dequant_f16(const uint32_t* qweight, const uint32_t* qsz, int flags, int64_t N,
                     int64_t K, int bits, int group, uint16_t* w, void* stream);

/*
 * y[M, N] = x[M, K] @ W_dq[N, K]^T (+ bias[N]) with the group-wise unpack + dequant fused into the
 * product; fp16 in/out, fp32 accumulation.  Replaces QuantLinear.forward's
 * fwd_func(input, weight, bias) = F.linear (quant/int_linear.py:62) on packed weights.
 *   qlin_gemv_f16: matrix-core GEMV, 1 <= M <= 16 (decode / small batches).
 *   qlin_gemm_f16: MFMA (v_mfma_f32_*_f16) tiles, any M >= 1 (prefill / PPL windows).
 *   qlin_linear_f16: picks from M: GEMV for M <= 64 (16-row chunks), MFMA GEMM above.
 *   workspace / workspace_bytes (qlin_gemm_f16): NULL / 0, or a device buffer (256-B aligned,
 *     contents need not be initialised) of workspace_bytes bytes: when that is at least
 *     qlin_linear_workspace_bytes(M, N, K, bits, group, 0), launches whose grid of 64 x 128 blocks
 *     leaves most CUs idle split K over up to 8 block groups and reduce the fp32 partials in a
 *     second pass (fixed order: deterministic, within fp32 rounding of the unsplit launch); with
 *     a smaller (or no) buffer they run unsplit — the call never writes past workspace_bytes.
 */
int qlin_gemv_f16(const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
                  const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K, int bits,
                  int group, void* stream);
int qlin_gemm_f16(const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
                  const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K, int bits,
                  int group, void* workspace, int64_t workspace_bytes, void* stream);
/*
 * Strided batch of independent decode products in one launch:
 *   y[b] = x[b] @ W_dq[b]^T (+ bias[b]),  b < batch (<= 65535), 1 <= M <= 16,
 * problem b's operands at qweight + b*qweight_stride, qsz + b*qsz_stride (uint32 words),
 * x + b*x_stride, bias + b*bias_stride, y + b*y_stride (fp16 elements); every problem has the
 * same M, N, K, bits, group and flags.
 * The same QuantLinear.forward F.linear (quant/int_linear.py:62) as qlin_gemv_f16, applied to
 * several independent QuantLinear modules of one shape at once (e.g. one decode step over the
 * modules of a ring of layers' weights); one kernel boundary per batch instead of per matrix.
 * x_stride / bias_stride may be 0 (one activation / bias shared by every problem); other strides
 * smaller than one problem's extent return QLIN_EINVAL.  M <= 4 with K % 512 == 0, group a
 * multiple of 128 (or 32 / 64) and 16-B aligned operands (qweight / qsz / x bases 16-B aligned,
 * qweight_stride and qsz_stride multiples of 4 words, x_stride a multiple of 8) runs the streaming
 * kernel: each output is one MFMA chain in k
 * order, bit-identical to qlin_gemm_f16 without workspace; other shapes run one qlin_gemv_f16
 * launch per problem.
 */
int qlin_gemv_batched_f16(const uint32_t* qweight, int64_t qweight_stride, const uint32_t* qsz,
                          int64_t qsz_stride, int flags, const uint16_t* x, int64_t x_stride,
                          const uint16_t* bias, int64_t bias_stride, uint16_t* y,
                          int64_t y_stride, int64_t batch, int64_t M, int64_t N, int64_t K,
                          int bits, int group, void* stream);
/*
 * The launch geometry qlin_gemv_batched_f16 uses for these arguments on the current device, without
 * launching (pointers are only checked for alignment): plan[0] = workgroups of the streaming
 * kernel, plan[1] = dynamic LDS bytes per workgroup, plan[2] = the instance's static LDS bytes,
 * plan[3] = resident workgroups per CU (occupancy query of that instance), plan[4] = tile rows per
 * wave (1 or 2); all 0 when the arguments take the per-problem path.  Introspection for tests and
 * tools (ABI 13); no reference counterpart.
 */
int qlin_gemv_batched_plan(const uint32_t* qweight, int64_t qweight_stride, const uint32_t* qsz,
                           int64_t qsz_stride, int flags, const uint16_t* x, int64_t x_stride,
                           int64_t batch, int64_t M, int64_t N, int64_t K, int bits, int group,
                           int64_t* plan);
int qlin_linear_f16(const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
                    const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K, int bits,
                    int group, void* stream);
/* Workspace bytes qlin_gemm_f16 / qlin_linear_ep_f16 use for this launch (act_bits as passed to
 * qlin_linear_ep_f16, 0 for qlin_gemm_f16): the act fake-quant x_dq region (when the quantizer
 * kernel runs) followed by the split-K partials; 0 = none; -1 = invalid arguments. */
int64_t qlin_linear_workspace_bytes(int64_t M, int64_t N, int64_t K, int bits, int group,
                                    int act_bits);

/*
 * Output columns per block that qlin_gemm_f16 picks for an M x N launch on the current device
 * (128, 256, 384 or 512; 128 = the 64-row x 128-column block for small grids, 255 = the 64-row x
 * 256-column block for grids a little larger), or -1 for invalid
 * arguments.  Introspection for tests and tools; no reference counterpart.
 */
int qlin_gemm_block_cols(int64_t M, int64_t N, int bits);

/*
 * Which kernel a one-token-row product (qlin_gemv_f16 / qlin_linear_ep_f16 at M = 1, 16-B aligned
 * x, and qlin_rmsnorm_linear_ep_f16) of this shape runs on the current device: 1 = the work-queue
 * kernel (wide matrices: each CU's workgroup takes chunks of 4 k-tiles of its tile rows from an LDS
 * counter and adds the chunks' partial sums per row in k order), 2 = the fast split-K kernel, 3 = the rows kernel (long K), 0 = the
 * general GEMV kernel (no M = 1 route: qlin_rmsnorm_linear_ep_f16 rejects the shape), -1 =
 * invalid arguments.  Introspection for tests and tools (ABI 12); no reference counterpart.
 */
int qlin_gemv_m1_route(int64_t N, int64_t K, int bits, int group);

/*
 * The packed linear with a fused output epilogue (the decoder layer's glue around two of its
 * linears, models/int_llama_layer.py of the reference) and optional activation fake-quant:
 *   QLIN_EP_RESIDUAL  y = RN16(residual + RN16(x @ W_dq^T + bias)) — o_proj / down_proj followed
 *                     by `hidden_states = residual + hidden_states` (:241-257); residual [M, N].
 *   QLIN_EP_SILU_MUL  W's rows interleaved in 8-row halves (rows 16j..16j+7 = gate rows
 *                     8j..8j+7, rows 16j+8..16j+15 = up rows 8j..8j+7; N % 16 == 0):
 *                     y[M, N/2] = RN16(RN16(silu(gate)) * up) with gate / up the fp16 F.linear
 *                     outputs — QuantLlamaMLP's act_fn(gate_proj(x)) * up_proj(x) (:44-45).
 *   QLIN_EP_NONE      == qlin_linear_f16.
 * act_bits != 0 additionally fake-quantizes x per token first — QuantLinear.forward's
 * act_quantizer(input) (quant/int_linear.py:59-60) with UniformAffineQuantizer(n_bits=act_bits,
 * dynamic_method="per_token") (quant/quantizer.py:132-159, :94-115), bit-exact; act_flags takes
 * QLIN_SYMMETRIC / QLIN_DISABLE_ZERO_POINT.  M <= 64 and N <= 16384: fused into the GEMV (each
 * block recomputes the token's min / max; x 16-byte aligned, K % 8 == 0); otherwise the quantizer
 * kernel writes x_dq to `workspace` (fp16 [M, K], required then) before the GEMV / GEMM.
 * Same kernels and dispatch as qlin_linear_f16 (GEMV for M <= 64, MFMA GEMM above).
 * workspace / workspace_bytes: NULL / 0 (only without the act quantizer kernel), or a buffer of
 * workspace_bytes bytes laid out as the x_dq region (when the quantizer kernel runs; a buffer
 * smaller than that region returns QLIN_EINVAL), then the split-K partials of qlin_gemm_f16 (run
 * unsplit when the rest is smaller than they need).  qlin_linear_workspace_bytes(M, N, K, bits,
 * group, act_bits) is the full size; the call never writes past workspace_bytes.
 */
#define QLIN_EP_NONE     0
#define QLIN_EP_RESIDUAL 1
#define QLIN_EP_SILU_MUL 2
int qlin_linear_ep_f16(const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
                       const uint16_t* bias, const uint16_t* residual, uint16_t* y, int64_t M,
                       int64_t N, int64_t K, int bits, int group, int epilogue, int act_bits,
                       int act_flags, uint16_t* workspace, int64_t workspace_bytes,
                       void* stream);

/*
 * RMSNorm + packed linear for ONE token row in one launch (the decoder layer's
 * input_layernorm -> fused q/k/v and post_attention_layernorm -> gate/up at decode; the norm is
 * OmniLlamaRMSNorm, quant/omni_norm.py:52-63 of the reference): x fp16 [K] is the hidden state
 * BEFORE the norm, norm_weight [K]: fp32 (8-B aligned; the fp16 weight upcast, exact) or, with
 * flags & QLIN_NORM_W16, the fp16 weight itself (4-B aligned; half the bytes, same result), eps
 * its variance epsilon.  The kernel normalises x at the reference's rounding point,
 * x_hat = RN16(weight * (x * rsqrt(mean(x^2) + eps))) with fp32 inside, and multiplies x_hat:
 * y = F.linear(x_hat, W_dq, bias), then `epilogue` as qlin_linear_ep_f16.  The sum of squares runs
 * in another order than torch's reduction (an fp32 ulp of the statistics can move an fp16 ulp of
 * x_hat).  Supported: M == 1, K % 128 == 0, group % 128 == 0 or group in {32, 64}, and K / 128 =
 * W * T with W <= 16 waves and T in {2, 4, 8} k-tiles per wave — qlin_rmsnorm_linear_supported()
 * says so (1) or not (0); otherwise QLIN_EINVAL.
 */
int qlin_rmsnorm_linear_supported(int64_t M, int64_t N, int64_t K, int bits, int group);
int qlin_rmsnorm_linear_ep_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                               const uint16_t* x, const void* norm_weight, float eps,
                               const uint16_t* bias, const uint16_t* residual, uint16_t* y,
                               int64_t M, int64_t N, int64_t K, int bits, int group, int epilogue,
                               void* stream);

/*
 * Fused decode attention (one query token per sequence), for the quantized LLaMA layer's
 * attention core (models/int_llama_layer.py:137-165 of the reference: repeat_kv, fp32 QK^T bmm,
 * / sqrt(head_dim), + mask, clamp at finfo(fp32).min, fp32 softmax, fp32 PV bmm) on an fp16 K/V
 * cache; fp32 arithmetic, equal to the reference up to fp32 summation order.
 *   q    fp32 [B, Hq, D] (after RoPE);  k, v  fp16 [B, Hkv, L, D], the L rows of (b, kv head h)
 *   at k + (b * Hkv + h) * kv_head_stride elements (0: L * D, contiguous; else a multiple of 8,
 *   >= L * D: a KV cache with spare rows, see qlin_rope_kv_f16);  mask  fp16 [B, L] additive or
 *   NULL;  out  [B, Hq, D] in out_dtype: QLIN_F32, or QLIN_F16 = the fp32 result rounded once
 *   (the layer's .to(fp16) before o_proj);  scale_div = sqrt(D) (the scores are divided by it).
 *   D == 128, Hq / Hkv in {1, 2, 4, 8}, L <= 4096.
 * The cache is split over blocks along L.  qlin_attn_decode_partials_bytes() returns the bytes
 * of `partials` scratch a call needs (0: none, pass NULL; -1: unsupported shapes); `counters` is
 * int32 [>= B * Hkv], zero-filled before its first use and left zero-filled by every call (the
 * merging block resets it), so one counter buffer serves all later calls on the same stream,
 * graph replays included; do not share it between streams running concurrently.
 * qlin_attn_decode_splits(): the split count S of a (B, Hkv, L) launch (1: no partials, -1:
 * unsupported arguments).
 */
int64_t qlin_attn_decode_partials_bytes(int64_t B, int Hq, int Hkv, int64_t L);
int qlin_attn_decode_splits(int64_t B, int Hkv, int64_t L);
int qlin_attn_decode(const float* q, const uint16_t* k, const uint16_t* v, const uint16_t* mask,
                     void* out, int out_dtype, int64_t B, int Hq, int Hkv, int64_t L, int D,
                     int64_t kv_head_stride, float scale_div, float* partials, int32_t* counters,
                     void* stream);

/*
 * qlin_rope_kv_f16 + qlin_attn_decode in one launch, for one query token per sequence with a KV
 * cache that has room for the new row: q / k / v are the step's projection rows BEFORE RoPE (fp16,
 * row b at q + b * q_row_stride, Hq resp. Hkv heads of D), cos / sin / position_ids as for
 * qlin_rope_f16; the caches fp16 [B, Hkv, rows, D] with head stride kv_head_stride (>= L * D)
 * hold rows 0 .. L - 2 and receive the rotated k and the v row at L - 1 from this launch, which
 * then attends over all L rows (mask fp16 [B, L] or NULL).  Same arithmetic as the two launches
 * (bit-identical output and cache rows); partials / counters as qlin_attn_decode.  B == 1 may
 * pass position_ids NULL with cos / sin pointing at the step's own rows.
 */
int qlin_attn_decode_rope(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                          int64_t k_row_stride, const uint16_t* v, int64_t v_row_stride,
                          const float* cos_cache, const float* sin_cache, int64_t cache_rows,
                          const int64_t* position_ids, int64_t pos_batch_stride, uint16_t* k_cache,
                          uint16_t* v_cache, int64_t kv_head_stride, const uint16_t* mask,
                          void* out, int out_dtype, int64_t B, int Hq, int Hkv, int64_t L, int D,
                          float scale_div, float* partials, int32_t* counters, void* stream);

/*
 * qlin_attn_decode_rope for a graph-replayed decode step (mask NULL, position_ids required): the
 * cache length is read on the device from len[0] (1 <= len[0] <= L_cap), so one captured launch
 * serves every step; L_cap (the cache capacity used at capture) sizes the grid and the partials
 * (qlin_attn_decode_partials_bytes(B, Hq, Hkv, L_cap)); blocks past the step's length exit.  The
 * split of the rows depends on L_cap, not on len[0]: same arithmetic as qlin_attn_decode_rope at
 * L = L_cap for the rows present (results agree with it to fp32 summation order).
 */
int qlin_attn_decode_rope_len(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                              int64_t k_row_stride, const uint16_t* v, int64_t v_row_stride,
                              const float* cos_cache, const float* sin_cache, int64_t cache_rows,
                              const int64_t* position_ids, int64_t pos_batch_stride,
                              uint16_t* k_cache, uint16_t* v_cache, int64_t kv_head_stride,
                              void* out, int out_dtype, int64_t B, int Hq, int Hkv, int64_t L_cap,
                              int D, float scale_div, float* partials, int32_t* counters,
                              const int32_t* len, void* stream);

/*
 * Fused prefill attention (many query tokens per sequence): the same attention core as
 * qlin_attn_decode — repeat_kv, fp32 QK^T, / sqrt(head_dim) (as torch: x the fp32 reciprocal),
 * + mask, clamp at finfo(fp32).min, fp32 softmax, fp32 PV (models/int_llama_layer.py:137-165 of
 * the reference, QuantMatMul qkt / pv of quant/int_matmul.py at A16) — as one kernel that keeps
 * the [S, L] scores on chip (online softmax) and multiplies on the fp32 matrix cores; equal to the
 * reference up to fp32 rounding (summation order), not bit for bit.
 *   q    fp32 [B, Hq, S, D] (after RoPE);  k, v  fp16 [B, Hkv, L, D], L >= S: query row i sits at
 *   key position L - S + i;  mask  [B', 1, S, L] additive, QLIN_F16 or QLIN_F32, batch b at
 *   mask + b * mask_batch_stride elements (0: broadcast), or NULL (no masking);
 *   causal = 1 (mask required): the caller guarantees mask[., i, j] <= -1e4 for every key
 *   j > L - S + i, so key blocks past a query block's diagonal are skipped (their exp()
 *   underflows to 0 in the reference as well); causal = 2: the mask is exactly that pattern
 *   (0 for j <= L - S + i, <= -1e4 above): it is applied arithmetically and never read (mask may
 *   be NULL); causal = 0: the mask (if any) is read everywhere and no key block is skipped;
 *   out  [B, S, Hq, D] (the layer's transpose(1, 2) layout) in out_dtype: QLIN_F32, or QLIN_F16 =
 *   the fp32 result rounded once (the layer's .to(fp16) before o_proj);  scale_div = sqrt(D).
 *   D == 128, Hq / Hkv in {1, 2, 4, 8}.
 */
int qlin_attn_prefill(const float* q, const uint16_t* k, const uint16_t* v, const void* mask,
                      int mask_dtype, int64_t mask_batch_stride, int causal, void* out,
                      int out_dtype, int64_t B, int Hq, int Hkv, int64_t S, int64_t L, int D,
                      float scale_div, void* stream);

/*
 * RMSNorm of the quantized LLaMA layer (OmniLlamaRMSNorm.forward, quant/omni_norm.py:52-63 of the
 * reference): y = (weight * (x * rsqrt(mean(x^2) + eps))).to(fp16), fp32 inside.
 *   x, y  fp16 [rows, H];  weight  fp32 [H] (the fp16 weight upcast: exact).
 * The sum of squares runs in another order than torch's reduction: y may differ by one fp16 ulp.
 */
int qlin_rmsnorm_f16(const uint16_t* x, const float* weight, uint16_t* y, int64_t rows, int64_t H,
                     float eps, void* stream);

/*
 * Rotary position embedding of QuantLlamaAttention.forward (models/int_llama_layer.py:116-125 of
 * the reference, transformers-4.37.2 apply_rotary_pos_emb): bit-exact, in one launch.
 *   q  fp16 rows of Hq*D, row (b, s) at q + (b*S + s)*q_row_stride (e.g. a column slice of the
 *      fused q/k/v output);  k  likewise with Hkv heads;
 *   cos_cache, sin_cache  fp32 [cache_rows, D] (the rotary cache; each value is cast to fp16 as
 *      the reference's rotary_emb(...).to(x.dtype) does); positions outside [0, cache_rows) are
 *      clamped (the reference's index raises instead);
 *   position_ids  int64, (b, s) at position_ids[b*pos_batch_stride + s];
 *   q_out  fp32 [B, Hq, S, D]: q.transpose(1, 2).float() * cos + rotate_half(.) * sin (fp32 ops);
 *   k_out  fp16 [B, Hkv, S, D]: the same in fp16 ops (each product and the sum rounded to fp16).
 */
int qlin_rope_f16(const uint16_t* q, int64_t q_row_stride, const uint16_t* k, int64_t k_row_stride,
                  const float* cos_cache, const float* sin_cache, int64_t cache_rows,
                  const int64_t* position_ids, int64_t pos_batch_stride, float* q_out, uint16_t* k_out, int64_t B, int64_t S,
                  int Hq, int Hkv, int D, void* stream);

/*
 * qlin_rope_f16 plus the KV-cache append of the same layer step (models/int_llama_layer.py:130-135
 * of the reference: torch.cat([past_key, key], dim=2), likewise for value): the rotated k rows and
 * the v rows (v  fp16 rows of Hkv*D at v + (b*S + s)*v_row_stride) are written straight into
 * caches k_cache / v_cache fp16 [B, Hkv, kv_rows, D] at rows kv0 .. kv0 + S - 1, so the cached
 * rows 0 .. kv0 - 1 are never copied.  Requires D % 8 == 0, q / k / v strides and pointers
 * 4-element aligned, cos / sin / q_out 16-B aligned and kv0 + S <= kv_rows (else
 * QLIN_EINVAL).  Same arithmetic as qlin_rope_f16 (bit-exact).
 */
int qlin_rope_kv_f16(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                     int64_t k_row_stride, const uint16_t* v, int64_t v_row_stride,
                     const float* cos_cache, const float* sin_cache, int64_t cache_rows,
                     const int64_t* position_ids, int64_t pos_batch_stride, float* q_out,
                     uint16_t* k_cache, uint16_t* v_cache, int64_t kv_rows, int64_t kv0,
                     int64_t B, int64_t S, int Hq, int Hkv, int D, void* stream);

/*
 * Attention scores of a prefill window, in place (models/int_llama_layer.py:143-157 of the
 * reference: attn_weights / sqrt(head_dim) + attention_mask, then torch.max(w, finfo(fp32).min)):
 * one pass instead of three, bit-exact (torch divides an fp32 tensor by a scalar as a
 * multiplication by the fp32 reciprocal).
 *   scores fp32 [B, H, T, L] contiguous, L % 4 == 0;  mask [B', 1, T, L] additive, QLIN_F16 or
 *   QLIN_F32, batch b at mask + b * mask_batch_stride elements (0: broadcast), or NULL (then only
 *   the division, as the reference applies the clamp only with a mask).
 */
int qlin_attn_scores_f32(float* scores, const void* mask, int mask_dtype, int64_t B, int64_t H,
                         int64_t T, int64_t L, int64_t mask_batch_stride, float scale_div,
                         void* stream);

#ifdef __cplusplus
}
#endif

#endif /* QLIN_GFX950_H */
