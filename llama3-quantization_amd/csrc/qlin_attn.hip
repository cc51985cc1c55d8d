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

#include "../../include/qlin_gfx950.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kD = 128;          // head_dim
// 4 waves per block: 8 took a cold launch 8.2 -> 7.6 us at L = 513 but the graph-replayed decode
// layer 43.25 -> 43.58 us (round 4, same box)
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxGroup = 8;     // query heads per KV head
constexpr int kMaxL = 4096;
constexpr int kSub = 64;         // positions per pass (8 lanes x 16 dims per K row)
constexpr int kRowsU = kThreads / 8;  // K rows per load set (8 lanes per row)
constexpr int kKU = kSub / kRowsU;    // load sets per pass
constexpr int kMaxChunk = 512;   // scores of one chunk live in LDS: 512 x 8 fp32 = 16 KB
constexpr int kMaxSplit = kMaxL / kSub;
// blocks a launch aims for (round 3 sweep: L = 4096 17.2 -> 14.7 us at 256, L <= 2048 +-0)
constexpr int kTargetBlocks = 256;

struct Split {
  int chunk, S;
};

Split choose_split(int64_t B, int Hkv, int64_t L) {
  const int64_t heads = B * Hkv;
  int64_t want = (kTargetBlocks + heads - 1) / heads;  // splits per (b, kv head)
  if (want < 1) want = 1;
  int64_t chunk = (L + want - 1) / want;
  chunk = (chunk + kSub - 1) / kSub * kSub;
  if (chunk > kMaxChunk) chunk = kMaxChunk;
  return Split{(int)chunk, (int)((L + chunk - 1) / chunk)};
}

// partials cross blocks at agent scope (sc1), acknowledged by vmcnt(0) before the count; a
// device-scope __threadfence() in every thread instead measured slower (round 3)
__device__ __forceinline__ void part_store(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float part_load(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// wave-wide max / sum: DPP inside each 16-lane row (quad xor 1, quad xor 2, half-row mirror, row
// mirror: after each step the partner group holds a uniform value, so mirrors act as xor 4 / 8),
// then the 4 row results through readlane — a fixed order, no ds_bpermute round trips
__device__ __forceinline__ float wave_max64(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(v));
  v = fmaxf(v, dpp_f32<0x4E>(v));
  v = fmaxf(v, dpp_f32<0x141>(v));
  v = fmaxf(v, dpp_f32<0x140>(v));
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

__device__ __forceinline__ float wave_sum64(float v) {
  v += dpp_f32<0xB1>(v);
  v += dpp_f32<0x4E>(v);
  v += dpp_f32<0x141>(v);
  v += dpp_f32<0x140>(v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return (r0 + r1) + (r2 + r3);
}

__device__ __forceinline__ float h2f(uint32_t w, int hi) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(hi ? (w >> 16) : (w & 0xFFFFu)));
}

// partials: [o fp32 B*Hkv*S*GRP*D][m, l fp32 B*Hkv*S*GRP*2]; counters: int32 [B*Hkv], zero

// ROPE: the step's RoPE and KV-cache append inside the attention launch (qlin_attn_decode_rope):
// q / k / v are the fused q/k/v projection's fp16 rows before RoPE; every block rotates the q
// rows of its query heads (qlin_rope_f16's fp32 arithmetic), and the block whose chunk holds the
// new cache row L - 1 rotates k (fp16 arithmetic), writes k and v into the cache row for later
// steps and uses them in place of that row's loads (the cache row is written by this launch)
struct RopeIn {
  const _Float16* q16;
  int64_t q_rs;
  const _Float16* k16;
  int64_t k_rs;
  const _Float16* v16;
  int64_t v_rs;
  const float* cosc;
  const float* sinc;
  int64_t cache_rows;
  const int64_t* pos;
  int64_t pos_bs;
  _Float16* kc;  // the caches k / v (writable views of the same buffers)
  _Float16* vc;
};

struct AttnArgs {
  const float* q;
  const _Float16* k;
  const _Float16* v;
  const _Float16* mask;
  void* out;
  int out_f16, Hq, Hkv, L;
  int64_t kv_hs;
  int chunk, S;
  float scale_div;
  int* counters;
  float* part_o;
  float* part_ml;
  RopeIn ri;
  const int* len;  // NULL, or the device-resident cache length (L is then the capacity: the
                   // grid and the partials are sized for it; blocks past the length exit)
};

template <int GRP, bool ROPE = false>
__device__ __forceinline__ void attn_decode_body(const AttnArgs& A, const int bh, const int split) {
  const float* __restrict__ q = A.q;
  const _Float16* __restrict__ k = A.k;
  const _Float16* __restrict__ v = A.v;
  const _Float16* __restrict__ mask = A.mask;
  void* __restrict__ out = A.out;
  const int out_f16 = A.out_f16, Hq = A.Hq, Hkv = A.Hkv, chunk = A.chunk;
  const int Sl = A.S;  // partials layout: split slots per (b, kv head)
  // device-resident length (graph-replayed decode steps): L and the split count of this step
  const int L = A.len ? min(max(__builtin_amdgcn_readfirstlane(*A.len), 1), A.L) : A.L;
  const int S = A.len ? (L + chunk - 1) / chunk : Sl;
  if (split >= S) return;  // block-uniform: past this step's length
  const int64_t kv_hs = A.kv_hs;
  const float scale_div = A.scale_div;
  int* __restrict__ counters = A.counters;
  float* __restrict__ part_o = A.part_o;
  float* __restrict__ part_ml = A.part_ml;
  const RopeIn& ri = A.ri;
  __shared__ float qs[GRP][kD];
  __shared__ __attribute__((aligned(16))) _Float16 knew[ROPE ? kD : 8];  // ROPE: the new k row
  __shared__ __attribute__((aligned(16))) _Float16 vnew[ROPE ? kD : 8];  // ... and v row
  __shared__ float sc[kMaxChunk][GRP];     // scores, then probabilities (position-major)
  __shared__ float po[kWaves][GRP * kD];   // per-wave P V (and merge) partial sums
  __shared__ float cm[GRP], cl[GRP];       // chunk max / sum; merged denominators
  __shared__ float mw[kMaxSplit][GRP];     // merge: chunk maxima, then weights
  __shared__ float ml_l[kMaxSplit][GRP];   // merge: chunk sums
  __shared__ int last;

  const int b = bh / Hkv, hk = bh % Hkv;  // bh = b * Hkv + kv head
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int sub = tid & 7, tl = tid >> 3;  // score passes: 8 lanes x 16 dims per K row
  const int t0 = split * chunk;
  const int n = min(chunk, L - t0);  // positions in this chunk (>= 1)
  const bool has_new = ROPE && split == S - 1;  // this block's chunk holds the new row L - 1
  constexpr int half = kD / 2;
  constexpr int QE = (GRP * kD + kThreads - 1) / kThreads;  // q elements per thread

  // ---- the q side first (its wait then does not wait for the K / V loads behind it) ----
  // ROPE: q / k / v rows of the step, the position id and the cos / sin rows at the guessed
  // position L - 1 (the new token's cache row; a padded sequence's position id differs and
  // takes the reload path below), so no load waits on another one
  float q_x[QE], q_rx[QE], c_q[QE], s_q[QE];
  float k_x = 0.f, k_rx = 0.f;
  _Float16 v_x = 0;
  int64_t p_guess = 0, p_raw = 0;
  const int dn = tid & (kD - 1), dp = dn < half ? dn + half : dn - half;
  if constexpr (ROPE) {
    p_guess = ri.pos ? min((int64_t)L - 1, ri.cache_rows - 1) : 0;
    if (ri.pos) p_raw = ri.pos[(int64_t)b * ri.pos_bs];  // scalar load (lgkmcnt)
#pragma unroll
    for (int e = 0; e < QE; ++e) {
      const int i = min(tid + kThreads * e, GRP * kD - 1);
      const int g = i / kD, d = i % kD;
      const _Float16* qr = ri.q16 + (int64_t)b * ri.q_rs + (int64_t)(hk * GRP + g) * kD;
      q_x[e] = (float)qr[d];
      q_rx[e] = (float)qr[d < half ? d + half : d - half];
      c_q[e] = ri.cosc[p_guess * kD + d];
      s_q[e] = ri.sinc[p_guess * kD + d];
    }
    const _Float16* kr = ri.k16 + (int64_t)b * ri.k_rs + (int64_t)hk * kD;
    k_x = (float)kr[dn];
    k_rx = (float)kr[dp];
    v_x = ri.v16[(int64_t)b * ri.v_rs + (int64_t)hk * kD + dn];
  } else {
    const float* qb = q + ((int64_t)b * Hq + (int64_t)hk * GRP) * kD;
#pragma unroll
    for (int e = 0; e < QE; ++e) q_x[e] = qb[min(tid + kThreads * e, GRP * kD - 1)];
  }
  asm volatile("" ::: "memory");  // the K / V loads are issued after the q side

  // cache rows of (b, kv head) bh start at bh * kv_hs (a KV cache with spare rows: kv_hs > L * kD)
  const _Float16* kb = k + (int64_t)bh * kv_hs + (int64_t)t0 * kD;
  const uint32_t* vb =
      reinterpret_cast<const uint32_t*>(v + (int64_t)bh * kv_hs + (int64_t)t0 * kD) + lane;
  // mask values are loaded unconditionally (from kb when there is no mask) and selected: a load
  // under a branch is followed by its own full wait
  const _Float16* mb = mask ? mask + (int64_t)b * L + t0 : kb;

  // issue the first pass's K rows, V words and mask before anything waits
  u32x4 kw[kKU][2];
  float mv[kKU];
  auto load_k = [&](int tb) {
#pragma unroll
    for (int u = 0; u < kKU; ++u) {
      const int t = min(tb + kRowsU * u + tl, n - 1);
      const u32x4* kr = reinterpret_cast<const u32x4*>(kb + (int64_t)t * kD + 16 * sub);
      kw[u][0] = __builtin_nontemporal_load(kr);
      kw[u][1] = __builtin_nontemporal_load(kr + 1);
      const float m = (float)mb[t];
      mv[u] = mask ? m : 0.f;
    }
  };
  uint32_t vw[kSub / kWaves];  // PV: lane = dim pair, wave = every 4th position
  auto load_v = [&](int tb) {
#pragma unroll
    for (int u = 0; u < kSub / kWaves; ++u) {
      const int t = min(tb + wave + kWaves * u, n - 1);
      vw[u] = __builtin_nontemporal_load(vb + (int64_t)t * (kD / 2));
    }
  };
  load_k(0);
  load_v(0);
  asm volatile("" ::: "memory");

  if constexpr (ROPE) {
#pragma clang fp contract(off)
    auto rope_apply = [&](const float* cr, const float* sr) {
#pragma unroll
      for (int e = 0; e < QE; ++e) {
        const int i = tid + kThreads * e;
        const int g = min(i, GRP * kD - 1) / kD, d = min(i, GRP * kD - 1) % kD;
        const float c = (float)(_Float16)cr[e], sn = (float)(_Float16)sr[e];
        const float rx = d < half ? -q_rx[e] : q_rx[e];
        if (i < GRP * kD) qs[g][d] = q_x[e] * c + rx * sn;  // fp32, each op rounded once
      }
      if (has_new && tid < kD) {
        // thread tid < 128 rotates k dim tid: q element tid (g = 0, d = tid) has its cos / sin
        const float c = (float)(_Float16)cr[0], sn = (float)(_Float16)sr[0];
        const float rx = tid < half ? -k_rx : k_rx;
        const float a0 = (float)(_Float16)(k_x * c), b0 = (float)(_Float16)(rx * sn);
        const _Float16 kn = (_Float16)(a0 + b0);  // fp16 ops, as the reference's k path
        knew[tid] = kn;
        vnew[tid] = v_x;
        const int64_t row = (int64_t)bh * kv_hs + (int64_t)(L - 1) * kD + tid;
        ri.kc[row] = kn;  // the cache row, for the following steps
        ri.vc[row] = v_x;
      }
    };
    rope_apply(c_q, s_q);
    const int64_t p_true = ri.pos ? min(max(p_raw, (int64_t)0), ri.cache_rows - 1) : 0;
    if (p_true != p_guess) {  // block-uniform; its own path, so the common one waits early
      float c2[QE], s2[QE];
#pragma unroll
      for (int e = 0; e < QE; ++e) {
        const int d = min(tid + kThreads * e, GRP * kD - 1) % kD;
        c2[e] = ri.cosc[p_true * kD + d];
        s2[e] = ri.sinc[p_true * kD + d];
      }
      rope_apply(c2, s2);
    }
  } else {
#pragma unroll
    for (int e = 0; e < QE; ++e) {
      const int i = tid + kThreads * e;
      if (i < GRP * kD) qs[i / kD][i % kD] = q_x[e];
    }
  }
  __syncthreads();

  // scores (the next pass's K rows are in flight while this pass computes)
  for (int tb = 0; tb < n; tb += kSub) {
    u32x4 kc[kKU][2];
    float mc[kKU];
#pragma unroll
    for (int u = 0; u < kKU; ++u) {
      kc[u][0] = kw[u][0];
      kc[u][1] = kw[u][1];
      mc[u] = mv[u];
      if (has_new && t0 + tb + kRowsU * u + tl == L - 1) {  // the new row: written by this launch
        kc[u][0] = *reinterpret_cast<const u32x4*>(&knew[16 * sub]);
        kc[u][1] = *reinterpret_cast<const u32x4*>(&knew[16 * sub + 8]);
      }
    }
    if (tb + kSub < n) load_k(tb + kSub);
#pragma unroll
    for (int u = 0; u < kKU; ++u) {
      const int t = tb + kRowsU * u + tl;
      float acc[GRP];
#pragma unroll
      for (int g = 0; g < GRP; ++g) acc[g] = 0.f;
      const _Float16* hv = reinterpret_cast<const _Float16*>(kc[u]);
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
#pragma unroll
        for (int g = 0; g < GRP; ++g) {
          const float4 qq = *reinterpret_cast<const float4*>(&qs[g][16 * sub + j]);
          acc[g] = fmaf(qq.x, (float)hv[j], acc[g]);
          acc[g] = fmaf(qq.y, (float)hv[j + 1], acc[g]);
          acc[g] = fmaf(qq.z, (float)hv[j + 2], acc[g]);
          acc[g] = fmaf(qq.w, (float)hv[j + 3], acc[g]);
        }
      }
#pragma unroll
      for (int g = 0; g < GRP; ++g) {
        // the xor-1 / xor-2 / xor-4 butterfly of the row's 8 lanes as DPP moves (ds_bpermute
        // would be 3 dependent LDS round trips per head): after the two quad steps every lane of
        // a quad holds the quad sum, so the half-row mirror (lane i <- 7 - i) reads the other
        // quad's sum exactly as xor 4 would
        acc[g] += dpp_f32<0xB1>(acc[g]);   // quad_perm [1, 0, 3, 2]
        acc[g] += dpp_f32<0x4E>(acc[g]);   // quad_perm [2, 3, 0, 1]
        acc[g] += dpp_f32<0x141>(acc[g]);  // row_half_mirror
      }
      if (t < n && sub < GRP) {
        // lane `sub` stores query head g = sub (select without dynamic register indexing)
        float a = acc[0];
#pragma unroll
        for (int g = 1; g < GRP; ++g) a = (sub == g) ? acc[g] : a;
        float s = a / scale_div + mc[u];
        s = (s != s) ? s : fmaxf(s, -3.402823466e38f);  // torch.max(w, finfo(fp32).min)
        sc[t][sub] = s;
      }
    }
  }
  __syncthreads();

  // chunk softmax statistics: wave w owns query heads w, w + 4 (wave-level reductions only)
  for (int g = wave; g < GRP; g += kWaves) {
    float m = -INFINITY;
    for (int t = lane; t < n; t += 64) m = fmaxf(m, sc[t][g]);
    m = wave_max64(m);
    float s = 0.f;
    for (int t = lane; t < n; t += 64) {
      const float e = expf(sc[t][g] - m);
      sc[t][g] = e;
      s += e;
    }
    s = wave_sum64(s);
    if (lane == 0) {
      cm[g] = m;
      cl[g] = s;
    }
  }
  __syncthreads();

  // P V: branch-free (rows past the chunk: clamped reads, results selected away), the
  // probabilities of RB rows read from LDS together (one LDS round trip per RB rows, not per row)
  {
    constexpr int VR = kSub / kWaves;         // V rows per wave and pass
    constexpr int RB = GRP <= 4 ? VR : VR / 2;  // rows per LDS batch (registers: RB x GRP)
    float a0[GRP], a1[GRP];
#pragma unroll
    for (int g = 0; g < GRP; ++g) a0[g] = a1[g] = 0.f;
    const uint32_t vn = has_new ? *reinterpret_cast<const uint32_t*>(&vnew[2 * lane]) : 0u;
    for (int tb = 0; tb < n; tb += kSub) {
      uint32_t vc[VR];
#pragma unroll
      for (int u = 0; u < VR; ++u) {
        const bool is_new = has_new && t0 + tb + wave + kWaves * u == L - 1;
        vc[u] = is_new ? vn : vw[u];
      }
      if (tb + kSub < n) load_v(tb + kSub);
#pragma unroll
      for (int r0 = 0; r0 < VR; r0 += RB) {
        float pr[RB][GRP];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int tc = min(tb + wave + kWaves * (r0 + r), n - 1);
#pragma unroll
          for (int g = 0; g < GRP; ++g) pr[r][g] = sc[tc][g];
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const bool ok = tb + wave + kWaves * (r0 + r) < n;
          const float v0 = h2f(vc[r0 + r], 0), v1 = h2f(vc[r0 + r], 1);
#pragma unroll
          for (int g = 0; g < GRP; ++g) {
            const float f0 = fmaf(pr[r][g], v0, a0[g]), f1 = fmaf(pr[r][g], v1, a1[g]);
            a0[g] = ok ? f0 : a0[g];
            a1[g] = ok ? f1 : a1[g];
          }
        }
      }
    }
#pragma unroll
    for (int g = 0; g < GRP; ++g) {
      po[wave][g * kD + 2 * lane] = a0[g];
      po[wave][g * kD + 2 * lane + 1] = a1[g];
    }
  }
  __syncthreads();

  const int64_t qh0 = (int64_t)b * Hq + (int64_t)hk * GRP;  // first query head of the group
  // output row of the group: fp32, or rounded once to fp16 (== the reference's .to(fp16))
  auto wave_total = [&](int o) {  // the per-wave partials of element o, added in wave order
    float r = po[0][o];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) r += po[w][o];
    return r;
  };
  auto put = [&](int o, float val) {
    if (out_f16) reinterpret_cast<_Float16*>(out)[qh0 * kD + o] = (_Float16)val;
    else reinterpret_cast<float*>(out)[qh0 * kD + o] = val;
  };
  auto put_all = [&]() {
    for (int o = tid; o < GRP * kD; o += kThreads)
      put(o, wave_total(o) / cl[o / kD]);
  };
  if (S == 1) {
    put_all();
    return;
  }

  // write this chunk's partials, then count in; the last block of (b, kv head) merges
  float* pob = part_o + ((int64_t)bh * Sl + split) * GRP * kD;
  for (int o = tid; o < GRP * kD; o += kThreads)
    part_store(pob + o, wave_total(o));
  if (tid < 2 * GRP) {
    float* ml = part_ml + ((int64_t)bh * Sl + split) * GRP * 2;
    part_store(ml + tid, (tid & 1) ? cl[tid >> 1] : cm[tid >> 1]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // sc1 stores acknowledged before the count
  __syncthreads();
  if (tid == 0)
    last = (__hip_atomic_fetch_add(&counters[bh], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            S - 1);
  __syncthreads();
  if (!last) return;

  // merge: the first kPre partial rows of every wave (s = wave + kWaves i) are requested with
  // the chunk statistics — one memory round trip instead of two at decode lengths (S <= 16)
  constexpr int J = GRP * kD / 64;
  constexpr int kPre = GRP <= 4 ? 4 : 2;
  const float* pb = part_o + (int64_t)bh * Sl * GRP * kD + lane;
  float xpre[kPre][J];
#pragma unroll
  for (int i = 0; i < kPre; ++i) {
    const int s = min(wave + kWaves * i, S - 1);
#pragma unroll
    for (int j = 0; j < J; ++j) xpre[i][j] = part_load(pb + (int64_t)s * GRP * kD + 64 * j);
  }
  // chunk statistics -> weights exp(m_s - M) and denominators sum_s w_s l_s
  const float* mlb = part_ml + (int64_t)bh * Sl * GRP * 2;
  for (int i = tid; i < S * GRP; i += kThreads) {
    mw[i / GRP][i % GRP] = part_load(mlb + 2 * i);
    ml_l[i / GRP][i % GRP] = part_load(mlb + 2 * i + 1);
  }
  __syncthreads();
  for (int g = wave; g < GRP; g += kWaves) {
    float M = -INFINITY;
    for (int s = lane; s < S; s += 64) M = fmaxf(M, mw[s][g]);
    M = wave_max64(M);
    float den = 0.f;
    for (int s = lane; s < S; s += 64) {
      const float w = expf(mw[s][g] - M);
      mw[s][g] = w;
      den += w * ml_l[s][g];
    }
    den = wave_sum64(den);
    if (lane == 0) cl[g] = den;
  }
  __syncthreads();
  // weighted sum of the S partial rows: wave w takes rows s = w, w + 4, ...; lane owns floats
  // o = lane + 64 j of the GRP x 128 row (one coalesced 256-B load per wave and j)
  {
    float acc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = 0.f;
    // rows s = wave + kWaves i, i < kPre, arrived with the statistics (same order as below)
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
      const int s = wave + kWaves * i;
      if (s < S) {
#pragma unroll
        for (int j = 0; j < J; ++j) acc[j] = fmaf(mw[s][(64 * j + lane) / kD], xpre[i][j], acc[j]);
      }
    }
    // the rest in rounds of kPre rows, every load of a round issued before its FMAs (long caches:
    // S = 64 at L = 4096 was 16 dependent round trips per wave)
    for (int s0 = wave + kWaves * kPre; s0 < S; s0 += kWaves * kPre) {
      float x[kPre][J];
#pragma unroll
      for (int i = 0; i < kPre; ++i) {
        const int s = min(s0 + kWaves * i, S - 1);
#pragma unroll
        for (int j = 0; j < J; ++j) x[i][j] = part_load(pb + (int64_t)s * GRP * kD + 64 * j);
      }
#pragma unroll
      for (int i = 0; i < kPre; ++i) {
        const int s = s0 + kWaves * i;
        if (s < S) {
#pragma unroll
          for (int j = 0; j < J; ++j) acc[j] = fmaf(mw[s][(64 * j + lane) / kD], x[i][j], acc[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < J; ++j) po[wave][lane + 64 * j] = acc[j];
  }
  __syncthreads();
  if (tid == 0) counters[bh] = 0;  // ready for the next launch (graph replay)
  put_all();
}

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
                   (int*)counters, part_o, part_ml, ri, len};
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

