/*
 * qlin_c_demo.c — the C ABI (include/qlin_gfx950.h) driven from plain C, as a non-Python host of
 * the reference's quantized-linear path would drive it: RTN-quantize + pack an fp16 weight on the
 * device (qlin_quantize), run the fused dequant-GEMV (qlin_gemv_f16), and check the result
 * against a host computation on the exact dequantized weight (qlin_dequant_f16).
 *
 *   gcc -O2 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ examples/qlin_c_demo.c \
 *       -L llama3-quantization_amd/csrc -lqlin_gfx950 -L /opt/rocm/lib -lamdhip64 -lm -o qlin_c_demo
 *   ./qlin_c_demo            # full run (needs a gfx950 GPU)
 *   ./qlin_c_demo --abi      # ABI version + argument validation only (no GPU touched)
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qlin_gfx950.h"

static uint16_t f2h(float f) { /* round-to-nearest-even fp32 -> fp16 (finite, normal range) */
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  int32_t e = (int32_t)((x >> 23) & 0xFF) - 127 + 15;
  uint32_t m = x & 0x7FFFFFu;
  if (e <= 0) return (uint16_t)sign; /* flush tiny values (not produced here) */
  uint32_t h = sign | ((uint32_t)e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)h;
}

static float h2f(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1F, m = h & 0x3FF;
  uint32_t x;
  if (e == 0) {
    if (m == 0) x = sign;
    else { float v = ldexpf((float)m, -24); return (h & 0x8000u) ? -v : v; }
  } else if (e == 31) {
    x = sign | 0x7F800000u | (m << 13);
  } else {
    x = sign | ((e + 112) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &x, 4);
  return f;
}

#define CHECK_HIP(c) do { hipError_t e_ = (c); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %d at %s:%d\n", (int)e_, __FILE__, __LINE__); return 2; } } while (0)
#define CHECK_QLIN(c) do { int r_ = (c); if (r_ != QLIN_OK) { \
  fprintf(stderr, "%s failed: %s\n", #c, qlin_error_string(r_)); return 2; } } while (0)

static int abi_only(void) {
  if (qlin_abi_version() != QLIN_ABI_VERSION) {
    fprintf(stderr, "ABI version %d, header %d\n", qlin_abi_version(), QLIN_ABI_VERSION);
    return 1;
  }
  /* every entry point validates its arguments before touching a device */
  int bad = 0;
  bad |= qlin_gemv_f16(NULL, NULL, 0, NULL, NULL, NULL, 1, 16, 64, 4, 64, NULL) != 1;
  bad |= qlin_gemm_f16(NULL, NULL, 0, NULL, NULL, NULL, 8, 16, 64, 4, 64, NULL, 0, NULL) != 1;
  bad |= qlin_dequant_f16(NULL, NULL, 0, 16, 64, 4, 64, NULL, NULL) != 1;
  bad |= qlin_pack_codes(NULL, 16, 64, 4, NULL, NULL) != 1;
  printf("abi %d, argument validation %s\n", qlin_abi_version(), bad ? "FAILED" : "ok");
  return bad;
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "--abi") == 0) return abi_only();
  const int N = 512, K = 1024, bits = 4, group = 128, Nt = (N + 15) / 16, Kt = (K + 127) / 128;
  const size_t n_w = (size_t)N * K, n_qw = (size_t)Nt * Kt * 64 * bits, n_sz = (size_t)Nt * (K / group) * 16;
  uint16_t* w = malloc(n_w * 2);
  uint16_t* wdq = malloc(n_w * 2);
  uint16_t* x = malloc((size_t)K * 2);
  uint16_t* y = malloc((size_t)N * 2);
  srand(1);
  for (size_t i = 0; i < n_w; ++i) w[i] = f2h(0.02f * ((float)rand() / RAND_MAX - 0.5f) * 3.4f);
  for (int k = 0; k < K; ++k) x[k] = f2h((float)rand() / RAND_MAX - 0.5f);

  void *d_w, *d_wdq, *d_x, *d_y;
  uint32_t *d_qw, *d_sz;
  CHECK_HIP(hipMalloc(&d_w, n_w * 2));
  CHECK_HIP(hipMalloc(&d_wdq, n_w * 2));
  CHECK_HIP(hipMalloc(&d_x, K * 2));
  CHECK_HIP(hipMalloc(&d_y, N * 2));
  CHECK_HIP(hipMalloc((void**)&d_qw, n_qw * 4));
  CHECK_HIP(hipMalloc((void**)&d_sz, n_sz * 4));
  CHECK_HIP(hipMemset(d_qw, 0, n_qw * 4));
  CHECK_HIP(hipMemset(d_sz, 0, n_sz * 4));
  CHECK_HIP(hipMemcpy(d_w, w, n_w * 2, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_x, x, K * 2, hipMemcpyHostToDevice));

  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));
  /* UniformAffineQuantizer(n_bits=4, group_size=128) forward + the real-quant pack, one launch */
  CHECK_QLIN(qlin_quantize(d_w, QLIN_F16, N, K, bits, group, 0, NULL, NULL, NULL, NULL, NULL,
                           d_qw, d_sz, st));
  /* QuantLinear.forward on the packed weight: fused unpack + dequant + GEMV */
  CHECK_QLIN(qlin_gemv_f16(d_qw, d_sz, 0, d_x, NULL, d_y, 1, N, K, bits, group, st));
  CHECK_QLIN(qlin_dequant_f16(d_qw, d_sz, 0, N, K, bits, group, d_wdq, st));
  CHECK_HIP(hipStreamSynchronize(st));
  CHECK_HIP(hipMemcpy(y, d_y, N * 2, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(wdq, d_wdq, n_w * 2, hipMemcpyDeviceToHost));

  double max_err = 0.0, max_ref = 0.0;
  for (int n = 0; n < N; ++n) {
    double ref = 0.0;
    for (int k = 0; k < K; ++k) ref += (double)h2f(wdq[(size_t)n * K + k]) * h2f(x[k]);
    max_err = fmax(max_err, fabs(h2f(y[n]) - ref));
    max_ref = fmax(max_ref, fabs(ref));
  }
  const double rel = max_err / max_ref;
  printf("int%d g%d %dx%d GEMV via the C ABI: max |y - x W_dq^T| / max|ref| = %.3g\n", bits, group,
         N, K, rel);
  hipFree(d_w); hipFree(d_wdq); hipFree(d_x); hipFree(d_y); hipFree(d_qw); hipFree(d_sz);
  hipStreamDestroy(st);
  free(w); free(wdq); free(x); free(y);
  return rel < 2e-3 ? 0 : 1;
}
