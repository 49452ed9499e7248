/* Host-side argument validation of libslx_hip.so's C-ABI under AddressSanitizer (SURVEY.md §5 "Race detection /
 * sanitizers"). Built against an ASan host build of the library (tools/asan_build.sh: every csrc .hip source compiled
 * with -Xarch_host -fsanitize=address); every call below must be refused on the host with a negative status and a
 * message in slx_last_error(), before any HIP call - so the program runs without a GPU. The pure host helpers
 * (workspace sizes, resampling tables, merge geometry) run to completion. Exit 0 = all checks passed and ASan found
 * nothing (ASan aborts the process on an error). */
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "slx.h"

static int fails = 0;

static void expect_err(int rc, const char* what, const char* needle) {
  const char* msg = slx_last_error();
  if (rc >= 0 || !msg || !msg[0] || (needle && !strstr(msg, needle))) {
    fprintf(stderr, "FAIL %s: rc=%d msg='%s' (want '%s')\n", what, rc, msg ? msg : "(null)", needle ? needle : "");
    ++fails;
  } else {
    printf("ok   %-28s rc=%d  %s\n", what, rc, msg);
  }
}

int main(void) {
  if (slx_abi_version() != 1) { fprintf(stderr, "FAIL abi version\n"); return 1; }
  /* GEMM: null desc, negative dims, K not a multiple of 8, misaligned operand, bad epilogue combinations */
  expect_err(slx_gemm_bf16(NULL, NULL), "gemm null desc", "null desc");
  slx_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.M = -1; g.N = 8; g.K = 8; g.batch = 1;
  expect_err(slx_gemm_bf16(&g, NULL), "gemm negative dims", "negative");
  g.M = 8; g.K = 7; g.lda = 8; g.ldb = 8;
  expect_err(slx_gemm_bf16(&g, NULL), "gemm K % 8", "multiple of 8");
  g.K = 8; g.lda = 12;
  expect_err(slx_gemm_bf16(&g, NULL), "gemm lda % 8", "lda/ldb");
  g.lda = 8; g.A = (const void*)(uintptr_t)0x1008; g.B = (const void*)(uintptr_t)0x2000;
  expect_err(slx_gemm_bf16(&g, NULL), "gemm misaligned A", "16B aligned");
  g.A = (const void*)(uintptr_t)0x1000; g.epilogue = SLX_EPI_GELU; g.layout = SLX_GEMM_NN;
  expect_err(slx_gemm_bf16(&g, NULL), "gemm GELU layout", "GELU needs NT");
  /* pair: mismatched layouts / K */
  slx_gemm_desc g2 = g;
  g.epilogue = SLX_EPI_STORE; g2.epilogue = SLX_EPI_STORE; g2.layout = SLX_GEMM_TN;
  expect_err(slx_gemm_bf16_pair(&g, &g2, NULL), "gemm pair layouts", "one layout and one K");
  expect_err(slx_gemm_bf16_pair(NULL, &g2, NULL), "gemm pair null", "null desc");
  /* attention: unsupported head_dim */
  slx_attn_desc a;
  memset(&a, 0, sizeof(a));
  a.head_dim = 128;
  expect_err(slx_attn_fwd(&a, NULL), "attn head_dim", "head_dim");
  /* host helpers: run fully */
  if (slx_norm_partial_ws_floats(1024) <= 0 || slx_colsum_ws_floats(4096) <= 0 || slx_dec_attn_ws_floats(14, 2, 1024) <= 0) {
    fprintf(stderr, "FAIL workspace-size helpers\n");
    ++fails;
  }
  int km = slx_resample_ksize(1024, 896);
  if (km <= 0 || km > 64) { fprintf(stderr, "FAIL resample ksize %d\n", km); ++fails; }
  else {
    int32_t* bounds = (int32_t*)malloc(sizeof(int32_t) * 2 * 896);
    int32_t* kk = (int32_t*)malloc(sizeof(int32_t) * (size_t)896 * km);
    if (slx_resample_coeffs(1024, 896, km, bounds, kk) != km) {  /* returns ksize */ fprintf(stderr, "FAIL resample coeffs\n"); ++fails; }
    free(bounds);
    free(kk);
  }
  {
    int32_t b2[4], k2[4];
    expect_err(slx_resample_coeffs(0, 896, 8, b2, k2), "resample bad size", "positive");
    expect_err(slx_resample_coeffs(1024, 2, 4, b2, k2), "resample kmax < ksize", "kmax");
    expect_err(slx_resample_coeffs(1024, 896, 64, NULL, NULL), "resample null out", "null");
  }
  if (slx_llava_merge_tokens(24, 48, 2) <= 0) { fprintf(stderr, "FAIL llava merge tokens\n"); ++fails; }
  printf("%s: %d failure(s)\n", fails ? "FAILED" : "PASSED", fails);
  return fails ? 1 : 0;
}
