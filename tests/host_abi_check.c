/* Host-side checks of the C-ABI that need no GPU: version, options, error strings, and the argument validation of
 * every entry point that refuses bad input before touching the device (VIT_REQUIRE paths), plus the pure host
 * helpers (workspace sizes, split-K hint, resize kernel size).  Built twice:
 *   - against the shipped library by tests/test_dropin_cpu.py (gcc, seconds);
 *   - against an AddressSanitizer build of the library's host code by tools/asan_host_check.sh
 *     (hipcc -Xarch_host -fsanitize=address), the SURVEY §5 "race detection / sanitizers" row for the host side.
 * Exit status 0 = every check passed; a failed check prints its line. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "vit_hip.h"

static int fails = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      fprintf(stderr, "host_abi_check: FAILED line %d: %s\n", __LINE__, #c); \
      ++fails;                                                         \
    }                                                                  \
  } while (0)

/* an entry point refused its arguments: VIT_ERR_INVALID and a non-empty message naming it */
static int refused(int rc, const char* name) {
  const char* e = vit_last_error();
  return rc == VIT_ERR_INVALID && e != NULL && strstr(e, name) != NULL;
}

int main(void) {
  CHECK(vit_abi_version() == VIT_ABI_VERSION);

  /* options: documented names, set / get / restore, unknown names refused */
  CHECK(vit_get_option("gemm_persist") == 1);
  CHECK(vit_set_option("gemm_persist", 0) == VIT_OK && vit_get_option("gemm_persist") == 0);
  CHECK(vit_set_option("gemm_persist", 1) == VIT_OK);
  CHECK(vit_get_option("no_such_option") == INT64_MIN);
  CHECK(refused(vit_set_option("no_such_option", 1), "vit_set_option"));
  CHECK(refused(vit_set_option(NULL, 1), "vit_set_option"));

  /* GEMM descriptor validation (all before any launch) */
  float dummy[64];
  vit_gemm_desc d;
  memset(&d, 0, sizeof(d));
  CHECK(refused(vit_gemm(NULL, NULL), "vit_gemm"));
  CHECK(refused(vit_gemm(&d, NULL), "vit_gemm"));                  /* null operands */
  d.a = dummy; d.b = dummy; d.c = dummy;
  d.m = 0; d.n = 8; d.k = 8;
  CHECK(refused(vit_gemm(&d, NULL), "vit_gemm"));                  /* bad shape */
  d.m = 8; d.in_dtype = 7;
  CHECK(refused(vit_gemm(&d, NULL), "vit_gemm"));                  /* bad dtype */
  d.in_dtype = VIT_F32; d.out_dtype = VIT_BF16; d.beta = 1.f;
  CHECK(refused(vit_gemm(&d, NULL), "vit_gemm"));                  /* beta needs f32 output */
  d.beta = 0.f; d.dropout_p = 1.5f;
  CHECK(refused(vit_gemm(&d, NULL), "vit_gemm"));                  /* dropout out of range */
  d.dropout_p = 0.f; d.in_dtype = VIT_BF16; d.lda = 7; d.ldb = 8;
  CHECK(refused(vit_gemm(&d, NULL), "vit_gemm"));                  /* bf16 leading dims */
  d.lda = 8;
  d.a_kcontig = 0; d.b_kcontig = 1;
  CHECK(refused(vit_gemm(&d, NULL), "vit_gemm"));                  /* layout not provided */

  /* host helpers */
  memset(&d, 0, sizeof(d));
  d.m = 50432; d.n = 768; d.k = 768; d.in_dtype = VIT_BF16; d.out_dtype = VIT_BF16; d.a_kcontig = d.b_kcontig = 1;
  CHECK(vit_gemm_workspace_bytes(&d) >= 0);
  CHECK(vit_gemm_workspace_bytes(NULL) == 0);
  CHECK(vit_gemm_split_k_hint(0, 8, 8, VIT_BF16) == 1);
  CHECK(vit_gemm_split_k_hint(3072, 768, 50432, VIT_BF16) >= 1);
  CHECK(vit_attn_bwd_uses_o32(256, 197, 12, 64, VIT_BF16) == 0);
  CHECK(vit_attn_bwd_uses_o32(64, 577, 12, 64, VIT_BF16) == 1);
  CHECK(vit_attn_bwd_uses_o32(4, 197, 2, 64, VIT_F32) == 0);
  CHECK(vit_attn_bwd_workspace_bytes(256, 197, 12, 64, VIT_BF16) == 256LL * 12 * 197 * 4);
  CHECK(vit_layernorm_bwd_parts(50432, 768) >= 1);
  CHECK(vit_colsum_workspace_bytes(50432, 768) > 0);
  CHECK(vit_resize_ksize(512, 224) >= 1);

  /* entry points that refuse before the device */
  CHECK(refused(vit_attn_fwd(NULL, NULL, NULL, NULL, NULL, 1, 1, 1, 64, 1.f, VIT_BF16, 0, NULL), "vit_attn_fwd"));
  CHECK(refused(vit_attn_bwd(NULL, NULL, NULL, NULL, NULL, NULL, 1, 1, 1, 64, 1.f, VIT_BF16, NULL, 0, NULL),
                "vit_attn_bwd"));
  CHECK(refused(vit_attn_fwd_row0(NULL, NULL, NULL, 1, 1, 1, 64, 1.f, VIT_BF16, NULL), "vit_attn_fwd_row0"));
  CHECK(refused(vit_attn_fwd_row0(dummy, dummy, (float*)dummy, 1, 5000, 1, 64, 1.f, VIT_BF16, NULL),
                "vit_attn_fwd_row0"));                                                 /* T > 4096 */
  CHECK(refused(vit_attn_bwd_row0(dummy, dummy, 8, dummy, 1, 5, 1, 64, 1.f, VIT_BF16, NULL),
                "vit_attn_bwd_row0"));                                                 /* ldo < H * hd */
  CHECK(refused(vit_colsum_finish(NULL, 1, 1, 1, dummy, NULL, NULL, 0.f, NULL), "vit_colsum_finish"));
  CHECK(refused(vit_colsum_finish(dummy, 1, 8, 2, dummy, NULL, NULL, 0.f, NULL), "vit_colsum_finish"));
  vit_colsum_job jobs[9];
  memset(jobs, 0, sizeof(jobs));
  CHECK(refused(vit_colsum_finish_batch(jobs, 0, NULL), "vit_colsum_finish_batch"));
  CHECK(refused(vit_colsum_finish_batch(jobs, 9, NULL), "vit_colsum_finish_batch"));
  jobs[0].part = dummy; jobs[0].nparts = 1; jobs[0].cols = 8; jobs[0].nsets = 2; jobs[0].out[0] = dummy;
  CHECK(refused(vit_colsum_finish_batch(jobs, 1, NULL), "vit_colsum_finish_batch"));   /* out[1] missing */
  CHECK(refused(vit_copy2d(NULL, 1, VIT_F32, dummy, 1, VIT_F32, 1, 1, 0, 0, 0.f, NULL), "vit_copy2d"));

  if (fails == 0) printf("host_abi_check: all checks passed (ABI %d)\n", vit_abi_version());
  return fails == 0 ? 0 : 1;
}
