/* Plain-C caller of libhbxgpu.so, mirroring the cgo stub of INTEGRATION.md
 * (the binding Hashback's Go code would use): hbx_chunk_hash on a file in
 * host memory, then the same file through hbx_arena_alloc + hbx_memcpy_h2d +
 * hbx_submit_device + hbx_wait (outputs in hbx_alloc_pinned memory, as cgo
 * requires), and the ABI's error conventions.  Test infrastructure
 * (tests/test_abi.py builds and runs it; tests/test_gpu_abi.py checks its
 * output against the oracle).
 *
 * usage: abi_driver <file> [--expect-nodev]
 * prints one line per chunk: "<cut end> <32 hex digits>" for each of the two
 * paths, then "content <type> <hex>" and "ok". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hbxgpu.h"

static void hex(const uint8_t *p, char *out) {
  for (int i = 0; i < 16; i++) sprintf(out + 2 * i, "%02x", p[i]);
}

static int fail(const char *what, int rc, hbx_ctx *ctx) {
  fprintf(stderr, "%s failed: %d %s\n", what, rc, ctx ? hbx_last_error(ctx) : "");
  return 1;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  int nd = 0;
  const int rc_dev = hbx_device_count(&nd);
  hbx_ctx *ctx = NULL;
  const int rc_ctx = hbx_ctx_create(0, &ctx);
  if (argc > 2 && strcmp(argv[2], "--expect-nodev") == 0) {
    /* no GPU: every entry point reports, nothing aborts */
    if (rc_dev != HBX_ERR_NODEV || nd != 0 || rc_ctx != HBX_ERR_NODEV || ctx) return 3;
    if (hbx_chunk_hash(NULL, NULL, 0, NULL, NULL, 0, NULL) != HBX_ERR_ARG) return 4;
    if (hbx_max_chunks(131072) != 3) return 5;
    if (hbx_set_join_lag(NULL, 1) != HBX_ERR_ARG) return 6;
    /* the operating point is host arithmetic: planned without a device (the
     * N = 8 share of configs[2]: 8 x 128 MiB per GPU, 282 GiB free) */
    hbx_plan_request q;
    memset(&q, 0, sizeof q);
    q.n_files = 8;
    q.arena_bytes = 8ull * (128ull << 20) + (64u << 10);
    q.longest_file = 128ull << 20;
    q.free_bytes = 282ull << 30;
    q.steps = 20;
    q.md5_slice = -1;
    q.lead = -1;
    hbx_pipeline_plan pl;
    if (hbx_plan_pipeline(NULL, &q, &pl) != HBX_OK) return 7;
    if (pl.join_lag != 2 || pl.lead != 3 || pl.k3_period != 4 || pl.resident < 200 ||
        (uint64_t)pl.md5_slice * pl.k3_period * pl.launches_per_batch < 131073u)
      return 8;
    q.join_lag = 9; /* refused, described by hbx_last_error(NULL) */
    if (hbx_plan_pipeline(NULL, &q, &pl) != HBX_ERR_ARG || !strstr(hbx_last_error(NULL), "join lag")) return 9;
    printf("plan R=%u slice=%u lag=%u lead=%u period=%u launches=%u\n", pl.resident, pl.md5_slice, pl.join_lag,
           pl.lead, pl.k3_period, pl.launches_per_batch);
    printf("nodev ok\n");
    return 0;
  }
  if (rc_ctx != HBX_OK) return fail("hbx_ctx_create", rc_ctx, NULL);

  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const uint64_t n = (uint64_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *data = malloc(n ? n : 1);
  if (n && fread(data, 1, n, f) != n) return 2;
  fclose(f);

  /* chunkHash of the cgo stub: one synchronous call */
  const uint64_t cap = hbx_max_chunks(n);
  uint64_t *cuts = calloc(cap, 8);
  uint8_t *ids = calloc(cap, 16);
  uint64_t k = 0;
  int rc = hbx_chunk_hash(ctx, data, n, cuts, ids, cap, &k);
  if (rc != HBX_OK) return fail("hbx_chunk_hash", rc, ctx);
  char h[33];
  for (uint64_t i = 0; i < k; i++) {
    hex(ids + 16 * i, h);
    printf("sync %llu %s\n", (unsigned long long)cuts[i], h);
  }
  /* too small a capacity: HBX_ERR_CAPACITY and the count needed */
  if (k > 1) {
    uint64_t k2 = 0;
    rc = hbx_chunk_hash(ctx, data, n, cuts, ids, k - 1, &k2);
    if (rc != HBX_ERR_CAPACITY || k2 != k) return fail("capacity check", rc, ctx);
  }

  /* the asynchronous form: device arena, pinned outputs, submit + wait */
  void *arena = NULL;
  if ((rc = hbx_arena_alloc(ctx, n, &arena)) != HBX_OK) return fail("hbx_arena_alloc", rc, ctx);
  if (n && (rc = hbx_memcpy_h2d(ctx, arena, data, n)) != HBX_OK) return fail("hbx_memcpy_h2d", rc, ctx);
  void *pin = NULL;
  const size_t need = cap * 8 + cap * 16 + sizeof(hbx_file_summary) + 3 * 8;
  if ((rc = hbx_alloc_pinned(need, &pin)) != HBX_OK) return fail("hbx_alloc_pinned", rc, ctx);
  uint64_t *acuts = (uint64_t *)pin;
  uint8_t *aids = (uint8_t *)(acuts + cap);
  hbx_file_summary *sum = (hbx_file_summary *)(aids + 16 * cap);
  uint64_t *meta = (uint64_t *)(sum + 1); /* offs, lens, out_base, caps live until the wait */
  meta[0] = 0;
  meta[1] = n;
  meta[2] = 0;
  uint64_t capv = cap;
  /* a join lag of 3 (the bench's small-batch setting): the wait's drain joins the batch */
  if ((rc = hbx_set_join_lag(ctx, 3)) != HBX_OK) return fail("hbx_set_join_lag", rc, ctx);
  if ((rc = hbx_submit_device(ctx, arena, 1, &meta[0], &meta[1], acuts, aids, &meta[2], &capv, sum)) != HBX_OK)
    return fail("hbx_submit_device", rc, ctx);
  if (hbx_pending(ctx) != 1) return fail("hbx_pending", hbx_pending(ctx), ctx);
  /* the slice is fixed while a batch is pending */
  if (hbx_set_md5_slice(ctx, 7) != HBX_ERR_STATE) return fail("hbx_set_md5_slice while pending", 0, ctx);
  if (hbx_set_join_lag(ctx, 1) != HBX_ERR_STATE) return fail("hbx_set_join_lag while pending", 0, ctx);
  if ((rc = hbx_wait(ctx)) != HBX_OK) return fail("hbx_wait", rc, ctx);
  if (sum->n_chunks != k) return fail("async chunk count", (int)sum->n_chunks, ctx);
  for (uint64_t i = 0; i < k; i++) {
    hex(aids + 16 * i, h);
    printf("async %llu %s\n", (unsigned long long)acuts[i], h);
  }
  hex(sum->content_id, h);
  printf("content %d %s\n", sum->content_type, h);
  /* an unaligned arena offset is refused and leaves nothing pending */
  meta[0] = 3;
  rc = hbx_submit_device(ctx, arena, 1, &meta[0], &meta[1], acuts, aids, &meta[2], &capv, sum);
  if (rc != HBX_ERR_ARG || hbx_pending(ctx) != 0) return fail("unaligned submit", rc, ctx);
  hbx_free_pinned(pin);
  hbx_arena_free(ctx, arena);
  hbx_ctx_destroy(ctx);
  free(cuts);
  free(ids);
  free(data);
  printf("ok\n");
  return 0;
}
