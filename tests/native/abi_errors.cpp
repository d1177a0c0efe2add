// Host-side argument validation of every C-ABI entry point (include/*.h), built with AddressSanitizer
// on the host code only (hipcc --cuda-host-only -fsanitize=address; tests/test_asan_abi.py) and run on
// a CPU-only machine: every call below must return its negative MINER_E* code before any device work
// (no HIP call is reached), and ASan must report nothing — no read or write outside an object in the
// validation, the size queries, the shape checks and miner_strerror (sanitizer builds of
// the native code). The pointers are host addresses that are never dereferenced by a correct
// validation: `buf` is 16-byte aligned, `mis` is not.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "miner_corpus.h"
#include "miner_fastformer.h"
#include "miner_metrics.h"
#include "miner_news.h"
#include "miner_score.h"
#include "miner_wide.h"

alignas(16) static unsigned char g_buf[4096];

static int g_fail = 0, g_calls = 0;
static void expect(const char* what, int rc, int want) {
  ++g_calls;
  const bool ok = want == 0 ? rc < 0 : rc == want;
  if (!ok) {
    fprintf(stderr, "FAIL %s: rc %d, want %s%d\n", what, rc, want == 0 ? "< 0, e.g. " : "", want);
    ++g_fail;
  }
}
#define EXPECT(call, want) expect(#call, (call), (want))

int main() {
  void* buf = g_buf;
  void* mis = g_buf + 4;
  const float* fb = (const float*)g_buf;
  float* fo = (float*)(g_buf + 1024);
  const int32_t* ib = (const int32_t*)g_buf;
  int32_t* io = (int32_t*)(g_buf + 2048);
  const uint8_t* ub = g_buf;
  void* st = nullptr;

  // ---- host-only queries: answers for any input, no out-of-bounds table reads ----
  for (int c = -64; c <= 64; ++c) {
    const char* s = miner_strerror(c);
    if (!s || strlen(s) > 200) { fprintf(stderr, "FAIL miner_strerror(%d)\n", c); ++g_fail; }
  }
  if (miner_abi_version() != MINER_ABI_VERSION) { fprintf(stderr, "FAIL abi version\n"); ++g_fail; }
  const int dts[] = {-1, 0, 1, 2, 3, 4, 5, 1 << 30};
  const int dims[] = {-2147483647 - 1, -1, 0, 1, 31, 32, 64, 768, 1 << 20, 2147483647};
  for (int dt : dts)
    for (int d : dims) {
      (void)miner_supported(dt, 50, d, 200, 32);
      (void)miner_supported(dt, d, 768, d, d);
      (void)miner_lds_bytes(dt, 0, 50, d, 200);
      (void)miner_lds_bytes(dt, 3, d, 768, d);
      (void)miner_news_supported(dt, d, 768, 200, 32);
      (void)miner_wide_supported(dt, d, 768, 200, d);
      (void)miner_packed_weights_bytes(dt, d, 200, 32);
      (void)miner_target_weights_bytes(dt, d);
      (void)miner_encoder_packed_bytes(dt, d, d, d);
      (void)miner_fastformer_packed_bytes(dt);
      (void)miner_fastformer_lds_bytes(dt);
      (void)miner_rank_topk_workspace_bytes(d, d);
      (void)miner_rank_topk_split_recommended(d);
      (void)miner_auc_workspace_bytes((int64_t)d * 4096);
    }
  EXPECT(miner_supported(7, 50, 768, 200, 32), MINER_EINVAL);
  EXPECT(miner_supported(MINER_DTYPE_F32_X6, 50, 768, 200, 32), MINER_EINVAL);   // a news-path form only
  EXPECT(miner_news_precompute(st, MINER_DTYPE_F32_X6, buf, 100, buf, 768, 200, 32, fo, buf), MINER_EINVAL);
  EXPECT(miner_supported(0, 50, 100, 200, 32), 0);          // d % 32
  EXPECT(miner_supported(0, 200, 768, 200, 32), 0);         // L > 64

  // ---- miner_score / gather / target_aware / packing ----
  EXPECT(miner_pack_weights(st, 0, nullptr, buf, buf, 768, 200, 32, buf), MINER_EINVAL);
  EXPECT(miner_pack_weights(st, 9, buf, buf, buf, 768, 200, 32, buf), 0);
  EXPECT(miner_pack_weights(st, 0, buf, buf, buf, 100, 200, 32, buf), 0);
  EXPECT(miner_pack_target_weights(st, 0, nullptr, 768, buf), 0);
  EXPECT(miner_pack_target_weights(st, 0, buf, -5, buf), 0);
  EXPECT(miner_score(st, 0, 0, nullptr, ub, nullptr, buf, nullptr, buf, 4, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score(st, 0, 9, buf, ub, nullptr, buf, nullptr, buf, 4, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score(st, 5, 0, buf, ub, nullptr, buf, nullptr, buf, 4, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score(st, 0, 0, buf, ub, nullptr, buf, nullptr, buf, -1, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score(st, 0, 0, buf, ub, nullptr, buf, nullptr, buf, 4, 65, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score(st, 0, 0, buf, ub, nullptr, buf, nullptr, buf, 4, 50, 40, 768, 200, 33, fo, nullptr), 0);
  EXPECT(miner_score(st, 0, 0, mis, ub, nullptr, buf, nullptr, buf, 4, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score_gather(st, 0, 0, nullptr, 100, ib, ub, nullptr, ib, nullptr, buf, 4, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score_gather(st, 0, 0, buf, 0, ib, ub, nullptr, ib, nullptr, buf, 4, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_score_gather(st, 0, 0, buf, -7, ib, ub, nullptr, ib, nullptr, buf, 4, 50, 40, 768, 200, 32, fo, nullptr), 0);
  EXPECT(miner_target_aware(st, 0, nullptr, buf, fb, nullptr, buf, 200, 4, 40, 768, 32, fo), 0);
  EXPECT(miner_target_aware(st, 0, buf, buf, fb, nullptr, buf, 200, 4, 40, 768, 99, fo), 0);

  // ---- news path ----
  EXPECT(miner_news_precompute(st, 0, nullptr, 100, buf, 768, 200, 32, fo, buf), 0);
  EXPECT(miner_news_precompute(st, 4, buf, 100, buf, 768, 200, 32, fo, buf), 0);
  // the fp32-MFMA form goes through the fp32 checks
  EXPECT(miner_news_precompute(st, MINER_DTYPE_F32_MFMA, buf, 100, buf, 100, 200, 32, fo, buf), MINER_ESHAPE);
  EXPECT(miner_news_precompute(st, MINER_DTYPE_F32_MFMA, mis, 100, buf, 768, 200, 32, fo, buf), MINER_EALIGN);
  EXPECT(miner_news_precompute(st, 0, buf, -1, buf, 768, 200, 32, fo, buf), 0);
  EXPECT(miner_score_news(st, 0, 0, nullptr, fb, buf, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, fo, nullptr), 0);
  EXPECT(miner_score_news(st, 0, 7, buf, fb, buf, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, fo, nullptr), 0);
  EXPECT(miner_score_news(st, 0, 0, buf, fb, buf, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 600, 768, 32, fo, nullptr), 0);
  EXPECT(miner_news_split_x2(st, nullptr, 10, 768, buf, fo), MINER_EINVAL);
  EXPECT(miner_news_split_x2(st, fb, 10, 100, buf, fo), MINER_ESHAPE);
  EXPECT(miner_news_split_x2(st, (const float*)mis, 10, 768, buf, fo), MINER_EALIGN);
  EXPECT(miner_score_news_x2(st, 9, buf, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, fo, nullptr, nullptr), MINER_EINVAL);
  EXPECT(miner_score_news_x2(st, 0, nullptr, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, fo, nullptr, nullptr), MINER_EINVAL);
  EXPECT(miner_score_news_x2(st, 0, buf, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 129, 40, 768, 32, fo, nullptr, nullptr), MINER_ESHAPE);
  EXPECT(miner_score_news_x2(st, 0, buf, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 68, fo, nullptr, nullptr), MINER_ESHAPE);
  EXPECT(miner_score_news_x2(st, 0, buf, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 100, 40, 768, 64, fo, nullptr, fo), MINER_ESHAPE);
  EXPECT(miner_score_news_x2(st, 0, buf, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 30, fo, nullptr, nullptr), MINER_ESHAPE);
  EXPECT(miner_score_news_x2(st, 0, buf, fb, fb, nullptr, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, fo, nullptr, nullptr), MINER_EINVAL);
  EXPECT(miner_score_news_x2(st, 3, buf, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, nullptr, nullptr, nullptr), MINER_EINVAL);
  EXPECT(miner_score_news_x2(st, 0, buf, fb, fb, buf, fb, 2000000, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, fo, nullptr, nullptr), MINER_ESHAPE);
  EXPECT(miner_score_news_x2(st, 0, mis, fb, fb, buf, fb, 100, ib, ub, nullptr, ib, nullptr, 4, 50, 40, 768, 32, fo, nullptr, nullptr), MINER_EALIGN);

  // ---- wide path ----
  EXPECT(miner_score_wide(st, 0, 0, nullptr, buf, buf, nullptr, 0, nullptr, nullptr, 4, 40, 768, 64, fo), 0);
  EXPECT(miner_score_wide(st, 0, 0, buf, buf, buf, nullptr, 0, nullptr, nullptr, 4, 40, 768, 65, fo), 0);
  EXPECT(miner_score_wide(st, 0, 8, buf, buf, buf, nullptr, 0, nullptr, nullptr, 4, 40, 768, 64, fo), 0);
  EXPECT(miner_wide_proj(st, 0, nullptr, buf, 10, 768, buf), 0);
  EXPECT(miner_wide_proj(st, 0, buf, buf, -3, 768, buf), 0);

  // ---- full-corpus ranking ----
  EXPECT(miner_encoder_pack(st, 0, nullptr, buf, buf, 768, 200, 64, buf), 0);
  EXPECT(miner_encode_users(st, 0, nullptr, nullptr, 0, ub, nullptr, buf, 4, 200, 768, 200, 64, fo, buf, buf), 0);
  EXPECT(miner_encode_users(st, 0, buf, nullptr, 0, ub, nullptr, buf, 4, 300, 768, 200, 64, fo, buf, buf), 0);
  EXPECT(miner_rank_topk(st, 2, 0, buf, buf, buf, 4, 1000, 768, 64, 0, fo, io), 0);
  EXPECT(miner_rank_topk(st, 2, 0, buf, nullptr, buf, 4, 1000, 768, 64, 10, fo, io), 0);
  EXPECT(miner_rank_topk(st, 2, 9, buf, buf, buf, 4, 1000, 768, 64, 10, fo, io), 0);
  EXPECT(miner_rank_topk_ws(st, 2, 0, buf, buf, buf, 4, 1000, 768, 64, 10, fo, io, mis, 1 << 20), MINER_EALIGN);
  EXPECT(miner_rank_topk_ws(st, 2, 0, buf, buf, buf, 4, 1000, 768, 64, 100000, fo, io, buf, 1 << 20), 0);

  // ---- FastFormer ----
  EXPECT(miner_fastformer_pack(st, 0, nullptr, buf), 0);
  EXPECT(miner_fastformer_pack(st, 5, fb, buf), 0);
  EXPECT(miner_fastformer_score(st, 0, nullptr, ub, buf, nullptr, buf, 4, 50, 40, fo, nullptr), 0);
  EXPECT(miner_fastformer_score(st, 0, buf, ub, buf, nullptr, buf, 4, 65, 40, fo, nullptr), 0);
  EXPECT(miner_fastformer_score_gather(st, 0, buf, 0, ib, ub, ib, nullptr, buf, 4, 50, 40, fo, nullptr), 0);

  // ---- metrics ----
  EXPECT(miner_impression_metrics(st, nullptr, ub, ib, 4, ib, 2, (double*)fo, nullptr), 0);
  EXPECT(miner_impression_metrics(st, fb, ub, ib, -1, ib, 2, (double*)fo, nullptr), 0);
  EXPECT(miner_global_auc(st, nullptr, ub, 100, buf, 4096, (double*)fo), 0);
  EXPECT(miner_global_auc(st, fb, ub, 100, buf, 1, (double*)fo), 0);        // workspace too small
  EXPECT(miner_global_auc(st, fb, ub, -5, buf, 4096, (double*)fo), 0);

  printf("abi_errors: %d calls, %d failures\n", g_calls, g_fail);
  return g_fail ? 1 : 0;
}
