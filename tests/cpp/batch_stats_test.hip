// batch_stats_test.hip — the per-layer error words of a batched launch set
// (csrc/batch_stats.hpp): one layer of a batch with unhashed
// chunks, the others clean.  Only that layer may report an error, with its
// own count and its own (layer-relative) first chunk id; the clean layers
// report none even though the launch set's counters are non-zero.
// Prints "PASS"; exit 1 on failure.
#include <stdio.h>
#include <string.h>

#include <vector>

#include "batch_stats.hpp"

#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                   \
    }                                                             \
  } while (0)
#define HIPOK(x) CHECK((x) == hipSuccess)

int main() {
  using namespace ngpu;
  const uint64_t first[] = {0, 700, 1300, 5000};  // layers of 700, 600 and 3700 chunks
  const uint32_t K = 3;
  const uint64_t N = first[K];
  std::vector<ngpu_result> res(N);
  memset(res.data(), 0, N * sizeof(ngpu_result));
  for (uint64_t i = 0; i < N; ++i) res[i].kind = NGPU_NEW;
  for (uint64_t i : {1300 + 3000ull, 1300 + 45ull, 1300 + 2999ull})  // layer 2: ids 45, 2999, 3000
    res[i].kind = NGPU_UNHASHED;
  std::vector<uint64_t> st(kStWords, 0);
  st[kStBadDesc] = 3;  // the launch set's counters
  st[kStUnhashed] = 3;
  st[kStUnhashedFirst] = ~(uint64_t)(1300 + 45);  // a batch-wide id
  std::vector<ngpu_layer_stats> lst(K);
  for (uint32_t k = 0; k < K; ++k) {
    memset(&lst[k], 0, sizeof lst[k]);
    lst[k].chunks = first[k + 1] - first[k];
  }
  ngpu_result *d_res;
  uint64_t *d_st, *d_first, *d_words;
  ngpu_layer_stats *d_lst;
  uint64_t **d_dst;
  HIPOK(hipMalloc(&d_res, N * sizeof(ngpu_result)));
  HIPOK(hipMalloc(&d_st, kStWords * 8));
  HIPOK(hipMalloc(&d_first, sizeof first));
  HIPOK(hipMalloc(&d_lst, K * sizeof(ngpu_layer_stats)));
  HIPOK(hipMalloc(&d_words, K * 32 * 8));
  HIPOK(hipMalloc(&d_dst, K * sizeof(uint64_t *)));
  std::vector<uint64_t *> dst(K);
  for (uint32_t k = 0; k < K; ++k) dst[k] = d_words + 32 * k;
  HIPOK(hipMemcpy(d_res, res.data(), N * sizeof(ngpu_result), hipMemcpyHostToDevice));
  HIPOK(hipMemcpy(d_st, st.data(), kStWords * 8, hipMemcpyHostToDevice));
  HIPOK(hipMemcpy(d_first, first, sizeof first, hipMemcpyHostToDevice));
  HIPOK(hipMemcpy(d_lst, lst.data(), K * sizeof(ngpu_layer_stats), hipMemcpyHostToDevice));
  HIPOK(hipMemcpy(d_dst, dst.data(), K * sizeof(uint64_t *), hipMemcpyHostToDevice));
  HIPOK(hipMemset(d_words, 0xAB, K * 32 * 8));
  hipLaunchKernelGGL(batch_stats_out, dim3(K), dim3(256), 0, 0, d_st, d_lst, d_res, d_first, d_dst);
  HIPOK(hipGetLastError());
  std::vector<uint64_t> w(K * 32);
  HIPOK(hipMemcpy(w.data(), d_words, K * 32 * 8, hipMemcpyDeviceToHost));
  for (uint32_t k = 0; k < K; ++k) {
    const uint64_t *x = w.data() + 32 * k;
    ngpu_layer_stats got;
    memcpy(&got, x + kStatsLayer, sizeof got);
    CHECK(got.chunks == first[k + 1] - first[k]);
    if (k == 2) {
      CHECK(x[kStUnhashed] == 3);
      CHECK(~x[kStUnhashedFirst] == 45);  // the layer's own chunk id
      CHECK(x[kStBadDesc] == 3);          // (the launch set's, for the message)
    } else {
      CHECK(x[kStUnhashed] == 0 && x[kStUnhashedFirst] == 0);
      CHECK(x[kStBadDesc] == 0 && x[kStOverlap] == 0);
    }
  }
  printf("PASS\n");
  return 0;
}
