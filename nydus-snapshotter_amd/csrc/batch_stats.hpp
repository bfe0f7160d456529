// batch_stats.hpp — each layer's stats out of a batched launch set
// (batch.hip): the call's counter words and the layer's own ngpu_layer_stats,
// into its pack's pinned read-back words (read_stats_parse layout).
//
// The error words are the layer's own: a batch's digest and dedup
// kernels count bad descriptors, overlaps and unhashed chunks for the whole
// launch set, and the first unhashed chunk id is a batch-wide id.  A chunk
// whose descriptor was bad, or that overlapped, reaches the dedup stage
// without a digest and is marked NGPU_UNHASHED in its record, so the layer
// that raised an error is the layer holding such a record: block k counts the
// NGPU_UNHASHED records of layer k and takes the smallest layer-relative id.
// A layer with none reports no error; a layer with some reports them and,
// for the message, the launch set's bad-descriptor / overlap counts.
// Included by batch.hip and by tests/cpp/batch_stats_test.hip.
#pragma once

#include "engine_internal.hpp"

namespace ngpu {

// Block k = layer k.  st: the launch set's counter words (kStWords); lst: the
// per-layer stats; res: the launch set's results (chunk i of layer k at
// lfirst[k] + i); dst[k]: layer k's pinned read-back words.
__global__ __launch_bounds__(256) void batch_stats_out(const uint64_t *__restrict__ st,
                                                       const ngpu_layer_stats *__restrict__ lst,
                                                       const ngpu_result *__restrict__ res,
                                                       const uint64_t *__restrict__ lfirst,
                                                       uint64_t *const *__restrict__ dst) {
  const uint32_t k = blockIdx.x, t = threadIdx.x;
  __shared__ unsigned long long cnt, first;
  if (t == 0) cnt = 0, first = ~0ull;
  __syncthreads();
  const uint64_t a = lfirst[k], b = lfirst[k + 1];
  unsigned long long c = 0, f = ~0ull;
  for (uint64_t i = a + t; i < b; i += blockDim.x)
    if (res[i].kind == NGPU_UNHASHED) {
      ++c;
      if (i - a < f) f = i - a;
    }
  if (c) {
    atomicAdd(&cnt, c);
    atomicMin(&first, f);
  }
  __syncthreads();
  constexpr uint32_t kL = sizeof(ngpu_layer_stats) / sizeof(uint64_t);
  static_assert(sizeof(ngpu_layer_stats) % sizeof(uint64_t) == 0, "layer stats are whole words");
  uint64_t *d = dst[k];
  if (t < (uint32_t)kStWords) {
    uint64_t v = st[t];
    if (t == kStBadDesc || t == kStOverlap) v = cnt ? v : 0;
    if (t == kStUnhashed) v = cnt;
    if (t == kStUnhashedFirst) v = cnt ? ~(uint64_t)first : 0;
    d[t] = v;
  }
  if (t < kL) d[kStatsLayer + t] = reinterpret_cast<const uint64_t *>(lst + k)[t];
}

}  // namespace ngpu
