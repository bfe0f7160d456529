// batch_lanes.hpp — which batch lane is free, as host state (csrc/batch.hip).
//
// A lane runs one batch at a time. A leader takes an idle lane for batch
// number s. The first of that batch's packs to see it end frees the lane, and
// only that batch can: a pack of the lane's previous batch that comes back
// late carries an older number and changes nothing. (When the end marker was
// set outside the batcher's lock, such a late pack freed a lane whose next
// batch was running, and the leader after it reused the lane's buffers under
// that batch.) All calls are made under the batcher's mutex; plain C++, no
// HIP, so tests/cpp/batch_lanes_test.cpp drives it on the CPU.
#pragma once
#include <stdint.h>

namespace ngpu {

template <int N>
struct LaneTable {
  bool running[N] = {};
  uint64_t lane_seq[N] = {};  // the batch each lane was last taken for
  uint64_t seq = 0;           // batches taken so far

  // An idle lane, or -1.
  int idle() const {
    for (int k = 0; k < N; ++k)
      if (!running[k]) return k;
    return -1;
  }
  // Take idle lane k for the next batch; returns that batch's number.
  uint64_t take(int k) {
    running[k] = true;
    lane_seq[k] = ++seq;
    return seq;
  }
  // Batch s on lane k was seen to end: true if that freed the lane (the
  // first report of the batch the lane runs now).
  bool end(int k, uint64_t s) {
    if (!running[k] || lane_seq[k] != s) return false;
    running[k] = false;
    return true;
  }
  // The launch of lane k's batch failed and was drained: the lane is free.
  void drop(int k) { running[k] = false; }
};

}  // namespace ngpu
