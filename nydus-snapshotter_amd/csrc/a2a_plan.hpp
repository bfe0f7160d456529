// a2a_plan.hpp — the argument sets of the node step's all-to-alls
// (node.hip, ngpu_node_process_step; SURVEY.md §8(e) "Collective"), shared by
// its two transports -- RCCL ncclAllToAllv and hipMemcpyPeerAsync -- and
// checked on the CPU by tests/cpp/a2a_plan_test.cpp (no GPU, no RCCL).
// Header-only, host-only; needs <stddef.h> and <stdint.h>.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace ngpu {

// One all-to-all-v of `row`-byte rows: rank i sends cnt(i, j) rows from row
// sdis(i, j) of its send buffer to rank j, which stores them at row
// rdis(j, i) of its receive buffer.  ncclAllToAllv takes, on rank i, byte
// counts and displacements per peer j (datatype ncclUint8):
//   sc[j] = cnt(i, j) row   sd[j] = sdis(i, j) row   (what i sends to j)
//   rc[j] = cnt(j, i) row   rd[j] = rdis(i, j) row   (what i receives from j)
// The peer-copy transport moves the same bytes: cnt(i, j) row bytes from
// src_i + sdis(i, j) row to dst_j + rdis(j, i) row.
template <class Cnt, class Sdis, class Rdis>
inline void a2a_rank_args(uint32_t W, uint32_t i, uint64_t row, Cnt cnt, Sdis sdis, Rdis rdis,
                          size_t *sc, size_t *sd, size_t *rc, size_t *rd) {
  for (uint32_t j = 0; j < W; ++j) {
    sc[j] = (size_t)(cnt(i, j) * row);
    sd[j] = (size_t)(sdis(i, j) * row);
    rc[j] = (size_t)(cnt(j, i) * row);
    rd[j] = (size_t)(rdis(i, j) * row);
  }
}

// The node step's padded layout: part i of W holds n[i] chunk rows.  Its
// digests, bucketed by owner (launch_route with seg_cap = n[i]), sit at rows
// [j n[i], j n[i] + c_ij) of its send buffer for owner j, the rest of each
// segment padding (row id ~0).  Every (i, j) pair therefore moves n[i] rows
// whatever c_ij is, so the transfer sizes are known on the host when the step
// is enqueued and the per-owner counts travel in band (one u32 per pair)
// instead of reaching the host mid-step.  Owner j keeps requester i's block
// at row off[i] = n[0] + ... + n[i-1] of its receive buffer (R = the sum of
// all n rows) and probes its first c_ij rows; the hits go back the same way.
struct PaddedStep {
  uint32_t W = 0;
  const uint64_t *n = nullptr;    // rows per part
  const uint64_t *off = nullptr;  // W + 1 prefix sums of n
  // digests, requester i -> owner j
  uint64_t fwd_cnt(uint32_t i, uint32_t) const { return n[i]; }
  uint64_t fwd_sdis(uint32_t i, uint32_t j) const { return (uint64_t)j * n[i]; }
  uint64_t fwd_rdis(uint32_t, uint32_t i) const { return off[i]; }
  // hits, owner j -> requester i
  uint64_t back_cnt(uint32_t, uint32_t i) const { return n[i]; }
  uint64_t back_sdis(uint32_t, uint32_t i) const { return off[i]; }
  uint64_t back_rdis(uint32_t i, uint32_t j) const { return (uint64_t)j * n[i]; }
  // counts (one u32 row per pair), requester i's cnt[j] -> owner j's rcnt[i]
  static uint64_t cnt_cnt(uint32_t, uint32_t) { return 1; }
  static uint64_t cnt_sdis(uint32_t, uint32_t j) { return j; }
  static uint64_t cnt_rdis(uint32_t, uint32_t i) { return i; }
};

}  // namespace ngpu
