// a2a_plan_test.cpp — the node step's all-to-all arguments (csrc/a2a_plan.hpp)
// on the CPU, no GPU and no RCCL.  For W = 1..8 parts with
// skewed row counts (empty parts, one owner taking most rows) it runs the
// whole padded step on host buffers -- route into padded segments, counts
// and digests to the owners, owner probe of the counted rows, hits back,
// scatter by row id -- once under ncclAllToAllv's semantics (rank i's
// sc/sd/rc/rd from a2a_rank_args) and once under the peer-copy transport's,
// and checks under both that every sender's count
// equals its receiver's, that no receive region overlaps another or leaves
// its buffer, and that every row gets exactly its owner's hit.
// usage: a2a_plan_test [seed]   -> prints "ok <cases>"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "a2a_plan.hpp"

using namespace ngpu;
typedef std::vector<uint8_t> Buf;

static int fails = 0;
#define CHECK(c, ...)                     \
  do {                                    \
    if (!(c)) {                           \
      fprintf(stderr, __VA_ARGS__);       \
      fprintf(stderr, "\n");              \
      ++fails;                            \
      return;                             \
    }                                     \
  } while (0)

// ncclAllToAllv on every rank at once: rank i sends sc[j] bytes at sd[j] to
// j; j receives rc[i] bytes at rd[i].
template <class C, class S, class R>
static void rccl_like(uint32_t W, uint64_t row, C cnt, S sdis, R rdis, const std::vector<Buf> &src,
                      std::vector<Buf> &dst) {
  std::vector<std::vector<size_t>> sc(W, std::vector<size_t>(W)), sd = sc, rc = sc, rd = sc;
  for (uint32_t i = 0; i < W; ++i)
    a2a_rank_args(W, i, row, cnt, sdis, rdis, sc[i].data(), sd[i].data(), rc[i].data(), rd[i].data());
  for (uint32_t j = 0; j < W; ++j) {
    std::vector<uint8_t> used(dst[j].size(), 0);
    for (uint32_t i = 0; i < W; ++i) {
      CHECK(sc[i][j] == rc[j][i], "W %u: rank %u sends %zu B to %u, which expects %zu", W, i,
            sc[i][j], j, rc[j][i]);
      CHECK(sd[i][j] + sc[i][j] <= src[i].size(), "W %u: send %u->%u past the buffer", W, i, j);
      CHECK(rd[j][i] + rc[j][i] <= dst[j].size(), "W %u: receive %u<-%u past the buffer", W, j, i);
      for (size_t b = 0; b < rc[j][i]; ++b) {
        CHECK(!used[rd[j][i] + b], "W %u: receive regions overlap on rank %u", W, j);
        used[rd[j][i] + b] = 1;
      }
      if (sc[i][j]) memcpy(dst[j].data() + rd[j][i], src[i].data() + sd[i][j], sc[i][j]);
    }
  }
}

// the peer-copy transport (node.hip step_alltoallv without RCCL)
template <class C, class S, class R>
static void peer_like(uint32_t W, uint64_t row, C cnt, S sdis, R rdis, const std::vector<Buf> &src,
                      std::vector<Buf> &dst) {
  for (uint32_t i = 0; i < W; ++i)
    for (uint32_t j = 0; j < W; ++j)
      if (cnt(i, j)) memcpy(dst[j].data() + rdis(j, i) * row, src[i].data() + sdis(i, j) * row, cnt(i, j) * row);
}

static uint32_t owner_of(uint64_t v, uint32_t W, uint32_t skew) {
  // skew: a hot owner 0 takes ~skew % of the rows
  const uint32_t h = (uint32_t)((v * 0x9E3779B97F4A7C15ull) >> 40);
  return (h % 100) < skew ? 0 : (uint32_t)(((uint64_t)(h & 0xFFFF) * W) >> 16);
}

static void run_case(uint32_t W, const std::vector<uint64_t> &n, uint32_t skew, bool rccl) {
  std::vector<uint64_t> off(W + 1, 0);
  for (uint32_t i = 0; i < W; ++i) off[i + 1] = off[i] + n[i];
  const PaddedStep ps{W, n.data(), off.data()};
  const uint64_t R = off[W];
  // route: requester i's rows into padded segments; a "digest" = (i, r)
  std::vector<Buf> xq(W), xrow(W), cnt(W), rcnt(W, Buf(W * 4, 0xEE)), rq(W, Buf(R * 8, 0xEE)),
      rh(W, Buf(R * 8, 0xEE)), sh(W);
  for (uint32_t i = 0; i < W; ++i) {
    xq[i].assign(W * n[i] * 8, 0xEE);
    xrow[i].assign(W * n[i] * 4, 0xFF);
    sh[i].assign(W * n[i] * 8, 0xEE);
    cnt[i].assign(W * 4, 0);
    uint32_t *c = (uint32_t *)cnt[i].data();
    for (uint64_t r = 0; r < n[i]; ++r) {
      const uint64_t v = (uint64_t)i << 32 | r;
      const uint32_t o = owner_of(v, W, skew);
      const uint64_t pos = o * n[i] + c[o]++;
      memcpy(xq[i].data() + pos * 8, &v, 8);
      const uint32_t rr = (uint32_t)r;
      memcpy(xrow[i].data() + pos * 4, &rr, 4);
    }
  }
  auto a2a = [&](uint64_t row, auto cntf, auto sdisf, auto rdisf, const std::vector<Buf> &src,
                 std::vector<Buf> &dst) {
    if (rccl)
      rccl_like(W, row, cntf, sdisf, rdisf, src, dst);
    else
      peer_like(W, row, cntf, sdisf, rdisf, src, dst);
  };
  a2a(4, PaddedStep::cnt_cnt, PaddedStep::cnt_sdis, PaddedStep::cnt_rdis, cnt, rcnt);
  a2a(8, [&](uint32_t i, uint32_t j) { return ps.fwd_cnt(i, j); },
      [&](uint32_t i, uint32_t j) { return ps.fwd_sdis(i, j); },
      [&](uint32_t j, uint32_t i) { return ps.fwd_rdis(j, i); }, xq, rq);
  // owner j probes the counted rows of each block: hit = digest * 3 + j
  for (uint32_t j = 0; j < W; ++j) {
    const uint32_t *rc = (const uint32_t *)rcnt[j].data();
    for (uint32_t i = 0; i < W; ++i) {
      CHECK(rc[i] == ((const uint32_t *)cnt[i].data())[j], "W %u: owner %u got count %u from %u", W,
            j, rc[i], i);
      CHECK(rc[i] <= n[i], "W %u: count past the block", W);
      for (uint64_t k = 0; k < rc[i]; ++k) {
        uint64_t v;
        memcpy(&v, rq[j].data() + (off[i] + k) * 8, 8);
        CHECK(owner_of(v, W, skew) == j && (v >> 32) == i, "W %u: owner %u got a row of owner %u", W,
              j, owner_of(v, W, skew));
        const uint64_t h = v * 3 + j;
        memcpy(rh[j].data() + (off[i] + k) * 8, &h, 8);
      }
    }
  }
  a2a(8, [&](uint32_t j, uint32_t i) { return ps.back_cnt(j, i); },
      [&](uint32_t j, uint32_t i) { return ps.back_sdis(j, i); },
      [&](uint32_t i, uint32_t j) { return ps.back_rdis(i, j); }, rh, sh);
  // scatter by row id, padding dropped; every row exactly its owner's hit
  for (uint32_t i = 0; i < W; ++i) {
    std::vector<uint64_t> hits(n[i], ~0ull);
    for (uint64_t k = 0; k < W * n[i]; ++k) {
      uint32_t r;
      memcpy(&r, xrow[i].data() + k * 4, 4);
      if (r == 0xFFFFFFFFu) continue;
      CHECK(hits[r] == ~0ull, "W %u: row %u of part %u scattered twice", W, r, i);
      memcpy(&hits[r], sh[i].data() + k * 8, 8);
    }
    for (uint64_t r = 0; r < n[i]; ++r) {
      const uint64_t v = (uint64_t)i << 32 | r;
      CHECK(hits[r] == v * 3 + owner_of(v, W, skew), "W %u: part %u row %llu wrong hit", W, i,
            (unsigned long long)r);
    }
  }
}

int main(int argc, char **argv) {
  std::mt19937_64 rng(argc > 1 ? strtoull(argv[1], nullptr, 10) : 5);
  int cases = 0;
  for (uint32_t W : {1u, 2u, 3u, 4u, 8u}) {
    for (int t = 0; t < 12; ++t) {
      std::vector<uint64_t> n(W);
      for (uint32_t i = 0; i < W; ++i) {
        const uint64_t k = rng() % 5;
        n[i] = k == 0 ? 0 : k == 1 ? 1 + rng() % 3 : k == 4 ? 2000 + rng() % 3000 : rng() % 700;
      }
      const uint32_t skew = (uint32_t)(t % 3 == 0 ? 0 : t % 3 == 1 ? 60 : 95);
      for (bool rccl : {true, false}) {
        run_case(W, n, skew, rccl);
        ++cases;
        if (fails) return 1;
      }
    }
  }
  printf("ok %d\n", cases);
  return 0;
}
