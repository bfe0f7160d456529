#!/usr/bin/env python3
"""Generates tools/valu_bank.hip: does the VGPR bank of a VALU op's sources
set its issue rate on gfx950, and how fast does the BLAKE3 compression
stream run under different register assignments?  (the
bare compression stream runs at 0.785 of the linear 2-/4-cycle issue model.)

Every variant is ONE inline-asm block per loop trip with physical VGPRs
(clobbered, so the compiler keeps its own values elsewhere); s_memtime
(shader clock) brackets the loop in every wave.  Bank of vN = N mod 4.
usage: tools/gen_valu_bank.py [blake3.s]  (the .s: the product kernel's
hot loop, replayed verbatim as variant `compiled`)"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]


def sched():
    cur, out = list(range(16)), []
    for _ in range(7):
        out.append(cur[:])
        cur = [cur[PERM[i]] for i in range(16)]
    return out


def g4(st, cols, ms, emit):
    """B3_G4's order: the 4 G of a step in lockstep (csrc/b3_compress.hpp)."""
    a = [st[c[0]] for c in cols]; b = [st[c[1]] for c in cols]
    c_ = [st[c[2]] for c in cols]; d = [st[c[3]] for c in cols]
    x, y = ms[:4], ms[4:]
    for i in range(4): emit(f"v_add3_u32 v{a[i]}, v{a[i]}, v{b[i]}, v{x[i]}")
    for i in range(4): emit(f"v_xor_b32 v{d[i]}, v{d[i]}, v{a[i]}")
    for i in range(4): emit(f"v_alignbit_b32 v{d[i]}, v{d[i]}, v{d[i]}, 16")
    for i in range(4): emit(f"v_add_u32 v{c_[i]}, v{c_[i]}, v{d[i]}")
    for i in range(4): emit(f"v_xor_b32 v{b[i]}, v{b[i]}, v{c_[i]}")
    for i in range(4): emit(f"v_alignbit_b32 v{b[i]}, v{b[i]}, v{b[i]}, 12")
    for i in range(4): emit(f"v_add3_u32 v{a[i]}, v{a[i]}, v{b[i]}, v{y[i]}")
    for i in range(4): emit(f"v_xor_b32 v{d[i]}, v{d[i]}, v{a[i]}")
    for i in range(4): emit(f"v_alignbit_b32 v{d[i]}, v{d[i]}, v{d[i]}, 8")
    for i in range(4): emit(f"v_add_u32 v{c_[i]}, v{c_[i]}, v{d[i]}")
    for i in range(4): emit(f"v_xor_b32 v{b[i]}, v{b[i]}, v{c_[i]}")
    for i in range(4): emit(f"v_alignbit_b32 v{b[i]}, v{b[i]}, v{b[i]}, 7")


COLS = [(0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15)]
DIAG = [(0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)]


def compression(st, mreg):
    out = []
    for s in sched():
        g4(st, COLS, [mreg[s[j]] for j in (0, 2, 4, 6, 1, 3, 5, 7)], out.append)
        g4(st, DIAG, [mreg[s[j]] for j in (8, 10, 12, 14, 9, 11, 13, 15)], out.append)
    return out


def streams(compiled_s=None):
    v = {}
    # single-op streams, 8 independent chains, 256 ops per trip
    def rep(fmt, n=256):
        return [fmt(i % 8) for i in range(n)]
    v["xor_same"] = rep(lambda i: f"v_xor_b32 v{i}, v{i}, v{8 + i}")          # banks equal
    v["xor_diff"] = rep(lambda i: f"v_xor_b32 v{i}, v{i}, v{9 + i}")          # banks differ
    v["add_same"] = rep(lambda i: f"v_add_u32 v{i}, v{i}, v{8 + i}")
    v["add_diff"] = rep(lambda i: f"v_add_u32 v{i}, v{i}, v{9 + i}")
    v["add3_same"] = rep(lambda i: f"v_add3_u32 v{i}, v{i}, v{8 + i}, v{16 + i}")
    v["add3_diff"] = rep(lambda i: f"v_add3_u32 v{i}, v{i}, v{9 + i}, v{18 + i}")
    v["align"] = rep(lambda i: f"v_alignbit_b32 v{i}, v{i}, v{i}, 7")
    v["bitop3_diff"] = rep(lambda i: f"v_bitop3_b32 v{i}, v{i}, v{9 + i}, v{18 + i} bitop3:0x96")
    v["bitop3_same"] = rep(lambda i: f"v_bitop3_b32 v{i}, v{i}, v{8 + i}, v{16 + i} bitop3:0x96")
    # xor / alignbit alternating in runs of 4 (the G shape)
    v["mix_x4a4_diff"] = [(f"v_xor_b32 v{i % 8}, v{i % 8}, v{9 + i % 8}" if (i // 4) % 2 == 0
                           else f"v_alignbit_b32 v{i % 8}, v{i % 8}, v{i % 8}, 7") for i in range(256)]
    v["mix_x4a4_same"] = [(f"v_xor_b32 v{i % 8}, v{i % 8}, v{8 + i % 8}" if (i // 4) % 2 == 0
                           else f"v_alignbit_b32 v{i % 8}, v{i % 8}, v{i % 8}, 7") for i in range(256)]
    # slow / fast runs of length n (alignbit then xor, 8 chains): the cost of
    # a switch between the 4-cycle and the 2-cycle ops
    for n in (1, 8, 16, 32):
        ops = []
        while len(ops) < 256:
            ops += [f"v_alignbit_b32 v{i % 8}, v{i % 8}, v{i % 8}, 7" for i in range(n)]
            ops += [f"v_xor_b32 v{i % 8}, v{i % 8}, v{9 + i % 8}" for i in range(n)]
        v[f"mix_s{n}f{n}"] = ops[:256]
    # the x4a4 mix with an s_barrier every k ops: waves of one workgroup
    # that share a SIMD kept in phase, so both sit in a 2-cycle run together
    for k in (32, 128):
        ops = []
        for i, o in enumerate(v["mix_x4a4_diff"]):
            ops.append(o)
            if (i + 1) % k == 0:
                ops.append("s_barrier")
        v[f"mix_x4a4_bar{k}"] = ops
    # one BLAKE3 compression (672 G ops) under three register assignments
    # state word k -> VGPR: "conflict" = k (a column step's a,b,c,d share a bank)
    v["comp_conflict"] = compression(list(range(16)), [16 + j for j in range(16)])
    # "distinct": bank = role (a 0, b 1, c 2, d 3); message words in banks 2 / 3
    role = [4 * (k % 4) + k // 4 for k in range(16)]
    v["comp_distinct"] = compression(role, [16 + 4 * (j // 2) + 2 + (j % 2) for j in range(16)])
    if compiled_s:
        v["compiled"] = compiled_stream(compiled_s)
        # the same G stream with the compiler's hazard pads kept (s_nop 0
        # after most pairs of ops, as the product kernel issues it), and with
        # pads placed by rule: s_nop K after every N VALU ops
        v["compiled_raw"] = compiled_stream(compiled_s, keep_nops=True)
        g = v["compiled"]
        for n_, k_ in ((1, 0), (2, 0), (4, 0), (2, 1), (2, 3), (8, 0)):
            ops = []
            for i, o in enumerate(g):
                ops.append(o)
                if (i + 1) % n_ == 0:
                    ops.append(f"s_nop {k_}")
            v[f"comp_nop{k_}_every{n_}"] = ops
        for k in (48, 96):  # a barrier after every (second) G4 step
            ops = []
            for i, o in enumerate(v["compiled"]):
                ops.append(o)
                if (i + 1) % k == 0:
                    ops.append("s_barrier")
            v[f"compiled_bar{k}"] = ops
    return v


def compiled_stream(path, keep_nops=False):
    """The product kernel's whole-leaf loop (b3_groups<3,0>, the block with
    the most v_alignbit) from 672 ops before its last G op: one compression's
    G stream with the compiler's registers."""
    text = open(path).read()
    k = "_ZN4ngpu12_GLOBAL__N_19b3_groupsILi3ELi0EE"
    body = text[text.index("\n" + k + "EvPKh") + 1:]
    body = body[body.index("\n") + 1: body.index(".Lfunc_end")]
    blocks, cur = [], []
    for line in body.splitlines():
        s = line.strip()
        if re.match(r"^\.LBB\w+:", s):
            blocks.append(cur)
            cur = []
            continue
        if s.startswith(("v_add3_u32", "v_xor_b32", "v_alignbit_b32", "v_add_u32")) or \
                (keep_nops and s.startswith("s_nop")):
            cur.append(s.split(";")[0].strip())
    blocks.append(cur)
    best = max(blocks, key=lambda b: sum(1 for m in b if m.startswith("v_alignbit")))
    # first run of 672 ops that starts with 4 v_add3 and holds 224 alignbit
    valu = [j for j, x in enumerate(best) if not x.startswith("s_nop")]
    for a in range(len(valu) - 672):
        seg = [best[j] for j in valu[a:a + 672]]
        if all(x.startswith("v_add3") for x in seg[:4]) and \
                sum(1 for x in seg if x.startswith("v_alignbit")) == 224:
            seg = best[valu[a]:valu[a + 671] + 1]  # with the pads between them, if kept
            return [x.replace("_e32", "").replace("_e64", "") for x in seg]
    raise SystemExit("no 672-op G stream in the hot block")


def regs(ops):
    r = set()
    for o in ops:
        r.update(int(x) for x in re.findall(r"\bv(\d+)\b", o))
    return sorted(r)


def main():
    vs = streams(sys.argv[1] if len(sys.argv) > 1 else None)
    out = ["// GENERATED by tools/gen_valu_bank.py -- see its docstring.",
           "#include <hip/hip_runtime.h>", "#include <stdint.h>", "#include <stdio.h>",
           "#include <stdlib.h>", "#include <string.h>", ""]
    names = []
    for name, ops in vs.items():
        rs = regs(ops)
        clob = ", ".join(f'"v{r}"' for r in rs)
        body = "\\n\\t".join(ops)
        out += [f"__global__ __launch_bounds__(1024) void k_{name}(uint64_t *rec, uint32_t iters) {{",
                "  uint64_t t0, t1;",
                '  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");',
                "  for (uint32_t it = 0; it < iters; ++it)",
                f'    asm volatile("{body}" ::: {clob});',
                '  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");',
                "  if ((threadIdx.x & 63) == 0) {",
                "    const uint64_t w = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64;",
                "    rec[4 * w] = t0; rec[4 * w + 1] = t1;",
                "    rec[4 * w + 2] = __builtin_amdgcn_s_getreg(0xF804);  // HW_REG_HW_ID, 32 bits",
                "    rec[4 * w + 3] = __builtin_amdgcn_s_getreg(0x7814);  // HW_REG_XCC_ID, 16 bits",
                "  }",
                "}", ""]
        names.append((name, sum(1 for o in ops if o.startswith("v_")), max(rs) + 1))
    out.append("struct V { const char *name; void (*k)(uint64_t *, uint32_t); int ops; int regs; };")
    out.append("static const V kV[] = {")
    out += [f'  {{"{n}", k_{n}, {c}, {r}}},' for n, c, r in names]
    out.append("};")
    out.append(MAIN)
    open(os.path.join(ROOT, "tools", "valu_bank.hip"), "w").write("\n".join(out) + "\n")


MAIN = r'''
#include <map>
#include <vector>
#include <algorithm>

// One launch: per-wave start / end (s_memtime, shader clock, per XCD),
// HW_ID and XCC_ID.  Reported: the waves per SIMD (histogram), and each
// SIMD's issue rate = (last end - first start) / (wave-instructions of its
// waves), by how many waves it held; the kernel's time = the slowest SIMD.
static void run(const V &v, int w, int threads, int rounds, uint64_t *d, uint64_t *h, int simds) {
  const int waves_total = simds * w * rounds;
  const int blocks = waves_total / (threads / 64);
  const uint32_t iters = (uint32_t)((v.ops > 300 ? 400 : 1000) / rounds);
  hipLaunchKernelGGL(v.k, dim3(blocks), dim3(threads), 0, 0, d, iters);  // warm / clock ramp
  hipLaunchKernelGGL(v.k, dim3(blocks), dim3(threads), 0, 0, d, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(v.k, dim3(blocks), dim3(threads), 0, 0, d, iters);
  (void)hipEventRecord(e1);
  if (hipEventSynchronize(e1) != hipSuccess) exit(2);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const size_t nw = (size_t)blocks * threads / 64;
  (void)hipMemcpy(h, d, nw * 32, hipMemcpyDeviceToHost);
  struct S { uint64_t t0 = ~0ull, t1 = 0; int n = 0; };
  std::map<uint64_t, S> simd;
  std::vector<uint64_t> life(nw);
  for (size_t i = 0; i < nw; ++i) {
    const uint64_t *r = h + 4 * i;
    const uint64_t key = (r[3] & 0xF) << 16 | ((r[2] >> 4) & 0xFFF);  // xcc | se/sh/cu/pipe/simd
    S &s = simd[key];
    s.t0 = std::min(s.t0, r[0]);
    s.t1 = std::max(s.t1, r[1]);
    s.n++;
    life[i] = r[1] - r[0];
  }
  std::sort(life.begin(), life.end());
  int hist[64] = {0};
  double cpi_n[64] = {0};
  uint64_t span_max = 0;
  for (auto &kv : simd) {
    const S &s = kv.second;
    const int n = s.n < 63 ? s.n : 63;
    hist[n]++;
    cpi_n[n] += (double)(s.t1 - s.t0) / ((double)s.n * iters * v.ops);
    span_max = std::max(span_max, s.t1 - s.t0);
  }
  printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"threads\": %d, \"rounds\": %d, "
         "\"ops_per_trip\": %d, \"vgprs_named\": %d, \"ms\": %.4f, \"simds_seen\": %zu, "
         "\"kernel_cycles_est\": %llu, \"clock_ghz_est\": %.3f, "
         "\"kernel_cpi_per_simd\": %.4f, \"wave_life_min_med_max\": [%llu, %llu, %llu], "
         "\"waves_per_simd_hist\": {",
         v.name, w, threads, rounds, v.ops, v.regs, ms, simd.size(),
         (unsigned long long)span_max, span_max / (ms * 1e6),
         (double)span_max / ((double)w * rounds * iters * v.ops), (unsigned long long)life[0],
         (unsigned long long)life[nw / 2], (unsigned long long)life[nw - 1]);
  bool first = true;
  for (int n = 1; n < 64; ++n)
    if (hist[n]) {
      printf("%s\"%d\": [%d, %.4f]", first ? "" : ", ", n, hist[n], cpi_n[n] / hist[n]);
      first = false;
    }
  printf("}}\n");
  fflush(stdout);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

// usage: valu_bank [variant-substring] [threads] [rounds]
//   -> one JSON line per (variant, waves/SIMD); hist "n": [SIMDs holding n
//   waves, their mean cycles per wave-instruction over the SIMD's busy span]
int main(int argc, char **argv) {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int simds = prop.multiProcessorCount * 4;
  const int threads = argc > 2 ? atoi(argv[2]) : 256;
  const int rounds = argc > 3 ? atoi(argv[3]) : 1;
  uint64_t *d;
  const size_t maxw = (size_t)simds * 8 * rounds;
  if (hipMalloc(&d, maxw * 32) != hipSuccess) return 1;
  uint64_t *h = (uint64_t *)malloc(maxw * 32);
  for (const V &v : kV) {
    if (argc > 1 && strcmp(argv[1], "all") && !strstr(v.name, argv[1])) continue;
    for (int w : {1, 2, 3, 4, 5, 6, 8}) {
      if (w * ((v.regs + 16 + 7) / 8 * 8) > 512) continue;  // cannot hold w waves per SIMD
      if ((simds * w * rounds) % (threads / 64)) continue;
      run(v, w, threads, rounds, d, h, simds);
    }
  }
  (void)hipFree(d);
  free(h);
  return 0;
}
'''

if __name__ == "__main__":
    main()
