#!/usr/bin/env python3
"""ISA mix of the dominant kernel's hot loop, for roofline.peak_mix (VERDICT
r3 item 4).  Emits gfx950 assembly of csrc/blake3.hip (hipcc -S), takes the
basic block of b3_groups<3,0> with the most v_alignbit_b32 (the whole-leaf
fast loop: two compressions per trip), and classes its VALU ops by the issue
cost measured on this chip (tools/valu_ops.hip, valu_ops2.hip;
profiles/r1/valu_*_issue_rates.jsonl): 3-operand / shift-left ops issue at 4
cycles per wave64 instruction, the 2-operand logic / add / move ops at 2.
The mix ceiling is 1024 SIMDs x 64 lanes x clock / (issue cycles per
algorithmic op).
usage: tools/isa_mix.py OUT.json [ASM.s]"""
import json
import os
import re
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FOUR = re.compile(r"^v_(alignbit|alignbyte|add3|xad|perm|bfi|lshlrev|lshl_add|lshl_or|and_or|or3|"
                  r"mad|bfe|lshl_b64|lshrrev_b64|cndmask)")
TWO = re.compile(r"^v_(xor_b32|add_u32|add_co|addc|or_b32|and_b32|lshrrev_b32|bitop3|mov_b32|"
                 r"sub_u32|not_b32)")
KERNEL = "_ZN4ngpu12_GLOBAL__N_19b3_groupsILi3ELi0EE"


def asm_text(path=None):
    if path:
        return open(path).read()
    out = "/tmp/isa_mix_blake3.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                           "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I",
                           os.path.join(ROOT, "nydus-snapshotter_amd", "csrc"),
                           os.path.join(ROOT, "nydus-snapshotter_amd", "csrc", "blake3.hip"),
                           "-o", out])
    return open(out).read()


def blocks(text, kernel):
    body = text[text.index("\n" + kernel + "EvPKh") + 1:]
    body = body[body.index("\n") + 1: body.index(".Lfunc_end")]
    cur, name = [], "entry"
    for line in body.splitlines():
        s = line.strip()
        if re.match(r"^\.LBB\w+:", s):
            yield name, cur
            cur, name = [], s.split(":")[0]
            continue
        if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
            continue
        cur.append(s.split()[0])
    yield name, cur


def main():
    out = sys.argv[1]
    text = asm_text(sys.argv[2] if len(sys.argv) > 2 else None)
    best = max(blocks(text, KERNEL), key=lambda b: sum(1 for m in b[1] if m.startswith("v_alignbit")))
    c = Counter(m.split("_e32")[0].split("_e64")[0] for m in best[1])
    valu = {k: v for k, v in c.items() if k.startswith("v_")}
    four = sum(v for k, v in valu.items() if FOUR.match(k))
    two = sum(v for k, v in valu.items() if TWO.match(k) and not FOUR.match(k))
    other = {k: v for k, v in valu.items() if not FOUR.match(k) and not TWO.match(k)}
    comps = round(c.get("v_alignbit_b32", 0) / 224)  # 4 rotations x 8 G x 7 rounds per compression
    cyc = 4 * four + 2 * two + 4 * sum(other.values())  # unknown classes priced at 4
    alg_ops = 680 * comps
    res = {"kernel": "b3_groups<3>", "block": best[0], "compressions_per_trip": comps,
           "valu_ops": sum(valu.values()), "four_cycle_ops": four, "two_cycle_ops": two,
           "other_valu_ops_priced_4": other, "issue_cycles_per_trip": cyc,
           "per_compression": {"four_cycle": four / comps, "two_cycle": two / comps,
                               "issue_cycles": cyc / comps, "algorithmic_ops": 680},
           "cycles_per_algorithmic_op": round(cyc / alg_ops, 4),
           "peak_mix_tops_at_2p4ghz": round(1024 * 64 * 2.4e9 * alg_ops / cyc / 1e12, 2),
           "mnemonics": dict(sorted(valu.items(), key=lambda kv: -kv[1])),
           "note": "issue costs per wave64 instruction measured on gfx950 "
                   "(profiles/r1/valu_*_issue_rates.jsonl): 3-operand and shift-left ops 4 cycles, "
                   "2-operand logic/add/mov 2 cycles"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "mnemonics"}))


if __name__ == "__main__":
    main()
