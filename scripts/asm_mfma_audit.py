#!/usr/bin/env python3
"""Audit a kernel's inline-asm MFMAs (lab/gemm_w4.h): hipcc does not pad hazards for an asm statement, so
check in the .s that (1) no compiler VALU write lands on an asm MFMA's A/B source registers within the
2 instructions before it, (2) no v_accvgpr_* moves sit inside the main loop, (3) no scratch access.
usage: asm_mfma_audit.py file.s kernel_substring"""
import re
import sys


def regs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok) or re.match(r"([va])(\d+)$", tok)
    if not m:
        return set()
    lo = int(m.group(2))
    hi = int(m.group(3)) if m.lastindex == 3 else lo
    return {f"{m.group(1)}{i}" for i in range(lo, hi + 1)}


def main():
    path, want = sys.argv[1], sys.argv[2]
    s = open(path).read()
    bad = 0
    for name in re.findall(r"^(\w*(?:" + want + r")\w*):", s, re.M):
        body = s[s.index(name + ":"):s.index(".Lfunc_end", s.index(name + ":"))].splitlines()
        ins = [l.strip() for l in body if l.strip() and not l.strip().startswith((";", ".")) and not l.strip().endswith(":")]
        hz = 0
        for i, l in enumerate(ins):
            if not l.startswith("v_mfma"):
                continue
            ops = [o.strip() for o in l.split(None, 1)[1].split(",")]
            srcs = regs(ops[1]) | regs(ops[2])
            for j in range(max(0, i - 2), i):
                p = ins[j]
                if p.startswith(("v_", )) and not p.startswith(("v_mfma", "v_accvgpr_read", "v_cmp")):
                    dst = regs(p.split(None, 1)[1].split(",")[0].strip()) if " " in p else set()
                    if dst & srcs:
                        hz += 1
                        print("hazard?", name[:60], "|", p, "->", l)
        loops = [i for i, l in enumerate(body) if "Loop Header" in l]
        acc_moves = 0
        if loops:
            lb = loops[0]
            hdr = body[lb].split(":")[0]
            ends = [i for i in range(lb, len(body)) if re.match(r"\s*s_(c?branch\w*)\s+" + re.escape(hdr) + r"\s*$", body[i])]
            le = ends[-1] if ends else lb
            acc_moves = sum(1 for l in body[lb:le] if "v_accvgpr" in l)
        scratch = sum(1 for l in ins if l.startswith("scratch_"))
        waterfall = sum(1 for l in ins if l.startswith("s_and_saveexec"))
        print(f"{name[:70]}: mfma {sum(l.startswith('v_mfma') for l in ins)}, VALU->MFMA-src hazards {hz}, "
              f"v_accvgpr in main loop {acc_moves}, scratch ops {scratch}, s_and_saveexec {waterfall}")
        bad += hz + acc_moves
    sys.exit(1 if bad else 0)


main()
