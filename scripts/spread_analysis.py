#!/usr/bin/env python3
"""Attribute the block-end spread of gemm_i8_fm's store tail from lab/build/w4_lab's
`spread` rows: blk,rep,block,xcd,tm,tn,start_us,loop_end_us,end_us,loop_clock_ghz.

For each launch: the tail of a block = end - loop end (its epilogue: dequantize + 256 KiB of fp32 stores).  The
question is whether the slow tails are tied to the memory channels the tile writes (its output columns tn and rows
tm), to its XCD, or simply to when its loop ended (late finishers store into an already draining queue).  Prints
the tail's mean by tn, by tm, by XCD, and by loop-end quartile, the variance each grouping explains (eta^2), and
the correlation of tail with loop end.

    python scripts/spread_analysis.py gpurun_out/.../spread.log
"""
import sys
from collections import defaultdict


def eta2(groups, allv):
    mu = sum(allv) / len(allv)
    sst = sum((v - mu) ** 2 for v in allv)
    ssb = sum(len(g) * (sum(g) / len(g) - mu) ** 2 for g in groups.values())
    return ssb / sst if sst else 0.0


def corr(x, y):
    n = len(x)
    mx, my = sum(x) / n, sum(y) / n
    sxy = sum((a - mx) * (b - my) for a, b in zip(x, y))
    sxx = sum((a - mx) ** 2 for a in x)
    syy = sum((b - my) ** 2 for b in y)
    return sxy / (sxx * syy) ** 0.5 if sxx and syy else 0.0


def main(path):
    reps = defaultdict(list)
    for line in open(path):
        if not line.startswith("blk,"):
            continue
        _, rep, b, xcd, tm, tn, st, le, en, clk = line.strip().split(",")
        reps[int(rep)].append(dict(b=int(b), xcd=int(xcd), tm=int(tm), tn=int(tn), st=float(st), le=float(le),
                                   en=float(en), clk=float(clk)))
    for rep, rows in sorted(reps.items()):
        tails = [r["en"] - r["le"] for r in rows]
        les = [r["le"] for r in rows]
        ens = [r["en"] for r in rows]
        print(f"launch {rep}: {len(rows)} blocks  loop ends {min(les):.2f}..{max(les):.2f} us  "
              f"block ends {min(ens):.2f}..{max(ens):.2f} us  tail {min(tails):.2f}..{max(tails):.2f} "
              f"(mean {sum(tails) / len(tails):.2f}) us")
        for key in ("tn", "tm", "xcd"):
            g = defaultdict(list)
            for r, t in zip(rows, tails):
                g[r[key]].append(t)
            means = " ".join(f"{k}:{sum(v) / len(v):.2f}" for k, v in sorted(g.items()))
            print(f"  tail by {key:3s} (eta2 {eta2(g, tails):.3f}): {means}")
        order = sorted(range(len(rows)), key=lambda i: les[i])
        q = defaultdict(list)
        for rank, i in enumerate(order):
            q[4 * rank // len(rows)].append(tails[i])
        means = " ".join(f"Q{k + 1}:{sum(v) / len(v):.2f}" for k, v in sorted(q.items()))
        print(f"  tail by loop-end quartile (eta2 {eta2(q, tails):.3f}): {means}")
        print(f"  corr(tail, loop end) {corr(tails, les):+.3f}   corr(block end, loop end) {corr(ens, les):+.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
