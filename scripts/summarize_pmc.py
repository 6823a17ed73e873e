#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc passes over bench.py into per-kernel HBM traffic and clock.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) reports half the bytes of a wide
coalesced streaming read on gfx950 (16 B/lane global_load and LDS-DMA alike), so read bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.  Infinity-Cache hits are
included (FETCH_SIZE counts L2 -> fabric requests).  Effective clock = GRBM_GUI_ACTIVE / 8 XCDs /
dispatch time; MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs).

usage: summarize_pmc.py <pmc dir (pass*_counter_collection.csv)> <out.json> [M N K]
"""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict


def short(name):
    if "mm_f32" in name and "<" in name:  # keep the tile configuration: attention QK^T and PV differ
        return "mm_f32<" + name.split("<")[1].split(">")[0] + ">"
    for key in ("gemm_i8", "outlier_flags", "pack_single_pass", "pack_rows_and_colmax", "pack_cols", "pack_rows", "colmax",
                "fill_uniform", "mm_f32", "error_partials", "error_final", "error_reference_mean"):
        if key in name:
            return key
    return name[-40:]


def main():
    d, out = sys.argv[1], sys.argv[2]
    M, N, K = (int(x) for x in sys.argv[3:6]) if len(sys.argv) > 5 else (4096, 4096, 4096)
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    durs = defaultdict(list)
    for f in sorted(glob.glob(f"{d}/pass*_counter_collection.csv")):
        disp = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            key = (k, r["Dispatch_Id"])
            disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
            disp[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        for (k, _), c in disp.items():
            for name, v in c.items():
                per[k][name].append(v)
    res = {}
    for k, c in per.items():
        med = {n: statistics.median(v) for n, v in c.items()}
        r = {"dispatch_us_profiled": round(med["_dur"] * 1e6, 2)}
        if "FETCH_SIZE" in med:
            r["read_bytes"] = 2 * med["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in med:
            r["write_bytes"] = med["WRITE_SIZE"] * 1024
        if "read_bytes" in r and "write_bytes" in r:
            r["hbm_bytes"] = r["read_bytes"] + r["write_bytes"]
        if "GRBM_GUI_ACTIVE" in med:
            cyc = med["GRBM_GUI_ACTIVE"] / 8
            r["clock_ghz"] = round(cyc / med["_dur"] / 1e9, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
                r["mfma_util"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4)
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in med and "SQ_WAVE_CYCLES" in med:
                    r[n.lower() + "_frac"] = round(med[n] / med["SQ_WAVE_CYCLES"], 3)
        if "TCC_HIT_sum" in med:
            r["l2_hit"] = round(med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 4)
        if "SQ_LDS_BANK_CONFLICT" in med:
            r["lds_bank_conflict_frac"] = round(med["SQ_LDS_BANK_CONFLICT"] / max(1.0, med["SQ_LDS_IDX_ACTIVE"]), 4)
        res[k] = r
    alg = {"gemm_i8": {"int8_ops": 2 * M * N * K,
                       "alg_bytes": M * K + N * K + 4 * M * N + 4 * (M + N)},
           "pack_single_pass": {"alg_bytes": 4 * M * K + M * K + 4 * K * N + K * N + 4 * (M + N)},
           "pack_rows_and_colmax": {"alg_bytes": 4 * M * K + M * K + 4 * K * N},
           "pack_cols": {"alg_bytes": 4 * K * N + K * N}}
    for k, a in alg.items():
        if k in res:
            res[k].update(a)
    json.dump({"M": M, "N": N, "K": K, "kernels": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
