#!/bin/bash
# Lab: in-kernel clocks of the ping-pong GEMM + one PMC pass (MFMA busy, waits, clock) over pp_lab.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pp_pmc; mkdir -p $OUT
L=lab/build/pp_lab
timeout -k 10 120 $L 4096 4096 4096 0 clock > $OUT/clock.log 2>&1; echo "clock rc=$?"; cat $OUT/clock.log
timeout -k 10 120 $L 4096 4096 4096 5 v3p,pp1,pp1_nostore,pp1_nodma_ns > $OUT/abl.log 2>&1; echo "abl rc=$?"; grep -v check $OUT/abl.log
P="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/sq -o sq -- $L 4096 4096 4096 2 v3p,pp1 > $OUT/sq.log 2>&1; echo "pmc rc=$?"
timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/sqpeak -o sq -- $L 0 0 0 0 peak > $OUT/sqpeak.log 2>&1; echo "pmc peak rc=$?"
python3 - <<'PY'
import csv, glob, statistics
from collections import defaultdict
for d in ("gpurun_out/pp_pmc/sq", "gpurun_out/pp_pmc/sqpeak"):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        disp = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]
            key = (k, r["Dispatch_Id"])
            disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
            disp[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        per = defaultdict(lambda: defaultdict(list))
        for (k, _), c in disp.items():
            for n, v in c.items(): per[k][n].append(v)
        for k, c in per.items():
            med = {n: statistics.median(v) for n, v in c.items()}
            cyc = med["GRBM_GUI_ACTIVE"] / 8
            print(f"{k:60s} n={len(c['_dur'])} dur={med['_dur']*1e6:.2f}us clk={cyc/med['_dur']/1e9:.3f}GHz "
                  f"mfma_util={med['SQ_VALU_MFMA_BUSY_CYCLES']/(cyc*1024):.4f} "
                  f"wait_any={med['SQ_WAIT_ANY']/med['SQ_WAVE_CYCLES']:.3f} wait_inst={med['SQ_WAIT_INST_ANY']/med['SQ_WAVE_CYCLES']:.3f} "
                  f"active={med['SQ_ACTIVE_INST_ANY']/med['SQ_WAVE_CYCLES']:.3f}")
PY
