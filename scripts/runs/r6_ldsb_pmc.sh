#!/bin/bash
# clock and MFMA busy of the B-through-LDS lab kernel against the product (lab/epi_lab.hip, 4096^3), one --pmc pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6ldsbpmc; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT -o pass1 -- lab/build/epi_lab 4096 4096 4096 3 prod,ldsb1 > $OUT/run.log 2>&1
echo "rc=$?"
