#!/bin/bash
# the store-policy lab (lab/c4_lab.hip at C2 and the C4 shard), then the round-4 final measurement set
set -o pipefail
bash scripts/runs/r4_c4nt.sh && bash scripts/runs/r4_final2.sh
