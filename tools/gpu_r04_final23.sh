#!/bin/bash
# Round 4 final build, calls 2 and 3 in one (when GPU slots are scarce).
set -o pipefail
bash tools/gpu_r04_final2.sh && bash tools/gpu_r04_final3.sh
