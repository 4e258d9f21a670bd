#!/bin/bash
# Round 4: the stack hand-off A/B and tests (gpu_r04t.sh), then the host
# harness and bench lines (gpu_r04e.sh), in one call.
set -o pipefail
bash tools/gpu_r04t.sh && bash tools/gpu_r04e.sh
