#!/bin/bash
# (Needs the session-a build in a worktree: git worktree add build/wt_a ba59b7f, then build its library there.)
# Round 4: config C on the session-a build (worktree build/wt_a, commit
# ba59b7f) and the current build, alternated on one box.
set -o pipefail
mkdir -p gpurun_out/r04j
R=$PWD
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r04j/cur_$i.json 2> gpurun_out/r04j/cur_$i.err &&
  (cd build/wt_a && timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e > $R/gpurun_out/r04j/old_$i.json 2> $R/gpurun_out/r04j/old_$i.err) || exit 1
done
