#!/bin/bash
# Round 4: r4r (pipelined lift-splat forward A/B) then r4q (BN finalize, benches, step table,
# 1x1-conv route A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_r4r.sh gpurun_out/r4r && bash scripts/gpu_r4q.sh gpurun_out/r4q
