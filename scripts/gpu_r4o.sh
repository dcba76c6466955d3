#!/bin/bash
# Round 4: r4m (BN statistics validation + benches + step table) then r4n (fp32 K order study)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_r4m.sh gpurun_out/r4m && bash scripts/gpu_r4n.sh gpurun_out/r4n
