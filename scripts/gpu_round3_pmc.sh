#!/bin/bash
# Round-3 counter evidence: kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes
# (separate runs) for C2 (headline), C3 (RGB path) and C4 at its configured
# 1024 spp, then the two SQ passes of C2 at 16 spp.  Each step has its own
# time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT"
set -o pipefail
bash scripts/gpu_pmc_cfg.sh pmc_c2 || exit $?
bash scripts/gpu_pmc_cfg.sh pmc_c3 --config c3 || exit $?
bash scripts/gpu_pmc_cfg.sh pmc_c4 --config c4 || exit $?
bash scripts/gpu_pmc_sq.sh || exit $?
echo "round3 pmc done"
