#!/bin/bash
# gpu_ab3.sh A/B (tests skipped unless RUN_TESTS=1), then the two SQ counter passes of the default variant.
cd "$GRAFT_REPO_ROOT"
if [ -z "$RUN_TESTS" ]; then export SKIP_TESTS=1; fi
bash scripts/gpu_ab3.sh "$@" || exit $?
bash scripts/gpu_pmc_sq.sh $SQ_ARGS
