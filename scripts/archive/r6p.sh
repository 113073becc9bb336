#!/bin/bash
# round 6: the GPU suite + smoke + driver-shape bench, then the blocked-sketch tail runs (r6o)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/archive/r6n.sh || exit $?
bash scripts/archive/r6o.sh
