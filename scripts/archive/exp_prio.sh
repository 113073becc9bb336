#!/bin/bash
# A/B of stream priorities for the 1-GPU headline pipeline (main = training stream).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 60 python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" || exit 1
run() { echo "== $*"; env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 20 | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value']/1e6)" || exit 1; }
run PSAMD_X=0
run PSAMD_MAIN_PRIORITY=-1
run PSAMD_MAIN_PRIORITY=-1 PSAMD_PREP_PRIORITY=0
run PSAMD_PREP_PRIORITY=0
run PSAMD_MAIN_PRIORITY=0 PSAMD_PREP_PRIORITY=1
run PSAMD_MAIN_PRIORITY=-1 PSAMD_PREP_PRIORITY=1
run PSAMD_X=0
