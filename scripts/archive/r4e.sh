# round 4 (e): event diagnostic, sequential + pipelined kernel profiles of the flat path, p2p rows
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { "$@"; rc=$?; echo "rc=$rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 120 python scripts/archive/diag_launchlist.py > $O/diag.log 2>&1
step env PSAMD_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --exchange p2p --consistency asp --steps 50 --warmup 10 > $O/p2p_2.log 2>&1
step env PSAMD_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 3 --exchange p2p --consistency asp --steps 50 --warmup 10 > $O/p2p_3.log 2>&1
step env PSAMD_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --consistency asp --steps 50 --warmup 10 > $O/padded_gloo_2.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_darlin" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_darlin.py" --rows 4000000 --passes 3 --device-data --tau32 1 > "$GRAFT_REPO_ROOT/$O/prof_darlin.log" 2>&1
