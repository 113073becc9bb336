# round 4 (f): native one-call iteration (events kept alive), p2p owner stream + bench rows, profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { "$@"; rc=$?; echo "rc=$rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_tpf_gpu.py tests/test_p2p_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
for i in 1 2; do
  step timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_native_$i.log 2>&1
  step env PSAMD_NATIVE_ITER=0 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_flat_eager_$i.log 2>&1
done
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b300_native.log 2>&1
step timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 > $O/b300_b10k.log 2>&1
step env PSAMD_NATIVE_ITER=0 timeout -k 10 120 python bench.py --steps 300 --warmup 10 --minibatch 10000 > $O/b300_b10k_eager.log 2>&1
step env PSAMD_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --exchange p2p --consistency asp --steps 50 --warmup 10 > $O/p2p_2.log 2>&1
step env PSAMD_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 3 --exchange p2p --consistency asp --steps 50 --warmup 10 > $O/p2p_3.log 2>&1
step env PSAMD_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --consistency asp --steps 50 --warmup 10 > $O/padded_gloo_2.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_seq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 --pipeline 0 > "$GRAFT_REPO_ROOT/$O/prof_seq.log" 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 10 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_darlin" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_darlin.py" --rows 4000000 --passes 3 --device-data --tau32 1 > "$GRAFT_REPO_ROOT/$O/prof_darlin.log" 2>&1
