#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python benchmarks/probe_host_costs.py > gpurun_out/r3_host_costs.log 2>&1 || exit $?
tail -1 gpurun_out/r3_host_costs.log
for c in 1 0; do
  PSAMD_COMM_CHAIN=$c timeout -k 10 240 python bench.py --steps 100 --warmup 20 --emulate-peers 8 > gpurun_out/r3_e8_chain$c.log 2>&1 || exit $?
  tail -1 gpurun_out/r3_e8_chain$c.log | cut -c 1-330
done
timeout -k 10 300 python benchmarks/train_check.py --steps 50 lr:sgd:e8asp2:alpha=0.001 lr:sgd:e8asp2:alpha=0.0003 lr:ftrl:e8asp2 lr:adagrad:e8asp2 > gpurun_out/r3_train2.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/train_check.py --steps 50 --minibatch 16384 fm fm:emb_lr=0.02,wide_alpha=0.05 fm:emb_lr=0.01 >> gpurun_out/r3_train2.log 2>&1 || exit $?
cat gpurun_out/r3_train2.log | grep spec | cut -c 1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_seq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --pipeline 0 --graph 0 > $GRAFT_REPO_ROOT/gpurun_out/r3_seq.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_darlin_gpu.py > gpurun_out/r3_pytest_darlin.log 2>&1 || { tail -20 gpurun_out/r3_pytest_darlin.log; exit 1; }
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --device-data > gpurun_out/r3_darlin_t1.log 2>&1 || exit $?
tail -1 gpurun_out/r3_darlin_t1.log | cut -c 1-300
timeout -k 10 300 python benchmarks/bench_darlin.py --rows 4000000 --passes 5 --tau 8 --device-data > gpurun_out/r3_darlin_t8.log 2>&1 || exit $?
tail -1 gpurun_out/r3_darlin_t8.log | cut -c 1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_darlin_prof -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_darlin.py --rows 4000000 --passes 3 --device-data > $GRAFT_REPO_ROOT/gpurun_out/r3_darlin_prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_p2p_gpu.py tests/test_sharded_kv.py > gpurun_out/r3_pytest_p2p.log 2>&1; rc=$?
tail -15 gpurun_out/r3_pytest_p2p.log; exit $rc
