#!/bin/bash
# One 1-GPU run per BASELINE.json config (multi-GPU configs with emulated peers:
# per-GPU device cost of the N-GPU step; the driver measures the real 8-GPU runs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/baseline_configs.log
: > $out
run() {
  local name="$1"; shift
  timeout -k 10 240 python bench.py --steps 100 --warmup 10 "$@" > gpurun_out/cfg.log 2>&1 || { echo "$name FAILED rc=$?" >> $out; tail -5 gpurun_out/cfg.log >> $out; return 1; }
  echo "## $name: python bench.py $*" >> $out
  tail -1 gpurun_out/cfg.log >> $out
}
run "config 2: AdaGrad, BSP, 1e8 features, 1 GPU" --algo adagrad --consistency bsp --num-features 1e8 &&
run "config 3: FTRL-L1, SSP 4, 1e9 features (1 GPU)" &&
run "config 3: FTRL-L1, SSP 4, 1e9 features, 8 emulated peers" --emulate-peers 8 --emulate-backend nccl &&
run "config 4: async (asp) FTRL, fixing-float 1 B + key caching, 1e9, 8 emulated peers" --consistency asp --fixing-float 1 --emulate-peers 8 --emulate-backend nccl &&
run "config 4: async (asp) SGD, fixing-float 2 B + key caching, 1e9, 8 emulated peers" --algo sgd --consistency asp --fixing-float 2 --emulate-peers 8 --emulate-backend nccl &&
run "1e10 features (KeyMix 34 bits, u64 keys), FTRL SSP 4, 1 GPU" --num-features 1e10 &&
run "1e10 features, 8 emulated peers" --num-features 1e10 --emulate-peers 8 --emulate-backend nccl &&
{ timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 > gpurun_out/cfg.log 2>&1 &&
  echo "## config 5: wide & deep 1e9 x 128 (auto GEMM), 1 GPU: python benchmarks/bench_wide_deep.py --steps 30" >> $out &&
  tail -1 gpurun_out/cfg.log >> $out; } &&
{ timeout -k 10 300 python benchmarks/bench_wide_deep.py --steps 30 --emulate-peers 8 > gpurun_out/cfg.log 2>&1 &&
  echo "## config 5: wide & deep, 8 emulated peers: python benchmarks/bench_wide_deep.py --steps 30 --emulate-peers 8" >> $out &&
  tail -1 gpurun_out/cfg.log >> $out; }
cat $out
