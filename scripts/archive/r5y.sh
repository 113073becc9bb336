cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r5y; mkdir -p $O
export PYTHONUNBUFFERED=1
j() { python -c "import sys,json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d.get('host_issue_ms_per_step') or 0,4), d['config'].get('native_iteration'))"; }
for p in 2 3; do
  PSAMD_ITER_GRAPH=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --minibatch 10000 --prep-streams $p > $O/g_p$p.log 2>&1 || exit 3; j $O/g_p$p.log "B10k itergraph prep=$p"
done
for i in 1 2; do
for m in "nat 1 0" "eager 0 0" "graph 0 1"; do set -- $m
  PSAMD_NATIVE_ITER=$2 PSAMD_ITER_GRAPH=$3 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_$1_$i.log 2>&1 || exit 3; j $O/b20_$1_$i.log "B65536-20 $1"
done
for m in "nat 1 0" "eager 0 0" "graph 0 1"; do set -- $m
  PSAMD_NATIVE_ITER=$2 PSAMD_ITER_GRAPH=$3 timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $O/b300_$1_$i.log 2>&1 || exit 3; j $O/b300_$1_$i.log "B65536-300 $1"
done
done
