#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
p() { echo -n "$1: "; env $1 timeout -k 10 100 python benchmarks/probe_graph_overhead.py 2>/dev/null | tail -1; }
p "X=0"
p "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"
p "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"
p "HIP_FORCE_DEV_KERNARG=1"
p "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"
p "ROC_SYSTEM_SCOPE_SIGNAL=0"
p "DEBUG_HIP_GRAPH_BATCH_SIZE=1"
