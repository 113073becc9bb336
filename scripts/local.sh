#!/bin/bash
# usage: ./local.sh num_servers num_workers program [args..]
# Same role/port layout semantics as the reference script/local.sh, all on 127.0.0.1.
if [ $# -lt 3 ]; then
  echo "usage: $0 num_servers num_workers program [args..]"; exit 1
fi
S=$1; shift; W=$1; shift
cd "$(dirname "$0")/.." && exec python -m parameter_server_amd.launch local "$S" "$W" -- "$@"
