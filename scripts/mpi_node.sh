#!/bin/bash
# One node of an MPI-launched job (reference script/mpi_node.sh): the node's rank
# comes from the MPI launcher and Van-style auto addressing (-my_rank) derives
# role, id, IP and port; rank 0 is the scheduler given by $PS_SCHEDULER.
#   mpirun -np $((1+S+W)) scripts/mpi_node.sh S W python -m parameter_server_amd.app.main -app_file x.conf
# (a root script would export PS_SCHEDULER="role:SCHEDULER,hostname:'<ip>',port:8001,id:'H'")
set -e
S=$1; W=$2; shift 2
RANK=${PMI_RANK:-${OMPI_COMM_WORLD_RANK:-${SLURM_PROCID:-${RANK:-0}}}}
SCH=${PS_SCHEDULER:-"role:SCHEDULER,hostname:'127.0.0.1',port:8001,id:'H'"}
exec "$@" -num_servers "$S" -num_workers "$W" -scheduler "$SCH" -my_rank "$RANK" ${PS_INTERFACE:+-interface $PS_INTERFACE}
