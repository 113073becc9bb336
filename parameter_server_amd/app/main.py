"""``ps`` node binary (reference build/ps: src/app/main/main.cc).

Starts a scheduler / server / worker node from gflags-style flags and runs the
app described by the text config (``-app_file`` / ``-app_conf``):

    python -m parameter_server_amd.launch local 2 2 -- \
        python -m parameter_server_amd.app.main -app_file example/linear/ctr/online_l1lr.conf
"""
from __future__ import annotations

import sys

from .. import ps
from ..utils.flags import parse_flags


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    flags = parse_flags(argv)
    po = ps.start_node(flags)
    po.run(timeout=flags.timeout)
    if flags.traffic_statistics:
        print(f"[{po.my_node.id}] traffic {po.van.stats()}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
