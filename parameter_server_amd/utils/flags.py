"""gflags-compatible command line flags.

The reference reads topology / transport / debug flags with gflags
(postoffice.cc:11-32, van.cc:9-15, remote_node.cc:8-9, ...): ``-flag value``,
``-flag=value``, ``--flag value`` and bare boolean ``-flag`` / ``-noflag`` forms.
Unknown flags are kept for the program (``ps.h``: flags are removed from argv,
positional arguments remain).
"""
from __future__ import annotations

from dataclasses import dataclass, field, fields


@dataclass
class Flags:
    num_servers: int = 0
    num_workers: int = 0
    num_threads: int = 2
    app_name: str = "app"
    app_conf: str = ""
    app_file: str = ""
    my_node: str = ""
    scheduler: str = ""
    my_rank: int = -1
    interface: str = ""
    bind_to: int = 0
    print_van: bool = False
    verbose: bool = False
    log_to_file: bool = False
    traffic_statistics: bool = False
    key_cache: bool = True
    message_compression: bool = False
    report_interval: float = 1.0
    heartbeat_interval: float = 0.0
    shuffle_fea_id: bool = False
    line_limit: int = -1
    input: str = ""
    output: str = ""
    format: str = ""
    num_replicas: int = 0
    enable_fault_tolerance: bool = False
    timeout: float = 600.0
    rest: list = field(default_factory=list)


def parse_flags(argv: list[str]) -> Flags:
    f = Flags()
    types = {x.name: x.type for x in fields(Flags)}
    i = 0
    rest = []
    while i < len(argv):
        a = argv[i]
        if a.startswith("-") and len(a) > 1 and not a[1:2].isdigit():
            name = a.lstrip("-")
            val = None
            if "=" in name:
                name, val = name.split("=", 1)
            neg = False
            if name not in types and name.startswith("no") and name[2:] in types:
                name, neg = name[2:], True
            if name in types:
                t = types[name]
                if t in ("bool", bool):
                    if val is None and i + 1 < len(argv) and argv[i + 1].lower() in ("true", "false", "1", "0"):
                        val = argv[i + 1]
                        i += 1
                    b = True if val is None else val.lower() in ("true", "1", "t", "yes")
                    setattr(f, name, (not b) if neg else b)
                else:
                    if val is None:
                        i += 1
                        val = argv[i]
                    conv = {"int": int, "float": float, "str": str}.get(t if isinstance(t, str) else t.__name__, str)
                    setattr(f, name, conv(val))
                i += 1
                continue
        rest.append(a)
        i += 1
    f.rest = rest
    return f
