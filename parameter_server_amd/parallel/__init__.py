from .comm import Comm, DistComm, LocalComm, init_from_env
from .consistency import INF, EventClock, VectorClock, parse_consistency
from .partition import KeyPartition, even_divide

__all__ = ["Comm", "DistComm", "LocalComm", "init_from_env", "INF", "EventClock", "VectorClock",
           "parse_consistency", "KeyPartition", "even_divide"]
