"""Tracing utility (utils/trace.py): phase ranges, traffic counters, per-rank JSON."""
import json

from parameter_server_amd.utils import trace


def test_ranges_and_traffic(tmp_path):
    trace.reset()
    trace.enable(False)
    with trace.trace_range("off"):
        pass
    assert "off" not in trace.snapshot()["phases"]
    trace.enable(True)
    try:
        for _ in range(3):
            with trace.trace_range("pull"):
                pass
    finally:
        trace.enable(False)
    trace.count_traffic("all_to_all", 100, 40)
    trace.count_traffic("all_to_all", 50, 10)
    snap = trace.snapshot({"sent_remote": 7})
    assert snap["phases"]["pull"]["count"] == 3
    assert snap["traffic"]["all_to_all"] == {"calls": 2, "bytes_sent": 150, "bytes_recv": 50}
    p = trace.dump(str(tmp_path / "t_{rank}.json"), rank=3, van_stats={"sent_remote": 7})
    d = json.load(open(p))
    assert p.endswith("t_3.json") and d["rank"] == 3 and d["van"]["sent_remote"] == 7
    assert "all_to_all: 2 calls" in trace.format_traffic(snap)
    trace.reset()
