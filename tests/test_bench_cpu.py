"""bench.py host logic that needs no GPU: the roofline `traffic` lookup."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_headline_traffic_is_attached_to_the_chain_schedule():
    t = bench.load_traffic("rq1.botnet.static")
    assert set(t) >= {"k_mlp", "k_survive"}
    assert {"k_genc"} <= set(t) or {"k_gen", "k_cons"} <= set(t)
    assert all(v > 0 for v in t.values())


def test_unmeasured_workload_gets_no_traffic():
    assert bench.load_traffic("synthetic.botnet.wide") == {}
