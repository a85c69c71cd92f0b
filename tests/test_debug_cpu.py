"""Score-table debug dump (koordinator_amd/debug.py) against TestDebugScores
(frameworkext/debug_test.go:91-176) and on hand-built planes."""
import json
import os

import numpy as np

from koordinator_amd import debug
from koordinator_amd.config import shipped_profile

GOLD = os.path.join(os.path.dirname(__file__), "golden", "debug_scores_kat.json")


def test_debug_scores_kat():
    k = json.load(open(GOLD))
    got = debug.render_scores(k["top_n"], k["pod"], k["plugin_scores"], k["nodes"])
    assert got == k["want"]


def test_debug_scores_top_n_truncates_and_ties_keep_node_order():
    t = debug.render_scores(2, "ns/p", {"B": [1, 5, 5], "A": [0, 0, 0]}, ["n0", "n1", "n2"])
    rows = t.splitlines()
    assert rows[0] == "| # | Pod | Node | Score | A | B |"
    assert rows[2:] == ["| 0 | ns/p | n1 | 5 | 0 | 5 |", "| 1 | ns/p | n2 | 5 | 0 | 5 |"]


def test_debug_dump_from_planes_weights_and_feasibility(monkeypatch):
    cfg = shipped_profile()
    P, N = 2, 70
    rng = np.random.default_rng(3)
    mask_bits = rng.random((P, 128)) < 0.6
    mask_bits[:, N:] = False
    res = {"mask": np.packbits(mask_bits, axis=1, bitorder="little").view(np.uint64),
           "scores": rng.integers(0, 101, (P, 128, 2), dtype=np.uint8),
           "numa_scores": rng.integers(0, 101, (P, 128), dtype=np.uint8),
           "rsv_scores": np.zeros((P, 128), np.uint8)}
    monkeypatch.setenv("KOORD_GPU_DEBUG_TOPN", "3")
    assert debug.debug_top_n() == 3
    tables = debug.dump_eval(cfg, res, N, debug.debug_top_n())
    assert len(tables) == P
    for p, t in enumerate(tables):
        nodes = np.flatnonzero(mask_bits[p, :N])
        tot = res["scores"][p, nodes, 0].astype(int) * int(cfg["weight_fit"]) + \
            res["scores"][p, nodes, 1].astype(int) * int(cfg["weight_loadaware"])
        plugins = int(cfg["enabled_plugins"])
        if plugins & 0x4:
            tot = tot + res["numa_scores"][p, nodes].astype(int) * int(cfg["weight_numa"])
        best = nodes[np.argsort(-tot, kind="stable")[:3]]
        lines = t.splitlines()[2:]
        assert [ln.split(" | ")[2] for ln in lines] == [f"node-{i}" for i in best]
        assert [int(ln.split(" | ")[3]) for ln in lines] == sorted(tot, reverse=True)[:3]
    monkeypatch.setenv("KOORD_GPU_DEBUG_TOPN", "0")
    assert debug.debug_top_n() == 0
