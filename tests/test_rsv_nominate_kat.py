"""Reservation known answers: TestFilterReservation (reservation/plugin_test.go:1559-1750) and
TestPreScoreWithNominateReservation (scoring_test.go:392-728), tests/golden/reservation_nominate_filter_kat.json,
through the oracle and the engine's per-pair code (kg_row_eval_rsv).  Both reference tests inject the matched
reservations into the cycle state; each case here is the node whose restore yields that state (the fixture's
note derives it)."""
import json
import os

import pytest

from koordinator_amd import engine
from koordinator_amd.config import make_config
from oracle import oracle
from rsv_cases import _kat_view

DOC = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reservation_nominate_filter_kat.json")))
CFG = make_config(plugins=("Reservation",))
RES = {"4C8G": {"cpu": 4000, "memory": 8 << 30}, "2C4G": {"cpu": 2000, "memory": 4 << 30}}


def _node(rsvs, matched):
    """The reserve pods of every reservation on the node; allocatable = Σ allocatable − Σ allocated of the
    matched ones, so fitsNode compares the request with the reservation's remainder alone."""
    req, alloc = {"cpu": 0, "memory": 0}, {"cpu": 0, "memory": 0}
    for r in rsvs:
        for k in req:
            req[k] += RES[r["r"]][k]
            alloc[k] += RES[r["r"]][k]
    for r in matched:
        for k in alloc:
            alloc[k] -= RES[r["allocated"]][k] if r.get("allocated") else 0
    return {"allocatable": alloc, "requested": req, "pod_count": len(rsvs), "allowed_pods": 110}


def _rsv(doc, node):
    d = {"node": node, "allocatable": RES[doc["r"]], "order": doc.get("order", 0),
         "allocate_once": doc.get("allocate_once", False), "n_assigned": doc.get("n_assigned", 0)}
    if doc.get("allocated"):
        d["allocated"] = RES[doc["allocated"]]
    return d


@pytest.mark.parametrize("case", DOC["filter_cases"], ids=lambda c: c["name"])
def test_filter_reservation_kat(case):
    rs = case["reservations"]
    usable_target = [r for r in rs if r.get("target") and not (r.get("allocate_once") and r.get("n_assigned"))]
    node = _node(rs, usable_target)
    rsv = [dict(_rsv(r, 0), affinity=bool(r.get("target"))) for r in rs]
    view = _kat_view([node], rsv, case["pod"], affinity=True)
    assert oracle.rsv_pair(CFG, view, 0, 0)[0] == case["want"]
    rows = engine.build_node_rows(CFG, view)
    prow = engine.build_pod_rows(CFG, view, [0])
    assert engine.row_eval_rsv(CFG, rows[0:1], view.rsv_arr, prow[0:1], view.now_ns)[0] == case["want"]


@pytest.mark.parametrize("case", DOC["nominate_cases"], ids=lambda c: c["name"])
def test_prescore_nominate_reservation_kat(case):
    nodes = [_node(rs, rs) for rs in case["nodes"]]
    rsv = [_rsv(r, j) for j, rs in enumerate(case["nodes"]) for r in rs]
    view = _kat_view(nodes, rsv, case["pod"])
    rows = engine.build_node_rows(CFG, view)
    prow = engine.build_pod_rows(CFG, view, [0])
    first = 0
    for j, rs in enumerate(case["nodes"]):
        want = case["want_nominated"][j]
        ok, _, nom = oracle.rsv_pair(CFG, view, 0, j)
        assert ok and nom == want
        slots = view.rsv_arr[first:first + len(rs)]
        f, *_, nominated = engine.row_eval_rsv(CFG, rows[j:j + 1], slots, prow[0:1], view.now_ns)
        assert f and nominated == want
        first += len(rs)
