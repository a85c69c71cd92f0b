"""Reservation known answers from the reference's own tests (tests/golden/
reservation_restore_filter_kat.json): the BeforePreFilter restore (TestRestoreReservation),
filterWithReservations (Test_filterWithReservations) and PreScore order + NormalizeScore
(TestScoreWithOrder), each through the oracle and through the engine's shared per-pair code."""
import numpy as np
import pytest

from koordinator_amd import engine
from koordinator_amd.config import make_config
from oracle import oracle
from rsv_cases import filter_view, order_view, restore_filter_doc, restore_view, restored_dict, rows_matrix5

DOC = restore_filter_doc()
CFG = make_config(plugins=("Reservation",))


def test_restore_reservation_kat():
    view = restore_view(DOC)
    want = DOC["restore"]["want"]
    assert restored_dict(oracle.rsv_restore(CFG, view, 0, 0)) == want
    rows = engine.build_node_rows(CFG, view)
    prow = engine.build_pod_rows(CFG, view, [0])
    assert restored_dict(engine.row_rsv_restore(CFG, rows[0:1], view.rsv_arr, prow[0:1])) == want


def test_restore_without_reservations_is_identity():
    view = restore_view(DOC)
    rows = engine.build_node_rows(CFG, view)
    prow = engine.build_pod_rows(CFG, view, [0])
    got = engine.row_rsv_restore(CFG, rows[0:1], view.rsv_arr[:0], prow[0:1])
    assert not got["has_state"] and got["n_matched"] == 0
    assert restored_dict(got)["requested"] == DOC["restore"]["node"]["requested"]
    assert int(got["pod_count"]) == DOC["restore"]["node"]["pod_count"]


@pytest.mark.parametrize("case", DOC["filter"]["cases"], ids=lambda c: c["name"])
def test_filter_with_reservations_kat(case):
    view = filter_view(DOC, case)
    ok, _, _ = oracle.rsv_pair(CFG, view, 0, 0)
    assert ok == case["want"]
    rows = engine.build_node_rows(CFG, view)
    prow = engine.build_pod_rows(CFG, view, [0])
    f, *_ = engine.row_eval_rsv(CFG, rows[0:1], view.rsv_arr, prow[0:1], view.now_ns)
    assert bool(f) == case["want"]


@pytest.mark.parametrize("case", [c for c in DOC["filter"]["cases"] if not c["want"]], ids=lambda c: c["name"])
def test_filter_failures_pass_without_required_affinity(case):
    """requiredFromReservation false: no satisfied reservation is not a failure (plugin.go:417-421)."""
    view = filter_view(DOC, dict(case, affinity=False))
    assert oracle.rsv_pair(CFG, view, 0, 0)[0]
    rows = engine.build_node_rows(CFG, view)
    prow = engine.build_pod_rows(CFG, view, [0])
    assert engine.row_eval_rsv(CFG, rows[0:1], view.rsv_arr, prow[0:1], view.now_ns)[0]


def test_score_with_order_kat():
    s = DOC["score_with_order"]
    view = order_view(DOC)
    raws = [oracle.rsv_pair(CFG, view, 0, j)[1] for j in range(4)]
    assert raws == [min(r, 100) for r in s["want_raw"]]   # scoreReservation before the preferred override
    m, _, _, _, rsv, top1 = oracle.eval_matrix5(CFG, view, np.arange(1), view.now_ns)
    assert m.all() and list(rsv[0]) == s["want"]
    got = rows_matrix5(CFG, view, np.arange(1), view.now_ns)
    np.testing.assert_array_equal(got[4], rsv)
    np.testing.assert_array_equal(got[5], top1)
    assert engine.decode_top1(top1)[0][0] == 3
