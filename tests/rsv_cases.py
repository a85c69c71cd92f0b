"""Config-5 (Reservation + ElasticQuota) test clusters: the TestScore known-answer node and a
host-row mirror of the engine's per-pod Reservation reduction (PreScore preferred node, Score
override, DefaultNormalizeScore) built on kg_row_eval / kg_row_eval_rsv."""
import json
import os

import numpy as np

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth

HERE = os.path.dirname(os.path.abspath(__file__))
INT64_MAX = (1 << 63) - 1


def _rl(d):
    out = np.zeros((), dtype=nat.RESOURCE_LIST)
    for k, v in (d or {}).items():
        r = {"cpu": nat.RES_CPU, "memory": nat.RES_MEMORY, "ephemeral-storage": nat.RES_EPHEMERAL_STORAGE}[k]
        out["v"][r] = v
        out["present"] |= np.uint32(1 << r)
    return out


def kat_doc():
    with open(os.path.join(HERE, "golden", "reservation_score_kat.json")) as f:
        return json.load(f)


def kat_cluster(doc, case):
    """One node with an empty NodeStatus, the case's reservations on it, one pod (owner class 0)."""
    nodes = np.zeros(1, dtype=nat.NODE_SPEC)
    nodes["numa"] = -1
    pods = np.zeros(1, dtype=nat.POD_SPEC)
    pods["n_containers"] = 1
    pods["label_priority_class"] = -1
    pods["label_qos"] = -1
    pods["rsv_owner_class"] = 0
    pods["rsv_affinity_class"] = -1
    pods["quota"] = -1
    cont = np.zeros(1, dtype=nat.CONTAINER)
    cont[0]["requests"] = _rl(case["pod"])
    rsv = np.zeros(len(case["reservations"]), dtype=nat.RESERVATION)
    for i, name in enumerate(case["reservations"]):
        rsv[i]["node"] = 0
        rsv[i]["flags"] = nat.RSV_AVAILABLE
        rsv[i]["owner_classes"] = 1
        rsv[i]["allocatable"] = _rl(doc["reservations"][name])
        alloc = case.get("allocated", {}).get(name)
        if alloc:
            rsv[i]["allocated"] = _rl(alloc)
            rsv[i]["n_assigned"] = 1
    return synth.SynthView(pods, cont, nodes, synth.NOW_NS, reservations=rsv)


def rsv_cluster(n_nodes, n_pods, seed, **kw):
    return synth.make_rsv_cluster(n_nodes, n_pods, seed, **kw)


def rows_matrix5(cfg, view, pod_index, now_ns):
    """mask, fit, la, reservation planes and top1 keys through the engine's per-pair host code
    (kg_row_eval for plain nodes, kg_row_eval_rsv for nodes with reservations) + the per-pod
    reduction of rsv_best_block, restated in numpy.  ElasticQuota is not applied here."""
    rows = engine.build_node_rows(cfg, view)
    prow = engine.build_pod_rows(cfg, view, pod_index)
    by_node = {}
    for r in view.rsv_arr:
        by_node.setdefault(int(r["node"]), []).append(r)
    N, P = len(rows), len(prow)
    mask = np.zeros((P, N), bool)
    fit = np.zeros((P, N), np.uint8)
    la = np.zeros((P, N), np.uint8)
    numa = np.zeros((P, N), np.uint8)
    rsvp = np.zeros((P, N), np.uint8)
    top1 = np.zeros(P, np.uint64)
    wf, wl, wr = int(cfg["weight_fit"]), int(cfg["weight_loadaware"]), int(cfg["weight_reservation"])
    wn = int(cfg["weight_numa"]) if int(cfg["enabled_plugins"]) & nat.PLUGIN_NUMA else 0
    for p in range(P):
        raw = np.zeros(N, np.int64)
        order = np.full(N, INT64_MAX, np.int64)
        for j in range(N):
            if j in by_node:
                f, a, b, n, rr, o, _ = engine.row_eval_rsv(cfg, rows[j:j + 1], np.array(by_node[j]), prow[p:p + 1],
                                                           now_ns)
                raw[j], order[j] = rr, o
            else:
                f, a, b, n = engine.row_eval(cfg, rows[j:j + 1], prow[p:p + 1], now_ns)
            mask[p, j], fit[p, j], la[p, j], numa[p, j] = f, a, b, n
        feas = mask[p]
        cand = np.where(feas & (order != INT64_MAX))[0]
        if len(cand):
            pref = cand[np.argmin(order[cand])]  # first minimum = lowest node
            raw[pref] = 1000
        mx = int(raw[feas].max()) if feas.any() else 0
        s = np.where(feas, (100 * raw) // mx if mx else 0, 0)
        rsvp[p] = s
        total = wf * fit[p].astype(np.int64) + wl * la[p].astype(np.int64) + wn * numa[p].astype(np.int64) + wr * s
        if feas.any():
            t = np.where(feas, total, -1)
            j = int(t.argmax())
            top1[p] = ((int(t[j]) + 1) << 32) | (0xFFFFFFFF - j)
    return mask, fit, la, numa, rsvp, top1


def restore_filter_doc():
    with open(os.path.join(HERE, "golden", "reservation_restore_filter_kat.json")) as f:
        return json.load(f)


def _kat_view(node_docs, rsv_docs, pod, affinity=False):
    """Nodes from {allocatable, requested, nonzero, pod_count, allowed_pods} dicts, reservations
    from {node, allocatable, allocated, n_assigned, matches_pod, policy, order} dicts, one
    single-container pod (owner class 0; affinity class 0 when `affinity`)."""
    nodes = np.zeros(len(node_docs), dtype=nat.NODE_SPEC)
    nodes["numa"] = -1
    for j, d in enumerate(node_docs):
        nodes[j]["allocatable"] = _rl(d["allocatable"])
        req = d.get("requested", {})
        nodes[j]["requested"] = _rl(req)
        nz = d.get("nonzero", req)
        nodes[j]["nonzero_requested"] = (nz.get("cpu", 0), nz.get("memory", 0))
        nodes[j]["pod_count"] = d.get("pod_count", 0)
        nodes[j]["allowed_pods"] = d.get("allowed_pods", 110)
    pods = np.zeros(1, dtype=nat.POD_SPEC)
    pods["n_containers"] = 1
    pods["label_priority_class"] = -1
    pods["label_qos"] = -1
    pods["rsv_owner_class"] = 0
    pods["rsv_affinity_class"] = 0 if affinity else -1
    pods["quota"] = -1
    cont = np.zeros(1, dtype=nat.CONTAINER)
    cont[0]["requests"] = _rl(pod)
    rsv = np.zeros(len(rsv_docs), dtype=nat.RESERVATION)
    pol = {"Default": nat.RSV_POLICY_DEFAULT, "Aligned": nat.RSV_POLICY_ALIGNED,
           "Restricted": nat.RSV_POLICY_RESTRICTED}
    for i, d in enumerate(rsv_docs):
        rsv[i]["node"] = d.get("node", 0)
        rsv[i]["flags"] = nat.RSV_AVAILABLE | (nat.RSV_ALLOCATE_ONCE if d.get("allocate_once") else 0)
        rsv[i]["policy"] = pol[d.get("policy", "Default")]
        rsv[i]["owner_classes"] = 1 if d.get("matches_pod", True) else 0
        rsv[i]["affinity_classes"] = 1 if d.get("affinity", d.get("matches_pod", True)) else 0
        rsv[i]["order"] = d.get("order", 0)
        rsv[i]["allocatable"] = _rl(d["allocatable"])
        rsv[i]["allocated"] = _rl(d.get("allocated"))
        rsv[i]["n_assigned"] = d.get("n_assigned", 0)
    return synth.SynthView(pods, cont, nodes, synth.NOW_NS, reservations=rsv)


def restore_view(doc):
    r = doc["restore"]
    return _kat_view([r["node"]], r["reservations"], r["pod"])


def filter_view(doc, case):
    f = doc["filter"]
    node = dict(f["node"], requested=case["pod_requested"])
    return _kat_view([node], [dict(f["reservation"], policy=case["policy"])], case["pod"], affinity=case["affinity"])


def order_view(doc):
    s = doc["score_with_order"]
    rsv = [dict(s["reservation"], node=j, order=o) for j, o in enumerate(s["orders"])]
    return _kat_view([s["node"]] * len(rsv), rsv, s["pod"])


def restored_dict(rec):
    """RSV_RESTORED → the JSON's units ({cpu, memory} maps, zero entries dropped)."""
    def rl(a):
        return {k: int(a[r]) for k, r in (("cpu", nat.RES_CPU), ("memory", nat.RES_MEMORY)) if int(a[r])}
    return {"pod_requested": rl(rec["pod_requested"]), "r_allocated": rl(rec["r_allocated"]),
            "requested": rl(rec["requested"]), "nonzero": rl(rec["nonzero"]),
            "pod_count": int(rec["pod_count"]), "n_matched": int(rec["n_matched"]),
            "has_state": bool(rec["has_state"])}
