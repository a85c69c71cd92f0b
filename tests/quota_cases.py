"""ElasticQuota PreFilter known answers (tests/golden/elasticquota_prefilter_kat.json) as one-node
clusters: the pod's quota group carries the case's usedLimit / used / min / non-preemptible used; the
node has room for any pod, so the pair's feasibility is the quota gate."""
import json
import os

import numpy as np

from koordinator_amd import _native as nat
from koordinator_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
KEYS = {"cpu": nat.RES_CPU, "memory": nat.RES_MEMORY, "gpu": nat.RES_EXTENDED}


def doc():
    with open(os.path.join(HERE, "golden", "elasticquota_prefilter_kat.json")) as f:
        return json.load(f)


def quota_config(case):
    from koordinator_amd.config import make_config
    return make_config(plugins=("NodeResourcesFit", "ElasticQuota"), eq_check_parent_quota=int(case.get("check_parent", 0)))


def _rl(d):
    out = np.zeros((), dtype=nat.RESOURCE_LIST)
    for k, v in (d or {}).items():
        out["v"][KEYS[k]] = v
        out["present"] |= np.uint32(1 << KEYS[k])
    return out


def quota_view(case):
    nodes = np.zeros(1, dtype=nat.NODE_SPEC)
    nodes["numa"] = -1
    nodes[0]["allocatable"] = _rl({"cpu": 1 << 40, "memory": 1 << 50, "gpu": 1 << 20})
    nodes[0]["allowed_pods"] = 110
    pods = np.zeros(1, dtype=nat.POD_SPEC)
    pods["n_containers"] = 1
    pods["label_priority_class"] = -1
    pods["label_qos"] = -1
    pods["rsv_owner_class"] = -1
    pods["rsv_affinity_class"] = -1
    pods["quota"] = 0
    pods["non_preemptible"] = 1 if case.get("non_preemptible") else 0
    cont = np.zeros(1, dtype=nat.CONTAINER)
    cont[0]["requests"] = _rl(case["pod"])
    chain = case.get("parents", [])
    q = np.zeros(1 + len(chain), dtype=nat.QUOTA)
    q[0]["used_limit"] = _rl(case["used_limit"])
    q[0]["used"] = _rl(case.get("used"))
    q[0]["min"] = _rl(case.get("min"))
    q[0]["non_preemptible_used"] = _rl(case.get("non_preemptible_used"))
    for i, a in enumerate(chain):  # group i's parent is group i + 1; the last one's parent is the root
        q[i + 1]["used_limit"] = _rl(a["used_limit"])
        q[i + 1]["used"] = _rl(a.get("used"))
    q["parent"] = np.arange(1, len(q) + 1)
    q["parent"][-1] = -1
    return synth.SynthView(pods, cont, nodes, synth.NOW_NS, quotas=q)


def used_tree_doc():
    with open(os.path.join(HERE, "golden", "elasticquota_used_tree_kat.json")) as f:
        return json.load(f)


def used_tree_view(case):
    """A one-node cluster with the case's groups (usedLimit / min far above every request) and its pods."""
    names = [g["name"] for g in case["groups"]]
    nodes = np.zeros(1, dtype=nat.NODE_SPEC)
    nodes["numa"] = -1
    nodes[0]["allocatable"] = _rl({"cpu": 1 << 40, "memory": 1 << 50})
    nodes[0]["allowed_pods"] = 110
    P = len(case["pods"])
    pods = np.zeros(P, dtype=nat.POD_SPEC)
    pods["n_containers"] = 1
    pods["first_container"] = np.arange(P)
    pods["label_priority_class"] = -1
    pods["label_qos"] = -1
    pods["rsv_owner_class"] = -1
    pods["rsv_affinity_class"] = -1
    cont = np.zeros(P, dtype=nat.CONTAINER)
    for i, p in enumerate(case["pods"]):
        pods[i]["quota"] = names.index(p["group"])
        pods[i]["non_preemptible"] = 1 if p["non_preemptible"] else 0
        cont[i]["requests"] = _rl({"cpu": p["cpu"], "memory": p["memory"]})
    q = np.zeros(len(names), dtype=nat.QUOTA)
    for i, g in enumerate(case["groups"]):
        q[i]["used_limit"] = _rl({"cpu": 1 << 40, "memory": 1 << 50})
        q[i]["min"] = _rl({"cpu": 1 << 40, "memory": 1 << 50})
        q[i]["parent"] = -1 if g["parent"] is None else names.index(g["parent"])
    return synth.SynthView(pods, cont, nodes, synth.NOW_NS, quotas=q), names


def used_tree_want(case, names):
    """want[group] → (used, nonPreemptibleUsed) as [NUM_RES] arrays."""
    out = []
    for name in names:
        w = case["want"].get(name, {"used": {}, "non_preemptible_used": {}})
        out.append((_rl(w["used"])["v"].copy(), _rl(w["non_preemptible_used"])["v"].copy()))
    return out
