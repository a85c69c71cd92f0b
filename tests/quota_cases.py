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
    q = np.zeros(1, dtype=nat.QUOTA)
    q[0]["used_limit"] = _rl(case["used_limit"])
    q[0]["used"] = _rl(case.get("used"))
    q[0]["min"] = _rl(case.get("min"))
    q[0]["non_preemptible_used"] = _rl(case.get("non_preemptible_used"))
    return synth.SynthView(pods, cont, nodes, synth.NOW_NS, quotas=q)
