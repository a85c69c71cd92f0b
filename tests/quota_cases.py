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
