"""Informer-event feeders (koordinator_amd/feeders.py).

* TestPodAssignCache_OnAdd / _OnUpdate / _OnDelete (loadaware/pod_assign_cache_test.go:35-253), case by
  case, on the feeder's podAssignCache (timeNowFn fixed as in the reference test);
* a seeded stream of node / pod / NodeMetric / NodeResourceTopology events: after every batch the rows
  the feeder emitted as deltas equal a fresh build of the final state, for every live node;
* the assign timestamps: an update re-stamps a bound pod (pod_assign_cache.go:90-100), which moves it
  from "assigned before the NodeMetric" to "estimated" in the LoadAware node term.
"""
import json

import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import feeders
from koordinator_amd.config import make_config, shipped_profile

NOW_NS = 1_700_000_000 * 10**9


def _pod(uid, name, node="", phase="Running", cpu="1", mem="1Gi", ns="default", status=None):
    p = {"metadata": {"uid": uid, "name": name, "namespace": ns, "labels": {}},
         "spec": {"nodeName": node, "containers": [{"resources": {"requests": {"cpu": cpu, "memory": mem},
                                                                  "limits": {"cpu": cpu, "memory": mem}}}]},
         "status": {"phase": phase}}
    if status is not None:
        p["metadata"]["annotations"] = {"scheduling.koordinator.sh/resource-status": json.dumps(status)}
    return p


class Clock:
    def __init__(self, t=NOW_NS, step=0):
        self.t, self.step = t, step

    def __call__(self):
        self.t += self.step
        return self.t


# ---- TestPodAssignCache_* ------------------------------------------------------------------------

FAKE_NOW = 12345   # fakeTimeNowFn: a fixed time


def _cache(events):
    f = feeders.SnapshotFeeder(make_config(), now_fn=lambda: FAKE_NOW)
    for ev in events:
        ev(f)
    return f.assign_cache


RUNNING = _pod("123456789", "test", node="test-node", phase="Running")
FAILED = _pod("123456789", "test", node="test-node", phase="Failed")


@pytest.mark.parametrize("pod, want", [
    ({"metadata": {"uid": "x"}, "spec": {}, "status": {}}, {}),                  # "update pending pod"
    (_pod("123456789", "test", node="test-node", phase="Failed"), {}),          # "update terminated pod"
    (RUNNING, {"test-node": {"123456789": FAKE_NOW}}),                           # "update scheduled running pod"
], ids=["pending", "terminated", "running"])
def test_pod_assign_cache_on_add(pod, want):
    """TestPodAssignCache_OnAdd (pod_assign_cache_test.go:35-107)."""
    assert _cache([lambda f: f.on_pod_add(pod)]) == want


@pytest.mark.parametrize("before, pod, want", [
    ([], {"metadata": {"uid": "x"}, "spec": {}, "status": {}}, {}),
    ([lambda f: f.on_pod_add(RUNNING)], FAILED, {}),
    ([], RUNNING, {"test-node": {"123456789": FAKE_NOW}}),
], ids=["pending", "terminated", "running"])
def test_pod_assign_cache_on_update(before, pod, want):
    """TestPodAssignCache_OnUpdate (pod_assign_cache_test.go:109-212): the cache holds the running pod in
    the "terminated" case; OnUpdate(nil, pod)."""
    assert _cache(before + [lambda f: f.on_pod_update(None, pod)]) == want


def test_pod_assign_cache_on_delete():
    """TestPodAssignCache_OnDelete (pod_assign_cache_test.go:214-253)."""
    assert _cache([lambda f: f.on_pod_add(RUNNING), lambda f: f.on_pod_delete(FAILED)]) == {}


# ---- event streams -------------------------------------------------------------------------------

def _node_obj(name, cpu, mem_gi, ann=None):
    return {"metadata": {"name": name, "annotations": ann or {}, "labels": {}},
            "status": {"allocatable": {"cpu": str(cpu), "memory": f"{mem_gi}Gi", "pods": "110",
                                       "kubernetes.io/batch-cpu": str(cpu * 300), "kubernetes.io/batch-memory": "8Gi"}}}


def _metric(name, upd_ns, cpu_m, mem_gi, pods=()):
    s = (upd_ns // 10**9)
    import datetime as dt
    ts = dt.datetime.fromtimestamp(s, dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
    return {"metadata": {"name": name}, "spec": {"metricCollectPolicy": {"reportIntervalSeconds": 60}},
            "status": {"updateTime": ts,
                       "nodeMetric": {"nodeUsage": {"resources": {"cpu": f"{cpu_m}m", "memory": f"{mem_gi}Gi"}}},
                       "podsMetric": [{"namespace": "default", "name": pn,
                                       "podUsage": {"resources": {"cpu": "300m", "memory": "512Mi"}}} for pn in pods]}}


def _nrt(name, zones):
    return {"metadata": {"name": name, "annotations": {}}, "topologyPolicies": ["SingleNUMANodePodLevel"],
            "zones": [{"name": f"node-{z}", "type": "Node",
                       "resources": [{"name": "cpu", "allocatable": str(c)}, {"name": "memory", "allocatable": f"{m}Gi"}]}
                      for z, (c, m) in enumerate(zones)]}


def _check(f, mirror):
    idx, rows, removed = f.take_deltas()
    for i in removed:
        mirror.pop(int(i), None)
    for i, r in zip(idx.tolist(), rows):
        mirror[i] = r.copy()
    fidx, frows = f.full_rows()
    assert sorted(mirror) == sorted(fidx.tolist())
    for i, r in zip(fidx.tolist(), frows):
        np.testing.assert_array_equal(mirror[i], r, err_msg=f"row {i}")


@pytest.mark.parametrize("plugins", ["shipped", "numa"])
def test_event_stream_deltas_equal_fresh_build(plugins):
    rng = np.random.default_rng(7)
    cfg = shipped_profile()
    if plugins == "numa":
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    clock = Clock(step=7 * 10**8)
    f = feeders.SnapshotFeeder(cfg, now_fn=clock)
    mirror = {}
    live_nodes, pods, next_uid = [], {}, [0]

    def new_pod(node=""):
        next_uid[0] += 1
        u = f"u{next_uid[0]}"
        cpu = ["250m", "500m", "1", "2"][rng.integers(4)]
        status = None
        if node and plugins == "numa" and rng.random() < 0.5:
            status = {"numaNodeResources": [{"node": int(rng.integers(2)), "resources": {"cpu": cpu, "memory": "1Gi"}}]}
        p = _pod(u, f"p{next_uid[0]}", node=node, cpu=cpu, mem=f"{int(rng.integers(1, 4))}Gi", status=status,
                 phase="Running" if node else "Pending")
        pods[u] = p
        f.on_pod_add(p)
        return p

    for step in range(12):
        for _ in range(int(rng.integers(1, 5))):                          # nodes join / change / leave
            r = rng.random()
            if r < 0.5 or len(live_nodes) < 3:
                name = f"n{len(live_nodes) + step * 10}"
                live_nodes.append(name)
                f.on_node_add(_node_obj(name, int(rng.choice([16, 32, 64])), int(rng.choice([64, 128]))))
                if plugins == "numa":
                    f.on_nrt(_nrt(name, [(8, 32), (8, 32)]))
            elif r < 0.8:
                name = live_nodes[int(rng.integers(len(live_nodes)))]
                f.on_node_update(_node_obj(name, 48, 96, ann={"node.koordinator.sh/raw-allocatable":
                                                              json.dumps({"cpu": "60"})}))
            else:
                name = live_nodes.pop(int(rng.integers(len(live_nodes))))
                f.on_node_delete(name)
                f.on_nrt_delete(name)
                f.on_node_metric_delete(name)
        for _ in range(int(rng.integers(5, 15))):                         # pods
            r = rng.random()
            bound = [u for u, p in pods.items() if p["spec"]["nodeName"] and p["status"]["phase"] == "Running"]
            if r < 0.35:
                new_pod(live_nodes[int(rng.integers(len(live_nodes)))])
            elif r < 0.5:
                new_pod("")                                               # pending
            elif r < 0.65:                                                # pending → bound (scheduled)
                pend = [u for u, p in pods.items() if not p["spec"]["nodeName"]]
                if pend:
                    u = pend[int(rng.integers(len(pend)))]
                    old, new = pods[u], json.loads(json.dumps(pods[u]))
                    new["spec"]["nodeName"] = live_nodes[int(rng.integers(len(live_nodes)))]
                    new["status"]["phase"] = "Running"
                    pods[u] = new
                    f.on_pod_update(old, new)
            elif r < 0.8 and bound:                                       # bound → Succeeded / Failed
                u = bound[int(rng.integers(len(bound)))]
                old, new = pods[u], json.loads(json.dumps(pods[u]))
                new["status"]["phase"] = ["Succeeded", "Failed"][rng.integers(2)]
                pods[u] = new
                f.on_pod_update(old, new)
            elif r < 0.9 and bound:                                       # label change: re-stamped
                u = bound[int(rng.integers(len(bound)))]
                old, new = pods[u], json.loads(json.dumps(pods[u]))
                new["metadata"]["labels"]["touched"] = str(step)
                pods[u] = new
                f.on_pod_update(old, new)
            elif pods:
                u = list(pods)[int(rng.integers(len(pods)))]
                f.on_pod_delete(pods.pop(u))
        for name in live_nodes:                                           # NodeMetric reports
            if rng.random() < 0.4:
                mine = [p["metadata"]["name"] for p in pods.values() if p["spec"]["nodeName"] == name]
                named = mine[: int(rng.integers(0, len(mine) + 1))] + (["ghost"] if rng.random() < 0.2 else [])
                f.on_node_metric(_metric(name, clock.t - int(rng.integers(0, 120)) * 10**9,
                                         int(rng.integers(100, 8000)), int(rng.integers(1, 30)), named))
        _check(f, mirror)
    assert len(mirror) >= 3 and f.assign_cache


def test_update_restamps_assign_time():
    """OnUpdate re-assigns a bound, non-terminated pod with timeNowFn() (pod_assign_cache.go:90-100): a pod
    assigned before the NodeMetric's UpdateTime − report interval counts with its PodsMetric usage, and
    after any update it is "estimated" again (load_aware.go:348-373), so the node term changes."""
    cfg = shipped_profile()
    clock = Clock()
    f = feeders.SnapshotFeeder(cfg, now_fn=clock)
    f.on_node_add(_node_obj("n0", 32, 64))
    p = _pod("a", "pa", node="n0", cpu="4", mem="8Gi")
    clock.t = NOW_NS - 600 * 10**9                 # assigned 10 minutes ago
    f.on_pod_add(p)
    clock.t = NOW_NS
    f.on_node_metric(_metric("n0", NOW_NS - 30 * 10**9, 2000, 4, pods=["pa"]))
    _, before = f.full_rows()
    p2 = json.loads(json.dumps(p))
    p2["metadata"]["labels"]["x"] = "y"
    f.on_pod_update(p, p2)                          # re-stamped at NOW_NS: after the UpdateTime
    assert f.assign_cache["n0"]["a"] == NOW_NS
    _, after = f.full_rows()
    assert (before["la_used"] != after["la_used"]).any()
