"""A seeded stream of informer events (nodes, pods, NodeMetrics, NodeResourceTopologies) for the
feeder tests (tests/test_feeders_cpu.py, tests/test_feeders_gpu.py)."""
import datetime as dt
import json

import numpy as np

NOW_NS = 1_700_000_000 * 10**9


def pod_obj(uid, name, node="", phase="Running", cpu="1", mem="1Gi", ns="default", status=None):
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


def node_obj(name, cpu, mem_gi, ann=None):
    return {"metadata": {"name": name, "annotations": ann or {}, "labels": {}},
            "status": {"allocatable": {"cpu": str(cpu), "memory": f"{mem_gi}Gi", "pods": "110",
                                       "kubernetes.io/batch-cpu": str(cpu * 300), "kubernetes.io/batch-memory": "8Gi"}}}


def metric_obj(name, upd_ns, cpu_m, mem_gi, pods=()):
    ts = dt.datetime.fromtimestamp(upd_ns // 10**9, dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
    return {"metadata": {"name": name}, "spec": {"metricCollectPolicy": {"reportIntervalSeconds": 60}},
            "status": {"updateTime": ts,
                       "nodeMetric": {"nodeUsage": {"resources": {"cpu": f"{cpu_m}m", "memory": f"{mem_gi}Gi"}}},
                       "podsMetric": [{"namespace": "default", "name": pn,
                                       "podUsage": {"resources": {"cpu": "300m", "memory": "512Mi"}}} for pn in pods]}}


def nrt_obj(name, zones):
    return {"metadata": {"name": name, "annotations": {}}, "topologyPolicies": ["SingleNUMANodePodLevel"],
            "zones": [{"name": f"node-{z}", "type": "Node",
                       "resources": [{"name": "cpu", "allocatable": str(c)}, {"name": "memory", "allocatable": f"{m}Gi"}]}
                      for z, (c, m) in enumerate(zones)]}


def run_stream(f, rng, clock, steps, numa=False, allow_delete=True, nodes_per_step=(1, 5), pods_per_step=(5, 15),
               on_step=None):
    """Drive feeder `f` with `steps` batches of events; on_step(step) after each batch.  Returns the pod
    objects that exist at the end (UID → object)."""
    live_nodes, pods, next_uid = [], {}, [0]

    def new_pod(node=""):
        next_uid[0] += 1
        u = f"u{next_uid[0]}"
        cpu = ["250m", "500m", "1", "2"][rng.integers(4)]
        status = None
        if node and numa and rng.random() < 0.5:
            status = {"numaNodeResources": [{"node": int(rng.integers(2)), "resources": {"cpu": cpu, "memory": "1Gi"}}]}
        p = pod_obj(u, f"p{next_uid[0]}", node=node, cpu=cpu, mem=f"{int(rng.integers(1, 4))}Gi", status=status,
                    phase="Running" if node else "Pending")
        pods[u] = p
        f.on_pod_add(p)

    def changed(u, edit):
        old, new = pods[u], json.loads(json.dumps(pods[u]))
        edit(new)
        pods[u] = new
        f.on_pod_update(old, new)

    for step in range(steps):
        for _ in range(int(rng.integers(*nodes_per_step))):              # nodes join / change / leave
            r = rng.random()
            if r < 0.5 or len(live_nodes) < 3:
                name = f"n{len(live_nodes) + step * 10}"
                live_nodes.append(name)
                f.on_node_add(node_obj(name, int(rng.choice([16, 32, 64])), int(rng.choice([64, 128]))))
                if numa:
                    f.on_nrt(nrt_obj(name, [(8, 32), (8, 32)]))
            elif r < 0.8 or not allow_delete:
                name = live_nodes[int(rng.integers(len(live_nodes)))]
                f.on_node_update(node_obj(name, 48, 96, ann={"node.koordinator.sh/raw-allocatable":
                                                             json.dumps({"cpu": "60"})}))
            else:
                name = live_nodes.pop(int(rng.integers(len(live_nodes))))
                f.on_node_delete(name)
                f.on_nrt_delete(name)
                f.on_node_metric_delete(name)
        for _ in range(int(rng.integers(*pods_per_step))):               # pods
            r = rng.random()
            bound = [u for u, p in pods.items() if p["spec"]["nodeName"] and p["status"]["phase"] == "Running"]
            if r < 0.35:
                new_pod(live_nodes[int(rng.integers(len(live_nodes)))])
            elif r < 0.5:
                new_pod("")                                              # pending
            elif r < 0.65:                                               # pending → bound (scheduled)
                pend = [u for u, p in pods.items() if not p["spec"]["nodeName"]]
                if pend:
                    target = live_nodes[int(rng.integers(len(live_nodes)))]

                    def bind(p, target=target):
                        p["spec"]["nodeName"] = target
                        p["status"]["phase"] = "Running"
                    changed(pend[int(rng.integers(len(pend)))], bind)
            elif r < 0.8 and bound:                                      # bound → Succeeded / Failed
                phase = ["Succeeded", "Failed"][rng.integers(2)]
                changed(bound[int(rng.integers(len(bound)))], lambda p: p["status"].update(phase=phase))
            elif r < 0.9 and bound:                                      # label change: re-stamped
                changed(bound[int(rng.integers(len(bound)))], lambda p: p["metadata"]["labels"].update(touched=str(step)))
            elif pods:
                u = list(pods)[int(rng.integers(len(pods)))]
                f.on_pod_delete(pods.pop(u))
        for name in live_nodes:                                          # NodeMetric reports
            if rng.random() < 0.4:
                mine = [p["metadata"]["name"] for p in pods.values() if p["spec"]["nodeName"] == name]
                named = mine[: int(rng.integers(0, len(mine) + 1))] + (["ghost"] if rng.random() < 0.2 else [])
                f.on_node_metric(metric_obj(name, clock.t - int(rng.integers(0, 120)) * 10**9,
                                            int(rng.integers(100, 8000)), int(rng.integers(1, 30)), named))
        if on_step is not None:
            on_step(step)
    return pods
