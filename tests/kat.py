"""Turn the transcribed reference known-answer tests (tests/golden/*.json) into objects."""
from __future__ import annotations

import json
import os

from koordinator_amd.config import make_config
from koordinator_amd.objects import Cluster, Container, Node, NodeMetric, Pod

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name: str) -> dict:
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def pod_from(d: dict) -> Pod:
    return Pod(namespace=d.get("namespace", "default"), name=d["name"],
               containers=[Container(requests=c.get("requests", {}), limits=c.get("limits", {}))
                           for c in d.get("containers", [])],
               priority=d.get("priority"), labels=d.get("labels", {}), daemonset=d.get("daemonset", False))


def metric_from(d):
    if d is None:
        return None
    return NodeMetric(update_time_s=d.get("update_time_s"), report_interval_s=d.get("report_interval_s"),
                      node_usage=d.get("node_usage"), aggregated=d.get("aggregated", []),
                      pods_metric=d.get("pods_metric", []))


def case_cluster(doc: dict, case: dict, pod_key: str):
    """Returns (cfg, view, pod_index, node_index=0) for one score/filter case."""
    args = dict(case.get("args", {}))
    if "score_according_prod_usage" in args:
        args["score_according_prod_usage"] = bool(args["score_according_prod_usage"])
    cfg = make_config(**args)
    nd = doc["node"]
    node = Node(nd["name"], allocatable=nd["allocatable"],
                custom_usage_thresholds=case.get("custom_usage_thresholds"),
                custom_prod_usage_thresholds=case.get("custom_prod_usage_thresholds"),
                custom_aggregated=case.get("custom_aggregated"))
    cl = Cluster()
    cl.add_node(node)
    m = metric_from(case.get("node_metric"))
    if m is not None:
        cl.set_metric(node.name, m)
    for lp in case.get("lister_pods", []):
        cl.add_lister_pod(pod_from(lp))
    for a in case.get("assigned", []):
        ap = pod_from(a["pod"])
        cl.add_lister_pod(ap)     # the test creates assigned pods through the clientset
        cl.assign(node.name, ap, a["age_s"])
    pod = pod_from(case[pod_key]) if case.get(pod_key) else Pod(name="empty")
    view = cl.view(extra_pods=[pod])
    return cfg, view, view.pod_index(pod), cl
