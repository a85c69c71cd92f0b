"""Snapshot ingest from k8s-shaped objects (koordinator_amd/ingest.py).

Pinned by the reference's own tests:
* TestTrimNodeAllocatableByNodeReservation (pkg/util/node_test.go:231-312);
* TestNodeReservationTransformer (pkg/util/transformer/node_transformer_test.go:89-259): every
  reservation spec on the three fake nodes, expected allocatable computed as that test computes it;
* TestTransformNode (node_transformer_test.go:261-): deprecated batch resource names;
* the LoadAwareScheduling known answers (tests/golden/loadaware_kat.json, load_aware_test.go) re-expressed
  as real objects — corev1.Node with its annotations, slov1alpha1.NodeMetric with an RFC 3339 updateTime,
  corev1.Pod — ingested, flattened and scored by the oracle and by the engine's own per-pair code.
"""
import datetime as dt
import json
from fractions import Fraction

import pytest

from kat import load
from koordinator_amd import engine, ingest
from koordinator_amd.config import make_config
from koordinator_amd.objects import Node
from oracle import oracle

Q = ingest.parse_quantity


def _node(alloc, annotations=None, name="n", labels=None, capacity=None):
    status = {"allocatable": alloc}
    if capacity is not None:
        status["capacity"] = capacity
    return {"metadata": {"name": name, "annotations": annotations or {}, "labels": labels or {}}, "status": status}


def _rl(d):
    return {k: Q(v) for k, v in d.items()}


# ---- TestTrimNodeAllocatableByNodeReservation ----------------------------------------------------

TRIM_ALLOC = {"cpu": "96", "memory": "512Gi", "kubernetes.io/batch-cpu": "16", "kubernetes.io/batch-memory": "32Gi",
              "nvidia.com/gpu": "8"}


@pytest.mark.parametrize("policy,want,trimmed", [
    ("Default", {"cpu": "80", "memory": "500Gi", "kubernetes.io/batch-cpu": "16",
                 "kubernetes.io/batch-memory": "32Gi", "nvidia.com/gpu": "8"}, True),
    ("ReservedCPUsOnly", TRIM_ALLOC, False),
])
def test_trim_node_allocatable_by_node_reservation(policy, want, trimmed):
    rsv = {"resources": {"cpu": "16", "memory": "12Gi"}, "applyPolicy": policy}
    got, got_trimmed = ingest.trim_allocatable_by_node_reservation(_node(TRIM_ALLOC, {ingest.NODE_RESERVATION: json.dumps(rsv)}))
    assert got == _rl(want) and got_trimmed == trimmed


# ---- TestNodeReservationTransformer ----------------------------------------------------------------

FAKE_ALLOC = {"cpu": "10", "memory": "10Gi", "pods": "200", "kubernetes.io/batch-cpu": "1",
              "ephemeral-storage": "10Gi", "kubernetes.io/batch-memory": "1Gi"}
RESERVATIONS = [
    {},
    {"resources": {"cpu": "1"}},
    {"resources": {"cpu": "1"}, "applyPolicy": "Default"},
    {"reservedCPUs": "0-1"},
    {"reservedCPUs": "0-1", "applyPolicy": "Default"},
    {"reservedCPUs": "0-1", "resources": {"cpu": "1"}},
    {"resources": {"memory": "2Gi"}},
    {"resources": {"memory": "2Gi", "cpu": "1"}},
    {"resources": {"memory": "1Gi"}, "reservedCPUs": "2"},
    {"resources": {"kubernetes.io/batch-memory": "1Gi"}},
    {"resources": {"kubernetes.io/batch-cpu": "1"}},
    {"reservedCPUs": "0-3", "applyPolicy": "ReservedCPUsOnly"},
]


@pytest.mark.parametrize("rsv", RESERVATIONS, ids=lambda r: json.dumps(r, sort_keys=True))
@pytest.mark.parametrize("variant", ["annotated", "no-annotations", "other-annotation"])
def test_node_reservation_transformer(rsv, variant):
    ann = {"annotated": {ingest.NODE_RESERVATION: json.dumps(rsv)}, "no-annotations": {},
           "other-annotation": {"k": "v"}}[variant]
    node = _node(FAKE_ALLOC, ann)
    reserved = {}
    if variant == "annotated" and rsv.get("applyPolicy", "") in ("", "Default"):
        reserved = ingest.reservation_resources(rsv)       # util.GetNodeReservationFromAnnotation
    orig = _rl(FAKE_ALLOC)
    want = {k: (v if k.startswith("kubernetes.io/batch-") else v - reserved.get(k, 0)) for k, v in orig.items()}
    got = ingest.resources(ingest.transform_node(node)["status"]["allocatable"])
    # framework.NewResource view: keys the reservation adds at zero do not change the Resource
    assert {k: v for k, v in got.items() if k in orig} == want
    assert all(got[k] == 0 for k in got if k not in orig)


# ---- TestTransformNode -----------------------------------------------------------------------------

def test_transform_node_deprecated_batch_resources():
    base = {"cpu": "32", "memory": "64Gi"}
    old = dict(base, **{"koordinator.sh/batch-cpu": "1000", "koordinator.sh/batch-memory": "10Gi"})
    new = dict(base, **{"kubernetes.io/batch-cpu": "1000", "kubernetes.io/batch-memory": "10Gi"})
    plain = ingest.transform_node(_node(base, capacity=base))["status"]
    assert ingest.resources(plain["allocatable"]) == _rl(base) == ingest.resources(plain["capacity"])
    got = ingest.transform_node(_node(old, capacity=old))["status"]
    assert ingest.resources(got["allocatable"]) == _rl(new) == ingest.resources(got["capacity"])
    both = dict(old, **new)        # current names present: the deprecated ones are left as they are
    got = ingest.transform_node(_node(both, capacity=both))["status"]
    assert ingest.resources(got["allocatable"]) == _rl(both) == ingest.resources(got["capacity"])


def test_transform_pod_deprecated_batch_resources():
    pod = {"metadata": {"name": "p"}, "spec": {"containers": [{"resources": {
        "requests": {"koordinator.sh/batch-cpu": "1000", "koordinator.sh/batch-memory": "1Gi"},
        "limits": {"koordinator.sh/batch-cpu": "1000", "koordinator.sh/batch-memory": "1Gi"}}}]}}
    p = ingest.pod_from_object(pod)
    assert p.containers[0].requests == {"kubernetes.io/batch-cpu": Fraction(1000), "kubernetes.io/batch-memory": Q("1Gi")}


def test_unsupported_pod_resource_is_refused():
    pod = {"metadata": {"name": "p"}, "spec": {"containers": [{"resources": {"requests": {"nvidia.com/gpu": "1"}}}]}}
    with pytest.raises(ingest.UnsupportedResource):
        ingest.pod_from_object(pod)


def test_pod_fit_request_init_containers_and_overhead():
    pod = {"metadata": {"name": "p"}, "spec": {
        "containers": [{"resources": {"requests": {"cpu": "1"}}}, {"resources": {"requests": {"memory": "1Gi"}}}],
        "initContainers": [{"resources": {"requests": {"cpu": "3"}}}],
        "overhead": {"cpu": "250m", "memory": "100Mi"}}}
    req, nz = ingest.pod_fit_request(ingest.pod_from_object(pod))
    assert req == {"cpu": Q("3.25"), "memory": Q("1Gi") + Q("100Mi")}
    # NonZero: (1000 + 100) vs init 3000 → 3000, + overhead 250; memory 200Mi + 1Gi (> init default), + 100Mi
    assert nz == (3250, 200 * 2**20 + 2**30 + 100 * 2**20)


# ---- NodeResourceTopology --------------------------------------------------------------------------

def test_nrt_zones_policy_and_cpu_topology():
    nrt = {"metadata": {"name": "n", "annotations": {ingest.CPU_TOPOLOGY: json.dumps(
        {"detail": [{"id": 0, "core": 0, "socket": 0, "node": 0}, {"id": 1, "core": 1, "socket": 0, "node": 1}]})}},
        "topologyPolicies": ["None", "Restricted"],
        "zones": [{"name": "node-1", "type": "Node", "resources": [{"name": "cpu", "allocatable": "26"},
                                                                    {"name": "memory", "allocatable": "64Gi"}]},
                  {"name": "node-0", "type": "Node", "resources": [{"name": "cpu", "allocatable": "26"}]},
                  {"name": "socket-0", "type": "Socket", "resources": []},
                  {"name": "nodeX", "type": "Node", "resources": []}]}
    n = ingest.node_from_object(_node({"cpu": "52", "memory": "128Gi", "pods": "110"}), nrt)
    assert n.numa_zone_ids == [0, 1] and n.numa_policy == "Restricted" and n.cpu_topology_valid and n.pods == 110
    assert n.numa_zones[1] == {"cpu": Q("26"), "memory": Q("64Gi")}
    labelled = ingest.node_from_object(_node({"cpu": "52"}, labels={ingest.NUMA_POLICY_LABEL: "SingleNUMANode"}), nrt)
    assert labelled.numa_policy == "SingleNUMANode"
    del nrt["metadata"]["annotations"][ingest.CPU_TOPOLOGY]
    assert not ingest.node_from_object(_node({"cpu": "52"}), nrt).cpu_topology_valid


def test_invalid_annotations_flatten_to_unparsable_state():
    n = ingest.node_from_object(_node({"cpu": "8"}, {ingest.RAW_ALLOCATABLE: "{bad", ingest.USAGE_THRESHOLDS: "[1"}))
    assert n.raw_allocatable_invalid and n.custom_thresholds_invalid
    from koordinator_amd.objects import Cluster
    view = Cluster().add_node(n).view()
    assert view.nodes[0]["raw_allocatable_state"] == -1 and view.nodes[0]["custom_thresholds_state"] == -1


# ---- LoadAwareScheduling known answers through real objects ----------------------------------------

DOC = load("loadaware_kat.json")
NOW_NS = 1_700_000_000 * 10**9


def _rfc3339(ns):
    return dt.datetime.fromtimestamp(ns // 10**9, dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _pod_obj(d, node_name=""):
    owners = [{"kind": "DaemonSet", "name": "ds", "controller": True}] if d.get("daemonset") else []
    return {"metadata": {"name": d["name"], "namespace": d.get("namespace", "default"), "labels": d.get("labels", {}),
                         "ownerReferences": owners},
            "spec": {"priority": d.get("priority"), "nodeName": node_name,
                     "containers": [{"resources": {"requests": c.get("requests", {}), "limits": c.get("limits", {})}}
                                    for c in d.get("containers", [])]}}


def _objects(case, pod_key):
    nd = DOC["node"]
    ann = {}
    thr = {}
    if case.get("custom_usage_thresholds"):
        thr["usageThresholds"] = case["custom_usage_thresholds"]
    if case.get("custom_prod_usage_thresholds"):
        thr["prodUsageThresholds"] = case["custom_prod_usage_thresholds"]
    if case.get("custom_aggregated"):
        ca = dict(case["custom_aggregated"])
        if "usageAggregatedDuration" in ca:
            ca["usageAggregatedDuration"] = f"{int(ca['usageAggregatedDuration'])}s"
        thr["aggregatedUsage"] = ca
    if thr:
        ann[ingest.USAGE_THRESHOLDS] = json.dumps(thr)
    node = _node(dict(nd["allocatable"]), ann, name=nd["name"])
    metrics = []
    m = case.get("node_metric")
    if m is not None:
        status = {}
        if m.get("update_time_s") is not None:
            assert float(m["update_time_s"]).is_integer()
            status["updateTime"] = _rfc3339(NOW_NS + int(m["update_time_s"]) * 10**9)
        if m.get("node_usage") is not None or m.get("aggregated"):
            status["nodeMetric"] = {
                "nodeUsage": {"resources": m.get("node_usage") or {}},
                "aggregatedNodeUsages": [{"duration": f"{int(a['duration'])}s",
                                          "usage": {t: {"resources": u} for t, u in a["usage"].items()}}
                                         for a in m.get("aggregated", [])]}
        if m.get("pods_metric"):
            status["podsMetric"] = [{"namespace": pm.get("namespace", "default"), "name": pm["name"],
                                     "podUsage": {"resources": pm["usage"]}} for pm in m["pods_metric"]]
        spec = {} if m.get("report_interval_s") is None else {"metricCollectPolicy": {"reportIntervalSeconds": m["report_interval_s"]}}
        metrics.append({"metadata": {"name": nd["name"]}, "spec": spec, "status": status})
    pods = [_pod_obj(lp) for lp in case.get("lister_pods", [])]
    pods += [_pod_obj(a["pod"]) for a in case.get("assigned", [])]
    cl = ingest.cluster_from_objects([node], pods, metrics, now_ns=NOW_NS)
    for a in case.get("assigned", []):      # podAssignCache: scheduler state, not an object
        cl.assign(nd["name"], cl.lister_pods[f"default/{a['pod']['name']}"], a["age_s"])
    pod = ingest.pod_from_object(_pod_obj(case[pod_key] if case.get(pod_key) else {"name": "empty"}))
    view = cl.view(extra_pods=[pod])
    args = dict(case.get("args", {}))
    if "score_according_prod_usage" in args:
        args["score_according_prod_usage"] = bool(args["score_according_prod_usage"])
    return make_config(**args), view, view.pod_index(pod), cl


@pytest.mark.parametrize("case", DOC["score_cases"], ids=lambda c: c["name"])
def test_loadaware_score_kat_from_objects(case):
    cfg, view, pi, cl = _objects(case, "pod")
    assert oracle.la_score(cfg, view, pi, 0, NOW_NS) == case["want"]
    ok, fit, la, _ = engine.row_eval(cfg, engine.build_node_rows(cfg, view), engine.build_pod_rows(cfg, view, [pi]),
                                     NOW_NS)
    assert la == case["want"]


@pytest.mark.parametrize("case", DOC["filter_cases"], ids=lambda c: c["name"])
def test_loadaware_filter_kat_from_objects(case):
    cfg, view, pi, cl = _objects(case, "test_pod")
    assert oracle.la_filter(cfg, view, pi, 0, NOW_NS) == case["want"]


def test_cluster_nodeinfo_from_bound_pods():
    pods = [_pod_obj({"name": "a", "containers": [{"requests": {"cpu": "2", "memory": "1Gi"}}]}, "n"),
            _pod_obj({"name": "b", "containers": [{}]}, "n"),
            dict(_pod_obj({"name": "done", "containers": [{"requests": {"cpu": "8"}}]}, "n"), status={"phase": "Succeeded"})]
    cl = ingest.cluster_from_objects([_node({"cpu": "16", "memory": "32Gi", "pods": "110"})], pods, now_ns=NOW_NS)
    view = cl.view()
    ns = view.nodes[0]
    assert int(ns["pod_count"]) == 2 and int(ns["allowed_pods"]) == 110
    assert int(ns["requested"]["v"][0]) == 2000 and int(ns["requested"]["v"][1]) == 2**30
    assert list(ns["nonzero_requested"]) == [2100, 2**30 + 200 * 2**20]
    assert isinstance(cl.nodes[0], Node)


def _cpu_topology_ann(sockets, cores_per_socket, threads):
    detail, cid = [], 0
    for s in range(sockets):
        for c in range(cores_per_socket):
            for _ in range(threads):
                detail.append({"id": cid, "core": s * cores_per_socket + c, "socket": s, "node": s})
                cid += 1
    return json.dumps({"detail": detail})


def test_cpuset_inputs_from_objects():
    """NodeResourceTopology CPU topology / kubelet policy / reserved CPUs, node reservation, bound pods'
    resource-status cpusets and a pending pod's resource-spec → the engine's cpuset counts and verdicts,
    the same as the oracle's literal Allocate."""
    nrt = {"metadata": {"name": "n", "annotations": {
        ingest.CPU_TOPOLOGY: _cpu_topology_ann(2, 4, 2),
        ingest.KUBELET_CPU_MANAGER_POLICY: json.dumps({"policy": "static", "reservedCPUs": "0"}),
        ingest.POD_CPU_ALLOCS: json.dumps([{"uid": "u1", "cpuset": "15", "managedByKubelet": True}])}},
        "zones": [{"name": "node-0", "type": "Node", "resources": [{"name": "cpu", "allocatable": "8"}]},
                  {"name": "node-1", "type": "Node", "resources": [{"name": "cpu", "allocatable": "8"}]}]}
    node = _node({"cpu": "16", "memory": "64Gi", "pods": "110"}, name="n")
    bound = {"metadata": {"name": "b", "annotations": {ingest.RESOURCE_STATUS: json.dumps({"cpuset": "2-5"}),
                                                       ingest.RESOURCE_SPEC: json.dumps({"preferredCPUExclusivePolicy": "PCPULevel"})},
                          "labels": {"koordinator.sh/qosClass": "LSR"}},
             "spec": {"nodeName": "n", "priority": 9999,
                      "containers": [{"resources": {"requests": {"cpu": "4"}, "limits": {"cpu": "4"}}}]}}
    cl = ingest.cluster_from_objects([node], [bound], nrts=[nrt], now_ns=NOW_NS)
    n = cl.nodes[0]
    assert n.reserved_cpus == [0, 15] and n.cpu_allocated == {c: (1, "PCPULevel") for c in range(2, 6)}
    assert n.cpu_bind_policy == "None"
    pend = []
    for name, spec, cpu in [("full", {"requiredCPUBindPolicy": "FullPCPUs"}, "6"),
                            ("full-too-many", {"requiredCPUBindPolicy": "FullPCPUs"}, "10"),
                            ("spread", {"requiredCPUBindPolicy": "SpreadByPCPUs"}, "5"),
                            ("odd-full", {"requiredCPUBindPolicy": "FullPCPUs"}, "3"),
                            ("preferred", {}, "8"), ("fractional", {}, "1500m")]:
        pend.append(ingest.pod_from_object({"metadata": {"name": name, "labels": {"koordinator.sh/qosClass": "LSR"},
                                                         "annotations": {ingest.RESOURCE_SPEC: json.dumps(spec)}},
                                            "spec": {"priority": 9999, "containers": [{"resources": {
                                                "requests": {"cpu": cpu}, "limits": {"cpu": cpu}}}]}}))
    view = cl.view(extra_pods=pend)
    cfg = make_config(plugins=("NodeNUMAResource",))
    rows = engine.build_node_rows(cfg, view)
    # free: cores {0,1}→cpus 1 (0 reserved); core 1 (2,3) held; core 2 (4,5) held; 6..14 free, 15 reserved
    assert (rows[0]["cpus_per_core"], rows[0]["cpuset_full_free_cpus"], rows[0]["cpuset_free_cores"]) == (2, 8, 6)
    want = {"full": True, "full-too-many": False, "spread": True, "odd-full": False, "preferred": True,
            "fractional": False}
    for p in pend:
        pi = view.pod_index(p)
        ok, _ = oracle.numa_eval(cfg, view, pi, 0)
        got = engine.row_eval(cfg, rows[0:1], engine.build_pod_rows(cfg, view, [pi]), NOW_NS)
        assert bool(ok) == bool(got[0]) == want[p.name], p.name


@pytest.mark.parametrize("ann, reserved", [
    (None, [0, 15]),
    (json.dumps({"cpuset": "6-9"}), [0, 6, 7, 8, 9, 15]),                        # cpusetExclusive defaults to true
    (json.dumps({"cpuset": "6-9", "cpusetExclusive": True}), [0, 6, 7, 8, 9, 15]),
    (json.dumps({"cpuset": "6-9", "cpusetExclusive": False}), [0, 15]),
    ("bad-format-str", [0, 15]),                                                 # GetSystemQOSResource error
    (json.dumps({"cpuset": "9-6"}), [0, 15]),                                    # cpuset.Parse error
])
def test_system_qos_exclusive_cpuset_is_reserved(ann, reserved):
    """NewTopologyOptions (topology_options.go:119-134) unions the exclusive system-QoS cpuset of
    node.koordinator.sh/system-qos-resource into ReservedCPUs (system_qos.go:35-38: exclusive unless
    cpusetExclusive is false; TestGetSystemQOSResource's "bad-format-str" is skipped); a FullPCPUs pod that
    needs the reserved cores then fails on the engine exactly as in the oracle's literal Allocate."""
    anns = {ingest.CPU_TOPOLOGY: _cpu_topology_ann(2, 4, 2),
            ingest.KUBELET_CPU_MANAGER_POLICY: json.dumps({"policy": "static", "reservedCPUs": "0"}),
            ingest.POD_CPU_ALLOCS: json.dumps([{"uid": "u1", "cpuset": "15", "managedByKubelet": True}])}
    if ann is not None:
        anns[ingest.SYSTEM_QOS_RESOURCE] = ann
    nrt = {"metadata": {"name": "n", "annotations": anns},
           "zones": [{"name": "node-0", "type": "Node", "resources": [{"name": "cpu", "allocatable": "8"}]},
                     {"name": "node-1", "type": "Node", "resources": [{"name": "cpu", "allocatable": "8"}]}]}
    node = _node({"cpu": "16", "memory": "64Gi", "pods": "110"}, name="n")
    cl = ingest.cluster_from_objects([node], [], nrts=[nrt], now_ns=NOW_NS)
    assert cl.nodes[0].reserved_cpus == reserved
    pend = ingest.pod_from_object({"metadata": {"name": "full8", "labels": {"koordinator.sh/qosClass": "LSR"},
                                                "annotations": {ingest.RESOURCE_SPEC: json.dumps(
                                                    {"requiredCPUBindPolicy": "FullPCPUs"})}},
                                   "spec": {"priority": 9999, "containers": [{"resources": {
                                       "requests": {"cpu": "10"}, "limits": {"cpu": "10"}}}]}})
    view = cl.view(extra_pods=[pend])
    cfg = make_config(plugins=("NodeNUMAResource",))
    rows = engine.build_node_rows(cfg, view)
    pi = view.pod_index(pend)
    ok, _ = oracle.numa_eval(cfg, view, pi, 0)
    got = engine.row_eval(cfg, rows[0:1], engine.build_pod_rows(cfg, view, [pi]), NOW_NS)
    # 16 CPUs, 2 per core: the whole free cores hold 12 CPUs with 0 and 15 reserved, 8 with 6-9 too
    assert bool(ok) == bool(got[0]) == (len(reserved) == 2)
