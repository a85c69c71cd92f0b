"""Object model of the inputs the koord-scheduler plugins read, and its flattening into the
C structs of ``include/koord_gpu.h`` (``kg_cluster_view``).

This is the Python face of the drop-in boundary: a Go shim builds the same structs from its
informer objects (corev1.Pod / corev1.Node / NodeInfo / slov1alpha1.NodeMetric and the
LoadAware podAssignCache).  Quantities follow k8s ``resource.Quantity``: cpu is stored as
``MilliValue()``, everything else as ``Value()`` (rounded up, as Quantity does).
"""
from __future__ import annotations

import contextlib
import dataclasses
import math
import re
from fractions import Fraction
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _native as nat

# The engine's resource slots: the fixed names, then the named scalar slots (kg_config.ext_resource_names) —
# extended resources and hugepages-<size> the deployment's pods request.  RES maps a resource name to its slot for
# the flattening and the config builders; the Go shim keeps the same map per profile.  Names outside it are dropped
# from nodes and make a pod that requests them unsupported (ingest.UnsupportedResource).
DEFAULT_EXTENDED = ("example.com/gpu",)


def resource_map(extended=DEFAULT_EXTENDED) -> Dict[str, int]:
    """name → slot for the fixed resources and `extended` (≤ NUM_EXT_RES names, slot RES_EXT0 + i; "" skips one)."""
    extended = tuple(extended)
    if len(extended) > nat.NUM_EXT_RES:
        raise ValueError(f"at most {nat.NUM_EXT_RES} named scalar resources, got {len(extended)}")
    out = {n: r for r, n in enumerate(nat.FIXED_RES_NAMES)}
    for i, n in enumerate(extended):
        if not n:
            continue
        if n in out:
            raise ValueError(f"named scalar resource {n!r} repeats or is a fixed resource")
        out[n] = nat.RES_EXT0 + i
    return out


RES: Dict[str, int] = {}
EXTENDED = DEFAULT_EXTENDED


def set_extended_resources(names=DEFAULT_EXTENDED) -> None:
    """Point the flattening (and the config builders' defaults) at the profile's named scalar slots."""
    global EXTENDED
    m = resource_map(names)
    RES.clear()
    RES.update(m)
    EXTENDED = tuple(names)


@contextlib.contextmanager
def extended_resources(names):
    """set_extended_resources for a block (tests and tools building clusters for one profile)."""
    old = EXTENDED
    set_extended_resources(names)
    try:
        yield
    finally:
        set_extended_resources(old)


set_extended_resources()
BATCH_CPU = "kubernetes.io/batch-cpu"
BATCH_MEMORY = "kubernetes.io/batch-memory"

PRIORITY_CLASS = {"koord-prod": nat.PRIO_PROD, "koord-mid": nat.PRIO_MID, "koord-batch": nat.PRIO_BATCH,
                  "koord-free": nat.PRIO_FREE}
QOS_CLASS = {"LSE": nat.QOS_LSE, "LSR": nat.QOS_LSR, "LS": nat.QOS_LS, "BE": nat.QOS_BE, "SYSTEM": nat.QOS_SYSTEM}
KUBE_QOS = {"": nat.KUBE_QOS_UNSET, "Guaranteed": nat.KUBE_QOS_GUARANTEED, "Burstable": nat.KUBE_QOS_BURSTABLE,
            "BestEffort": nat.KUBE_QOS_BESTEFFORT}
AGG = {"": nat.AGG_UNSET, "avg": nat.AGG_AVG, "p50": nat.AGG_P50, "p90": nat.AGG_P90, "p95": nat.AGG_P95,
       "p99": nat.AGG_P99}

PRIORITY_PROD_MAX, PRIORITY_PROD_MIN = 9999, 9000
PRIORITY_MID_MAX, PRIORITY_MID_MIN = 7999, 7000
PRIORITY_BATCH_MAX, PRIORITY_BATCH_MIN = 5999, 5000
PRIORITY_FREE_MAX, PRIORITY_FREE_MIN = 3999, 3000

_SUFFIX = {
    "": 1, "m": Fraction(1, 1000), "k": 10**3, "M": 10**6, "G": 10**9, "T": 10**12, "P": 10**15, "E": 10**18,
    "Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60,
}
_QRE = re.compile(r"^([+-]?[0-9.]+)([eE][+-]?[0-9]+)?([a-zA-Z]*)$")


def parse_quantity(s) -> Fraction:
    """resource.MustParse → exact rational value in base units."""
    if isinstance(s, (int, Fraction)):
        return Fraction(s)
    m = _QRE.match(str(s).strip())
    if not m:
        raise ValueError(f"bad quantity {s!r}")
    num, exp, suf = m.groups()
    v = Fraction(num)
    if exp:
        v *= Fraction(10) ** int(exp[1:])
    if suf not in _SUFFIX:
        raise ValueError(f"bad quantity suffix {s!r}")
    return v * _SUFFIX[suf]


def quantity_value(name: str, q) -> int:
    """getResourceValue semantics: MilliValue for cpu, Value otherwise (ceil, as Quantity)."""
    v = parse_quantity(q)
    if name == "cpu":
        v *= 1000
    return int(math.ceil(v))


def resource_list(d: Optional[Dict[str, object]]) -> np.ndarray:
    out = np.zeros((), dtype=nat.RESOURCE_LIST)
    for k, q in (d or {}).items():
        r = RES[k]
        out["v"][r] = quantity_value(k, q)
        out["present"] |= np.uint32(1 << r)
    return out


@dataclasses.dataclass
class Container:
    requests: Dict[str, object] = dataclasses.field(default_factory=dict)
    limits: Dict[str, object] = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class Pod:
    namespace: str = "default"
    name: str = ""
    containers: List[Container] = dataclasses.field(default_factory=list)
    init_containers: List[Container] = dataclasses.field(default_factory=list)
    overhead: Optional[Dict[str, object]] = None
    priority: Optional[int] = None
    labels: Dict[str, str] = dataclasses.field(default_factory=dict)
    qos_status: str = ""
    # annotation scheduling.koordinator.sh/resource-spec (ResourceSpec)
    cpu_bind_required: str = ""
    cpu_bind_preferred: str = ""
    cpu_exclusive: str = ""
    daemonset: bool = False
    terminated: bool = False
    node_name: str = ""

    @property
    def key(self) -> str:
        return f"{self.namespace}/{self.name}"


@dataclasses.dataclass
class Node:
    name: str
    allocatable: Dict[str, object] = dataclasses.field(default_factory=dict)
    pods: int = 110
    annotations_raw_allocatable: Optional[Dict[str, object]] = None   # node.koordinator.sh/raw-allocatable
    raw_allocatable_invalid: bool = False                             # that annotation does not unmarshal
    custom_thresholds_invalid: bool = False                           # usage-thresholds does not unmarshal
    custom_usage_thresholds: Optional[Dict[str, int]] = None          # scheduling.koordinator.sh/usage-thresholds
    custom_prod_usage_thresholds: Optional[Dict[str, int]] = None
    custom_aggregated: Optional[dict] = None   # {"usageThresholds": {...}, "usageAggregationType": "p95", "usageAggregatedDuration": seconds}
    # NodeNUMAResource topology options: zones in NodeResourceTopology order
    numa_policy: str = ""                                   # "", "BestEffort", "Restricted", "SingleNUMANode"
    numa_zones: Optional[List[Dict[str, object]]] = None    # NUMANodeResources[i].Resources (None ⇔ no options)
    numa_zone_ids: Optional[List[int]] = None               # NUMANodeResource.Node (default 0..Z-1)
    numa_allocated: Optional[Dict[int, Dict[str, object]]] = None   # allocatedResources by zone id
    cpu_amplification_ratio: float = 0.0
    cpu_topology_valid: bool = True          # CPUTopology.IsValid() of the NodeResourceTopology (nil without zones)
    cpuset_cpus: int = 0                     # CPUs held by cpuset pods (NodeAllocation.allocatedCPUs)
    zone_cpuset_cpus: Optional[Dict[int, int]] = None   # those CPUs by zone id
    # cpuset binding: label node.koordinator.sh/cpu-bind-policy ("", "None", "FullPCPUsOnly", "SpreadByPCPUs"),
    # the reported CPU topology as (socket, NUMA node, core) per cpu id, the node allocation's cpus
    # {cpu: (refcount, exclusive policy)}, TopologyOptions.ReservedCPUs and MaxRefCount; with cpu_detail the
    # counts above are derived from it
    cpu_bind_policy: str = ""
    cpu_detail: Optional[List[tuple]] = None
    cpu_allocated: Optional[Dict[int, tuple]] = None
    reserved_cpus: Sequence[int] = ()
    max_ref_count: int = 1
    numa_allocate_strategy: str = ""         # label node.koordinator.sh/numa-allocate-strategy


NUMA_POLICY = {"": nat.NUMA_NONE, "BestEffort": nat.NUMA_BEST_EFFORT, "Restricted": nat.NUMA_RESTRICTED,
               "SingleNUMANode": nat.NUMA_SINGLE_NUMA_NODE}
CPU_BIND = {"": nat.CPU_BIND_UNSET, "Default": nat.CPU_BIND_DEFAULT, "FullPCPUs": nat.CPU_BIND_FULL_PCPUS,
            "SpreadByPCPUs": nat.CPU_BIND_SPREAD_BY_PCPUS, "ConstrainedBurst": nat.CPU_BIND_CONSTRAINED_BURST}
CPU_EXCLUSIVE = {"": nat.CPU_EXCL_UNSET, "None": nat.CPU_EXCL_NONE, "PCPULevel": nat.CPU_EXCL_PCPU_LEVEL,
                 "NUMANodeLevel": nat.CPU_EXCL_NUMA_NODE_LEVEL}
NUMA_ALLOCATE = {"": nat.NUMA_ALLOC_DEFAULT, "MostAllocated": nat.NUMA_ALLOC_MOST,
                 "LeastAllocated": nat.NUMA_ALLOC_LEAST, "DistributeEvenly": nat.NUMA_ALLOC_DISTRIBUTE_EVENLY}
NODE_CPU_BIND = {"": nat.NODE_CPU_BIND_NONE, "None": nat.NODE_CPU_BIND_NONE,
                 "FullPCPUsOnly": nat.NODE_CPU_BIND_FULL_PCPUS_ONLY, "SpreadByPCPUs": nat.NODE_CPU_BIND_SPREAD_BY_PCPUS}


def numa_spec_record(n: "Node", cpus: Optional[list] = None) -> np.ndarray:
    rec = np.zeros((), dtype=nat.NUMA_SPEC)
    rec["policy"] = NUMA_POLICY[n.numa_policy]
    zones = n.numa_zones or []
    ids = n.numa_zone_ids if n.numa_zone_ids is not None else list(range(len(zones)))
    rec["n_zones"] = len(zones)
    for z, (zid, res) in enumerate(zip(ids, zones)):
        rec["zone_id"][z] = zid
        rec["zone_total"][z] = resource_list(res)
        if n.numa_allocated and zid in n.numa_allocated:
            rec["zone_allocated"][z] = resource_list(n.numa_allocated[zid])
    rec["cpu_amplification_ratio"] = n.cpu_amplification_ratio
    # no NodeResourceTopology (a node with only the amplification annotation): CPUTopology is nil
    rec["cpu_topology_valid"] = -1 if n.numa_zones is None and n.cpu_detail is None else int(n.cpu_topology_valid)
    rec["cpuset_cpus"] = n.cpuset_cpus
    for z, zid in enumerate(ids):
        rec["zone_cpuset_cpus"][z] = (n.zone_cpuset_cpus or {}).get(zid, 0)
    rec["node_cpu_bind_policy"] = NODE_CPU_BIND[n.cpu_bind_policy]
    rec["max_ref_count"] = n.max_ref_count
    rec["numa_allocate_strategy"] = NUMA_ALLOCATE[n.numa_allocate_strategy]
    if n.cpu_detail is not None and cpus is not None:
        alloc = n.cpu_allocated or {}
        rec["first_cpu"], rec["n_cpus"] = len(cpus), len(n.cpu_detail)
        reserved = set(n.reserved_cpus)
        for c, (sk, nd, co) in enumerate(n.cpu_detail):
            ci = np.zeros((), dtype=nat.CPU_INFO)
            ci["socket"], ci["node"], ci["core"] = sk, nd, co
            ref, ex = alloc.get(c, (0, ""))
            ci["refcount"], ci["exclusive"] = ref, CPU_EXCLUSIVE[ex] if ref > 0 else 0
            ci["reserved"] = int(c in reserved)
            cpus.append(ci)
        # the node allocation's counts follow from the detail (allocatedCPUs, CPUsInNUMANodes)
        held = [c for c in alloc if alloc[c][0] > 0]
        rec["cpuset_cpus"] = len(held)
        for z, zid in enumerate(ids):
            rec["zone_cpuset_cpus"][z] = sum(1 for c in held if n.cpu_detail[c][1] == zid)
    return rec


@dataclasses.dataclass
class NodeMetric:
    update_time_s: Optional[float] = None             # Status.UpdateTime as seconds relative to `now` (None ⇒ nil)
    report_interval_s: Optional[int] = None           # Spec.CollectPolicy.ReportIntervalSeconds
    node_usage: Optional[Dict[str, object]] = None    # None ⇒ Status.NodeMetric == nil
    aggregated: List[dict] = dataclasses.field(default_factory=list)  # [{"duration": s, "usage": {"p95": {...}}}]
    pods_metric: List[dict] = dataclasses.field(default_factory=list)  # [{"namespace","name","usage": {...}}]


class Cluster:
    """Holds objects and flattens them into the C arrays of a ``kg_cluster_view``."""

    def __init__(self, now_ns: int = 1_700_000_000 * 10**9):
        self.now_ns = int(now_ns)
        self.nodes: List[Node] = []
        self.node_info: Dict[str, dict] = {}
        self.metrics: Dict[str, NodeMetric] = {}
        self.lister_pods: Dict[str, Pod] = {}
        self.assigned: Dict[str, List[tuple]] = {}
        self._names: Dict[str, int] = {}

    # -- building -------------------------------------------------------------------------
    def add_node(self, node: Node, requested: Optional[Dict[str, object]] = None,
                 nonzero_requested: Optional[Dict[str, object]] = None, pod_count: int = 0) -> "Cluster":
        self.nodes.append(node)
        self.node_info[node.name] = {"requested": requested or {}, "nonzero": nonzero_requested, "pods": pod_count}
        return self

    def add_node_with_pods(self, node: Node, pods: Sequence[Pod]) -> "Cluster":
        """NodeInfo built from pods (framework.NewNodeInfo(pods...))."""
        req: Dict[str, int] = {}
        nz = [0, 0]
        for p in pods:
            row = pod_request(p)
            for k, r in RES.items():
                if row["request"][r] or (r in (0, 1, 2)):
                    req[k] = req.get(k, 0) + int(row["request"][r])
            nz[0] += int(row["nonzero"][0])
            nz[1] += int(row["nonzero"][1])
        self.nodes.append(node)
        self.node_info[node.name] = {"requested_raw": req, "nonzero_raw": nz, "pods": len(pods)}
        return self

    def set_metric(self, node_name: str, m: NodeMetric) -> "Cluster":
        self.metrics[node_name] = m
        return self

    def add_lister_pod(self, pod: Pod) -> "Cluster":
        self.lister_pods[pod.key] = pod
        return self

    def assign(self, node_name: str, pod: Pod, age_s: float) -> "Cluster":
        """podAssignCache entry with timestamp now − age_s."""
        return self.assign_at(node_name, pod, self.now_ns - int(round(age_s * 10**9)))

    def assign_at(self, node_name: str, pod: Pod, timestamp_ns: int) -> "Cluster":
        """podAssignCache entry with an absolute timestamp (pod_assign_cache.go:53-68 timeNowFn())."""
        self.assigned.setdefault(node_name, []).append((pod, int(timestamp_ns)))
        return self

    def name_id(self, key: str) -> int:
        return self._names.setdefault(key, len(self._names) + 1)

    # -- flattening -----------------------------------------------------------------------
    def view(self, extra_pods: Sequence[Pod] = ()) -> "FlatView":
        fv = FlatView(self)
        for p in self.lister_pods.values():
            fv.pod_index(p)
        for p in extra_pods:
            fv.pod_index(p)
        nodes = np.zeros(len(self.nodes), dtype=nat.NODE_SPEC)
        for i, n in enumerate(self.nodes):
            ns = nodes[i]
            ns["allocatable"] = resource_list(n.allocatable)
            info = self.node_info[n.name]
            if "requested_raw" in info:
                rl = np.zeros((), dtype=nat.RESOURCE_LIST)
                for k, v in info["requested_raw"].items():
                    rl["v"][RES[k]] = v
                    rl["present"] |= np.uint32(1 << RES[k])
                ns["requested"] = rl
                ns["nonzero_requested"] = info["nonzero_raw"]
            else:
                ns["requested"] = resource_list(info["requested"])
                nz = info["nonzero"]
                if nz is None:
                    ns["nonzero_requested"] = [ns["requested"]["v"][0], ns["requested"]["v"][1]]
                else:
                    ns["nonzero_requested"] = [quantity_value("cpu", nz.get("cpu", 0)),
                                               quantity_value("memory", nz.get("memory", 0))]
            ns["pod_count"] = info["pods"]
            ns["allowed_pods"] = n.pods
            if n.raw_allocatable_invalid:
                ns["raw_allocatable_state"] = -1
            elif n.annotations_raw_allocatable is not None:
                ns["raw_allocatable_state"] = 1
                ns["raw_allocatable"] = resource_list(n.annotations_raw_allocatable)
            if n.custom_thresholds_invalid:
                ns["custom_thresholds_state"] = -1
            elif (n.custom_usage_thresholds or n.custom_prod_usage_thresholds or n.custom_aggregated) is not None:
                ns["custom_thresholds_state"] = 1
                ns["custom_usage_thresholds"] = _thresholds(n.custom_usage_thresholds)
                ns["custom_prod_usage_thresholds"] = _thresholds(n.custom_prod_usage_thresholds)
                if n.custom_aggregated is not None:
                    ca = n.custom_aggregated
                    ns["custom_has_aggregated"] = 1
                    ns["custom_agg_usage_type"] = AGG[ca.get("usageAggregationType", "")]
                    ns["custom_agg_usage_thresholds"] = _thresholds(ca.get("usageThresholds"))
                    ns["custom_agg_duration_ns"] = int(ca.get("usageAggregatedDuration", 0) * 10**9)
            m = self.metrics.get(n.name)
            if m is not None:
                ns["has_node_metric"] = 1
                if m.update_time_s is not None:
                    ns["has_update_time"] = 1
                    ns["update_time_ns"] = self.now_ns + int(round(m.update_time_s * 10**9))
                if m.report_interval_s is not None:
                    ns["has_report_interval"] = 1
                    ns["report_interval_seconds"] = m.report_interval_s
                if m.node_usage is not None:
                    ns["has_node_metric_info"] = 1
                    ns["node_usage"] = resource_list(m.node_usage)
                ns["first_aggregated"] = len(fv.aggregated)
                for a in m.aggregated:
                    rec = np.zeros((), dtype=nat.AGGREGATED_USAGE)
                    rec["duration_ns"] = int(a["duration"] * 10**9)
                    for t, u in a["usage"].items():
                        rec["usage"][AGG[t]] = resource_list(u)
                    fv.aggregated.append(rec)
                ns["n_aggregated"] = len(m.aggregated)
                ns["first_pod_metric"] = len(fv.pod_metrics)
                for pm in m.pods_metric:
                    rec = np.zeros((), dtype=nat.POD_METRIC)
                    key = f"{pm.get('namespace', 'default')}/{pm['name']}"
                    rec["name_id"] = self.name_id(key)
                    lp = self.lister_pods.get(key)
                    rec["lister_pod"] = fv.pod_index(lp) if lp is not None else -1
                    rec["usage"] = resource_list(pm["usage"])
                    fv.pod_metrics.append(rec)
                ns["n_pod_metric"] = len(m.pods_metric)
            ns["first_assigned"] = len(fv.assigned)
            for pod, ts in self.assigned.get(n.name, []):
                rec = np.zeros((), dtype=nat.ASSIGNED_POD)
                rec["pod"] = fv.pod_index(pod)
                rec["timestamp_ns"] = ts
                fv.assigned.append(rec)
            ns["n_assigned"] = len(self.assigned.get(n.name, []))
            ns["numa"] = -1
            if (n.numa_zones is not None or n.cpu_amplification_ratio > 1 or n.cpu_detail is not None
                    or NODE_CPU_BIND[n.cpu_bind_policy] != nat.NODE_CPU_BIND_NONE):
                ns["numa"] = len(fv.numa)
                fv.numa.append(numa_spec_record(n, fv.cpus))
        fv.nodes = nodes
        return fv.finish()


def _thresholds(d: Optional[Dict[str, int]]) -> np.ndarray:
    out = np.zeros((), dtype=nat.RESOURCE_LIST)
    for k, v in (d or {}).items():
        out["v"][RES[k]] = int(v)
        out["present"] |= np.uint32(1 << RES[k])
    return out


def pod_spec_record(p: Pod, containers: list, name_id: int) -> np.ndarray:
    rec = np.zeros((), dtype=nat.POD_SPEC)
    rec["first_container"] = len(containers)
    for c in p.containers:
        containers.append((resource_list(c.requests), resource_list(c.limits)))
    rec["n_containers"] = len(p.containers)
    rec["first_init_container"] = len(containers)
    for c in p.init_containers:
        containers.append((resource_list(c.requests), resource_list(c.limits)))
    rec["n_init_containers"] = len(p.init_containers)
    if p.overhead is not None:
        rec["overhead"] = resource_list(p.overhead)
    if p.priority is not None:
        rec["has_priority"] = 1
        rec["priority"] = p.priority
    pc = p.labels.get("koordinator.sh/priority-class")
    rec["label_priority_class"] = -1 if pc is None else PRIORITY_CLASS.get(pc, nat.PRIO_NONE)
    q = p.labels.get("koordinator.sh/qosClass")
    rec["label_qos"] = -1 if q is None else QOS_CLASS.get(q, nat.QOS_NONE)
    rec["status_qos"] = KUBE_QOS[p.qos_status]
    rec["is_daemonset"] = int(p.daemonset)
    rec["is_terminated"] = int(p.terminated)
    rec["cpu_bind_required"] = CPU_BIND.get(p.cpu_bind_required, nat.CPU_BIND_OTHER)
    rec["cpu_bind_preferred"] = CPU_BIND.get(p.cpu_bind_preferred, nat.CPU_BIND_OTHER)
    rec["cpu_exclusive"] = CPU_EXCLUSIVE[p.cpu_exclusive]
    rec["name_id"] = name_id
    rec["rsv_owner_class"] = getattr(p, "rsv_owner_class", -1)
    rec["rsv_affinity_class"] = getattr(p, "rsv_affinity_class", -1)
    rec["quota"] = getattr(p, "quota", -1)
    rec["non_preemptible"] = int(getattr(p, "non_preemptible", False))
    return rec


def pod_request(p: Pod) -> dict:
    """Fit request / nonzero request of a pod (for NodeInfo built from pods)."""
    req = np.zeros(nat.NUM_RES, dtype=np.int64)
    for c in p.containers:
        rl = resource_list(c.requests)
        for r in range(nat.NUM_RES):
            if rl["present"] >> r & 1:
                req[r] += rl["v"][r]
    nz = [0, 0]
    for c in p.containers:
        rl = resource_list(c.requests)
        nz[0] += int(rl["v"][0]) if rl["present"] & 1 else 100
        nz[1] += int(rl["v"][1]) if rl["present"] & 2 else 200 * 1024 * 1024
    return {"request": req, "nonzero": nz}


class FlatView:
    """Owns the numpy arrays behind one ``kg_cluster_view``."""

    def __init__(self, cluster: Cluster):
        self.cluster = cluster
        self._pods: List[np.ndarray] = []
        self._containers: list = []
        self._index: Dict[int, int] = {}
        self.aggregated: List[np.ndarray] = []
        self.pod_metrics: List[np.ndarray] = []
        self.assigned: List[np.ndarray] = []
        self.numa: List[np.ndarray] = []
        self.cpus: List[np.ndarray] = []
        self.nodes = None

    def pod_index(self, p: Pod) -> int:
        k = id(p)
        if k not in self._index:
            self._index[k] = len(self._pods)
            self._pods.append(pod_spec_record(p, self._containers, self.cluster.name_id(p.key)))
        return self._index[k]

    def finish(self) -> "FlatView":
        self.pods = _stack(self._pods, nat.POD_SPEC)
        cont = np.zeros(len(self._containers), dtype=nat.CONTAINER)
        for i, (rq, lm) in enumerate(self._containers):
            cont[i]["requests"] = rq
            cont[i]["limits"] = lm
        self.containers = cont
        self.aggregated_arr = _stack(self.aggregated, nat.AGGREGATED_USAGE)
        self.pod_metrics_arr = _stack(self.pod_metrics, nat.POD_METRIC)
        self.assigned_arr = _stack(self.assigned, nat.ASSIGNED_POD)
        self.numa_arr = _stack(self.numa, nat.NUMA_SPEC)
        self.cpu_arr = _stack(self.cpus, nat.CPU_INFO)
        self.c_view = nat.make_view(self.pods, self.containers, self.nodes, self.aggregated_arr, self.pod_metrics_arr,
                                    self.assigned_arr, self.numa_arr, cpus=self.cpu_arr)
        return self

    def add_pods(self, pods: Sequence[Pod]) -> List[int]:
        """Append pending pods after finish(); returns their indices."""
        idx = [self.pod_index(p) for p in pods]
        return self.refresh(idx)

    def refresh(self, idx):
        self.finish()
        return idx


def _stack(recs: List[np.ndarray], dtype) -> np.ndarray:
    out = np.zeros(len(recs), dtype=dtype)
    for i, r in enumerate(recs):
        out[i] = r
    return out
