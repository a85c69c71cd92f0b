"""Snapshot ingest from the Kubernetes / Koordinator objects the scheduler's informers hold (SURVEY §8
row f4): corev1.Node (with the informer transform koord-scheduler installs), corev1.Pod,
slo/v1alpha1.NodeMetric and topology/v1alpha1.NodeResourceTopology, given as their JSON objects (dicts as
``json.load`` / ``yaml.safe_load`` return them), turned into the ``objects`` model that flattens into the
C-ABI records.  The Go shim does the same from the typed objects; this module is the
reference for what each field means.

Restated from:
* ``TransformNode`` (pkg/util/transformer/node_transformer.go:40-75): the node-reservation trim
  (``TrimNodeAllocatableByNodeReservation``, pkg/util/node.go:88-146) and the deprecated batch / device
  resource names (apis/extension/deprecated.go:48-60, ``replaceAndEraseResource`` pod_transformer.go:112-139);
* ``TransformPod`` (pod_transformer.go:28-110): the same resource-name mapping on containers and overhead;
* NodeMetric (apis/slo/v1alpha1/nodemetric_types.go:38-136, ``ResourceMap`` resources.go:25-28);
* ``NewTopologyOptions`` (nodenumaresource/topology_options.go:90-211): NUMA zones from the NRT's
  ``Node`` zones (``node-<id>``, sorted by id), the topology-manager policy (``convertToNUMATopologyPolicy``,
  overridden by the node label, util.go:52-58), the reported CPU topology's validity
  (cpu_topology.go:77-79) and the amplification ratios (node_resource_amplification.go:45-57);
* the Fit request of a pod as NodeInfo accounts it (``calculateResource``, mirrored in
  reservation/transformer.go:316-346): Σ containers, max with each init container, + overhead; the
  NonZero cpu / memory defaults 100m / 200Mi per container.

Resources outside the engine's fixed set (``objects.RES``) are dropped from nodes (no plugin on the path
reads a resource a pod does not request); a pod that requests one raises ``UnsupportedResource`` so the
caller falls back to the reference plugins for it (SURVEY §5's error → CPU-fallback contract).
"""
from __future__ import annotations

import copy
import datetime as _dt
import json
import math
import re
from fractions import Fraction
from typing import Dict, Iterable, List, Optional, Tuple

from . import objects as ob
from .objects import parse_quantity

NODE_RESERVATION = "node.koordinator.sh/reservation"
RAW_ALLOCATABLE = "node.koordinator.sh/raw-allocatable"
AMPLIFICATION_RATIO = "node.koordinator.sh/resource-amplification-ratio"
USAGE_THRESHOLDS = "scheduling.koordinator.sh/usage-thresholds"
NUMA_POLICY_LABEL = "node.koordinator.sh/numa-topology-policy"
CPU_TOPOLOGY = "node.koordinator.sh/cpu-topology"
NODE_CPU_BIND_LABEL = "node.koordinator.sh/cpu-bind-policy"
NUMA_ALLOCATE_STRATEGY_LABEL = "node.koordinator.sh/numa-allocate-strategy"   # numa_aware.go:52-53
KUBELET_CPU_MANAGER_POLICY = "kubelet.koordinator.sh/cpu-manager-policy"
POD_CPU_ALLOCS = "node.koordinator.sh/pod-cpu-allocs"
SYSTEM_QOS_RESOURCE = "node.koordinator.sh/system-qos-resource"
RESOURCE_SPEC = "scheduling.koordinator.sh/resource-spec"
RESOURCE_STATUS = "scheduling.koordinator.sh/resource-status"
CPU_BIND_POLICIES = ("", "Default", "FullPCPUs", "SpreadByPCPUs", "ConstrainedBurst")
CPU_EXCLUSIVE_POLICIES = ("", "None", "PCPULevel", "NUMANodeLevel")

BATCH_CPU, BATCH_MEMORY = "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory"
# apis/extension/deprecated.go:48-60 (deprecated name → current name)
DEPRECATED_BATCH = {"koordinator.sh/batch-cpu": BATCH_CPU, "koordinator.sh/batch-memory": BATCH_MEMORY}
DEPRECATED_DEVICE = {
    "kubernetes.io/rdma": "koordinator.sh/rdma", "kubernetes.io/fpga": "koordinator.sh/fpga",
    "kubernetes.io/gpu": "koordinator.sh/gpu", "kubernetes.io/gpu-core": "koordinator.sh/gpu-core",
    "kubernetes.io/gpu-memory": "koordinator.sh/gpu-memory",
    "kubernetes.io/gpu-memory-ratio": "koordinator.sh/gpu-memory-ratio",
}
# nrtv1alpha1 topology-manager policies → NUMATopologyPolicy (topology_options.go:213-226)
NRT_POLICY = {"BestEffort": "BestEffort", "Restricted": "Restricted", "SingleNUMANodePodLevel": "SingleNUMANode"}

NONZERO_CPU_MILLI = 100
NONZERO_MEMORY = 200 * 1024 * 1024


class UnsupportedResource(ValueError):
    """A pod requests a resource the engine does not model: evaluate it with the reference plugins."""


Resources = Dict[str, Fraction]


def resources(d: Optional[dict]) -> Resources:
    return {k: parse_quantity(v) for k, v in (d or {}).items()}


def _milli_to_unit(q: Fraction) -> Fraction:
    # replaceAndEraseResource: a cpu quantity moved to another name keeps its MilliValue (ceil) as Value
    return Fraction(math.ceil(q * 1000))


def replace_and_erase(rl: Resources, mapping: Dict[str, str]) -> bool:
    """replaceAndEraseResource over a mapper (pod_transformer.go:112-139)."""
    done = False
    for src, dst in mapping.items():
        if not dst or dst in rl or src not in rl:
            continue
        q = rl.pop(src)
        rl[dst] = _milli_to_unit(q) if src == "cpu" else q
        done = True
    return done


def parse_cpuset(s: str) -> List[int]:
    """cpuset.Parse (pkg/util/cpuset): "0-3,8,10-11" → [0, 1, 2, 3, 8, 10, 11]."""
    out = set()
    for part in filter(None, (p.strip() for p in (s or "").split(","))):
        if "-" in part:
            a, b = (int(x) for x in part.split("-", 1))
            if b < a:
                raise ValueError(f"bad cpuset {s!r}")
            out.update(range(a, b + 1))
        else:
            out.add(int(part))
    return sorted(out)


def cpuset_size(s: str) -> int:
    """cpuset.Parse(s).Size()."""
    return len(parse_cpuset(s))


def node_reservation(annotations: dict) -> Optional[dict]:
    s = (annotations or {}).get(NODE_RESERVATION, "")
    if not s:
        return None
    return json.loads(s)


def reservation_resources(rsv: dict) -> Resources:
    """GetNodeReservationResources (node.go:104-119): reservedCPUs overrides the cpu quantity."""
    rl = resources(rsv.get("resources"))
    if rsv.get("reservedCPUs"):
        rl["cpu"] = Fraction(cpuset_size(rsv["reservedCPUs"]))
    return rl


def trim_allocatable_by_node_reservation(node: dict) -> Tuple[Resources, bool]:
    """TrimNodeAllocatableByNodeReservation (node.go:121-146)."""
    alloc = resources(node.get("status", {}).get("allocatable"))
    try:
        rsv = node_reservation(node.get("metadata", {}).get("annotations"))
    except (ValueError, TypeError):
        return alloc, False
    if rsv is None or rsv.get("applyPolicy", "") not in ("", "Default"):
        return alloc, False
    try:
        reserved = reservation_resources(rsv)
    except ValueError:
        return alloc, False
    if all(v == 0 for v in reserved.values()):
        return alloc, False
    # quotav1.SubtractWithNonNegativeResult: keys of both lists, floored at zero
    trimmed = {k: max(v - reserved.get(k, 0), Fraction(0)) for k, v in alloc.items()}
    for k in reserved:
        trimmed.setdefault(k, Fraction(0))
    # koord-manager already subtracted the reservation from the batch resources
    trimmed[BATCH_MEMORY] = alloc.get(BATCH_MEMORY, Fraction(0))
    trimmed[BATCH_CPU] = alloc.get(BATCH_CPU, Fraction(0))
    return trimmed, trimmed != alloc


def _dump(rl: Resources) -> dict:
    return {k: str(v) if v.denominator == 1 else f"{int(v * 1000)}m" for k, v in rl.items()}


def transform_node(node: dict) -> dict:
    """TransformNode (node_transformer.go:40-75) on a copy of the object."""
    node = copy.deepcopy(node)
    status = node.setdefault("status", {})
    trimmed, _ = trim_allocatable_by_node_reservation(node)
    alloc = trimmed
    cap = resources(status.get("capacity"))
    for rl in (alloc, cap):
        replace_and_erase(rl, DEPRECATED_BATCH)
        replace_and_erase(rl, DEPRECATED_DEVICE)
    status["allocatable"] = _dump(alloc)
    if "capacity" in status:
        status["capacity"] = _dump(cap)
    return node


def transform_pod(pod: dict) -> dict:
    """TransformPod's resource-name mapping (pod_transformer.go:62-110) on a copy of the object."""
    pod = copy.deepcopy(pod)
    spec = pod.setdefault("spec", {})
    for key in ("initContainers", "containers"):
        for c in spec.get(key) or []:
            r = c.setdefault("resources", {})
            for part in ("requests", "limits"):
                if part in r:
                    rl = resources(r[part])
                    replace_and_erase(rl, DEPRECATED_BATCH)
                    replace_and_erase(rl, DEPRECATED_DEVICE)
                    r[part] = _dump(rl)
    if spec.get("overhead") is not None:
        rl = resources(spec["overhead"])
        replace_and_erase(rl, DEPRECATED_BATCH)
        replace_and_erase(rl, DEPRECATED_DEVICE)
        spec["overhead"] = _dump(rl)
    return pod


# ---- pods ------------------------------------------------------------------------------------

def _engine_resources(rl: Resources, what: str) -> Dict[str, Fraction]:
    out = {}
    for k, v in rl.items():
        if k in ob.RES:
            out[k] = v
        elif v != 0:
            raise UnsupportedResource(f"{what} requests {k!r}, which the engine does not model")
    return out


def pod_from_object(pod: dict) -> ob.Pod:
    """corev1.Pod (after TransformPod) → objects.Pod."""
    pod = transform_pod(pod)
    meta, spec, status = pod.get("metadata", {}), pod.get("spec", {}), pod.get("status", {})
    name = f"{meta.get('namespace', 'default')}/{meta.get('name', '')}"

    def containers(key):
        out = []
        for c in spec.get(key) or []:
            r = c.get("resources", {})
            out.append(ob.Container(requests=_engine_resources(resources(r.get("requests")), name),
                                    limits={k: v for k, v in resources(r.get("limits")).items() if k in ob.RES}))
        return out

    owners = meta.get("ownerReferences") or []
    spec_ann = resource_spec((meta.get("annotations") or {}))
    return ob.Pod(
        namespace=meta.get("namespace", "default"), name=meta.get("name", ""),
        containers=containers("containers"), init_containers=containers("initContainers"),
        overhead=_engine_resources(resources(spec["overhead"]), name) if spec.get("overhead") else None,
        priority=spec.get("priority"), labels=dict(meta.get("labels") or {}),
        qos_status=status.get("qosClass", ""),
        cpu_bind_required=spec_ann["requiredCPUBindPolicy"], cpu_bind_preferred=spec_ann["preferredCPUBindPolicy"],
        cpu_exclusive=spec_ann["preferredCPUExclusivePolicy"],
        daemonset=any(o.get("kind") == "DaemonSet" and o.get("controller", False) for o in owners),
        terminated=status.get("phase") in ("Succeeded", "Failed"),
        node_name=spec.get("nodeName", ""))


def resource_spec(annotations: dict) -> dict:
    """GetResourceSpec (numa_aware.go:190-205); a policy the engine does not know binds no cpuset, as a
    non-empty ConstrainedBurst does."""
    d = {}
    s = annotations.get(RESOURCE_SPEC)
    if s:
        d = json.loads(s)
    out = {}
    for k in ("requiredCPUBindPolicy", "preferredCPUBindPolicy"):
        v = d.get(k, "")
        out[k] = v if v in CPU_BIND_POLICIES else "ConstrainedBurst"
    v = d.get("preferredCPUExclusivePolicy", "")
    out["preferredCPUExclusivePolicy"] = v if v in CPU_EXCLUSIVE_POLICIES else "None"
    return out


def pod_fit_request(p: ob.Pod) -> Tuple[Dict[str, Fraction], Tuple[int, int]]:
    """The pod's contribution to NodeInfo.Requested / NonZeroRequested (calculateResource)."""
    req: Dict[str, Fraction] = {}
    nz = [0, 0]
    for c in p.containers:
        rq = resources(c.requests)
        for k, v in rq.items():
            req[k] = req.get(k, Fraction(0)) + v
        nz[0] += ob.quantity_value("cpu", rq["cpu"]) if "cpu" in rq else NONZERO_CPU_MILLI
        nz[1] += ob.quantity_value("memory", rq["memory"]) if "memory" in rq else NONZERO_MEMORY
    for c in p.init_containers:
        rq = resources(c.requests)
        for k, v in rq.items():
            req[k] = max(req.get(k, Fraction(0)), v)
        nz[0] = max(nz[0], ob.quantity_value("cpu", rq["cpu"]) if "cpu" in rq else NONZERO_CPU_MILLI)
        nz[1] = max(nz[1], ob.quantity_value("memory", rq["memory"]) if "memory" in rq else NONZERO_MEMORY)
    if p.overhead:
        oh = resources(p.overhead)
        for k, v in oh.items():
            req[k] = req.get(k, Fraction(0)) + v
        nz[0] += ob.quantity_value("cpu", oh["cpu"]) if "cpu" in oh else 0
        nz[1] += ob.quantity_value("memory", oh["memory"]) if "memory" in oh else 0
    return req, (nz[0], nz[1])


# ---- NodeMetric ------------------------------------------------------------------------------

_DUR = re.compile(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)")
_DUR_S = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_duration(s) -> float:
    """metav1.Duration JSON (Go time.ParseDuration) → seconds."""
    if isinstance(s, (int, float)):
        return float(s)
    s = str(s).strip()
    if s in ("0", ""):
        return 0.0
    pos, total = 0, 0.0
    for m in _DUR.finditer(s):
        if m.start() != pos:
            raise ValueError(f"bad duration {s!r}")
        total += float(m.group(1)) * _DUR_S[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"bad duration {s!r}")
    return total


def parse_time_ns(s: str) -> int:
    """metav1.Time JSON (RFC 3339, whole seconds) → Unix ns."""
    t = _dt.datetime.fromisoformat(s.replace("Z", "+00:00"))
    if t.tzinfo is None:
        t = t.replace(tzinfo=_dt.timezone.utc)
    d = t - _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)
    return (d.days * 86400 + d.seconds) * 10**9 + d.microseconds * 1000


def _resource_map(rm: Optional[dict]) -> Dict[str, Fraction]:
    # ResourceMap{ResourceList `json:"resources"`, Devices}: only the resources the engine models
    return {k: v for k, v in resources((rm or {}).get("resources")).items() if k in ob.RES}


def node_metric_from_object(nm: dict, now_ns: int) -> ob.NodeMetric:
    """slov1alpha1.NodeMetric → objects.NodeMetric (times relative to ``now_ns``)."""
    spec, status = nm.get("spec") or {}, nm.get("status") or {}
    policy = spec.get("metricCollectPolicy") or {}
    out = ob.NodeMetric()
    if status.get("updateTime"):
        out.update_time_s = (parse_time_ns(status["updateTime"]) - now_ns) / 1e9
    if policy.get("reportIntervalSeconds") is not None:
        out.report_interval_s = int(policy["reportIntervalSeconds"])
    info = status.get("nodeMetric")
    if info is not None:
        out.node_usage = _resource_map(info.get("nodeUsage"))
        for agg in info.get("aggregatedNodeUsages") or []:
            out.aggregated.append({"duration": parse_duration(agg.get("duration", 0)),
                                   "usage": {t: _resource_map(u) for t, u in (agg.get("usage") or {}).items()
                                             if t in ob.AGG}})
    for pm in status.get("podsMetric") or []:
        out.pods_metric.append({"namespace": pm.get("namespace", "default"), "name": pm.get("name", ""),
                                "usage": _resource_map(pm.get("podUsage"))})
    return out


# ---- NodeResourceTopology --------------------------------------------------------------------

def numa_zones_from_nrt(nrt: dict) -> List[Tuple[int, Dict[str, Fraction]]]:
    """extractNUMANodeResources (topology_options.go:181-211): zones of type Node named node-<id>."""
    zones = []
    for z in nrt.get("zones") or []:
        if z.get("type") != "Node":
            continue
        parts = str(z.get("name", "")).split("node-")
        if len(parts) != 2:
            continue
        try:
            zid = int(parts[1])
        except ValueError:
            continue
        zones.append((zid, {r["name"]: parse_quantity(r.get("allocatable", 0)) for r in z.get("resources") or []}))
    zones.sort(key=lambda x: x[0])
    return zones


def nrt_policy(nrt: Optional[dict]) -> str:
    for p in (nrt or {}).get("topologyPolicies") or []:
        if p in NRT_POLICY:
            return NRT_POLICY[p]
    return ""


def cpu_topology_valid(nrt: dict) -> bool:
    """CPUTopology.IsValid() of the reported topology: every count non-zero ⇔ at least one CPU."""
    s = (nrt.get("metadata", {}).get("annotations") or {}).get(CPU_TOPOLOGY, "")
    if not s:
        return False
    try:
        detail = json.loads(s).get("detail") or []
    except (ValueError, AttributeError):
        return False
    return len(detail) > 0


def cpu_detail_from_nrt(nrt: dict) -> Optional[List[Tuple[int, int, int]]]:
    """convertCPUTopology (topology_options.go:173-179): (socket, NUMA node, core) per cpu id; the engine
    indexes CPUs by id, so the reported ids must be 0..n-1."""
    s = (nrt.get("metadata", {}).get("annotations") or {}).get(CPU_TOPOLOGY, "")
    if not s:
        return None
    detail = sorted(json.loads(s).get("detail") or [], key=lambda d: d["id"])
    if [d["id"] for d in detail] != list(range(len(detail))):
        raise UnsupportedResource("CPU ids of the reported topology are not 0..n-1")
    return [(int(d["socket"]), int(d["node"]), int(d["core"])) for d in detail]


def kubelet_cpu_policy(nrt: Optional[dict]) -> Optional[dict]:
    s = ((nrt or {}).get("metadata", {}).get("annotations") or {}).get(KUBELET_CPU_MANAGER_POLICY)
    return json.loads(s) if s else None


def system_qos_cpus(annotations: dict) -> List[int]:
    """The exclusive system-QoS cpuset of GetSystemQOSResource (apis/extension/system_qos.go:35-55): the
    cpuset of node.koordinator.sh/system-qos-resource when cpusetExclusive is absent or true; nothing for
    a missing annotation, unparsable JSON or an unparsable cpuset (the reference logs and skips those,
    topology_options.go:124-134)."""
    s = (annotations or {}).get(SYSTEM_QOS_RESOURCE)
    if s is None:
        return []
    try:
        res = json.loads(s)
    except ValueError:
        return []
    if not isinstance(res, dict) or res.get("cpusetExclusive", True) is False:
        return []
    try:
        return parse_cpuset(res.get("cpuset") or "")
    except ValueError:
        return []


def reserved_cpus_from_nrt(nrt: dict) -> List[int]:
    """TopologyOptions.ReservedCPUs (topology_options.go:119-134): kubelet-managed pod cpusets, the kubelet
    reserved CPUs, the node reservation's reservedCPUs and the exclusive system-QoS cpuset."""
    ann = nrt.get("metadata", {}).get("annotations") or {}
    out = set()
    for a in json.loads(ann.get(POD_CPU_ALLOCS, "[]") or "[]"):
        if a.get("managedByKubelet") and a.get("uid") and a.get("cpuset"):
            out.update(parse_cpuset(a["cpuset"]))
    pol = kubelet_cpu_policy(nrt)
    if pol and pol.get("reservedCPUs"):
        out.update(parse_cpuset(pol["reservedCPUs"]))
    rsv = node_reservation(ann)
    if rsv and rsv.get("reservedCPUs"):
        out.update(parse_cpuset(rsv["reservedCPUs"]))
    out.update(system_qos_cpus(ann))
    return sorted(out)


def node_cpu_bind_policy(labels: dict, nrt: Optional[dict]) -> str:
    """GetNodeCPUBindPolicy (numa_aware.go:314-325)."""
    v = labels.get(NODE_CPU_BIND_LABEL, "")
    pol = kubelet_cpu_policy(nrt)
    if v == "FullPCPUsOnly" or (pol and pol.get("policy") == "static" and
                                (pol.get("options") or {}).get("full-pcpus-only") == "true"):
        return "FullPCPUsOnly"
    return "SpreadByPCPUs" if v == "SpreadByPCPUs" else "None"


def amplification_ratios(annotations: Optional[dict]) -> Optional[Dict[str, float]]:
    s = (annotations or {}).get(AMPLIFICATION_RATIO)
    if s is None:
        return None
    return {k: float(v) for k, v in json.loads(s).items()}


# ---- nodes -----------------------------------------------------------------------------------

def node_from_object(node: dict, nrt: Optional[dict] = None) -> ob.Node:
    """corev1.Node (through TransformNode) + its NodeResourceTopology → objects.Node."""
    node = transform_node(node)
    meta = node.get("metadata", {})
    ann, labels = meta.get("annotations") or {}, meta.get("labels") or {}
    alloc = resources(node["status"].get("allocatable"))
    pods = int(alloc.pop("pods", 0))
    n = ob.Node(meta.get("name", ""), allocatable={k: v for k, v in alloc.items() if k in ob.RES}, pods=pods)
    if RAW_ALLOCATABLE in ann:
        try:
            n.annotations_raw_allocatable = {k: v for k, v in resources(json.loads(ann[RAW_ALLOCATABLE])).items()
                                             if k in ob.RES}
        except (ValueError, TypeError):
            n.raw_allocatable_invalid = True
    if USAGE_THRESHOLDS in ann:
        try:
            t = json.loads(ann[USAGE_THRESHOLDS])
            n.custom_usage_thresholds = {k: int(v) for k, v in (t.get("usageThresholds") or {}).items() if k in ob.RES}
            n.custom_prod_usage_thresholds = {k: int(v) for k, v in (t.get("prodUsageThresholds") or {}).items()
                                              if k in ob.RES}
            agg = t.get("aggregatedUsage")
            if agg is not None:
                n.custom_aggregated = {
                    "usageThresholds": {k: int(v) for k, v in (agg.get("usageThresholds") or {}).items() if k in ob.RES},
                    "usageAggregationType": agg.get("usageAggregationType", ""),
                    "usageAggregatedDuration": parse_duration(agg.get("usageAggregatedDuration") or 0)}
        except (ValueError, TypeError, AttributeError):
            n.custom_thresholds_invalid = True
    ratios = amplification_ratios(ann) or {}
    n.cpu_amplification_ratio = float(ratios.get("cpu", 0.0))
    label_policy = labels.get(NUMA_POLICY_LABEL, "")
    if nrt is not None:
        zones = numa_zones_from_nrt(nrt)
        n.numa_zones = [{k: v for k, v in res.items() if k in ob.RES} for _, res in zones]
        n.numa_zone_ids = [zid for zid, _ in zones]
        n.numa_policy = label_policy or nrt_policy(nrt)
        n.cpu_topology_valid = cpu_topology_valid(nrt)
        if n.cpu_topology_valid:
            n.cpu_detail = cpu_detail_from_nrt(nrt)
            n.cpu_allocated = {}
            n.reserved_cpus = reserved_cpus_from_nrt(nrt)
        if not ratios:
            nrt_ratios = amplification_ratios(nrt.get("metadata", {}).get("annotations")) or {}
            n.cpu_amplification_ratio = float(nrt_ratios.get("cpu", 0.0))
    elif label_policy:
        n.numa_policy = label_policy
    n.cpu_bind_policy = node_cpu_bind_policy(labels, nrt)
    # GetNUMAAllocateStrategy (util.go:35-41): any non-empty label value replaces the plugin default; the CPU
    # accumulator only tells NUMAMostAllocated from the rest
    v = labels.get(NUMA_ALLOCATE_STRATEGY_LABEL, "")
    n.numa_allocate_strategy = v if v in ob.NUMA_ALLOCATE else ("LeastAllocated" if v else "")
    return n


def cluster_from_objects(nodes: Iterable[dict], pods: Iterable[dict] = (), node_metrics: Iterable[dict] = (),
                         nrts: Iterable[dict] = (), now_ns: int = 1_700_000_000 * 10**9,
                         assign_cache: Optional[Dict[str, Dict[str, int]]] = None) -> ob.Cluster:
    """A scheduler snapshot: nodes with the NodeInfo of their bound, non-terminated pods, NodeMetrics and
    NodeResourceTopologies by node name; every pod also goes to the pod lister (PodsMetric lookups).
    assign_cache: LoadAware's podAssignCache, node name → pod UID → assign timestamp (ns) of pods among
    `pods` (feeders.SnapshotFeeder keeps it event by event); None leaves it empty."""
    by_nrt = {n.get("metadata", {}).get("name"): n for n in nrts}
    cl = ob.Cluster(now_ns)
    bound: Dict[str, List[ob.Pod]] = {}
    status_of: Dict[int, dict] = {}
    by_uid: Dict[str, ob.Pod] = {}
    for pj in pods:
        p = pod_from_object(pj)
        by_uid[(pj.get("metadata") or {}).get("uid", "")] = p
        cl.add_lister_pod(p)
        if p.node_name and not p.terminated:
            bound.setdefault(p.node_name, []).append(p)
            s = (pj.get("metadata", {}).get("annotations") or {}).get(RESOURCE_STATUS)
            if s:
                status_of[id(p)] = json.loads(s)
    for nj in nodes:
        n = node_from_object(nj, by_nrt.get(nj.get("metadata", {}).get("name")))
        req: Dict[str, Fraction] = {}
        nz = [0, 0]
        for p in bound.get(n.name, []):
            r, z = pod_fit_request(p)
            for k, v in r.items():
                req[k] = req.get(k, Fraction(0)) + v
            nz[0] += z[0]
            nz[1] += z[1]
        # the plugin's NodeAllocation from the bound pods' resource status (pod_eventhandler.go:93-136;
        # resourceManager.Update records nothing on an invalid topology)
        if n.cpu_topology_valid and n.numa_zones is not None:
            for p in bound.get(n.name, []):
                st = status_of.get(id(p))
                if not st:
                    continue
                for c in parse_cpuset(st.get("cpuset", "")):
                    ref, _ = (n.cpu_allocated or {}).get(c, (0, ""))
                    if n.cpu_allocated is not None:
                        n.cpu_allocated[c] = (ref + 1, p.cpu_exclusive or "None")
                for zr in st.get("numaNodeResources") or []:
                    zid = int(zr["node"])
                    acc = (n.numa_allocated or {}).get(zid, {})
                    for k, v in resources(zr.get("resources")).items():
                        if k in ob.RES:
                            acc[k] = acc.get(k, Fraction(0)) + v
                    n.numa_allocated = dict(n.numa_allocated or {}, **{zid: acc})
        cl.add_node(n, requested={k: v for k, v in req.items() if k in ob.RES},
                    nonzero_requested={"cpu": f"{nz[0]}m", "memory": str(nz[1])}, pod_count=len(bound.get(n.name, [])))
    for m in node_metrics:
        cl.set_metric(m.get("metadata", {}).get("name"), node_metric_from_object(m, now_ns))
    for node_name, items in (assign_cache or {}).items():
        for uid, ts in sorted(items.items(), key=lambda kv: kv[1]):
            cl.assign_at(node_name, by_uid[uid], ts)
    return cl
