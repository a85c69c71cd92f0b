"""Seeded synthetic clusters for the BASELINE.json configs, built straight into
the ``kg_cluster_view`` arrays with numpy (100k–1M nodes in well under a second per 100k).

Config 1/2 distributions:
  nodes  cpu ∈ {32,48,64,96,128} cores, memory ∈ {64,128,256,512} GiB, 110 pods;
         batch-cpu / batch-memory allocatable 20–60 % of cpu / memory (colocation nodes);
         Requested uniform 0–70 % of each allocatable; NonZeroRequested = Requested;
         NodeMetric usage 0–80 % cpu, 0–90 % memory, UpdateTime = now − 30 s;
         5 % of nodes without a NodeMetric, 2 % expired (UpdateTime = now − 400 s).
  pods   cpu ∈ {250,500,1000,2000,4000} m, memory ∈ {256Mi … 16Gi};
         50 % limit = request (Guaranteed → LSR → prod), 30 % limit = 2 × request
         (Burstable → LS → prod), 20 % BestEffort batch pods requesting only
         batch-cpu / batch-memory.
Every quantity is an exact integer in its base unit (cpu in milli).

Node-side LoadAware inputs beyond the base distributions (``decorate``, on by default) so that every
branch of the node terms is exercised at scale: a fraction of the nodes carry already-assigned pods
(podAssignCache entries assigned long before, inside the report interval before, or after the
NodeMetric UpdateTime), PodsMetric entries (for most of those pods, plus NotFound and duplicated
ones), AggregatedNodeUsages (one or two durations, some percentile types missing), best-effort pods
that make NonZeroRequested exceed Requested, custom usage-threshold annotations (valid and
unparsable) and raw-allocatable annotations (EstimateNode ≠ Allocatable).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _native as nat

NOW_NS = 1_700_000_000 * 10**9
GI = 1 << 30
MI = 1 << 20


class SynthView:
    """Same attribute surface as objects.FlatView (pods, containers, nodes, c_view …)."""

    def __init__(self, pods, containers, nodes, now_ns, numa=None, reservations=None, quotas=None, aggregated=None,
                 pod_metrics=None, assigned=None):
        self.pods = pods
        self.containers = containers
        self.nodes = nodes
        self.aggregated_arr = np.zeros(0, dtype=nat.AGGREGATED_USAGE) if aggregated is None else aggregated
        self.pod_metrics_arr = np.zeros(0, dtype=nat.POD_METRIC) if pod_metrics is None else pod_metrics
        self.assigned_arr = np.zeros(0, dtype=nat.ASSIGNED_POD) if assigned is None else assigned
        self.numa_arr = np.zeros(0, dtype=nat.NUMA_SPEC) if numa is None else numa
        self.rsv_arr = np.zeros(0, dtype=nat.RESERVATION) if reservations is None else reservations
        self.quota_arr = np.zeros(0, dtype=nat.QUOTA) if quotas is None else quotas
        self.now_ns = now_ns
        self.c_view = nat.make_view(self.pods, self.containers, self.nodes, self.aggregated_arr, self.pod_metrics_arr,
                                    self.assigned_arr, self.numa_arr, self.rsv_arr, self.quota_arr)

    def with_nodes(self, nodes: np.ndarray, pods: Optional[np.ndarray] = None) -> "SynthView":
        """The same cluster with other node (and pod) specs; every side array is kept, so the nodes'
        indices into them stay valid."""
        return SynthView(self.pods if pods is None else pods, self.containers, nodes, self.now_ns, self.numa_arr,
                         self.rsv_arr, self.quota_arr, self.aggregated_arr, self.pod_metrics_arr, self.assigned_arr)

    def subset_nodes(self, begin: int, end: int) -> "SynthView":
        return self.with_nodes(np.ascontiguousarray(self.nodes[begin:end]))


def _rl_fill(arr, r, values, mask=None):
    """arr: structured array of RESOURCE_LIST; set resource r = values where mask."""
    if mask is None:
        arr["v"][:, r] = values
        arr["present"] |= np.uint32(1 << r)
    else:
        arr["v"][mask, r] = values[mask] if np.ndim(values) else values
        arr["present"][mask] |= np.uint32(1 << r)


def make_nodes(n: int, seed: int, now_ns: int = NOW_NS, no_metric_frac: float = 0.05,
               expired_frac: float = 0.02) -> np.ndarray:
    rng = np.random.default_rng(seed)
    nodes = np.zeros(n, dtype=nat.NODE_SPEC)
    cpu = rng.choice(np.array([32, 48, 64, 96, 128], np.int64), n) * 1000
    mem = rng.choice(np.array([64, 128, 256, 512], np.int64), n) * GI
    bcpu = (cpu * rng.integers(20, 61, n)) // 100
    bmem = (mem // 100) * rng.integers(20, 61, n)
    alloc = nodes["allocatable"]
    _rl_fill(alloc, nat.RES_CPU, cpu)
    _rl_fill(alloc, nat.RES_MEMORY, mem)
    _rl_fill(alloc, nat.RES_BATCH_CPU, bcpu)
    _rl_fill(alloc, nat.RES_BATCH_MEMORY, bmem)
    req = nodes["requested"]
    rcpu = (cpu * rng.integers(0, 71, n)) // 100
    rmem = (mem // 100) * rng.integers(0, 71, n)
    _rl_fill(req, nat.RES_CPU, rcpu)
    _rl_fill(req, nat.RES_MEMORY, rmem)
    _rl_fill(req, nat.RES_EPHEMERAL_STORAGE, np.zeros(n, np.int64))
    _rl_fill(req, nat.RES_BATCH_CPU, (bcpu * rng.integers(0, 71, n)) // 100)
    _rl_fill(req, nat.RES_BATCH_MEMORY, (bmem // 100) * rng.integers(0, 71, n))
    nodes["nonzero_requested"][:, 0] = rcpu
    nodes["nonzero_requested"][:, 1] = rmem
    nodes["allowed_pods"] = 110
    nodes["pod_count"] = rng.integers(0, 60, n)
    u = rng.random(n)
    has_metric = u >= no_metric_frac
    expired = (u >= no_metric_frac) & (u < no_metric_frac + expired_frac)
    nodes["has_node_metric"] = has_metric
    nodes["has_update_time"] = has_metric
    nodes["update_time_ns"] = np.where(expired, now_ns - 400 * 10**9, now_ns - 30 * 10**9)
    nodes["has_report_interval"] = has_metric
    nodes["report_interval_seconds"] = 60
    nodes["has_node_metric_info"] = has_metric
    usage = nodes["node_usage"]
    _rl_fill(usage, nat.RES_CPU, (cpu * rng.integers(0, 81, n)) // 100)
    _rl_fill(usage, nat.RES_MEMORY, (mem // 100) * rng.integers(0, 91, n))
    nodes["numa"] = -1
    return nodes


def make_pods(p: int, seed: int, distinct: bool = False):
    """Pending pods of the config-1/2 distribution.  distinct: cpu uniform in [100, 4000] m and memory uniform
    in [128 Mi, 16 Gi] bytes instead of the 5 × 7 request shapes, so (almost) every pod's row is its own
    (the bench's config2_distinct section: no two pods share an evaluation)."""
    rng = np.random.default_rng(seed + 1_000_003)
    pods = np.zeros(p, dtype=nat.POD_SPEC)
    cont = np.zeros(p, dtype=nat.CONTAINER)
    if distinct:
        cpu = rng.integers(100, 4001, p).astype(np.int64)
        mem = rng.integers(128 * MI, 16 * GI + 1, p).astype(np.int64)
    else:
        cpu = rng.choice(np.array([250, 500, 1000, 2000, 4000], np.int64), p)
        mem = rng.choice(np.array([256, 512, 1024, 2048, 4096, 8192, 16384], np.int64), p) * MI
    kind = rng.random(p)
    guaranteed = kind < 0.5
    burstable = (kind >= 0.5) & (kind < 0.8)
    batch = kind >= 0.8
    ls = ~batch
    rq, lm = cont["requests"], cont["limits"]
    _rl_fill(rq, nat.RES_CPU, cpu, ls)
    _rl_fill(rq, nat.RES_MEMORY, mem, ls)
    _rl_fill(lm, nat.RES_CPU, np.where(burstable, 2 * cpu, cpu), ls)
    _rl_fill(lm, nat.RES_MEMORY, np.where(burstable, 2 * mem, mem), ls)
    _rl_fill(rq, nat.RES_BATCH_CPU, cpu, batch)       # batch-cpu in milli-cores (Value)
    _rl_fill(rq, nat.RES_BATCH_MEMORY, mem, batch)
    _rl_fill(lm, nat.RES_BATCH_CPU, cpu, batch)
    _rl_fill(lm, nat.RES_BATCH_MEMORY, mem, batch)
    pods["first_container"] = np.arange(p)
    pods["n_containers"] = 1
    pods["first_init_container"] = np.arange(p)
    pods["label_priority_class"] = -1
    pods["label_qos"] = -1
    pods["name_id"] = np.arange(p) + 10_000_000
    pods["rsv_owner_class"] = -1
    pods["rsv_affinity_class"] = -1
    pods["quota"] = -1
    return pods, cont


def decorate(nodes: np.ndarray, pods: np.ndarray, cont: np.ndarray, seed: int, assigned_frac: float = 0.2,
             aggregated_frac: float = 0.3, besteffort_frac: float = 0.3, custom_frac: float = 0.04,
             raw_alloc_frac: float = 0.02):
    """Node-side LoadAware inputs (see the module docstring), in place on `nodes`.  Existing pods are
    appended after the pending ones (pods[len(pods):]), so pending pod i keeps index i.  Returns
    (pods, containers, aggregated, pod_metrics, assigned)."""
    rng = np.random.default_rng(seed + 313)
    n, p0, c0 = len(nodes), len(pods), len(cont)
    metric = (nodes["has_node_metric"] != 0) & (nodes["has_node_metric_info"] != 0)
    upd = nodes["update_time_ns"]
    cpu = nodes["allocatable"]["v"][:, nat.RES_CPU]
    mem = nodes["allocatable"]["v"][:, nat.RES_MEMORY]
    # NonZeroRequested > Requested: best-effort pods count 100m / 200Mi each (schedutil.GetNonzeroRequests)
    be = np.where(rng.random(n) < besteffort_frac, rng.integers(1, 4, n), 0)
    nodes["nonzero_requested"][:, 0] += be * 100
    nodes["nonzero_requested"][:, 1] += be * 200 * MI
    nodes["pod_count"] = np.minimum(nodes["pod_count"] + be, 100)
    # already-assigned pods (podAssignCache) with their PodsMetric
    host = np.flatnonzero(metric & (rng.random(n) < assigned_frac))
    k = rng.integers(1, 5, len(host))
    m = int(k.sum())
    xp, xc = make_pods(m, seed + 17)
    xp["first_container"] += c0
    xp["first_init_container"] += c0
    xp["name_id"] = np.arange(m) + 20_000_000 + 1_000_000 * (seed % 7)
    pods = np.concatenate([pods, xp])
    cont = np.concatenate([cont, xc])
    owner = np.repeat(host, k)
    assigned = np.zeros(m, dtype=nat.ASSIGNED_POD)
    assigned["pod"] = p0 + np.arange(m)
    interval = nodes["report_interval_seconds"][owner] * 10**9
    when = rng.random(m)   # long before / inside the report interval before / after UpdateTime
    assigned["timestamp_ns"] = np.where(when < 0.4, upd[owner] - 5 * interval,
                                        np.where(when < 0.7, upd[owner] - interval // 3, upd[owner] + 5 * 10**9))
    first = np.zeros(n, np.int64)
    first[host] = np.concatenate([[0], np.cumsum(k)[:-1]])
    nodes["first_assigned"][host] = first[host]
    nodes["n_assigned"][host] = k
    # PodsMetric: 80 % of the assigned pods, plus NotFound entries and repeated names on some nodes
    rq = xc["requests"]["v"]
    req_cpu = np.maximum(rq[:, nat.RES_CPU], rq[:, nat.RES_BATCH_CPU])
    req_mem = np.maximum(rq[:, nat.RES_MEMORY], rq[:, nat.RES_BATCH_MEMORY])
    reported = rng.random(m) < 0.8
    extra = rng.random(len(host)) < 0.3
    entries = []
    pos = 0
    for h_i, node in enumerate(host):
        idx = np.arange(pos, pos + k[h_i])
        pos += k[h_i]
        mine = [(int(xp["name_id"][j]), int(p0 + j), j) for j in idx if reported[j]]
        if extra[h_i]:
            mine.append((90_000_000 + int(node), -1, -1))            # lister NotFound: skipped
            if mine[0][2] >= 0:
                mine.append(mine[0])                                  # repeated name: the last one wins
        entries.append(mine)
    pm_count = np.array([len(e) for e in entries], np.int64)
    pm = np.zeros(int(pm_count.sum()), dtype=nat.POD_METRIC)
    flat = [x for e in entries for x in e]
    if flat:
        pm["name_id"] = [x[0] for x in flat]
        pm["lister_pod"] = [x[1] for x in flat]
        src = np.array([x[2] for x in flat])
        scale = rng.integers(30, 121, len(flat))
        ucpu = np.where(src >= 0, req_cpu[np.maximum(src, 0)] * scale // 100, 1000)
        umem = np.where(src >= 0, (req_mem[np.maximum(src, 0)] // 100) * scale, GI)
        _rl_fill(pm["usage"], nat.RES_CPU, ucpu)
        _rl_fill(pm["usage"], nat.RES_MEMORY, umem)
    pfirst = np.concatenate([[0], np.cumsum(pm_count)[:-1]]) if len(host) else np.zeros(0, np.int64)
    nodes["first_pod_metric"][host] = pfirst
    nodes["n_pod_metric"][host] = pm_count
    # AggregatedNodeUsages: one or two durations; p95 missing on some
    ag_nodes = np.flatnonzero(metric & (rng.random(n) < aggregated_frac))
    na = rng.integers(1, 3, len(ag_nodes))
    agg = np.zeros(int(na.sum()), dtype=nat.AGGREGATED_USAGE)
    owner_a = np.repeat(ag_nodes, na)
    slot = np.concatenate([np.arange(c) for c in na]) if len(na) else np.zeros(0, np.int64)
    agg["duration_ns"] = np.where(slot == 0, 300, 600) * 10**9
    ucpu = nodes["node_usage"]["v"][owner_a, nat.RES_CPU]
    umem = nodes["node_usage"]["v"][owner_a, nat.RES_MEMORY]
    drop_p95 = rng.random(len(agg)) < 0.2
    for t, f in ((nat.AGG_AVG, 80), (nat.AGG_P50, 85), (nat.AGG_P90, 100), (nat.AGG_P95, 105), (nat.AGG_P99, 110)):
        live = ~drop_p95 if t == nat.AGG_P95 else np.ones(len(agg), bool)
        _rl_fill(agg["usage"][:, t], nat.RES_CPU, np.minimum(ucpu * f // 100, cpu[owner_a]), live)
        _rl_fill(agg["usage"][:, t], nat.RES_MEMORY, np.minimum((umem // 100) * f, mem[owner_a]), live)
    afirst = np.concatenate([[0], np.cumsum(na)[:-1]]) if len(na) else np.zeros(0, np.int64)
    nodes["first_aggregated"][ag_nodes] = afirst
    nodes["n_aggregated"][ag_nodes] = na
    # annotations: custom usage thresholds (valid / unparsable) and raw allocatable
    u = rng.random(n)
    custom = u < custom_frac
    nodes["custom_thresholds_state"] = np.where(custom, 1, np.where(u < custom_frac * 1.25, -1, 0))
    _rl_fill(nodes["custom_usage_thresholds"], nat.RES_CPU, np.full(n, 70), custom)
    _rl_fill(nodes["custom_usage_thresholds"], nat.RES_MEMORY, np.full(n, 90), custom)
    prod_thr = custom & (rng.random(n) < 0.3)
    _rl_fill(nodes["custom_prod_usage_thresholds"], nat.RES_CPU, np.full(n, 50), prod_thr)
    raw = rng.random(n) < raw_alloc_frac
    nodes["raw_allocatable_state"] = np.where(raw, 1, 0)
    _rl_fill(nodes["raw_allocatable"], nat.RES_CPU, cpu * 6 // 5, raw)
    return pods, cont, agg, pm, assigned


def make_cluster(n_nodes: int, n_pods: int, seed: int, now_ns: int = NOW_NS, decorated: bool = True,
                 distinct_pods: bool = False, **kw) -> SynthView:
    nodes = make_nodes(n_nodes, seed, now_ns, **kw)
    pods, cont = make_pods(n_pods, seed, distinct=distinct_pods)
    if not decorated:
        return SynthView(pods, cont, nodes, now_ns)
    pods, cont, agg, pm, asg = decorate(nodes, pods, cont, seed)
    return SynthView(pods, cont, nodes, now_ns, aggregated=agg, pod_metrics=pm, assigned=asg)


def make_numa_cluster(n_nodes: int, n_pods: int, seed: int, now_ns: int = NOW_NS, zones=(4, 6, 8),
                      ls_frac: float = 0.6, distinct_pods: bool = False) -> SynthView:
    """BASELINE config 3: nodes with Z ∈ `zones` NUMA zones (equal split of the node's
    cpu / memory allocatable; zone allocated uniform 0–70 %), policy mix 40 % SingleNUMANode, 30 %
    Restricted, 30 % None; pods 60 % LS (cpu / memory requests) and 40 % batch (batch-cpu /
    batch-memory).  Node Requested carries the zone allocations (they are pods on the node)."""
    rng = np.random.default_rng(seed + 77)
    nodes = make_nodes(n_nodes, seed, now_ns)
    cpu = nodes["allocatable"]["v"][:, nat.RES_CPU].copy()
    mem = nodes["allocatable"]["v"][:, nat.RES_MEMORY].copy()
    Z = rng.choice(np.array(zones, np.int64), n_nodes)
    u = rng.random(n_nodes)
    policy = np.where(u < 0.4, nat.NUMA_SINGLE_NUMA_NODE, np.where(u < 0.7, nat.NUMA_RESTRICTED, nat.NUMA_NONE))
    numa = np.zeros(n_nodes, dtype=nat.NUMA_SPEC)
    numa["policy"] = policy
    numa["n_zones"] = Z
    numa["cpu_topology_valid"] = 1
    req_cpu = np.zeros(n_nodes, np.int64)
    req_mem = np.zeros(n_nodes, np.int64)
    for z in range(max(zones)):
        live = z < Z
        zc = np.where(live, (cpu // Z) // 1000 * 1000, 0)
        zm = np.where(live, (mem // Z) // (1 << 20) * (1 << 20), 0)
        ac = (zc * rng.integers(0, 71, n_nodes)) // 100 // 1000 * 1000
        am = (zm // 100) * rng.integers(0, 71, n_nodes)
        numa["zone_id"][:, z] = np.where(live, z, 0)
        _rl_fill(numa["zone_total"][:, z], nat.RES_CPU, zc, live)
        _rl_fill(numa["zone_total"][:, z], nat.RES_MEMORY, zm, live)
        _rl_fill(numa["zone_allocated"][:, z], nat.RES_CPU, ac, live)
        _rl_fill(numa["zone_allocated"][:, z], nat.RES_MEMORY, am, live)
        req_cpu += np.where(live, ac, 0)
        req_mem += np.where(live, am, 0)
    # the zone allocations are pods on the node: NodeInfo.Requested / NonZeroRequested hold them
    rv = nodes["requested"]["v"]
    rv[:, nat.RES_CPU] = np.maximum(rv[:, nat.RES_CPU], req_cpu)
    rv[:, nat.RES_MEMORY] = np.maximum(rv[:, nat.RES_MEMORY], req_mem)
    nodes["nonzero_requested"][:, 0] = rv[:, nat.RES_CPU]
    nodes["nonzero_requested"][:, 1] = rv[:, nat.RES_MEMORY]
    nodes["numa"] = np.arange(n_nodes)
    pods, cont = make_pods(n_pods, seed, distinct=distinct_pods)   # distinct: continuous requests, no repeated rows
    # 60 % LS / 40 % batch mix
    rng2 = np.random.default_rng(seed + 991)
    batch = rng2.random(n_pods) >= ls_frac
    rq, lm = cont["requests"], cont["limits"]
    cpu_r = np.where(rq["present"] & (1 << nat.RES_CPU), rq["v"][:, nat.RES_CPU], rq["v"][:, nat.RES_BATCH_CPU])
    mem_r = np.where(rq["present"] & (1 << nat.RES_MEMORY), rq["v"][:, nat.RES_MEMORY], rq["v"][:, nat.RES_BATCH_MEMORY])
    for arr in (rq, lm):
        arr["v"][:] = 0
        arr["present"][:] = 0
    _rl_fill(rq, nat.RES_CPU, cpu_r, ~batch)
    _rl_fill(rq, nat.RES_MEMORY, mem_r, ~batch)
    _rl_fill(lm, nat.RES_CPU, cpu_r, ~batch)
    _rl_fill(lm, nat.RES_MEMORY, mem_r, ~batch)
    _rl_fill(rq, nat.RES_BATCH_CPU, cpu_r, batch)
    _rl_fill(rq, nat.RES_BATCH_MEMORY, mem_r, batch)
    _rl_fill(lm, nat.RES_BATCH_CPU, cpu_r, batch)
    _rl_fill(lm, nat.RES_BATCH_MEMORY, mem_r, batch)
    return SynthView(pods, cont, nodes, now_ns, numa)


def make_rsv_cluster(n_nodes: int, n_pods: int, seed: int, now_ns: int = NOW_NS, rsv_node_frac: float = 0.10,
                     owner_classes: int = 16, n_quotas: int = 64, quota_ratio: float = 0.8,
                     owned_frac: float = 0.8, affinity_frac: float = 0.1, non_preemptible_frac: float = 0.1,
                     max_rsv_per_node: int = 2, quota_tree: bool = False) -> SynthView:
    """BASELINE config 5: colocation burst of batch pods (batch-cpu / batch-memory
    requests) with Reservations and ElasticQuota.  `rsv_node_frac` of the nodes carry 1–2
    reservations of batch resources (10–30 % of the node's batch allocatable; 95 % available, 5 %
    unschedulable, 20 % allocate-once; policy 70 % Default / 20 % Aligned / 10 % Restricted; owner
    classes: one or two of `owner_classes`; an order label on 30 %; 0–3 assigned pods holding 0–100 %
    of it).  The reserve pods and their assigned pods are pods of the node (Requested, pod count).
    Pods: `owned_frac` belong to an owner class, `affinity_frac` of those require a matching
    reservation; each pod is in one of `n_quotas` quota groups whose runtime is `quota_ratio` of the
    group's total demand (min = half of it); `non_preemptible_frac` are non-preemptible."""
    rng = np.random.default_rng(seed + 555)
    nodes = make_nodes(n_nodes, seed, now_ns)
    rsv = _reservations(nodes, rng, rsv_node_frac, owner_classes, (nat.RES_BATCH_CPU, nat.RES_BATCH_MEMORY),
                        max_rsv_per_node)
    pods, cont = make_pods(n_pods, seed)
    rq, lm = cont["requests"], cont["limits"]
    cpu_r = np.where(rq["present"] & (1 << nat.RES_CPU), rq["v"][:, nat.RES_CPU], rq["v"][:, nat.RES_BATCH_CPU])
    mem_r = np.where(rq["present"] & (1 << nat.RES_MEMORY), rq["v"][:, nat.RES_MEMORY], rq["v"][:, nat.RES_BATCH_MEMORY])
    for arr in (rq, lm):
        arr["v"][:] = 0
        arr["present"][:] = 0
    for arr in (rq, lm):
        _rl_fill(arr, nat.RES_BATCH_CPU, cpu_r)
        _rl_fill(arr, nat.RES_BATCH_MEMORY, mem_r)
    quotas = _owners_and_quotas(pods, cont, seed, owner_classes, n_quotas, quota_ratio, owned_frac, affinity_frac,
                                non_preemptible_frac, quota_tree)
    return SynthView(pods, cont, nodes, now_ns, reservations=rsv, quotas=quotas)


def _reservations(nodes, rng, rsv_node_frac, owner_classes, res, max_per_node=2):
    """`rsv_node_frac` of the nodes carry 1–`max_per_node` reservations of the two resources `res` (10–30 %
    of the node's allocatable of them); the reserve pods and their assigned pods are pods of the node."""
    n_nodes = len(nodes)
    rn = np.sort(rng.choice(n_nodes, int(round(rsv_node_frac * n_nodes)), replace=False))
    node_of = np.repeat(rn, rng.integers(1, max_per_node + 1, len(rn)))
    R = len(node_of)
    rsv = np.zeros(R, dtype=nat.RESERVATION)
    rsv["node"] = node_of
    flags = np.where(rng.random(R) < 0.95, nat.RSV_AVAILABLE, 0)
    flags |= np.where(rng.random(R) < 0.05, nat.RSV_UNSCHEDULABLE, 0)
    flags |= np.where(rng.random(R) < 0.2, nat.RSV_ALLOCATE_ONCE, 0)
    rsv["flags"] = flags
    pu = rng.random(R)
    rsv["policy"] = np.where(pu < 0.7, nat.RSV_POLICY_DEFAULT, np.where(pu < 0.9, nat.RSV_POLICY_ALIGNED,
                                                                       nat.RSV_POLICY_RESTRICTED))
    o1 = rng.integers(0, owner_classes, R)
    o2 = rng.integers(0, owner_classes, R)
    owners = (np.uint32(1) << o1.astype(np.uint32)) | np.where(rng.random(R) < 0.3,
                                                               np.uint32(1) << o2.astype(np.uint32), np.uint32(0))
    rsv["owner_classes"] = owners
    rsv["affinity_classes"] = owners
    rsv["order"] = np.where(rng.random(R) < 0.3, rng.integers(1, 101, R), 0)
    r0, r1 = res
    bcpu = nodes["allocatable"]["v"][node_of, r0]
    bmem = nodes["allocatable"]["v"][node_of, r1]
    ac = bcpu * rng.integers(10, 31, R) // 100
    am = (bmem // 100) * rng.integers(10, 31, R)
    if r0 == nat.RES_CPU:
        ac = ac // 1000 * 1000
    _rl_fill(rsv["allocatable"], r0, ac)
    _rl_fill(rsv["allocatable"], r1, am)
    assigned = rng.integers(0, 4, R)
    fill = np.where(assigned > 0, rng.integers(0, 101, R), 0)
    xc = ac * fill // 100
    xm = (am // 100) * fill
    has = assigned > 0
    _rl_fill(rsv["allocated"], r0, xc, has)
    _rl_fill(rsv["allocated"], r1, xm, has)
    rsv["n_assigned"] = assigned
    rv = nodes["requested"]["v"]
    np.add.at(rv[:, r0], node_of, ac + xc)
    np.add.at(rv[:, r1], node_of, am + xm)
    if r0 == nat.RES_CPU:
        np.add.at(nodes["nonzero_requested"][:, 0], node_of, ac + xc)
        np.add.at(nodes["nonzero_requested"][:, 1], node_of, am + xm)
    else:
        np.add.at(nodes["nonzero_requested"][:, 0], node_of, 100 * (1 + assigned))
        np.add.at(nodes["nonzero_requested"][:, 1], node_of, 200 * MI * (1 + assigned))
    np.add.at(nodes["pod_count"], node_of, 1 + assigned)
    return rsv


def _owners_and_quotas(pods, cont, seed, owner_classes, n_quotas, quota_ratio, owned_frac, affinity_frac,
                       non_preemptible_frac, quota_tree=False):
    """Reservation owner / affinity classes, quota groups and non-preemptible flags of the pods; each
    group's runtime (used limit) is `quota_ratio` of its total demand of every requested resource
    (min = half of it).  quota_tree: the groups form a binary heap (group g's parent is (g - 1) // 2,
    group 0's the root) and a group's limit is `quota_ratio` of its whole subtree's demand."""
    n_pods = len(pods)
    prng = np.random.default_rng(seed + 4242)
    owned = prng.random(n_pods) < owned_frac
    owner = prng.integers(0, owner_classes, n_pods)
    pods["rsv_owner_class"] = np.where(owned, owner, -1)
    pods["rsv_affinity_class"] = np.where(owned & (prng.random(n_pods) < affinity_frac), owner, -1)
    q = prng.integers(0, n_quotas, n_pods)
    pods["quota"] = q
    pods["non_preemptible"] = prng.random(n_pods) < non_preemptible_frac
    quotas = np.zeros(n_quotas, dtype=nat.QUOTA)
    g = np.arange(n_quotas)
    quotas["parent"] = np.where(quota_tree & (g > 0), (g - 1) // 2, -1)
    rq = cont["requests"]
    for r in (nat.RES_CPU, nat.RES_MEMORY, nat.RES_BATCH_CPU, nat.RES_BATCH_MEMORY):
        has = (rq["present"] & np.uint32(1 << r)) != 0
        if not has.any():
            continue
        d = np.bincount(q, weights=np.where(has, rq["v"][:, r], 0), minlength=n_quotas).astype(np.int64)
        if quota_tree:
            for k in range(n_quotas - 1, 0, -1):
                d[(k - 1) // 2] += d[k]
        lim = (d * int(quota_ratio * 100)) // 100 if r in (nat.RES_CPU, nat.RES_BATCH_CPU) else \
            (d // 100) * int(quota_ratio * 100)
        _rl_fill(quotas["used_limit"], r, lim)
        _rl_fill(quotas["min"], r, lim // 2)
    return quotas


def make_profile_cluster(n_nodes: int, n_pods: int, seed: int, now_ns: int = NOW_NS, rsv_node_frac: float = 0.1,
                         owner_classes: int = 16, n_quotas: int = 32, quota_ratio: float = 0.8,
                         owned_frac: float = 0.6, affinity_frac: float = 0.1, non_preemptible_frac: float = 0.1,
                         zones=(2, 4, 8), quota_tree: bool = False) -> SynthView:
    """The shipped profile with every engine plugin (Fit, LoadAware, NodeNUMAResource, Reservation,
    ElasticQuota): config-3 nodes (NUMA zones, policy mix) and LS / batch pods, with reservations of
    cpu / memory on `rsv_node_frac` of the nodes (so the restored NodeInfo moves NodeNUMAResource's
    node-level terms), owner / affinity classes and quota groups over every requested resource."""
    cl = make_numa_cluster(n_nodes, n_pods, seed, now_ns, zones=zones)
    nodes = cl.nodes
    rng = np.random.default_rng(seed + 556)
    rsv = _reservations(nodes, rng, rsv_node_frac, owner_classes, (nat.RES_CPU, nat.RES_MEMORY))
    pods, cont = cl.pods, cl.containers
    quotas = _owners_and_quotas(pods, cont, seed, owner_classes, n_quotas, quota_ratio, owned_frac, affinity_frac,
                                non_preemptible_frac, quota_tree)
    return SynthView(pods, cont, nodes, now_ns, numa=cl.numa_arr, reservations=rsv, quotas=quotas)


# BASELINE.json configs (single-GPU bench uses config 2)
CONFIGS = {
    1: dict(n_nodes=5_000, n_pods=1_000, seed=1),
    2: dict(n_nodes=100_000, n_pods=10_000, seed=2),
    4: dict(n_nodes=1_000_000, n_pods=10_000, seed=4),
}


def make_la_extra_cluster(n_nodes: int, n_pods: int, seed: int, now_ns: int = NOW_NS) -> SynthView:
    """A config-2 cluster whose LoadAware inputs also carry the resources beyond cpu / memory that
    resourceWeights may name: ephemeral-storage and an extended resource in allocatable (some nodes
    without them), node usage of ephemeral-storage / batch-cpu / batch-memory / the extended resource,
    pod requests and limits of ephemeral-storage and the extended resource, and those resources in the
    assigned pods' PodsMetric."""
    base = make_cluster(n_nodes, n_pods, seed, now_ns)
    rng = np.random.default_rng(seed + 4242)
    nodes = base.nodes.copy()
    n = len(nodes)
    eph = rng.integers(50, 500, n) * GI
    gpu = rng.integers(0, 9, n)
    has_eph, has_gpu = rng.random(n) < 0.85, rng.random(n) < 0.5
    _rl_fill(nodes["allocatable"], nat.RES_EPHEMERAL_STORAGE, eph, has_eph)
    _rl_fill(nodes["allocatable"], nat.RES_EXTENDED, gpu, has_gpu)
    _rl_fill(nodes["requested"], nat.RES_EXTENDED, (gpu * rng.integers(0, 3, n)) // 4, has_gpu)
    usage = nodes["node_usage"]
    live = usage["present"] != 0
    _rl_fill(usage, nat.RES_EPHEMERAL_STORAGE, (eph // 100) * rng.integers(0, 101, n), live & has_eph)
    ba = nodes["allocatable"]["v"]
    _rl_fill(usage, nat.RES_BATCH_CPU, (ba[:, nat.RES_BATCH_CPU] * rng.integers(0, 91, n)) // 100, live)
    _rl_fill(usage, nat.RES_BATCH_MEMORY, (ba[:, nat.RES_BATCH_MEMORY] // 100) * rng.integers(0, 91, n), live)
    _rl_fill(usage, nat.RES_EXTENDED, (gpu * rng.integers(0, 5, n)) // 4, live & has_gpu)
    cont = base.containers.copy()
    c = len(cont)
    rq, lm = cont["requests"], cont["limits"]
    e_req = rng.integers(1, 40, c) * GI
    want_eph, want_gpu = rng.random(c) < 0.6, rng.random(c) < 0.25
    _rl_fill(rq, nat.RES_EPHEMERAL_STORAGE, e_req, want_eph)
    _rl_fill(lm, nat.RES_EPHEMERAL_STORAGE, e_req * rng.integers(1, 3, c), want_eph & (rng.random(c) < 0.5))
    g_req = rng.integers(1, 3, c)
    _rl_fill(rq, nat.RES_EXTENDED, g_req, want_gpu)
    _rl_fill(lm, nat.RES_EXTENDED, g_req, want_gpu)
    pm = base.pod_metrics_arr.copy()
    m = len(pm)
    if m:
        _rl_fill(pm["usage"], nat.RES_EPHEMERAL_STORAGE, rng.integers(0, 30, m) * GI, rng.random(m) < 0.7)
        _rl_fill(pm["usage"], nat.RES_BATCH_CPU, rng.integers(0, 4000, m), rng.random(m) < 0.4)
        _rl_fill(pm["usage"], nat.RES_EXTENDED, rng.integers(0, 3, m), rng.random(m) < 0.2)
    return SynthView(base.pods, cont, nodes, now_ns, aggregated=base.aggregated_arr, pod_metrics=pm,
                     assigned=base.assigned_arr)


SCALAR_NAMES = ("nvidia.com/gpu", "koordinator.sh/gpu-core", "koordinator.sh/rdma", "hugepages-2Mi")


def make_scalar_cluster(n_nodes: int, n_pods: int, seed: int, now_ns: int = NOW_NS) -> SynthView:
    """A config-2 cluster whose nodes and pods also carry the named scalar slots RES_EXT0..3 (the profile names them
    SCALAR_NAMES: GPUs, GPU cores, RDMA devices, 2 MiB hugepages): every node reports each with probability 0.6 (some
    already partly requested, some fully: Insufficient), 40 % of the pods request one to three of them at once (a
    zero-valued key now and then: a scalar key with a zero request still takes part in the compare)."""
    base = make_cluster(n_nodes, n_pods, seed, now_ns)
    rng = np.random.default_rng(seed + 5151)
    nodes = base.nodes.copy()
    n = len(nodes)
    caps = {nat.RES_EXT0: (0, 9), nat.RES_EXT1: (0, 801), nat.RES_EXT2: (0, 5), nat.RES_EXT3: (0, 65)}
    for r, (lo, hi) in caps.items():
        has = rng.random(n) < 0.6
        a = rng.integers(lo, hi, n)
        if r == nat.RES_EXT3:
            a = a * 2 * MI
        _rl_fill(nodes["allocatable"], r, a, has)
        _rl_fill(nodes["requested"], r, (a * rng.integers(0, 5, n)) // 4, has & (rng.random(n) < 0.7))
    cont = base.containers.copy()
    c = len(cont)
    rq, lm = cont["requests"], cont["limits"]
    wants = rng.random(c) < 0.4
    k = rng.integers(1, 4, c)
    for j, (r, (lo, hi)) in enumerate(caps.items()):
        pick = wants & (rng.random(c) < k / 4.0)
        v = rng.integers(0, max(2, hi // 3), c)
        if r == nat.RES_EXT3:
            v = v * 2 * MI
        _rl_fill(rq, r, v, pick)
        _rl_fill(lm, r, v, pick)
    return SynthView(base.pods, cont, nodes, now_ns, aggregated=base.aggregated_arr, pod_metrics=base.pod_metrics_arr,
                     assigned=base.assigned_arr)
