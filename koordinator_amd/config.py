"""Plugin args → ``kg_config`` (pkg/scheduler/apis/config/types.go:30-114).

``load_aware_args(...)`` mirrors v1beta2.SetDefaults_LoadAwareSchedulingArgs
(pkg/scheduler/apis/config/v1beta2/defaults.go:78-100): a map given explicitly replaces the
default map as a whole (UsageThresholds, ResourceWeights), EstimatedScalingFactors is merged
key by key, and nil pointers get their defaults.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from . import _native as nat
from . import objects
from .objects import AGG

DEFAULT_USAGE_THRESHOLDS = {"cpu": 65, "memory": 95}
DEFAULT_RESOURCE_WEIGHTS = {"cpu": 1, "memory": 1}
DEFAULT_SCALING_FACTORS = {"cpu": 85, "memory": 70}


def _rl(d: Optional[Dict[str, int]], res: Dict[str, int]) -> np.ndarray:
    out = np.zeros((), dtype=nat.RESOURCE_LIST)
    for k, v in (d or {}).items():
        out["v"][res[k]] = int(v)
        out["present"] |= np.uint32(1 << res[k])
    return out


def make_config(*, plugins=("NodeResourcesFit", "LoadAwareScheduling"), weight_fit: int = 1,
                weight_loadaware: int = 1, fit_strategy: str = "LeastAllocated",
                fit_resources: Optional[Dict[str, int]] = None,
                filter_expired_node_metrics: Optional[bool] = None,
                node_metric_expiration_seconds: Optional[int] = None,
                resource_weights: Optional[Dict[str, int]] = None,
                usage_thresholds: Optional[Dict[str, int]] = None,
                prod_usage_thresholds: Optional[Dict[str, int]] = None,
                score_according_prod_usage: bool = False,
                estimated_scaling_factors: Optional[Dict[str, int]] = None,
                aggregated: Optional[dict] = None,
                weight_numa: int = 1, numa_strategy: str = "LeastAllocated",
                numa_hint_strategy: str = "LeastAllocated", numa_resources: Optional[Dict[str, int]] = None,
                numa_default_cpu_bind_policy: str = "FullPCPUs",
                weight_reservation: int = 1, eq_check_parent_quota: int = 0, device: int = 0,
                place_chunk: int = 16, extended_resources=None) -> np.ndarray:
    """extended_resources: the names of the named scalar slots (kg_config.ext_resource_names, ≤ 5; default the
    flattening's current ones, objects.EXTENDED — "example.com/gpu" unless set_extended_resources changed it).
    Flatten clusters for this config under objects.extended_resources(the same names)."""
    ext = tuple(objects.EXTENDED if extended_resources is None else extended_resources)
    RES = objects.resource_map(ext)
    c = np.zeros((), dtype=nat.CONFIG)
    for i, n in enumerate(ext):
        c["ext_resource_names"][i] = n.encode()
    c["abi_version"] = nat.ABI_VERSION
    bits = 0
    for p in plugins:
        bits |= {"NodeResourcesFit": nat.PLUGIN_FIT, "LoadAwareScheduling": nat.PLUGIN_LOADAWARE,
                 "NodeNUMAResource": nat.PLUGIN_NUMA, "Reservation": nat.PLUGIN_RESERVATION,
                 "ElasticQuota": nat.PLUGIN_ELASTICQUOTA}[p]
    c["enabled_plugins"] = bits
    c["weight_fit"] = weight_fit
    c["weight_loadaware"] = weight_loadaware
    c["fit_strategy"] = {"LeastAllocated": nat.STRATEGY_LEAST_ALLOCATED,
                         "MostAllocated": nat.STRATEGY_MOST_ALLOCATED}[fit_strategy]
    for k, w in (fit_resources or {"cpu": 1, "memory": 1}).items():
        c["fit_resource_weight"][RES[k]] = w
    # SetDefaults_LoadAwareSchedulingArgs
    c["la_filter_expired_node_metrics"] = int(True if filter_expired_node_metrics is None else filter_expired_node_metrics)
    c["la_has_expiration"] = 1
    c["la_expiration_seconds"] = 180 if node_metric_expiration_seconds is None else node_metric_expiration_seconds
    for k, w in (resource_weights or DEFAULT_RESOURCE_WEIGHTS).items():
        c["la_resource_weight"][RES[k]] = w
    c["la_usage_thresholds"] = _rl(usage_thresholds if usage_thresholds else DEFAULT_USAGE_THRESHOLDS, RES)
    c["la_prod_usage_thresholds"] = _rl(prod_usage_thresholds, RES)
    sf = dict(estimated_scaling_factors or {})
    for k, v in DEFAULT_SCALING_FACTORS.items():
        sf.setdefault(k, v)
    for k, v in sf.items():
        c["la_scaling_factor"][RES[k]] = v
    c["la_score_according_prod_usage"] = int(score_according_prod_usage)
    if aggregated is not None:
        c["la_has_aggregated"] = 1
        c["la_agg_usage_thresholds"] = _rl(aggregated.get("usageThresholds"), RES)
        c["la_agg_usage_type"] = AGG[aggregated.get("usageAggregationType", "")]
        c["la_agg_score_type"] = AGG[aggregated.get("scoreAggregationType", "")]
        c["la_agg_usage_duration_ns"] = int(aggregated.get("usageAggregatedDuration", 0) * 10**9)
        c["la_agg_score_duration_ns"] = int(aggregated.get("scoreAggregatedDuration", 0) * 10**9)
    # NodeNUMAResourceArgs (SetDefaults_NodeNUMAResourceArgs, v1beta2/defaults.go:101-137)
    strategies = {"LeastAllocated": nat.STRATEGY_LEAST_ALLOCATED, "MostAllocated": nat.STRATEGY_MOST_ALLOCATED}
    c["weight_numa"] = weight_numa
    c["numa_strategy"] = strategies[numa_strategy]
    c["numa_hint_strategy"] = strategies[numa_hint_strategy]
    # NodeNUMAResourceArgs.DefaultCPUBindPolicy (v1beta2 defaults.go:50)
    c["numa_default_cpu_bind_policy"] = {"": nat.CPU_BIND_UNSET, "FullPCPUs": nat.CPU_BIND_FULL_PCPUS,
                                         "SpreadByPCPUs": nat.CPU_BIND_SPREAD_BY_PCPUS,
                                         "ConstrainedBurst": nat.CPU_BIND_CONSTRAINED_BURST}[numa_default_cpu_bind_policy]
    for k, w in (numa_resources or {"cpu": 1, "memory": 1}).items():
        c["numa_resource_weight"][RES[k]] = w
    c["weight_reservation"] = weight_reservation  # profile weight (the shipped profile: 5000)
    c["device"] = device
    c["place_chunk"] = place_chunk
    c["eq_check_parent_quota"] = eq_check_parent_quota  # ElasticQuotaArgs.EnableCheckParentQuota
    return c


def shipped_profile(**kw) -> np.ndarray:
    """config/manager/scheduler-config.yaml:17-45 (Fit scores batch resources too)."""
    base = dict(fit_resources={"cpu": 1, "memory": 1, "kubernetes.io/batch-cpu": 1, "kubernetes.io/batch-memory": 1},
                filter_expired_node_metrics=False, node_metric_expiration_seconds=300, weight_reservation=5000)
    base.update(kw)
    return make_config(**base)
