"""ctypes binding of ``libkoordgpu.so`` (the C-ABI in ``include/koord_gpu.h``).

numpy structured dtypes mirror every ABI struct; ``check_abi()`` compares their sizes with
``kg_struct_size`` so a layout drift fails loudly.  The library is built in-tree by
``koordinator_amd/build.py``; there is no fallback: importing the engine without the library
raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ENGINE_SO = os.environ.get("KG_ENGINE_SO") or os.path.join(_HERE, "lib", "libkoordgpu.so")

ABI_VERSION = 12
COMM_ID_BYTES = 128   # KG_COMM_ID_BYTES
COMM_NONE, COMM_RCCL, COMM_LOOPBACK = 0, 1, 2   # kg_comm_kind
# kg_set_forms bits (include/koord_gpu.h)
FORM_PLACE_PIPELINE, FORM_PLACE_SEQUENTIAL, FORM_NUMA_QUEUED, FORM_NUMA_CHUNK_TILE = 0x1, 0x2, 0x4, 0x8
FORM_NUMA_NO_CACHE = 0x10
FORM_NUMA_FUSED = 0x20
NUM_RES = 12
NUM_EXT_RES = 5        # KG_NUM_EXT_RES: the named scalar slots RES_EXT0 .. RES_EXT4
RES_NAME_MAX = 64      # KG_RES_NAME_MAX
(RES_CPU, RES_MEMORY, RES_EPHEMERAL_STORAGE, RES_BATCH_CPU, RES_BATCH_MEMORY, RES_MID_CPU, RES_MID_MEMORY,
 RES_EXT0, RES_EXT1, RES_EXT2, RES_EXT3, RES_EXT4) = range(12)
RES_EXTENDED = RES_EXT0   # the default name of slot 0: "example.com/gpu"
FIXED_RES_NAMES = ("cpu", "memory", "ephemeral-storage", "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory",
                   "kubernetes.io/mid-cpu", "kubernetes.io/mid-memory")
PRIO_NONE, PRIO_PROD, PRIO_MID, PRIO_BATCH, PRIO_FREE = range(5)
QOS_NONE, QOS_LSE, QOS_LSR, QOS_LS, QOS_BE, QOS_SYSTEM = range(6)
KUBE_QOS_UNSET, KUBE_QOS_GUARANTEED, KUBE_QOS_BURSTABLE, KUBE_QOS_BESTEFFORT = range(4)
AGG_UNSET, AGG_AVG, AGG_P50, AGG_P90, AGG_P95, AGG_P99 = range(6)
NUM_AGG_TYPES = 6
STRATEGY_LEAST_ALLOCATED, STRATEGY_MOST_ALLOCATED = 0, 1
PLUGIN_FIT, PLUGIN_LOADAWARE, PLUGIN_NUMA, PLUGIN_RESERVATION, PLUGIN_ELASTICQUOTA = 0x1, 0x2, 0x4, 0x8, 0x10
RSV_POLICY_DEFAULT, RSV_POLICY_ALIGNED, RSV_POLICY_RESTRICTED = range(3)
RSV_AVAILABLE, RSV_UNSCHEDULABLE, RSV_ALLOCATE_ONCE = 0x1, 0x2, 0x4
MAX_RSV_PER_NODE = 16
NUMA_NONE, NUMA_BEST_EFFORT, NUMA_RESTRICTED, NUMA_SINGLE_NUMA_NODE = range(4)
MAX_ZONES = 8

POD_HAS_REQUEST, POD_DAEMONSET, POD_PROD, POD_LA_PROD_SCORE, POD_VALID = 0x1, 0x2, 0x4, 0x8, 0x80000000
POD_NUMA_SKIP, POD_NUMA_CPU_BIND, POD_NON_PREEMPTIBLE, POD_NUMA_BIND_INVALID = 0x10, 0x20, 0x40, 0x100
CPU_BIND_UNSET, CPU_BIND_DEFAULT, CPU_BIND_FULL_PCPUS, CPU_BIND_SPREAD_BY_PCPUS, CPU_BIND_CONSTRAINED_BURST, CPU_BIND_OTHER = range(6)
CPU_EXCL_UNSET, CPU_EXCL_NONE, CPU_EXCL_PCPU_LEVEL, CPU_EXCL_NUMA_NODE_LEVEL = range(4)
NODE_CPU_BIND_NONE, NODE_CPU_BIND_FULL_PCPUS_ONLY, NODE_CPU_BIND_SPREAD_BY_PCPUS = range(3)
NUMA_ALLOC_DEFAULT, NUMA_ALLOC_MOST, NUMA_ALLOC_LEAST, NUMA_ALLOC_DISTRIBUTE_EVENLY = range(4)
NOT_FOUND = 1   # KG_NOT_FOUND
NODE_VALID, NODE_HAS_METRIC, NODE_HAS_UPDATE_TIME, NODE_LA_PASS_NONPROD, NODE_LA_PASS_PROD = 0x1, 0x2, 0x4, 0x8, 0x10
NODE_NUMA_OPTIONS, NODE_NUMA_TOPO_VALID, NODE_NUMA_TOPO_INVALID = 0x40, 0x80, 0x100

CODE_SUCCESS, CODE_ERROR, CODE_UNSCHEDULABLE, CODE_UNSCHEDULABLE_AND_UNRESOLVABLE = 0, 1, 2, 3
TILE = 1024
PLACE_CHUNK_MAX = 1024
PARTIAL_SLOTS = 16      # KG_PARTIAL_SLOTS: uint32 per (pod, tile) in the placement-chunk partial buffer

RESOURCE_LIST = np.dtype([("v", "<i8", (NUM_RES,)), ("present", "<u4"), ("_pad", "<u4")], align=True)

CONFIG = np.dtype([
    ("abi_version", "<i4"), ("enabled_plugins", "<u4"), ("weight_fit", "<i4"), ("weight_loadaware", "<i4"),
    ("fit_strategy", "<i4"), ("_pad0", "<i4"), ("fit_resource_weight", "<i8", (NUM_RES,)),
    ("la_filter_expired_node_metrics", "<i4"), ("la_has_expiration", "<i4"), ("la_expiration_seconds", "<i8"),
    ("la_resource_weight", "<i8", (NUM_RES,)), ("la_scaling_factor", "<i8", (NUM_RES,)),
    ("la_usage_thresholds", RESOURCE_LIST), ("la_prod_usage_thresholds", RESOURCE_LIST),
    ("la_score_according_prod_usage", "<i4"), ("la_has_aggregated", "<i4"),
    ("la_agg_usage_thresholds", RESOURCE_LIST), ("la_agg_usage_type", "<i4"), ("la_agg_score_type", "<i4"),
    ("la_agg_usage_duration_ns", "<i8"), ("la_agg_score_duration_ns", "<i8"),
    ("weight_numa", "<i4"), ("numa_strategy", "<i4"), ("numa_hint_strategy", "<i4"),
    ("numa_default_cpu_bind_policy", "<i4"),
    ("numa_resource_weight", "<i8", (NUM_RES,)),
    ("device", "<i4"), ("place_chunk", "<i4"),
    ("weight_reservation", "<i4"), ("eq_check_parent_quota", "<i4"),
    ("ext_resource_names", f"S{RES_NAME_MAX}", (NUM_EXT_RES,)),
], align=True)

CONTAINER = np.dtype([("requests", RESOURCE_LIST), ("limits", RESOURCE_LIST)], align=True)

POD_SPEC = np.dtype([
    ("first_container", "<i4"), ("n_containers", "<i4"), ("first_init_container", "<i4"), ("n_init_containers", "<i4"),
    ("overhead", RESOURCE_LIST), ("has_priority", "<i4"), ("priority", "<i4"), ("label_priority_class", "<i4"),
    ("label_qos", "<i4"), ("status_qos", "<i4"), ("is_daemonset", "<i4"), ("is_terminated", "<i4"),
    ("cpu_bind_required", "<i4"),
    ("name_id", "<i8"),
    ("rsv_owner_class", "<i4"), ("rsv_affinity_class", "<i4"), ("quota", "<i4"), ("non_preemptible", "<i4"),
    ("cpu_bind_preferred", "<i4"), ("cpu_exclusive", "<i4"),
], align=True)

AGGREGATED_USAGE = np.dtype([("duration_ns", "<i8"), ("usage", RESOURCE_LIST, (NUM_AGG_TYPES,))], align=True)
POD_METRIC = np.dtype([("name_id", "<i8"), ("lister_pod", "<i4"), ("_pad", "<i4"), ("usage", RESOURCE_LIST)], align=True)
ASSIGNED_POD = np.dtype([("pod", "<i4"), ("_pad", "<i4"), ("timestamp_ns", "<i8")], align=True)

NODE_SPEC = np.dtype([
    ("allocatable", RESOURCE_LIST), ("requested", RESOURCE_LIST), ("nonzero_requested", "<i8", (2,)),
    ("allowed_pods", "<i4"), ("pod_count", "<i4"), ("raw_allocatable_state", "<i4"), ("custom_thresholds_state", "<i4"),
    ("raw_allocatable", RESOURCE_LIST), ("custom_usage_thresholds", RESOURCE_LIST),
    ("custom_prod_usage_thresholds", RESOURCE_LIST), ("custom_has_aggregated", "<i4"), ("custom_agg_usage_type", "<i4"),
    ("custom_agg_usage_thresholds", RESOURCE_LIST), ("custom_agg_duration_ns", "<i8"),
    ("has_node_metric", "<i4"), ("has_update_time", "<i4"), ("update_time_ns", "<i8"),
    ("has_report_interval", "<i4"), ("has_node_metric_info", "<i4"), ("report_interval_seconds", "<i8"),
    ("node_usage", RESOURCE_LIST), ("first_aggregated", "<i4"), ("n_aggregated", "<i4"),
    ("first_pod_metric", "<i4"), ("n_pod_metric", "<i4"), ("first_assigned", "<i4"), ("n_assigned", "<i4"),
    ("numa", "<i4"), ("_pad_numa", "<i4"),
], align=True)

NUMA_SPEC = np.dtype([
    ("policy", "<i4"), ("n_zones", "<i4"), ("zone_id", "<i4", (MAX_ZONES,)),
    ("zone_total", RESOURCE_LIST, (MAX_ZONES,)), ("zone_allocated", RESOURCE_LIST, (MAX_ZONES,)),
    ("cpu_amplification_ratio", "<f8"), ("cpu_topology_valid", "<i4"), ("cpuset_cpus", "<i4"),
    ("zone_cpuset_cpus", "<i4", (MAX_ZONES,)),
    ("node_cpu_bind_policy", "<i4"), ("max_ref_count", "<i4"), ("first_cpu", "<i4"), ("n_cpus", "<i4"),
    ("numa_allocate_strategy", "<i4"), ("_pad_s", "<i4"),
], align=True)

CPU_INFO = np.dtype([("socket", "<i4"), ("node", "<i4"), ("core", "<i4"), ("refcount", "<i4"), ("exclusive", "<i4"),
                     ("reserved", "<i4")], align=True)

POD_ROW = np.dtype([
    ("request", "<i8", (NUM_RES,)), ("fit_score_request", "<i8", (NUM_RES,)), ("nonzero_request", "<i8", (2,)),
    ("la_estimate", "<i8", (2,)), ("request_present", "<u4"), ("flags", "<u4"),
    ("numa_request", "<i8", (NUM_RES,)), ("numa_request_present", "<u4"), ("cpu_bind", "<u4"),
    ("rsv_owner_class", "<i4"), ("rsv_affinity_class", "<i4"), ("quota", "<i4"), ("_pad2", "<i4"),
    ("la_estimate_x", "<i8", (NUM_RES - 2,)),
], align=True)

NODE_ROW = np.dtype([
    ("alloc", "<i8", (NUM_RES,)), ("requested", "<i8", (NUM_RES,)), ("nonzero_requested", "<i8", (2,)),
    ("la_alloc", "<i8", (2,)), ("la_used", "<i8", (2, 2)), ("metric_update_ns", "<i8"),
    ("pod_count", "<i4"), ("allowed_pods", "<i4"), ("alloc_present", "<u4"), ("flags", "<u4"),
    ("numa_policy", "<i4"), ("n_zones", "<i4"), ("zone_id", "<i4", (MAX_ZONES,)),
    ("zone_total", "<i8", (MAX_ZONES, 2)), ("zone_allocated", "<i8", (MAX_ZONES, 2)),
    ("zone_keys", "<u4"), ("zone_alloc_keys", "<u4"), ("cpu_amplification_ratio", "<f8"),
    ("cpuset_milli", "<i8"), ("cpuset_amp_milli", "<i8"), ("zone_cpuset_amp", "<i8", (MAX_ZONES,)),
    ("node_cpu_bind", "<i4"), ("cpus_per_core", "<i4"), ("cpuset_full_free_cpus", "<i4"), ("cpuset_free_cores", "<i4"),
    ("la_alloc_x", "<i8", (NUM_RES - 2,)), ("la_used_x", "<i8", (2, NUM_RES - 2)),
    ("cpuset_avail_cpus", "<i4"), ("_pad_cpu", "<i4"), ("zone_cpus_avail", "<i2", (MAX_ZONES,)),
    ("zone_cpus_full", "<i2", (MAX_ZONES,)), ("zone_cores_free", "<i2", (MAX_ZONES,)), ("_pad_row", "<i8"),
], align=True)

RESERVATION = np.dtype([
    ("node", "<i4"), ("flags", "<u4"), ("policy", "<i4"), ("n_assigned", "<i4"), ("owner_classes", "<u4"),
    ("affinity_classes", "<u4"), ("order", "<i8"), ("allocatable", RESOURCE_LIST), ("allocated", RESOURCE_LIST),
], align=True)

QUOTA = np.dtype([
    ("used_limit", RESOURCE_LIST), ("used", RESOURCE_LIST), ("min", RESOURCE_LIST),
    ("non_preemptible_used", RESOURCE_LIST), ("parent", "<i4"), ("_pad", "<i4"),
], align=True)

RSV_RESTORED = np.dtype([
    ("requested", "<i8", (NUM_RES,)), ("pod_requested", "<i8", (NUM_RES,)), ("r_allocated", "<i8", (NUM_RES,)),
    ("nonzero", "<i8", (2,)), ("pod_count", "<i4"), ("n_matched", "<i4"), ("has_state", "<i4"), ("_pad", "<i4"),
], align=True)

COUNTERS = np.dtype([(k, "<u8") for k in ("eval_calls", "evals", "out_bytes", "resolved", "placed", "h2d_bytes",
                                            "timed_launches", "kernel_ns")])

STRUCT_IDS = [RESOURCE_LIST, CONFIG, CONTAINER, POD_SPEC, AGGREGATED_USAGE, POD_METRIC, ASSIGNED_POD, NODE_SPEC,
              None, POD_ROW, NODE_ROW, None, NUMA_SPEC, RESERVATION, QUOTA, RSV_RESTORED, CPU_INFO, COUNTERS]


class ClusterView(ctypes.Structure):
    _fields_ = [
        ("pods", ctypes.c_void_p), ("n_pods", ctypes.c_int32), ("_p0", ctypes.c_int32),
        ("containers", ctypes.c_void_p), ("n_containers", ctypes.c_int32), ("_p1", ctypes.c_int32),
        ("nodes", ctypes.c_void_p), ("n_nodes", ctypes.c_int32), ("_p2", ctypes.c_int32),
        ("aggregated", ctypes.c_void_p), ("n_aggregated", ctypes.c_int32), ("_p3", ctypes.c_int32),
        ("pod_metrics", ctypes.c_void_p), ("n_pod_metrics", ctypes.c_int32), ("_p4", ctypes.c_int32),
        ("assigned", ctypes.c_void_p), ("n_assigned", ctypes.c_int32), ("_p5", ctypes.c_int32),
        ("numa", ctypes.c_void_p), ("n_numa", ctypes.c_int32), ("_p6", ctypes.c_int32),
        ("reservations", ctypes.c_void_p), ("n_reservations", ctypes.c_int32), ("_p7", ctypes.c_int32),
        ("quotas", ctypes.c_void_p), ("n_quotas", ctypes.c_int32), ("_p8", ctypes.c_int32),
        ("cpus", ctypes.c_void_p), ("n_cpus", ctypes.c_int32), ("_p9", ctypes.c_int32),
    ]


class EvalOut(ctypes.Structure):
    _fields_ = [("mask", ctypes.c_void_p), ("scores", ctypes.c_void_p), ("top1", ctypes.c_void_p),
                ("out_on_device", ctypes.c_int32), ("_pad", ctypes.c_int32), ("numa_scores", ctypes.c_void_p),
                ("rsv_scores", ctypes.c_void_p)]


def ptr(a) -> ctypes.c_void_p:
    if a is None:
        return ctypes.c_void_p(0)
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    return ctypes.c_void_p(a.ctypes.data)


def make_view(pods, containers, nodes, aggregated, pod_metrics, assigned, numa=None, reservations=None,
              quotas=None, cpus=None) -> ClusterView:
    if numa is None:
        numa = np.zeros(0, dtype=NUMA_SPEC)
    if reservations is None:
        reservations = np.zeros(0, dtype=RESERVATION)
    if quotas is None:
        quotas = np.zeros(0, dtype=QUOTA)
    if cpus is None:
        cpus = np.zeros(0, dtype=CPU_INFO)
    v = ClusterView()
    for name, arr in (("pods", pods), ("containers", containers), ("nodes", nodes), ("aggregated", aggregated),
                      ("pod_metrics", pod_metrics), ("assigned", assigned), ("numa", numa),
                      ("reservations", reservations), ("quotas", quotas), ("cpus", cpus)):
        assert arr.flags["C_CONTIGUOUS"]
        setattr(v, name, arr.ctypes.data if len(arr) else 0)
    v.n_pods, v.n_containers, v.n_nodes = len(pods), len(containers), len(nodes)
    v.n_aggregated, v.n_pod_metrics, v.n_assigned = len(aggregated), len(pod_metrics), len(assigned)
    v.n_numa, v.n_reservations, v.n_quotas, v.n_cpus = len(numa), len(reservations), len(quotas), len(cpus)
    v._keep = (pods, containers, nodes, aggregated, pod_metrics, assigned, numa, reservations, quotas, cpus)
    return v


EXPORTED = [
    "kg_abi_version", "kg_struct_size", "kg_config_default", "kg_config_shipped_profile", "kg_config_validate",
    "kg_build_pod_rows", "kg_build_node_rows", "kg_row_commit", "kg_row_eval", "kg_engine_create", "kg_engine_destroy",
    "kg_last_error", "kg_set_stream", "kg_sync", "kg_snapshot_reset", "kg_snapshot_upsert", "kg_snapshot_remove",
    "kg_snapshot_download", "kg_set_shard", "kg_pods_set", "kg_eval", "kg_place", "kg_num_tiles",
    "kg_place_chunk_eval", "kg_place_chunk_resolve", "kg_commit", "kg_set_profiling", "kg_eval_kernel_times",
    "kg_rsv_set", "kg_rsv_download", "kg_quota_set", "kg_quota_download", "kg_row_eval_rsv", "kg_row_rsv_restore",
    "kg_snapshot_generation", "kg_cpuset_take", "kg_row_reserve", "kg_cpus_set", "kg_cpus_download",
    "kg_place_chunk_resolve_prev", "kg_set_eval_stream", "kg_set_forms", "kg_comm_unique_id", "kg_comm_init",
    "kg_place_sharded", "kg_counters_get", "kg_counters_reset", "kg_comm_init_loopback", "kg_comm_kind",
]

_lib = None


def lib() -> ctypes.CDLL:
    """Load the in-tree engine library; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    # test hook (tests/test_sanitizers_cpu.py): a sanitizer build of the host code alone; the engine
    # entry points are absent from it, so any GPU call fails
    host_only = os.environ.get("KG_SANITIZED_HOST_SO")
    # measurement builds of the engine (tools/ablate_mat.sh): an alternative in-tree library
    so = host_only or os.environ.get("KG_ENGINE_SO") or ENGINE_SO
    if not os.path.exists(so):
        raise RuntimeError(f"{so} is missing: build it with `python koordinator_amd/build.py` "
                           "(there is no CPU fallback for the engine)")
    L = ctypes.CDLL(so)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "kg_abi_version": (i32, []), "kg_struct_size": (i64, [i32]),
        "kg_config_default": (None, [vp]), "kg_config_shipped_profile": (None, [vp]),
        "kg_config_validate": (i32, [vp, ctypes.c_char_p, i32]),
        "kg_build_pod_rows": (i32, [vp, vp, vp, i32, vp]), "kg_build_node_rows": (i32, [vp, vp, vp, i32, vp]),
        "kg_row_commit": (i32, [vp, vp, vp]),
        "kg_row_eval": (i32, [vp, vp, vp, i64, vp, vp, vp, vp]),
        "kg_engine_create": (i32, [vp, ctypes.POINTER(vp)]), "kg_engine_destroy": (None, [vp]),
        "kg_last_error": (ctypes.c_char_p, [vp]), "kg_set_stream": (i32, [vp, vp]), "kg_sync": (i32, [vp]),
        "kg_snapshot_reset": (i32, [vp, i32]), "kg_snapshot_upsert": (i32, [vp, vp, vp, i32]),
        "kg_snapshot_remove": (i32, [vp, i32]), "kg_snapshot_download": (i32, [vp, i32, i32, vp]),
        "kg_set_shard": (i32, [vp, i32, i32]), "kg_pods_set": (i32, [vp, vp, i32]),
        "kg_eval": (i32, [vp, i64, vp]), "kg_place": (i32, [vp, i64, vp, vp]), "kg_num_tiles": (i32, [vp]),
        "kg_place_chunk_eval": (i32, [vp, i64, i32, i32, vp]),
        "kg_place_chunk_resolve": (i32, [vp, i64, i32, i32, vp, vp, vp]),
        "kg_commit": (i32, [vp, i32, i32]),
        "kg_set_profiling": (i32, [vp, i32]), "kg_eval_kernel_times": (i32, [vp, vp, i32]),
        "kg_rsv_set": (i32, [vp, vp, i32]), "kg_rsv_download": (i32, [vp, vp, i32]),
        "kg_quota_set": (i32, [vp, vp, i32]), "kg_quota_download": (i32, [vp, vp, i32]),
        "kg_row_eval_rsv": (i32, [vp, vp, vp, i32, vp, i64, vp, vp, vp, vp, vp, vp, vp]),
        "kg_row_rsv_restore": (i32, [vp, vp, vp, i32, vp, vp]),
        "kg_snapshot_generation": (i32, [vp, ctypes.POINTER(ctypes.c_uint64)]),
        "kg_cpuset_take": (i32, [vp, i32, i32, vp, i32, i32, i32, i32, vp]),
        "kg_row_reserve": (i32, [vp, vp, vp, vp, i32, i32, i32, vp]),
        "kg_cpus_set": (i32, [vp, vp, vp, vp, i32]), "kg_cpus_download": (i32, [vp, i32, vp, i32]),
        "kg_place_chunk_resolve_prev": (i32, [vp, i64, i32, i32, vp, vp, vp, vp, i32]),
        "kg_set_eval_stream": (i32, [vp, vp]), "kg_set_forms": (i32, [vp, ctypes.c_uint32]),
        "kg_comm_unique_id": (i32, [vp]), "kg_comm_init": (i32, [vp, i32, i32, vp]),
        "kg_place_sharded": (i32, [vp, ctypes.c_int64, vp, vp]), "kg_counters_get": (i32, [vp, vp]), "kg_counters_reset": (i32, [vp]),
        "kg_comm_init_loopback": (i32, [vp, i32, i32, ctypes.c_char_p]), "kg_comm_kind": (i32, [vp]),
    }
    for name, (res, args) in sig.items():
        if host_only and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    check_abi(L)
    return L


def check_abi(L=None) -> None:
    L = L or lib()
    if L.kg_abi_version() != ABI_VERSION:
        raise RuntimeError("engine ABI version mismatch")
    for sid, dt in enumerate(STRUCT_IDS):
        if dt is None:
            continue
        got = L.kg_struct_size(sid)
        if got != dt.itemsize:
            raise RuntimeError(f"struct id {sid}: C size {got} != numpy {dt.itemsize}")
    if L.kg_struct_size(8) != ctypes.sizeof(ClusterView) or L.kg_struct_size(11) != ctypes.sizeof(EvalOut):
        raise RuntimeError("view/eval_out struct size mismatch")
