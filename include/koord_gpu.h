/*
 * koord_gpu.h — C-ABI of the MI355X batched Filter/Score engine for koord-scheduler.
 *
 * This is the drop-in boundary between the (Go) koord-scheduler plugins and the
 * HIP engine.  Every entry point takes plain pointers and sizes; no torch / HIP
 * types appear in the signatures (streams are passed as opaque `void*`).
 *
 * Which reference surface each entry replaces (paths relative to the reference
 * repository PeterChg/koordinator @ 2025-01-12):
 *
 *   kg_engine_create        plugin construction: loadaware.New (pkg/scheduler/plugins/loadaware/load_aware.go:76-110),
 *                           NodeResourcesFit (upstream k8s v1.24.15 noderesources.NewFit; profile
 *                           config/manager/scheduler-config.yaml:17-31)
 *   kg_build_pod_rows       PreFilter-time pod preprocessing: NodeResourcesFit computePodResourceRequest
 *                           (in-repo mirror reservation/transformer.go:316-346), estimator.EstimatePod
 *                           (loadaware/estimator/default_estimator.go:57-108), GetPodPriorityClassWithDefault
 *                           (apis/extension/priority_utils.go:26-47), isDaemonSetPod (loadaware/helper.go:189-196)
 *   kg_build_node_rows      snapshot ingest of NodeInfo + NodeMetric + podAssignCache: the node-only parts of
 *                           LoadAware.Filter (load_aware.go:123-254) and LoadAware.Score (load_aware.go:269-376),
 *                           EstimateNode (default_estimator.go:110-129)
 *   kg_snapshot_upsert      informer/event feeders: podAssignCache.OnAdd/OnUpdate/OnDelete
 *                           (loadaware/pod_assign_cache.go:82-117), upstream Cache.UpdateSnapshot
 *   kg_eval                 per-(pod,node) hot loops: framework.FilterPlugin.Filter and ScorePlugin.Score of
 *                           LoadAwareScheduling (load_aware.go:123, :269) and NodeResourcesFit (upstream
 *                           fitsRequest / LeastAllocated), plus the per-pod max of upstream selectHost
 *   kg_place                the sequential scheduling cycle (upstream scheduleOne → Filter → Score → selectHost →
 *                           Reserve) for a queue of pods, with Reserve deltas of LoadAware.Reserve
 *                           (load_aware.go:260-267) and NodeInfo.AddPod (mirror reservation/transformer.go:293-306)
 *   kg_commit               one Reserve (AssumePod + LoadAware.Reserve) of a pod on a node
 *   kg_rsv_set              reservation cache feed (reservation/cache.go:249-269 forEachAvailableReservationOnNode,
 *                           frameworkext/reservation_info.go:200-300): per-node reservation slots for the
 *                           Reservation plugin's restore / Filter / Score / Reserve (reservation/transformer.go:49-291,
 *                           plugin.go:311-476, scoring.go:42-203, nominator.go:76-135)
 *   kg_quota_set            ElasticQuota group state for its PreFilter / Reserve (elasticquota/plugin.go:210-255,
 *                           :323-337; core/group_quota_manager.go:613-650, :791-797)
 *
 * Units follow k8s Quantity conversions used by the plugins: cpu-like resources
 * (KG_RES_CPU) in milli-units (Quantity.MilliValue), every other resource in
 * base units (Quantity.Value).  batch-cpu / mid-cpu are stored as their Value()
 * (the reference encodes them in milli-cores already).
 *
 * Error model: every function returns kg_status (0 = ok, < 0 = error); the
 * message of the last error of an engine is available from kg_last_error().
 * Threading: one engine = one HIP stream; calls on one engine must be serialized
 * by the caller (the Go side holds a mutex), results are plain host memory.
 */
#ifndef KOORD_GPU_H
#define KOORD_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KG_ABI_VERSION 12
#define KG_QUOTA_MAX_DEPTH 64 /* longest kg_quota parent chain (cycles are rejected) */

/* largest kg_config.place_chunk / kg_place_chunk_resolve chunk (the resolve kernel's touched list) */
#define KG_PLACE_CHUNK_MAX 1024

/* kg_place_chunk_eval / _resolve partial buffer: KG_PARTIAL_SLOTS uint32 per (pod, 1024-node tile) —
 * the tile's best keys in descending order, 0-padded (nodes outside the fp64 fast-path bounds are not
 * listed: the resolve re-scores them from the engine's slow-node list).  Slots of a tile come from one
 * rank only, so ranks merge buffers with an element-wise max. */
#define KG_PARTIAL_SLOTS 16

/* ------------------------------------------------------------------ */
/* status codes                                                          */
/* ------------------------------------------------------------------ */
typedef int32_t kg_status;
#define KG_OK 0
#define KG_ERR_INVALID_ARG (-1)
#define KG_ERR_HIP (-2)
#define KG_ERR_UNSUPPORTED (-3)
#define KG_ERR_RANGE (-4)
#define KG_ERR_STATE (-5)
#define KG_NOT_FOUND 1       /* a search found nothing (kg_cpuset_take: no cpuset satisfies the request) */

/* upstream framework.Code values used in filter results */
#define KG_CODE_SUCCESS 0
#define KG_CODE_ERROR 1
#define KG_CODE_UNSCHEDULABLE 2
#define KG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE 3

/* ------------------------------------------------------------------ */
/* resources                                                             */
/* ------------------------------------------------------------------ */
#define KG_NUM_RES 12
#define KG_NUM_EXT_RES 5          /* named scalar slots KG_RES_EXT0 .. KG_RES_EXT4 */
#define KG_RES_NAME_MAX 64        /* bytes of a slot name in kg_config.ext_resource_names, NUL included */
enum kg_resource {
    KG_RES_CPU = 0,               /* "cpu"                         MilliValue */
    KG_RES_MEMORY = 1,            /* "memory"                      Value      */
    KG_RES_EPHEMERAL_STORAGE = 2, /* "ephemeral-storage"           Value      */
    KG_RES_BATCH_CPU = 3,         /* "kubernetes.io/batch-cpu"     Value      */
    KG_RES_BATCH_MEMORY = 4,      /* "kubernetes.io/batch-memory"  Value      */
    KG_RES_MID_CPU = 5,           /* "kubernetes.io/mid-cpu"       Value      */
    KG_RES_MID_MEMORY = 6,        /* "kubernetes.io/mid-memory"    Value      */
    /* the named scalar slots: extended resources (nvidia.com/gpu, koordinator.sh/gpu-core, koordinator.sh/rdma,
     * ...) and hugepages-<size>, named by kg_config.ext_resource_names (default: slot 0 "example.com/gpu", the
     * others unused).  Every plugin on the path treats them as the ScalarResources of framework.Resource:
     * NodeResourcesFit compares each requested one (fitsRequest), scores those its ScoringStrategy weighs,
     * LoadAware weighs those its resourceWeights name, Reservation / ElasticQuota add them up. */
    KG_RES_EXT0 = 7, KG_RES_EXT1 = 8, KG_RES_EXT2 = 9, KG_RES_EXT3 = 10, KG_RES_EXT4 = 11,
    KG_RES_EXTENDED = KG_RES_EXT0
};
/* resources that upstream schedutil.IsScalarResourceName() treats as scalar */
#define KG_SCALAR_RES_MASK 0xFF8u

/* A corev1.ResourceList restricted to the resources above: `present` is the
 * key set (bit r ⇔ key r exists in the map), v[r] the converted value. */
typedef struct kg_resource_list {
    int64_t v[KG_NUM_RES];
    uint32_t present;
    uint32_t _pad;
} kg_resource_list;

/* ------------------------------------------------------------------ */
/* enums                                                                 */
/* ------------------------------------------------------------------ */
enum kg_priority_class { /* apis/extension/priority.go:28-34 */
    KG_PRIO_NONE = 0,
    KG_PRIO_PROD = 1,
    KG_PRIO_MID = 2,
    KG_PRIO_BATCH = 3,
    KG_PRIO_FREE = 4
};
enum kg_qos_class { /* apis/extension/qos.go */
    KG_QOS_NONE = 0,
    KG_QOS_LSE = 1,
    KG_QOS_LSR = 2,
    KG_QOS_LS = 3,
    KG_QOS_BE = 4,
    KG_QOS_SYSTEM = 5
};
enum kg_kube_qos { /* corev1.PodQOSClass */
    KG_KUBE_QOS_UNSET = 0,
    KG_KUBE_QOS_GUARANTEED = 1,
    KG_KUBE_QOS_BURSTABLE = 2,
    KG_KUBE_QOS_BESTEFFORT = 3
};
enum kg_aggregation_type { /* apis/extension AggregationType */
    KG_AGG_UNSET = 0, /* "" */
    KG_AGG_AVG = 1,
    KG_AGG_P50 = 2,
    KG_AGG_P90 = 3,
    KG_AGG_P95 = 4,
    KG_AGG_P99 = 5
};
#define KG_NUM_AGG_TYPES 6

enum kg_scoring_strategy {
    KG_STRATEGY_LEAST_ALLOCATED = 0,
    KG_STRATEGY_MOST_ALLOCATED = 1
};

#define KG_PLUGIN_FIT 0x1u       /* NodeResourcesFit       */
#define KG_PLUGIN_LOADAWARE 0x2u /* LoadAwareScheduling    */
#define KG_PLUGIN_NUMA 0x4u      /* NodeNUMAResource (zone fit + score, cpuset binding) */
#define KG_PLUGIN_RESERVATION 0x8u  /* Reservation (restore, Filter, Score + NormalizeScore, Reserve) */
#define KG_PLUGIN_ELASTICQUOTA 0x10u /* ElasticQuota (PreFilter quota gate, Reserve used accounting) */

/* NUMA topology policies (apis/extension/numa_aware.go; node label node.koordinator.sh/numa-topology-policy
 * or the NodeResourceTopology kubelet policy, pkg/scheduler/plugins/nodenumaresource/util.go:52-58) */
/* CPU bind policies of NodeNUMAResource (apis/extension/numa_aware.go:86-118) */
enum kg_cpu_bind_policy {          /* ResourceSpec Required/PreferredCPUBindPolicy, args.DefaultCPUBindPolicy */
    KG_CPU_BIND_UNSET = 0,         /* "" */
    KG_CPU_BIND_DEFAULT = 1,       /* "Default" (the plugin's DefaultCPUBindPolicy) */
    KG_CPU_BIND_FULL_PCPUS = 2,
    KG_CPU_BIND_SPREAD_BY_PCPUS = 3,
    KG_CPU_BIND_CONSTRAINED_BURST = 4,
    KG_CPU_BIND_OTHER = 5,         /* any other annotation value (PreFilter binds nothing for it) */
};
enum kg_cpu_exclusive_policy {     /* ResourceSpec.PreferredCPUExclusivePolicy / CPUInfo.ExclusivePolicy */
    KG_CPU_EXCL_UNSET = 0, KG_CPU_EXCL_NONE = 1, KG_CPU_EXCL_PCPU_LEVEL = 2, KG_CPU_EXCL_NUMA_NODE_LEVEL = 3,
};
enum kg_node_cpu_bind_policy {     /* GetNodeCPUBindPolicy: label node.koordinator.sh/cpu-bind-policy, or the
                                      kubelet static policy with full-pcpus-only (numa_aware.go:314-325) */
    KG_NODE_CPU_BIND_NONE = 0, KG_NODE_CPU_BIND_FULL_PCPUS_ONLY = 1, KG_NODE_CPU_BIND_SPREAD_BY_PCPUS = 2,
};

enum kg_numa_allocate_strategy {   /* label node.koordinator.sh/numa-allocate-strategy (numa_aware.go:52-53, util.go:35-41) */
    KG_NUMA_ALLOC_DEFAULT = 0,     /* label absent: the plugin default (NUMAMostAllocated iff NUMAScoringStrategy.Type is
                                      MostAllocated, util.go:27-33) */
    KG_NUMA_ALLOC_MOST = 1, KG_NUMA_ALLOC_LEAST = 2, KG_NUMA_ALLOC_DISTRIBUTE_EVENLY = 3
};

enum kg_numa_policy {
    KG_NUMA_NONE = 0,
    KG_NUMA_BEST_EFFORT = 1,
    KG_NUMA_RESTRICTED = 2,
    KG_NUMA_SINGLE_NUMA_NODE = 3
};
#define KG_MAX_ZONES 8
#define KG_MAX_NODE_CPUS 1024     /* logical CPUs of one node in kg_cluster_view.cpus */

/* ------------------------------------------------------------------ */
/* engine configuration = plugin args (pkg/scheduler/apis/config/types.go)  */
/* ------------------------------------------------------------------ */
typedef struct kg_config {
    int32_t abi_version;       /* must be KG_ABI_VERSION */
    uint32_t enabled_plugins;  /* KG_PLUGIN_* : enabled at Filter AND Score */
    int32_t weight_fit;        /* profile score weight of NodeResourcesFit    */
    int32_t weight_loadaware;  /* profile score weight of LoadAwareScheduling */

    /* NodeResourcesFitArgs.ScoringStrategy (upstream v1.24.15) */
    int32_t fit_strategy;                  /* kg_scoring_strategy */
    int32_t _pad0;
    int64_t fit_resource_weight[KG_NUM_RES]; /* 0 ⇔ resource not listed */

    /* LoadAwareSchedulingArgs (types.go:30-76) */
    int32_t la_filter_expired_node_metrics;   /* *FilterExpiredNodeMetrics (nil ⇒ 0) */
    int32_t la_has_expiration;                /* NodeMetricExpirationSeconds != nil  */
    int64_t la_expiration_seconds;
    int64_t la_resource_weight[KG_NUM_RES];   /* ResourceWeights (0 ⇔ absent).  Weights on resources other than
                                                 cpu / memory take the exact int64 pair path on every node
                                                 (correct, not the fp64 fast kernels) */
    int64_t la_scaling_factor[KG_NUM_RES];    /* EstimatedScalingFactors (missing key ⇒ 0) */
    kg_resource_list la_usage_thresholds;     /* UsageThresholds */
    kg_resource_list la_prod_usage_thresholds;/* ProdUsageThresholds */
    int32_t la_score_according_prod_usage;    /* ScoreAccordingProdUsage */
    int32_t la_has_aggregated;                /* Aggregated != nil */
    kg_resource_list la_agg_usage_thresholds; /* Aggregated.UsageThresholds */
    int32_t la_agg_usage_type;                /* Aggregated.UsageAggregationType */
    int32_t la_agg_score_type;                /* Aggregated.ScoreAggregationType */
    int64_t la_agg_usage_duration_ns;         /* Aggregated.UsageAggregatedDuration (0 ⇒ max) */
    int64_t la_agg_score_duration_ns;         /* Aggregated.ScoreAggregatedDuration (0 ⇒ max) */

    /* NodeNUMAResourceArgs (types.go:103-114); both scorers weigh ScoringStrategy.Resources
     * (nodenumaresource/scoring.go:38,46) */
    int32_t weight_numa;                      /* profile score weight of NodeNUMAResource */
    int32_t numa_strategy;                    /* ScoringStrategy.Type (node / allocated-zone score) */
    int32_t numa_hint_strategy;               /* NUMAScoringStrategy.Type (per-mask hint score) */
    int32_t numa_default_cpu_bind_policy;     /* DefaultCPUBindPolicy (kg_cpu_bind_policy; v1beta2 default FullPCPUs) */
    int64_t numa_resource_weight[KG_NUM_RES]; /* ScoringStrategy.Resources (0 ⇔ absent) */

    /* engine knobs */
    int32_t device;            /* HIP device ordinal */
    int32_t place_chunk;       /* pods per refresh in kg_place (0 ⇒ default 16; at most KG_PLACE_CHUNK_MAX) */

    /* Reservation (profile weight, config/manager/scheduler-config.yaml:82-91 ships 5000) */
    int32_t weight_reservation;
    /* ElasticQuotaArgs.EnableCheckParentQuota: PreFilter also checks every ancestor group below the root
     * (plugin.go:250-252, plugin_helper.go:281-297 checkQuotaRecursive) */
    int32_t eq_check_parent_quota;
    /* names of the scalar slots KG_RES_EXT0 + i ("" ⇔ unused): the resource-name keys the ingest maps to them,
     * and their place in the sorted-name order the topology merge walks (policy.go:108: Go map order, fixed to
     * sorted names here).  Distinct, not one of the fixed names above. */
    char ext_resource_names[KG_NUM_EXT_RES][KG_RES_NAME_MAX];
} kg_config;

/* ------------------------------------------------------------------ */
/* object-level specs (what the Go plugin reads from its informers)        */
/* ------------------------------------------------------------------ */
typedef struct kg_container {
    kg_resource_list requests;
    kg_resource_list limits;
} kg_container;

typedef struct kg_pod_spec {
    int32_t first_container, n_containers;      /* into kg_cluster_view.containers */
    int32_t first_init_container, n_init_containers;
    kg_resource_list overhead;                  /* present == 0 ⇔ Spec.Overhead == nil */
    int32_t has_priority;                       /* Spec.Priority != nil */
    int32_t priority;
    int32_t label_priority_class;               /* -1 label absent, else kg_priority_class of the label value */
    int32_t label_qos;                          /* -1 label absent, else kg_qos_class of the label value */
    int32_t status_qos;                         /* kg_kube_qos of Status.QOSClass (UNSET ⇒ computed) */
    int32_t is_daemonset;                       /* an OwnerReference of Kind DaemonSet */
    int32_t is_terminated;                      /* util.IsPodTerminated */
    int32_t cpu_bind_required;                  /* annotation scheduling.koordinator.sh/resource-spec
                                                   RequiredCPUBindPolicy (kg_cpu_bind_policy) */
    int64_t name_id;                            /* identity of namespace/name */
    /* Reservation: the pod's owner class (reservation.Match(pod) ⇔ bit owner_class of the reservation's
     * owner_classes; −1 ⇔ matches none) and its required reservation affinity class (−1 ⇔ no
     * scheduling.koordinator.sh/reservation-affinity; else the reservation must have bit affinity_class
     * in affinity_classes: reservationAffinity.Match(fakeNode), transformer.go:348-372) */
    int32_t rsv_owner_class;
    int32_t rsv_affinity_class;
    /* ElasticQuota: index into kg_cluster_view.quotas (−1 ⇔ no quota: PreFilter skips) */
    int32_t quota;
    int32_t non_preemptible;                    /* extension.IsPodNonPreemptible */
    int32_t cpu_bind_preferred;                 /* ResourceSpec.PreferredCPUBindPolicy (kg_cpu_bind_policy) */
    int32_t cpu_exclusive;                      /* ResourceSpec.PreferredCPUExclusivePolicy (kg_cpu_exclusive_policy) */
} kg_pod_spec;

typedef struct kg_aggregated_usage { /* slov1alpha1.AggregatedUsage */
    int64_t duration_ns;
    kg_resource_list usage[KG_NUM_AGG_TYPES];   /* map[AggregationType]ResourceMap */
} kg_aggregated_usage;

typedef struct kg_pod_metric { /* slov1alpha1.PodMetricInfo */
    int64_t name_id;      /* namespace/name */
    int32_t lister_pod;   /* index of the pod in kg_cluster_view.pods, -1 ⇔ podLister NotFound */
    int32_t _pad;
    kg_resource_list usage;
} kg_pod_metric;

typedef struct kg_assigned_pod { /* podAssignCache item */
    int32_t pod;          /* index into kg_cluster_view.pods */
    int32_t _pad;
    int64_t timestamp_ns;
} kg_assigned_pod;

typedef struct kg_node_spec {
    /* framework.NodeInfo */
    kg_resource_list allocatable;   /* Allocatable (scalar keys = ScalarResources keys) */
    kg_resource_list requested;     /* Requested */
    int64_t nonzero_requested[2];   /* NonZeroRequested cpu, memory */
    int32_t allowed_pods;           /* Allocatable.AllowedPodNumber */
    int32_t pod_count;              /* len(NodeInfo.Pods) */
    /* annotation node.koordinator.sh/raw-allocatable: 0 absent, 1 present, -1 unparsable */
    int32_t raw_allocatable_state;
    /* annotation scheduling.koordinator.sh/usage-thresholds: 0 absent, 1 present, -1 unparsable */
    int32_t custom_thresholds_state;
    kg_resource_list raw_allocatable;
    kg_resource_list custom_usage_thresholds;
    kg_resource_list custom_prod_usage_thresholds;
    int32_t custom_has_aggregated;          /* AggregatedUsage != nil */
    int32_t custom_agg_usage_type;
    kg_resource_list custom_agg_usage_thresholds;
    int64_t custom_agg_duration_ns;         /* 0 ⇔ nil/zero */
    /* NodeMetric (nodeMetricLister.Get(node.Name)) */
    int32_t has_node_metric;                /* 0 ⇔ NotFound */
    int32_t has_update_time;                /* Status.UpdateTime != nil */
    int64_t update_time_ns;
    int32_t has_report_interval;            /* Spec.CollectPolicy.ReportIntervalSeconds != nil */
    int32_t has_node_metric_info;           /* Status.NodeMetric != nil */
    int64_t report_interval_seconds;
    kg_resource_list node_usage;            /* Status.NodeMetric.NodeUsage */
    int32_t first_aggregated, n_aggregated; /* Status.NodeMetric.AggregatedNodeUsages */
    int32_t first_pod_metric, n_pod_metric; /* Status.PodsMetric */
    int32_t first_assigned, n_assigned;     /* podAssignCache.podInfoItems[node] */
    int32_t numa;                           /* index into kg_cluster_view.numa, −1 ⇔ no topology options */
    int32_t _pad_numa;
} kg_node_spec;

/* NodeNUMAResource view of one node: TopologyOptions (nodenumaresource/topology_options.go:90-153)
 * and the plugin's NodeAllocation (node_allocation.go). */
typedef struct kg_numa_spec {
    int32_t policy;                                  /* kg_numa_policy (label, else NRT policy) */
    int32_t n_zones;                                 /* len(NUMANodeResources) */
    int32_t zone_id[KG_MAX_ZONES];                   /* NUMANodeResource.Node: the zone's affinity bit (< 64) */
    kg_resource_list zone_total[KG_MAX_ZONES];       /* NUMANodeResources[i].Resources (before amplification) */
    kg_resource_list zone_allocated[KG_MAX_ZONES];   /* allocatedResources[zone] (present == 0 ⇔ none) */
    double cpu_amplification_ratio;                  /* annotation resource-amplification-ratio cpu (≤ 1 ⇔ none) */
    int32_t cpu_topology_valid;                      /* TopologyOptions.CPUTopology: 1 valid (IsValid()), 0 reported but
                                                        invalid, −1 nil (no NodeResourceTopology).  Reserve records
                                                        allocations only when valid; with a cpu amplification ratio
                                                        > 1, 0 makes filterAmplifiedCPUs reject cpu requests
                                                        (plugin.go:359-362, resource_manager.go:390-397) */
    int32_t cpuset_cpus;                             /* |NodeAllocation.allocatedCPUs|: CPUs held by cpuset pods
                                                        (GetAvailableCPUs' allocated, no preferred CPUs) */
    int32_t zone_cpuset_cpus[KG_MAX_ZONES];          /* allocatedCPUs.CPUsInNUMANodes(zone_id[z]) (node_allocation.go:165) */
    /* cpuset binding (the CPU accumulator's inputs): the node's CPU bind policy, TopologyOptions.MaxRefCount,
       and its logical CPUs (CPUTopology.CPUDetails + NodeAllocation.allocatedCPUs + ReservedCPUs) as
       kg_cluster_view.cpus[first_cpu, first_cpu + n_cpus), cpu id = position; n_cpus == 0 ⇔ no detail
       (the count fields above then stand alone) */
    int32_t node_cpu_bind_policy;                    /* kg_node_cpu_bind_policy */
    int32_t max_ref_count;                           /* ≥ 1 */
    int32_t first_cpu, n_cpus;
    int32_t numa_allocate_strategy;                  /* kg_numa_allocate_strategy: which CPUs a Reserve takes */
    int32_t _pad_s;
} kg_numa_spec;

/* One logical CPU of a node (CPUInfo of cpu_topology.go + the node allocation's view of it). */
typedef struct kg_cpu_info {
    int32_t socket, node, core;   /* SocketID, NodeID (NUMA node = zone id), CoreID as reported */
    int32_t refcount;             /* NodeAllocation.allocatedCPUs[cpu].RefCount (0 ⇔ not allocated) */
    int32_t exclusive;            /* its ExclusivePolicy (kg_cpu_exclusive_policy) while allocated */
    int32_t reserved;             /* in TopologyOptions.ReservedCPUs (kubelet / node reservation / system QoS) */
} kg_cpu_info;

/* One reservation as the reservation cache holds it (frameworkext.ReservationInfo). */
enum kg_rsv_policy { /* schedulingv1alpha1.ReservationAllocatePolicy */
    KG_RSV_POLICY_DEFAULT = 0,   /* "" */
    KG_RSV_POLICY_ALIGNED = 1,
    KG_RSV_POLICY_RESTRICTED = 2
};
#define KG_RSV_AVAILABLE 0x1u      /* IsAvailable() && ParseError == nil */
#define KG_RSV_UNSCHEDULABLE 0x2u  /* Spec.Unschedulable || terminating */
#define KG_RSV_ALLOCATE_ONCE 0x4u  /* IsAllocateOnce() */
typedef struct kg_reservation {
    int32_t node;                  /* node index (reservationsOnNode key) */
    uint32_t flags;                /* KG_RSV_* */
    int32_t policy;                /* kg_rsv_policy */
    int32_t n_assigned;            /* len(AssignedPods) */
    uint32_t owner_classes;        /* bit c ⇔ Match(pod) for pods of owner class c */
    uint32_t affinity_classes;     /* bit a ⇔ a reservation-affinity class a selects this reservation */
    int64_t order;                 /* label scheduling.koordinator.sh/reservation-order (0 ⇔ absent / unparsable) */
    kg_resource_list allocatable;  /* Allocatable; present = ResourceNames */
    kg_resource_list allocated;    /* Allocated */
} kg_reservation;

/* One ElasticQuota group (core.QuotaInfo) as its PreFilter reads it. */
typedef struct kg_quota {
    kg_resource_list used_limit;           /* getQuotaInfoUsedLimit: runtime (EnableRuntimeQuota) or max */
    kg_resource_list used;                 /* Used */
    kg_resource_list min;                  /* CalculateInfo.Min (non-preemptible gate) */
    kg_resource_list non_preemptible_used; /* NonPreemptibleUsed */
    /* ParentName as an index into the same list; -1 ⇔ the parent is the root quota (or is not tracked).
     * Reserve adds the pod's requests to the group and every ancestor (group_quota_manager.go:227-238,
     * :334-354); kg_quota_set rejects indices out of range and chains deeper than KG_QUOTA_MAX_DEPTH. */
    int32_t parent;
    int32_t _pad;
} kg_quota;

typedef struct kg_cluster_view {
    const kg_pod_spec *pods;                 int32_t n_pods;       int32_t _p0;
    const kg_container *containers;          int32_t n_containers; int32_t _p1;
    const kg_node_spec *nodes;               int32_t n_nodes;      int32_t _p2;
    const kg_aggregated_usage *aggregated;   int32_t n_aggregated; int32_t _p3;
    const kg_pod_metric *pod_metrics;        int32_t n_pod_metrics; int32_t _p4;
    const kg_assigned_pod *assigned;         int32_t n_assigned;   int32_t _p5;
    const kg_numa_spec *numa;                int32_t n_numa;       int32_t _p6;
    const kg_reservation *reservations;      int32_t n_reservations; int32_t _p7;
    const kg_quota *quotas;                  int32_t n_quotas;     int32_t _p8;
    const kg_cpu_info *cpus;                 int32_t n_cpus;       int32_t _p9;
} kg_cluster_view;

/* ------------------------------------------------------------------ */
/* engine rows (pod-only / node-only precompute; what the kernels read)    */
/* ------------------------------------------------------------------ */
#define KG_POD_HAS_REQUEST 0x1u    /* Fit: request not all-zero (fit.go fitsRequest early return) */
#define KG_POD_DAEMONSET 0x2u      /* LoadAware.Filter passes (load_aware.go:129) */
#define KG_POD_PROD 0x4u           /* GetPodPriorityClassWithDefault == koord-prod */
#define KG_POD_LA_PROD_SCORE 0x8u  /* prodPod && ScoreAccordingProdUsage (load_aware.go:291) */
#define KG_POD_NUMA_SKIP 0x10u     /* NodeNUMAResource PreFilter skip: all requests zero (plugin.go:225-231) */
#define KG_POD_NUMA_CPU_BIND 0x20u /* PreFilter requestCPUBind: LSE/LSR prod with a FullPCPUs / SpreadByPCPUs
                                      policy and a cpu request (plugin.go:232-262) */
#define KG_POD_NUMA_BIND_INVALID 0x100u /* PreFilter ErrInvalidRequestedCPUs (cpu request not whole cores):
                                           NodeNUMAResource fails on every node */
#define KG_POD_NON_PREEMPTIBLE 0x40u /* ElasticQuota: extension.IsPodNonPreemptible (min gate) */
#define KG_POD_VALID 0x80000000u

typedef struct kg_pod_row {
    int64_t request[KG_NUM_RES];        /* Fit PreFilter request (computePodResourceRequest) */
    int64_t fit_score_request[KG_NUM_RES]; /* Fit score pod request per resource (nonzero cpu/mem) */
    int64_t nonzero_request[2];         /* schedutil.GetNonzeroRequests sum (AssumePod NonZeroRequested delta) */
    int64_t la_estimate[2];             /* EstimatePod(pod)[cpu], [memory] */
    uint32_t request_present;           /* ScalarResources key set of the Fit request */
    uint32_t flags;                     /* KG_POD_* */
    int64_t numa_request[KG_NUM_RES];   /* PodRequestsAndLimits requests (NodeNUMAResource PreFilter,
                                           Reservation podRequests, ElasticQuota podRequest) */
    uint32_t numa_request_present;      /* key set of those requests */
    uint32_t cpu_bind;                  /* PreFilter state: required policy | preferred (effective) policy << 4 |
                                           exclusive policy << 8 (kg_cpu_bind_policy / kg_cpu_exclusive_policy) */
    int32_t rsv_owner_class;            /* kg_pod_spec.rsv_owner_class */
    int32_t rsv_affinity_class;         /* kg_pod_spec.rsv_affinity_class */
    int32_t quota;                      /* kg_pod_spec.quota */
    int32_t _pad2;
    int64_t la_estimate_x[KG_NUM_RES - 2]; /* EstimatePod(pod)[r] for r = 2..11 (0 unless resourceWeights name r) */
} kg_pod_row;

#define KG_NODE_VALID 0x1u
#define KG_NODE_HAS_METRIC 0x2u          /* nodeMetricLister found the NodeMetric */
#define KG_NODE_HAS_UPDATE_TIME 0x4u     /* Status.UpdateTime != nil */
#define KG_NODE_LA_PASS_NONPROD 0x8u     /* threshold check result for non-prod pods */
#define KG_NODE_LA_PASS_PROD 0x10u       /* threshold check result for prod pods */
#define KG_NODE_LA_AGG_MISSING 0x20u     /* score aggregation requested but not reported (info) */
#define KG_NODE_NUMA_OPTIONS 0x40u       /* the node has NodeNUMAResource topology options */
#define KG_NODE_NUMA_TOPO_VALID 0x80u    /* CPUTopology valid: Reserve records zone allocations */
#define KG_NODE_NUMA_TOPO_INVALID 0x100u /* CPUTopology reported but invalid (GetAvailableCPUs fails) */

typedef struct kg_node_row {
    int64_t alloc[KG_NUM_RES];          /* NodeInfo.Allocatable */
    int64_t requested[KG_NUM_RES];      /* NodeInfo.Requested */
    int64_t nonzero_requested[2];       /* NodeInfo.NonZeroRequested */
    int64_t la_alloc[2];                /* EstimateNode(node)[cpu], [memory] */
    int64_t la_used[2][2];              /* [nonProd, prod][cpu, memory]: assigned-pod estimates + usage term */
    int64_t metric_update_ns;           /* NodeMetric Status.UpdateTime */
    int32_t pod_count;
    int32_t allowed_pods;
    uint32_t alloc_present;             /* Allocatable.ScalarResources key set */
    uint32_t flags;                     /* KG_NODE_* */
    /* NodeNUMAResource: zones of cpu (milli, amplified) and memory; zone z = affinity bit zone_id[z] */
    int32_t numa_policy;                /* kg_numa_policy */
    int32_t n_zones;                    /* 0 ⇔ no NUMA resources */
    int32_t zone_id[KG_MAX_ZONES];
    int64_t zone_total[KG_MAX_ZONES][2];
    int64_t zone_allocated[KG_MAX_ZONES][2];
    uint32_t zone_keys;                 /* bit 2z+r: zone z's total has resource r (cpu 0, memory 1) */
    uint32_t zone_alloc_keys;           /* bit 2z+r: zone z's allocation has resource r */
    double cpu_amplification_ratio;     /* ≤ 1 ⇔ none */
    /* cpuset pods on the node (the amplified-CPU terms of filterAmplifiedCPUs / scoreWithAmplifiedCPUs /
       getAvailableNUMANodeResources); zero unless the CPU topology is valid */
    int64_t cpuset_milli;               /* cpuset_cpus · 1000 */
    int64_t cpuset_amp_milli;           /* Amplify(cpuset_milli, ratio) */
    int64_t zone_cpuset_amp[KG_MAX_ZONES]; /* Amplify(c, ratio) − c, c = zone z's cpuset CPUs · 1000: added to the
                                              zone's allocated cpu while the zone has an allocation entry */
    /* cpuset binding on a node without a NUMA topology policy (the Filter's Allocate reduces to counts:
       takeCPUs always succeeds on a large enough available set, and the required-policy filter leaves
       whole free cores / one CPU per core with a free CPU) */
    int32_t node_cpu_bind;              /* kg_node_cpu_bind_policy */
    int32_t cpus_per_core;              /* CPUTopology.CPUsPerCore() (0 ⇔ no CPU detail) */
    int32_t cpuset_full_free_cpus;      /* CPUs of the cores whose every CPU is available (getAvailableCPUs) */
    int32_t cpuset_free_cores;          /* cores with at least one available CPU */
    /* LoadAwareScheduling resourceWeights beyond cpu / memory (resources 2..11; zero unless weighted):
       EstimateNode(node)[r] and the [nonProd, prod] node terms of r */
    int64_t la_alloc_x[KG_NUM_RES - 2];
    int64_t la_used_x[2][KG_NUM_RES - 2];
    /* cpusets on a node with a NUMA topology policy (trimNUMANodeResources, allocateCPUSet): the node's
       available CPUs, and per zone its available CPUs, the CPUs of its wholly available cores and its
       cores with an available CPU */
    int32_t cpuset_avail_cpus;
    int32_t _pad_cpu;
    int16_t zone_cpus_avail[KG_MAX_ZONES];
    int16_t zone_cpus_full[KG_MAX_ZONES];
    int16_t zone_cores_free[KG_MAX_ZONES];
    int64_t _pad_row;
} kg_node_row;

/* ------------------------------------------------------------------ */
/* engine                                                                 */
/* ------------------------------------------------------------------ */
typedef struct kg_engine kg_engine;

/* Output of kg_eval (matrix mode).  Any pointer may be NULL (not produced).
 * Columns cover the evaluated node range [B, E) (the shard; the whole snapshot by default),
 * W = ceil((E - B) / 64), column c ⇔ node B + c:
 *   mask     [P][W] uint64: bit (c % 64) of word c/64 ⇔ pod p feasible on node B + c
 *            (AND of every enabled Filter plugin)
 *   scores   [P][64·W][2] uint8: {NodeResourcesFit score, LoadAwareScheduling score} ∈ [0,100]
 *            (0 where a plugin is disabled; row stride 64·W pairs).  Like the reference, where Score
 *            runs only on the nodes that passed Filter, a score is meaningful only where the pair's
 *            mask bit is set: the planes of a pod failing a node-independent gate (ElasticQuota
 *            PreFilter, a required reservation) keep the per-pair plugin scores of the plain nodes.
 *   numa_scores [P][64·W] uint8: NodeNUMAResource score (when KG_PLUGIN_NUMA is enabled)
 *   top1     [P] uint64: (total+1) << 32 | (0xFFFFFFFF − node) of the best feasible node,
 *            total = Σ weight·score, ties → lowest node index; 0 ⇔ no feasible node
 * When out_on_device != 0 the pointers are device pointers on the engine's device
 * (results stay resident; no copy back). */
typedef struct kg_eval_out {
    uint64_t *mask;
    uint8_t *scores;
    uint64_t *top1;
    int32_t out_on_device;
    int32_t _pad;
    uint8_t *numa_scores;    /* [P][64·W] NodeNUMAResource score (KG_PLUGIN_NUMA only; may be NULL) */
    uint8_t *rsv_scores;     /* [P][64·W] Reservation score after NormalizeScore (KG_PLUGIN_RESERVATION; may be NULL) */
} kg_eval_out;

int32_t kg_abi_version(void);
/* sizeof() of every ABI struct, in the order of kg_struct_id, for binding checks */
enum kg_struct_id {
    KG_SID_RESOURCE_LIST = 0, KG_SID_CONFIG, KG_SID_CONTAINER, KG_SID_POD_SPEC,
    KG_SID_AGGREGATED_USAGE, KG_SID_POD_METRIC, KG_SID_ASSIGNED_POD, KG_SID_NODE_SPEC,
    KG_SID_CLUSTER_VIEW, KG_SID_POD_ROW, KG_SID_NODE_ROW, KG_SID_EVAL_OUT, KG_SID_NUMA_SPEC,
    KG_SID_RESERVATION, KG_SID_QUOTA, KG_SID_RSV_RESTORED, KG_SID_CPU_INFO, KG_SID_COUNTERS, KG_SID_COUNT
};
int64_t kg_struct_size(int32_t sid);

/* Fill a config with the v1beta2 defaults (pkg/scheduler/apis/config/v1beta2/defaults.go:32-137)
 * and NodeResourcesFit LeastAllocated cpu:1 memory:1, both plugins enabled with weight 1. */
void kg_config_default(kg_config *cfg);
/* Shipped profile overrides (config/manager/scheduler-config.yaml:17-45). */
void kg_config_shipped_profile(kg_config *cfg);
kg_status kg_config_validate(const kg_config *cfg, char *err, int32_t err_len);

/* Host-side row builders (pure CPU, no GPU needed). */
kg_status kg_build_pod_rows(const kg_config *cfg, const kg_cluster_view *view,
                            const int32_t *pod_index, int32_t n, kg_pod_row *out);
kg_status kg_build_node_rows(const kg_config *cfg, const kg_cluster_view *view,
                             const int32_t *node_index, int32_t n, kg_node_row *out);
/* Reserve delta (AssumePod + LoadAware.Reserve + NodeNUMAResource.Reserve zone allocations) applied
 * to a host-side row. */
kg_status kg_row_commit(const kg_config *cfg, kg_node_row *node, const kg_pod_row *pod);
/* Filter + Score of one (pod, node) pair on host rows, through the same per-pair code the kernels
 * run: the single-node checks of a scheduling cycle (RunFilterPluginsWithNominatedPods for one
 * node, preemption's SelectVictimsOnNode, framework_extender.go:354-372) without a device.
 * Scores are the plugin scores (0..100) of the enabled plugins, 0 otherwise. */
kg_status kg_row_eval(const kg_config *cfg, const kg_node_row *node, const kg_pod_row *pod, int64_t now_ns,
                      int32_t *feasible, int32_t *fit_score, int32_t *la_score, int32_t *numa_score);
/* Reserve of a pod that may bind a cpuset, on host rows (NodeNUMAResource.Reserve, plugin.go:375-419):
 * requestCPUBind on the node (util.go:105-122), then resourceManager.Allocate (resource_manager.go:171-195) —
 * allocateResourcesByHint on the Filter's hint with the original requests and allocateCPUSet (:273-360), the
 * CPU accumulator zone by zone — and Update (node_allocation.go:57-100): the taken CPUs' RefCount + 1 and
 * ExclusivePolicy, the zone allocations, AssumePod / LoadAware deltas, and the row's cpuset counts re-derived
 * from `cpus` (the node's logical CPUs as kg_cluster_view.cpus holds them; updated in place).
 * numa_allocate_strategy: kg_numa_allocate_strategy of the node (DEFAULT ⇒ the plugin default from cfg).
 * KG_OK: reserved, taken[n_cpus] marks the cpuset (all zero when the pod binds none);
 * KG_NOT_FOUND: Allocate fails ("not enough cpus available to satisfy request" or a required policy that the
 * take cannot satisfy) — the Reserve fails and nothing is changed (Unreserve + ForgetPod). */
kg_status kg_row_reserve(const kg_config *cfg, kg_node_row *node, const kg_pod_row *pod, kg_cpu_info *cpus,
                         int32_t n_cpus, int32_t max_ref_count, int32_t numa_allocate_strategy, uint8_t *taken);

/* Reservation-aware Filter + Score of one (pod, node) pair on host rows through the kernels' per-pair
 * code (kg_rsv_pair): the node's reservation slots `rsv` (≤ KG_MAX_RSV_PER_NODE, in cache order) are
 * restored for the pod (transformer.go:49-291), Fit / LoadAware / NodeNUMAResource / Reservation.Filter
 * run on the restored NodeInfo, and *rsv_raw / *order / *nominated are the pod's PreScore inputs for this node
 * (scoreReservation of the nominated reservation, its order label, its slot; −1 none).  The
 * preferred-node override and NormalizeScore are per-pod reductions over nodes (not per pair). */
kg_status kg_row_eval_rsv(const kg_config *cfg, const kg_node_row *node, const kg_reservation *rsv, int32_t n_rsv,
                          const kg_pod_row *pod, int64_t now_ns, int32_t *feasible, int32_t *fit_score,
                          int32_t *la_score, int32_t *numa_score, int32_t *rsv_raw, int64_t *order,
                          int32_t *nominated);

/* The Reservation restore of one (pod, node) pair as the plugins see it (BeforePreFilter,
 * transformer.go:49-291): NodeInfo after restoring the unmatched reservations' remainders and removing
 * the matched reserve pods, and the nodeReservationState the Filter / nomination read. */
typedef struct kg_rsv_restored {
    int64_t requested[KG_NUM_RES];      /* NodeInfo.Requested after the restore */
    int64_t pod_requested[KG_NUM_RES];  /* nodeRState.podRequested (after the unmatched part) */
    int64_t r_allocated[KG_NUM_RES];    /* nodeRState.rAllocated (Σ Allocated of the matched) */
    int64_t nonzero[2];                 /* NodeInfo.NonZeroRequested after the restore */
    int32_t pod_count;                  /* len(NodeInfo.Pods) after the restore */
    int32_t n_matched;                  /* matched reservations (their slots: rsv[] order) */
    int32_t has_state;                  /* nodeReservationStates has the node */
    int32_t _pad;
} kg_rsv_restored;
kg_status kg_row_rsv_restore(const kg_config *cfg, const kg_node_row *node, const kg_reservation *rsv, int32_t n_rsv,
                             const kg_pod_row *pod, kg_rsv_restored *out);

/* Engine lifecycle. */
kg_status kg_engine_create(const kg_config *cfg, kg_engine **out);
void kg_engine_destroy(kg_engine *eng);
const char *kg_last_error(const kg_engine *eng);
kg_status kg_set_stream(kg_engine *eng, void *hip_stream); /* NULL ⇒ engine-owned stream */
kg_status kg_sync(kg_engine *eng);

/* Node snapshot (HBM-resident). */
kg_status kg_snapshot_reset(kg_engine *eng, int32_t n_nodes);
kg_status kg_snapshot_upsert(kg_engine *eng, const int32_t *node_index, const kg_node_row *rows, int32_t n);
kg_status kg_snapshot_remove(kg_engine *eng, int32_t node_index);
kg_status kg_snapshot_download(kg_engine *eng, int32_t first, int32_t n, kg_node_row *out);
/* Snapshot generation (SURVEY §5 error contract; replaces the Go cache's generation check in
 * Cache.UpdateSnapshot, a per-cycle staleness test): the count of successful snapshot mutations —
 * kg_snapshot_reset, kg_snapshot_upsert / _remove, kg_commit and each placement resolve (kg_place,
 * kg_place_chunk_resolve).  After a HIP error the device state is stale: this returns KG_ERR_STATE (with
 * the generation reached), every other entry point fails with KG_ERR_STATE, and the caller falls back to
 * the CPU plugins until kg_snapshot_reset + upsert reload the snapshot. */
kg_status kg_snapshot_generation(kg_engine *eng, uint64_t *out);

/* NodeNUMAResource's CPU accumulator on one node's logical CPUs: the cpuset a Reserve takes
 * (takeCPUs, nodenumaresource/cpu_accumulator.go:87-822) from `available` (per cpu id), with the node's
 * allocated CPUs' RefCount / ExclusivePolicy from `cpus`.  bind_policy / exclusive_policy:
 * kg_cpu_bind_policy / kg_cpu_exclusive_policy; numa_strategy: kg_scoring_strategy (NUMAAllocateStrategy).
 * KG_OK ⇔ `need` CPUs marked in result[n_cpus]; KG_NOT_FOUND ⇔ the accumulator fails.  The engine runs the
 * same code at Reserve in kg_place / kg_commit; exposed for host tools and tests. */
kg_status kg_cpuset_take(const kg_cpu_info *cpus, int32_t n_cpus, int32_t max_ref_count, const uint8_t *available,
                         int32_t need, int32_t bind_policy, int32_t exclusive_policy, int32_t numa_strategy,
                         uint8_t *result);
/* The logical CPUs of snapshot nodes (NodeNUMAResource's NodeAllocation.allocatedCPUs + CPUTopology +
 * ReservedCPUs, with MaxRefCount and the node's NUMA allocate strategy): for k < n, snapshot node
 * snap_index[k] takes the CPU detail of view node view_index[k] (either array NULL ⇔ k itself); a listed node
 * without CPU detail loses its table, unlisted nodes keep theirs (the feeders push the nodes an event
 * changed, next to their rows).  kg_snapshot_reset drops every table, kg_snapshot_remove the node's.
 * kg_place / kg_commit take cpusets from these tables at Reserve (the host runs the CPU accumulator for the
 * chosen node between device chunks) and write the node's cpuset counts back to its row.
 * kg_cpus_download reads one node's table (n = its CPU count). */
kg_status kg_cpus_set(kg_engine *eng, const kg_cluster_view *view, const int32_t *view_index, const int32_t *snap_index,
                      int32_t n);
kg_status kg_cpus_download(kg_engine *eng, int32_t node, kg_cpu_info *out, int32_t n);
/* Restrict kg_eval/kg_place evaluation to nodes [begin, end) (node sharding across GPUs);
 * node indices stay global.  begin must be a multiple of 1024 unless the shard is empty. */
kg_status kg_set_shard(kg_engine *eng, int32_t begin, int32_t end);

/* Pod batch (uploaded once; HBM-resident until replaced). */
kg_status kg_pods_set(kg_engine *eng, const kg_pod_row *pods, int32_t n_pods);

/* Matrix mode: every (pod, node) Filter+Score of the uploaded batch against the snapshot. */
kg_status kg_eval(kg_engine *eng, int64_t now_ns, const kg_eval_out *out);

/* Placement mode: schedule the uploaded batch in queue order exactly like the sequential
 * cycle (Filter all nodes → Score → argmax, lowest index on ties → Reserve), committing
 * each placement to the snapshot.  out_node[p] = node or −1, out_score[p] = total score
 * (−1 when unschedulable, or when its Reserve fails: a cpuset the CPU accumulator cannot take).
 * Pods that may bind a cpuset end their device chunk; their Reserve takes the CPUs on the host
 * (kg_cpus_set tables) before the next chunk is evaluated. */
kg_status kg_place(kg_engine *eng, int64_t now_ns, int32_t *out_node, int64_t *out_score);

/* Native multi-GPU placement: one engine per GPU, each holding the whole (replicated) snapshot and
 * restricted to its node shard (kg_set_shard).  kg_comm_unique_id (one rank) makes the RCCL id every rank passes
 * to kg_comm_init (librccl is loaded on first use; KG_ERR_UNSUPPORTED without it).  kg_place_sharded is kg_place
 * over the shards: per chunk each rank evaluates its tiles, the chunk's per-(pod, tile) partial keys are merged
 * with one ncclAllReduce(max) on the engine stream (beside the resolve in the pipelined form), and every rank runs
 * the same resolve and host Reserve steps (cpusets included) on identical inputs, so the replicas stay identical
 * and the placements equal kg_place's.  Every rank calls it with the same batch; outputs as kg_place. */
#define KG_COMM_ID_BYTES 128
kg_status kg_comm_unique_id(void *out /* KG_COMM_ID_BYTES */);
kg_status kg_comm_init(kg_engine *eng, int32_t rank, int32_t world, const void *unique_id);
/* The loopback communicator: the ranks (processes of one host, on one GPU or several) merge the partial keys
 * through a POSIX shared-memory segment `name` ("/…", the same on every rank; unlinked once every rank has joined)
 * instead of RCCL, running the same chunk loop — the rehearsal of kg_place_sharded where RCCL cannot form a
 * communicator (two ranks on one device).  Needs the snapshot loaded (the slots follow its tile count); a rank that
 * does not arrive within 120 s fails the others' waits with KG_ERR_STATE instead of hanging them. */
kg_status kg_comm_init_loopback(kg_engine *eng, int32_t rank, int32_t world, const char *name);
#define KG_COMM_NONE 0
#define KG_COMM_RCCL 1
#define KG_COMM_LOOPBACK 2
int32_t kg_comm_kind(const kg_engine *eng);
/* Failure contract: the ranks first agree (one status all-reduce) that each set up its loop; if any failed, none
 * enters it — that rank returns its error, the others KG_ERR_STATE, nothing is placed.  A step that fails inside
 * the loop (not a HIP fault) turns the rest of that rank's loop into merges of zero keys flagged as failed, so no
 * peer blocks in a collective; every rank then returns an error and is stale (reload the snapshot).  A HIP fault
 * leaves the device unusable: RCCL peers may then block in their next collective (loopback peers time out). */
kg_status kg_place_sharded(kg_engine *eng, int64_t now_ns, int32_t *out_node, int64_t *out_score);

/* Multi-GPU building blocks of kg_place (see koordinator_amd/dist.py); pods that bind cpusets are refused
 * here (KG_ERR_UNSUPPORTED: the sharded resolve has no host Reserve step):
 * chunk_eval writes per-(pod, 1024-node tile) partial keys of the shard for pods
 * [pod_begin, pod_begin+n) into partial_dev ([n][tiles_total][KG_PARTIAL_SLOTS] uint32, tile index
 * global; the caller zeroes nothing, chunk_eval clears the buffer's n rows itself);
 * chunk_resolve commits those pods sequentially given the partials of ALL tiles. */
int32_t kg_num_tiles(const kg_engine *eng);
kg_status kg_place_chunk_eval(kg_engine *eng, int64_t now_ns, int32_t pod_begin, int32_t n, uint32_t *partial_dev);
kg_status kg_place_chunk_resolve(kg_engine *eng, int64_t now_ns, int32_t pod_begin, int32_t n,
                                 const uint32_t *partial_dev, int32_t *out_node_dev, int64_t *out_score_dev);
/* The pipelined form (dist.place_sharded): chunk i + 1 is evaluated — on the eval stream, beside its partial
 * merge — while chunk i is resolved on the engine stream, so its partials may predate chunk i's commits.
 * kg_place_chunk_resolve_prev takes the nodes chunk i placed (prev_nodes_dev[0..n_prev), device, −1 = none)
 * and re-scores them like nodes this chunk touches (their keys in the lists are not trusted), exactly as the
 * one-GPU kg_place pipeline does.  The caller orders the streams: eval(i + 1) after resolve(i − 1), resolve(i)
 * after eval(i) and its merge.  Not with reservations (their per-pod entries are written by chunk_eval).
 * kg_set_eval_stream: the stream kg_place_chunk_eval launches on (NULL ⇒ the engine stream); no sync.  A resolve
 * waits (on the device) for the kg_place_chunk_eval that last wrote its partial_dev, not for later evaluations. */
kg_status kg_place_chunk_resolve_prev(kg_engine *eng, int64_t now_ns, int32_t pod_begin, int32_t n,
                                      const uint32_t *partial_dev, int32_t *out_node_dev, int64_t *out_score_dev,
                                      const int32_t *prev_nodes_dev, int32_t n_prev);
kg_status kg_set_eval_stream(kg_engine *eng, void *hip_stream);

/* Kernel forms the engine picks by batch and snapshot size, forced so that parity tests reach each form on
 * small clusters (0, the default: chosen by size).  Every form answers identically.
 *  KG_FORM_PLACE_PIPELINE    kg_place evaluates chunk i + 1 beside chunk i's resolve for every batch (by size:
 *                            NodeNUMAResource batches, whose chunk evaluation is long)
 *  KG_FORM_PLACE_SEQUENTIAL  kg_place never pipelines
 *  KG_FORM_NUMA_QUEUED       NodeNUMAResource matrix launches take the queued work-item form (by size: launches
 *                            with at least one work item per resident wave, and placement chunks)
 *  KG_FORM_NUMA_CHUNK_TILE   NodeNUMAResource placement chunks write one key per tile through the matrix kernel
 *                            (by size: chunks above 16 pods; smaller ones take per-tile top-16 lists)
 *  KG_FORM_NUMA_NO_CACHE     pipelined NodeNUMAResource placement evaluates every chunk pair by pair (by size: a
 *                            batch of repeated pod rows reads the distinct rows' outcomes from a per-node cache,
 *                            refreshed for each chunk's committed nodes)
 *  KG_FORM_NUMA_FUSED        NodeNUMAResource matrix launches evaluate Fit + LoadAware inside k_eval_numa2 (by size:
 *                            a matrix launch with planes runs the Fit + LoadAware pass first and k_eval_numa2
 *                            adds the NodeNUMAResource term to its planes) */
#define KG_FORM_PLACE_PIPELINE 0x1u
#define KG_FORM_PLACE_SEQUENTIAL 0x2u
#define KG_FORM_NUMA_QUEUED 0x4u
#define KG_FORM_NUMA_CHUNK_TILE 0x8u
#define KG_FORM_NUMA_NO_CACHE 0x10u
#define KG_FORM_NUMA_FUSED 0x20u
kg_status kg_set_forms(kg_engine *eng, uint32_t forms);

/* Reservation cache (KG_PLUGIN_RESERVATION): replaces every reservation slot; a node holds at most
 * KG_MAX_RSV_PER_NODE.  Nodes carrying slots are evaluated on the exact per-pair path with the
 * restore of transformer.go:49-291.  Under kg_set_shard every rank still evaluates every reservation
 * node (the slots are replicated): the per-pod preferred-reservation choice and Reservation
 * NormalizeScore's maximum (plugin.go Score / NormalizeScore) are global and identical on each rank,
 * the planes cover the shard's columns only, and top1 includes every reservation node, so a max over
 * the ranks' top1 keys equals the unsharded result.
 * kg_rsv_download returns the slots (allocated / n_assigned after placements) in kg_rsv_set order. */
#define KG_MAX_RSV_PER_NODE 16
kg_status kg_rsv_set(kg_engine *eng, const kg_reservation *rsv, int32_t n);
kg_status kg_rsv_download(kg_engine *eng, kg_reservation *out, int32_t n);
/* ElasticQuota groups (KG_PLUGIN_ELASTICQUOTA); kg_pod_row.quota indexes them. */
kg_status kg_quota_set(kg_engine *eng, const kg_quota *q, int32_t n);
kg_status kg_quota_download(kg_engine *eng, kg_quota *out, int32_t n);

/* Single Reserve on the device snapshot (pod = index in the uploaded batch); a cpuset pod takes its CPUs
 * from the node's kg_cpus_set table.  KG_NOT_FOUND ⇔ its Allocate fails (nothing changed). */
kg_status kg_commit(kg_engine *eng, int32_t pod, int32_t node);

/* Measurement: when on, every k_eval launch (kg_eval, kg_place_chunk_eval) is bracketed by a
 * pair of HIP events on the engine stream (ring of 256).  kg_eval_kernel_times writes the
 * durations (ms) of the last min(n, recorded) launches, oldest first, and returns that count
 * (< 0 on error). */
kg_status kg_set_profiling(kg_engine *eng, int32_t on);
int32_t kg_eval_kernel_times(kg_engine *eng, float *ms, int32_t n);

/* Engine counters since creation or kg_counters_reset (SURVEY §5 "Metrics"; the reference's analogue is the
 * scheduler's Prometheus set, pkg/scheduler/metrics/metrics.go:28-41): pod×node pairs evaluated (matrix mode
 * and placement chunk evaluations), matrix-mode output bytes written, pods walked by placement resolves and
 * pods placed (kg_place / kg_commit, where the outcome reaches the host), host→device bytes uploaded, and the
 * device time of the k_eval launches timed under kg_set_profiling (evals ÷ that time = evals/s, output
 * bytes ÷ it = the achieved write rate). */
typedef struct kg_counters {
    uint64_t eval_calls;        /* kg_eval + kg_place_chunk_eval calls */
    uint64_t evals;             /* pod × node pairs evaluated */
    uint64_t out_bytes;         /* mask + score planes + top-1 bytes written by matrix mode */
    uint64_t resolved;          /* pods walked by placement resolves (kg_place, kg_place_chunk_resolve*) */
    uint64_t placed;            /* pods placed by kg_place / kg_commit */
    uint64_t h2d_bytes;         /* host → device bytes (snapshot rows, pod rows, class tables, reservations, ...) */
    uint64_t timed_launches;    /* k_eval launches whose device time is in kernel_ns */
    uint64_t kernel_ns;         /* their device time (HIP events, kg_set_profiling) */
} kg_counters;
kg_status kg_counters_get(kg_engine *eng, kg_counters *out);
kg_status kg_counters_reset(kg_engine *eng);

/* Helpers for consumers of matrix-mode output. */
static inline int kg_mask_test(const uint64_t *mask, int32_t n_nodes, int32_t p, int32_t n) {
    int32_t words = (n_nodes + 63) / 64;
    return (int)((mask[(int64_t)p * words + n / 64] >> (n % 64)) & 1u);
}

#ifdef __cplusplus
}
#endif
#endif /* KOORD_GPU_H */
