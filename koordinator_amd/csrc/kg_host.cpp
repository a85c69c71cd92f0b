// kg_host.cpp — host side of the engine: plugin args, and the row builders that turn the
// objects a koord-scheduler plugin reads from its informers (Pod, Node/NodeInfo, NodeMetric,
// podAssignCache) into the pod-only / node-only rows the HIP kernels consume.
//
// Everything that does not depend on the (pod, node) pair is hoisted here:
//   pod rows   NodeResourcesFit PreFilter request (upstream fit.go computePodResourceRequest; in-repo
//              mirror reservation/transformer.go:316-346), Fit score pod request (upstream
//              resource_allocation.go calculatePodResourceRequest), EstimatePod
//              (loadaware/estimator/default_estimator.go:57-108), priority class
//              (apis/extension/priority_utils.go:26-47), isDaemonSetPod (loadaware/helper.go:189-196)
//   node rows  EstimateNode (default_estimator.go:110-129); the threshold checks of LoadAware.Filter
//              (load_aware.go:149-254) for a non-prod and a prod pod; the node-side terms of
//              LoadAware.Score (load_aware.go:291-327 + estimatedAssignedPodUsed :337-376) for the
//              non-prod and the prod-usage variant.
// Time-dependent checks (NodeMetric expiry) stay in the kernels, which take `now`.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "kg_common.h"
#include "kg_host.h"

namespace {

constexpr int64_t kDefaultMilliCPU = 250;                       // default_estimator.go:36
constexpr int64_t kDefaultMemory = 200LL * 1024 * 1024;         // default_estimator.go:38
constexpr int64_t kNonZeroMilliCPU = 100;                        // upstream schedutil.DefaultMilliCPURequest
constexpr int64_t kNonZeroMemory = 200LL * 1024 * 1024;          // upstream schedutil.DefaultMemoryRequest

inline bool bit(uint32_t m, int r) { return (m >> r) & 1u; }
inline bool scalar_res(int r) { return bit(KG_SCALAR_RES_MASK, r); }
inline int64_t val(const kg_resource_list &l, int r) { return bit(l.present, r) ? l.v[r] : 0; }
inline int nkeys(const kg_resource_list &l) { return __builtin_popcount(l.present); }

void set_thr(kg_resource_list &l, int r, int64_t v) {
    l.v[r] = v;
    l.present |= 1u << r;
}

// ---- pod classification ----------------------------------------------------------------

struct PodView {
    const kg_cluster_view &v;
    const kg_pod_spec &p;
    const kg_container &container(int i) const { return v.containers[p.first_container + i]; }
    const kg_container &init(int i) const { return v.containers[p.first_init_container + i]; }
};

// corev1 qos helper (k8s v1.24 GetPodQOS), cpu and memory only
int kube_qos_of(const PodView &pv) {
    if (pv.p.status_qos != KG_KUBE_QOS_UNSET) return pv.p.status_qos;
    int64_t req[2] = {0, 0}, lim[2] = {0, 0};
    bool rq[2] = {false, false}, lm[2] = {false, false};
    bool guaranteed = true;
    auto visit = [&](const kg_container &c) {
        int found = 0;
        for (int r = 0; r < 2; r++) {
            if (bit(c.requests.present, r) && c.requests.v[r] > 0) { req[r] += c.requests.v[r]; rq[r] = true; }
            if (bit(c.limits.present, r) && c.limits.v[r] > 0) { lim[r] += c.limits.v[r]; lm[r] = true; found |= 1 << r; }
        }
        if (found != 3) guaranteed = false;
    };
    for (int i = 0; i < pv.p.n_containers; i++) visit(pv.container(i));
    for (int i = 0; i < pv.p.n_init_containers; i++) visit(pv.init(i));
    if (!rq[0] && !rq[1] && !lm[0] && !lm[1]) return KG_KUBE_QOS_BESTEFFORT;
    for (int r = 0; r < 2 && guaranteed; r++)
        if (rq[r] && (!lm[r] || lim[r] != req[r])) guaranteed = false;
    if (guaranteed && (int(rq[0]) + int(rq[1])) == (int(lm[0]) + int(lm[1]))) return KG_KUBE_QOS_GUARANTEED;
    return KG_KUBE_QOS_BURSTABLE;
}

int priority_class_of(const PodView &pv) {
    int pc = KG_PRIO_NONE;
    if (pv.p.label_priority_class >= 0) {
        pc = pv.p.label_priority_class;
    } else if (pv.p.has_priority) {
        const int32_t x = pv.p.priority;
        pc = (x >= 9000 && x <= 9999)   ? KG_PRIO_PROD
             : (x >= 7000 && x <= 7999) ? KG_PRIO_MID
             : (x >= 5000 && x <= 5999) ? KG_PRIO_BATCH
             : (x >= 3000 && x <= 3999) ? KG_PRIO_FREE
                                        : KG_PRIO_NONE;
    }
    if (pc != KG_PRIO_NONE) return pc;
    int qos = KG_QOS_NONE;
    if (pv.p.label_qos > KG_QOS_NONE) {
        qos = pv.p.label_qos;
    } else {
        switch (kube_qos_of(pv)) {
            case KG_KUBE_QOS_GUARANTEED: qos = KG_QOS_LSR; break;
            case KG_KUBE_QOS_BURSTABLE: qos = KG_QOS_LS; break;
            case KG_KUBE_QOS_BESTEFFORT: qos = KG_QOS_BE; break;
        }
    }
    if (qos == KG_QOS_SYSTEM || qos == KG_QOS_LSE || qos == KG_QOS_LSR || qos == KG_QOS_LS) return KG_PRIO_PROD;
    if (qos == KG_QOS_BE) return KG_PRIO_BATCH;
    return KG_PRIO_NONE;
}

// PodRequestsAndLimits: sums over containers, max with init containers, + overhead
void requests_and_limits(const PodView &pv, kg_resource_list &req, kg_resource_list &lim) {
    memset(&req, 0, sizeof(req));
    memset(&lim, 0, sizeof(lim));
    for (int i = 0; i < pv.p.n_containers; i++) {
        const kg_container &c = pv.container(i);
        for (int r = 0; r < KG_NUM_RES; r++) {
            if (bit(c.requests.present, r)) set_thr(req, r, val(req, r) + c.requests.v[r]);
            if (bit(c.limits.present, r)) set_thr(lim, r, val(lim, r) + c.limits.v[r]);
        }
    }
    for (int i = 0; i < pv.p.n_init_containers; i++) {
        const kg_container &c = pv.init(i);
        for (int r = 0; r < KG_NUM_RES; r++) {
            if (bit(c.requests.present, r) && (!bit(req.present, r) || c.requests.v[r] > req.v[r])) set_thr(req, r, c.requests.v[r]);
            if (bit(c.limits.present, r) && (!bit(lim.present, r) || c.limits.v[r] > lim.v[r])) set_thr(lim, r, c.limits.v[r]);
        }
    }
    for (int r = 0; r < KG_NUM_RES; r++) {
        if (!bit(pv.p.overhead.present, r)) continue;
        set_thr(req, r, val(req, r) + pv.p.overhead.v[r]);
        if (bit(lim.present, r)) lim.v[r] += pv.p.overhead.v[r];
    }
}

int translate_resource(int pc, int r) {  // -1 ⇔ "" (no such resource)
    if (pc == KG_PRIO_PROD || pc == KG_PRIO_NONE) return r;
    if (r != KG_RES_CPU && r != KG_RES_MEMORY) return -1;
    if (pc == KG_PRIO_BATCH) return r == KG_RES_CPU ? KG_RES_BATCH_CPU : KG_RES_BATCH_MEMORY;
    if (pc == KG_PRIO_MID) return r == KG_RES_CPU ? KG_RES_MID_CPU : KG_RES_MID_MEMORY;
    return -1;
}

// EstimatePod (default_estimator.go:57-70): every resource resourceWeights names (0 elsewhere)
void estimate_pod(const kg_config &cfg, const PodView &pv, int64_t out[KG_NUM_RES]) {
    kg_resource_list req, lim;
    requests_and_limits(pv, req, lim);
    const int pc = priority_class_of(pv);
    for (int r = 0; r < KG_NUM_RES; r++) {
        out[r] = 0;
        if (cfg.la_resource_weight[r] == 0) continue;
        const int real = translate_resource(pc, r);
        if (real < 0) continue;
        int64_t limit = val(lim, real), request = val(req, real), q, scaling = cfg.la_scaling_factor[r];
        if (limit > request) {
            q = limit;
            scaling = 100;
        } else {
            q = request;
        }
        if (q == 0) {
            out[r] = (real == KG_RES_CPU || real == KG_RES_BATCH_CPU)          ? kDefaultMilliCPU
                     : (real == KG_RES_MEMORY || real == KG_RES_BATCH_MEMORY) ? kDefaultMemory
                                                                              : 0;
            continue;
        }
        int64_t e = (int64_t)round((double)q * (double)scaling / 100.0);
        if (limit > 0 && e > limit) e = limit;
        out[r] = e;
    }
}

// schedutil.GetRequestForResource(r, requests, nonZero=true) for one container
int64_t nonzero_request_of(const kg_resource_list &rq, int r) {
    if (!bit(rq.present, r)) return r == KG_RES_CPU ? kNonZeroMilliCPU : r == KG_RES_MEMORY ? kNonZeroMemory : 0;
    return rq.v[r];
}

// ---- node-side LoadAware ---------------------------------------------------------------------

void estimate_node(const kg_node_spec &n, kg_resource_list &out) {
    out = n.allocatable;
    if (n.raw_allocatable_state != 1 || n.raw_allocatable.present == 0) return;
    bool same = n.raw_allocatable.present == n.allocatable.present;
    for (int r = 0; same && r < KG_NUM_RES; r++)
        if (bit(n.raw_allocatable.present, r) && n.raw_allocatable.v[r] != n.allocatable.v[r]) same = false;
    if (same) return;
    for (int r = 0; r < KG_NUM_RES; r++)
        if (bit(n.raw_allocatable.present, r)) set_thr(out, r, n.raw_allocatable.v[r]);
}

const kg_resource_list *aggregated_usage(const kg_cluster_view &v, const kg_node_spec &n, int64_t duration_ns, int type) {
    if (!n.has_node_metric_info || n.n_aggregated == 0) return nullptr;
    const kg_aggregated_usage *a = v.aggregated + n.first_aggregated;
    if (duration_ns == 0) {
        int best = 0;
        int64_t best_d = 0;
        for (int i = 0; i < n.n_aggregated; i++)
            if (a[i].duration_ns > best_d) { best_d = a[i].duration_ns; best = i; }
        return nkeys(a[best].usage[type]) ? &a[best].usage[type] : nullptr;
    }
    for (int i = 0; i < n.n_aggregated; i++)
        if (a[i].duration_ns == duration_ns && nkeys(a[i].usage[type])) return &a[i].usage[type];
    return nullptr;
}

struct Thresholds {
    kg_resource_list usage{}, prod{};
    bool agg = false;
    kg_resource_list agg_thr{};
    int agg_type = 0;
    int64_t agg_dur = 0;
};

Thresholds thresholds_of(const kg_config &c, const kg_node_spec &n) {
    Thresholds t;
    const bool args_agg = c.la_has_aggregated && nkeys(c.la_agg_usage_thresholds) > 0 && c.la_agg_usage_type != KG_AGG_UNSET;
    if (n.custom_thresholds_state == 1) {
        t.usage = n.custom_usage_thresholds;
        t.prod = n.custom_prod_usage_thresholds;
        if (n.custom_has_aggregated && nkeys(n.custom_agg_usage_thresholds) > 0 && n.custom_agg_usage_type != KG_AGG_UNSET) {
            t.agg = true;
            t.agg_thr = n.custom_agg_usage_thresholds;
            t.agg_type = n.custom_agg_usage_type;
            t.agg_dur = n.custom_agg_duration_ns;
        }
    }
    if (!nkeys(t.usage)) t.usage = c.la_usage_thresholds;
    if (!nkeys(t.prod)) t.prod = c.la_prod_usage_thresholds;
    if (!t.agg && args_agg) {
        t.agg = true;
        t.agg_thr = c.la_agg_usage_thresholds;
        t.agg_type = c.la_agg_usage_type;
        t.agg_dur = c.la_agg_usage_duration_ns;
    }
    return t;
}

bool exceeds(const kg_resource_list &thr, const kg_resource_list &alloc, const kg_resource_list *used) {
    for (int r = 0; r < KG_NUM_RES; r++) {
        if (!bit(thr.present, r) || thr.v[r] == 0) continue;
        const int64_t total = val(alloc, r);
        if (total == 0 || used == nullptr) continue;
        const int64_t scale = r == KG_RES_CPU ? 1 : 1000;  // Quantity.MilliValue
        const double ratio = (double)(val(*used, r) * scale) / (double)(total * scale);
        if ((int64_t)round(ratio * 100.0) >= thr.v[r]) return true;
    }
    return false;
}

struct MetricIndex {  // buildPodMetricMap: name → usage (last entry wins)
    std::unordered_map<int64_t, const kg_resource_list *> usage;
    std::vector<int64_t> order;
};

MetricIndex pod_metric_map(const kg_cluster_view &v, const kg_node_spec &n, bool prod_only) {
    MetricIndex m;
    for (int i = 0; i < n.n_pod_metric; i++) {
        const kg_pod_metric &pm = v.pod_metrics[n.first_pod_metric + i];
        if (pm.lister_pod < 0) continue;
        if (prod_only && priority_class_of(PodView{v, v.pods[pm.lister_pod]}) != KG_PRIO_PROD) continue;
        if (!m.usage.count(pm.name_id)) m.order.push_back(pm.name_id);
        m.usage[pm.name_id] = &pm.usage;
    }
    return m;
}

// node-side sum of LoadAware.Score for one variant (0 = non-prod, 1 = prod usage)
void loadaware_node_term(const kg_config &c, const kg_cluster_view &v, const kg_node_spec &n, int variant,
                         int64_t out[KG_NUM_RES]) {
    const bool prod = variant == 1;
    const MetricIndex pm = pod_metric_map(v, n, prod);
    const bool score_agg = c.la_has_aggregated && c.la_agg_score_type != KG_AGG_UNSET;
    const kg_resource_list *agg = score_agg ? aggregated_usage(v, n, c.la_agg_score_duration_ns, c.la_agg_score_type) : nullptr;
    const int64_t upd = n.has_update_time ? n.update_time_ns : INT64_MIN;
    const int64_t interval = (n.has_report_interval ? n.report_interval_seconds : 60) * 1000000000LL;
    for (int r = 0; r < KG_NUM_RES; r++) out[r] = 0;
    std::unordered_set<int64_t> estimated;
    for (int i = 0; i < n.n_assigned; i++) {
        const kg_assigned_pod &a = v.assigned[n.first_assigned + i];
        const PodView ap{v, v.pods[a.pod]};
        if (prod && priority_class_of(ap) != KG_PRIO_PROD) continue;
        auto it = pm.usage.find(ap.p.name_id);
        const kg_resource_list *usage = it == pm.usage.end() ? nullptr : it->second;
        const bool recent = a.timestamp_ns > upd || (a.timestamp_ns < upd && upd - a.timestamp_ns < interval);
        if (usage == nullptr || nkeys(*usage) == 0 || recent || (score_agg && agg == nullptr)) {
            int64_t est[KG_NUM_RES];
            estimate_pod(c, ap, est);
            for (int r = 0; r < KG_NUM_RES; r++) {
                if (c.la_resource_weight[r] == 0) continue;
                int64_t x = est[r];
                if (usage && bit(usage->present, r) && usage->v[r] > x) x = usage->v[r];
                out[r] += x;
            }
            estimated.insert(ap.p.name_id);
        }
    }
    int64_t actual[KG_NUM_RES] = {}, est_actual[KG_NUM_RES] = {};
    for (int64_t name : pm.order) {
        const kg_resource_list *u = pm.usage.at(name);
        int64_t *dst = estimated.count(name) ? est_actual : actual;
        for (int r = 0; r < KG_NUM_RES; r++) dst[r] += val(*u, r);
    }
    if (prod) {
        for (int r = 0; r < KG_NUM_RES; r++) out[r] += actual[r];
    } else if (n.has_node_metric_info) {
        const kg_resource_list *nu = score_agg ? agg : &n.node_usage;
        if (nu) {
            for (int r = 0; r < KG_NUM_RES; r++) {
                if (!bit(nu->present, r)) continue;
                int64_t q = nu->v[r];
                if (est_actual[r] != 0 && q >= est_actual[r]) q -= est_actual[r];
                out[r] += q;
            }
        }
    }
}

}  // namespace

extern "C" {

int32_t kg_abi_version(void) { return KG_ABI_VERSION; }

int64_t kg_struct_size(int32_t sid) {
    switch (sid) {
        case KG_SID_RESOURCE_LIST: return sizeof(kg_resource_list);
        case KG_SID_CONFIG: return sizeof(kg_config);
        case KG_SID_CONTAINER: return sizeof(kg_container);
        case KG_SID_POD_SPEC: return sizeof(kg_pod_spec);
        case KG_SID_AGGREGATED_USAGE: return sizeof(kg_aggregated_usage);
        case KG_SID_POD_METRIC: return sizeof(kg_pod_metric);
        case KG_SID_ASSIGNED_POD: return sizeof(kg_assigned_pod);
        case KG_SID_NODE_SPEC: return sizeof(kg_node_spec);
        case KG_SID_CLUSTER_VIEW: return sizeof(kg_cluster_view);
        case KG_SID_POD_ROW: return sizeof(kg_pod_row);
        case KG_SID_NODE_ROW: return sizeof(kg_node_row);
        case KG_SID_EVAL_OUT: return sizeof(kg_eval_out);
        case KG_SID_NUMA_SPEC: return sizeof(kg_numa_spec);
        case KG_SID_RESERVATION: return sizeof(kg_reservation);
        case KG_SID_QUOTA: return sizeof(kg_quota);
        case KG_SID_RSV_RESTORED: return sizeof(kg_rsv_restored);
        case KG_SID_CPU_INFO: return sizeof(kg_cpu_info);
        case KG_SID_COUNTERS: return sizeof(kg_counters);
    }
    return -1;
}

void kg_config_default(kg_config *c) {
    memset(c, 0, sizeof(*c));
    c->abi_version = KG_ABI_VERSION;
    c->enabled_plugins = KG_PLUGIN_FIT | KG_PLUGIN_LOADAWARE;
    c->weight_fit = 1;
    c->weight_loadaware = 1;
    c->fit_strategy = KG_STRATEGY_LEAST_ALLOCATED;
    c->fit_resource_weight[KG_RES_CPU] = 1;
    c->fit_resource_weight[KG_RES_MEMORY] = 1;
    // v1beta2/defaults.go:32-48, 78-100
    c->la_filter_expired_node_metrics = 1;
    c->la_has_expiration = 1;
    c->la_expiration_seconds = 180;
    c->la_resource_weight[KG_RES_CPU] = 1;
    c->la_resource_weight[KG_RES_MEMORY] = 1;
    set_thr(c->la_usage_thresholds, KG_RES_CPU, 65);
    set_thr(c->la_usage_thresholds, KG_RES_MEMORY, 95);
    c->la_scaling_factor[KG_RES_CPU] = 85;
    c->la_scaling_factor[KG_RES_MEMORY] = 70;
    // SetDefaults_NodeNUMAResourceArgs (v1beta2/defaults.go:101-137): LeastAllocated cpu:1 memory:1 for both
    c->weight_numa = 1;
    c->numa_strategy = KG_STRATEGY_LEAST_ALLOCATED;
    c->numa_hint_strategy = KG_STRATEGY_LEAST_ALLOCATED;
    c->numa_default_cpu_bind_policy = KG_CPU_BIND_FULL_PCPUS;   // v1beta2 defaults.go:50
    c->numa_resource_weight[KG_RES_CPU] = 1;
    c->numa_resource_weight[KG_RES_MEMORY] = 1;
    c->place_chunk = 16;
    snprintf(c->ext_resource_names[0], KG_RES_NAME_MAX, "%s", "example.com/gpu");
}

}  // extern "C"

// the resource-name keys of the slots: the fixed ones, then kg_config.ext_resource_names ("" ⇔ unused)
const char *kg_res_name(const kg_config &c, int r) {
    static const char *const fixed[KG_RES_EXT0] = {"cpu", "memory", "ephemeral-storage", "kubernetes.io/batch-cpu",
                                                   "kubernetes.io/batch-memory", "kubernetes.io/mid-cpu",
                                                   "kubernetes.io/mid-memory"};
    return r < KG_RES_EXT0 ? fixed[r] : c.ext_resource_names[r - KG_RES_EXT0];
}

// resource ids by name (Go string order, bytewise); unused slots last
void kg_res_sorted_order(const kg_config &c, int8_t out[KG_NUM_RES]) {
    int ids[KG_NUM_RES];
    for (int r = 0; r < KG_NUM_RES; r++) ids[r] = r;
    std::stable_sort(ids, ids + KG_NUM_RES, [&](int a, int b) {
        const char *na = kg_res_name(c, a), *nb = kg_res_name(c, b);
        if (!na[0] || !nb[0]) return na[0] && !nb[0];
        return strcmp(na, nb) < 0;
    });
    for (int r = 0; r < KG_NUM_RES; r++) out[r] = (int8_t)ids[r];
}

extern "C" {

void kg_config_shipped_profile(kg_config *c) {
    // config/manager/scheduler-config.yaml:17-45
    c->fit_resource_weight[KG_RES_BATCH_CPU] = 1;
    c->fit_resource_weight[KG_RES_BATCH_MEMORY] = 1;
    c->la_filter_expired_node_metrics = 0;
    c->la_has_expiration = 1;
    c->la_expiration_seconds = 300;
    c->weight_reservation = 5000;  // scheduler-config.yaml:82-91
}

kg_status kg_config_validate(const kg_config *c, char *err, int32_t err_len) {
    auto fail = [&](const char *m) {
        if (err && err_len > 0) snprintf(err, (size_t)err_len, "%s", m);
        return KG_ERR_INVALID_ARG;
    };
    if (!c) return fail("null config");
    if (c->abi_version != KG_ABI_VERSION) return fail("abi_version mismatch");
    if (c->enabled_plugins &
        ~(KG_PLUGIN_FIT | KG_PLUGIN_LOADAWARE | KG_PLUGIN_NUMA | KG_PLUGIN_RESERVATION | KG_PLUGIN_ELASTICQUOTA))
        return fail("unsupported plugin bit");
    if (c->eq_check_parent_quota != 0 && c->eq_check_parent_quota != 1) return fail("eq_check_parent_quota must be 0 or 1");
    int64_t fw = 0, lw = 0, nw = 0;
    for (int r = 0; r < KG_NUM_RES; r++) {
        if (c->fit_resource_weight[r] < 0 || c->la_resource_weight[r] < 0 || c->numa_resource_weight[r] < 0)
            return fail("negative resource weight");
        fw += c->fit_resource_weight[r];
        lw += c->la_resource_weight[r];
        nw += c->numa_resource_weight[r];
    }
    if (fw > 600 || lw > 600 || nw > 600) return fail("resource weight sum too large (max 600)");
    if ((c->enabled_plugins & KG_PLUGIN_NUMA) && nw == 0) return fail("NodeNUMAResource needs scoringStrategy resources");
    if (c->numa_strategy != KG_STRATEGY_LEAST_ALLOCATED && c->numa_strategy != KG_STRATEGY_MOST_ALLOCATED)
        return fail("unsupported NodeNUMAResource scoring strategy");
    if (c->numa_default_cpu_bind_policy != KG_CPU_BIND_UNSET && c->numa_default_cpu_bind_policy != KG_CPU_BIND_FULL_PCPUS &&
        c->numa_default_cpu_bind_policy != KG_CPU_BIND_SPREAD_BY_PCPUS &&
        c->numa_default_cpu_bind_policy != KG_CPU_BIND_CONSTRAINED_BURST)
        return fail("unsupported NodeNUMAResource defaultCPUBindPolicy");
    if (c->numa_hint_strategy != KG_STRATEGY_LEAST_ALLOCATED && c->numa_hint_strategy != KG_STRATEGY_MOST_ALLOCATED)
        return fail("unsupported NodeNUMAResource NUMA scoring strategy");
    if ((c->enabled_plugins & KG_PLUGIN_LOADAWARE) && lw == 0) return fail("LoadAwareScheduling needs resourceWeights");
    // totals are packed as ((total + 1) << 10) | node into 32-bit per-tile keys: 100·Σweights < 2^22
    if (c->weight_fit < 0 || c->weight_loadaware < 0 || c->weight_numa < 0 || c->weight_reservation < 0 ||
        (int64_t)c->weight_fit + c->weight_loadaware + ((c->enabled_plugins & KG_PLUGIN_NUMA) ? c->weight_numa : 0) +
                ((c->enabled_plugins & KG_PLUGIN_RESERVATION) ? c->weight_reservation : 0) >
            40000)
        return fail("plugin weight out of range (each >= 0, sum <= 40000)");
    if (c->fit_strategy != KG_STRATEGY_LEAST_ALLOCATED && c->fit_strategy != KG_STRATEGY_MOST_ALLOCATED)
        return fail("unsupported NodeResourcesFit scoring strategy");
    // kg_place: 0 ⇒ the default chunk (8); at most the resolve kernel's touched-list capacity
    if (c->place_chunk < 0 || c->place_chunk > KG_PLACE_CHUNK_MAX) return fail("place_chunk out of range (0..1024)");
    // the named scalar slots: NUL-terminated, printable, distinct, none a fixed name
    for (int i = 0; i < KG_NUM_EXT_RES; i++) {
        const char *n = c->ext_resource_names[i];
        if (!memchr(n, 0, KG_RES_NAME_MAX)) return fail("ext_resource_names: a name is not NUL-terminated");
        for (const char *q = n; *q; q++)
            if ((unsigned char)*q <= ' ' || (unsigned char)*q >= 127) return fail("ext_resource_names: unprintable name");
        if (!n[0]) continue;
        for (int r = 0; r < KG_NUM_RES; r++)
            if (r != KG_RES_EXT0 + i && !strcmp(n, kg_res_name(*c, r)))
                return fail("ext_resource_names: a name repeats or is a fixed resource name");
    }
    return KG_OK;
}

kg_status kg_build_pod_rows(const kg_config *cfg, const kg_cluster_view *view, const int32_t *pod_index, int32_t n,
                            kg_pod_row *out) {
    if (!cfg || !view || (!pod_index && n > 0) || (!out && n > 0) || n < 0) return KG_ERR_INVALID_ARG;
    for (int32_t k = 0; k < n; k++) {
        const int32_t pi = pod_index[k];
        if (pi < 0 || pi >= view->n_pods) return KG_ERR_RANGE;
        const PodView pv{*view, view->pods[pi]};
        kg_pod_row &row = out[k];
        memset(&row, 0, sizeof(row));
        // Fit PreFilter request: Resource.Add per container, SetMaxResource per init container, + overhead
        uint32_t keys = 0;
        for (int i = 0; i < pv.p.n_containers; i++) {
            const kg_resource_list &rq = pv.container(i).requests;
            for (int r = 0; r < KG_NUM_RES; r++)
                if (bit(rq.present, r)) { row.request[r] += rq.v[r]; if (scalar_res(r)) keys |= 1u << r; }
        }
        for (int i = 0; i < pv.p.n_init_containers; i++) {
            const kg_resource_list &rq = pv.init(i).requests;
            for (int r = 0; r < KG_NUM_RES; r++) {
                if (!bit(rq.present, r)) continue;
                if (rq.v[r] > row.request[r] || (scalar_res(r) && !bit(keys, r))) row.request[r] = std::max(row.request[r], rq.v[r]);
                if (scalar_res(r)) keys |= 1u << r;
            }
        }
        for (int r = 0; r < KG_NUM_RES; r++)
            if (bit(pv.p.overhead.present, r)) { row.request[r] += pv.p.overhead.v[r]; if (scalar_res(r)) keys |= 1u << r; }
        row.request_present = keys;
        if (row.request[KG_RES_CPU] || row.request[KG_RES_MEMORY] || row.request[KG_RES_EPHEMERAL_STORAGE] || keys)
            row.flags |= KG_POD_HAS_REQUEST;
        // Fit score pod request and AssumePod NonZeroRequested delta
        for (int r = 0; r < KG_NUM_RES; r++) {
            int64_t s = 0;
            for (int i = 0; i < pv.p.n_containers; i++) s += nonzero_request_of(pv.container(i).requests, r);
            for (int i = 0; i < pv.p.n_init_containers; i++) s = std::max(s, nonzero_request_of(pv.init(i).requests, r));
            int64_t nz = s;
            if (bit(pv.p.overhead.present, r)) {
                const int64_t o = pv.p.overhead.v[r];
                nz += o;
                s += r == KG_RES_CPU ? (o + 999) / 1000 : o;  // upstream adds Quantity.Value() here
            }
            row.fit_score_request[r] = s;
            if (r < 2) row.nonzero_request[r] = nz;
        }
        {
            int64_t est[KG_NUM_RES];
            estimate_pod(*cfg, pv, est);
            row.la_estimate[0] = est[KG_RES_CPU];
            row.la_estimate[1] = est[KG_RES_MEMORY];
            for (int r = 2; r < KG_NUM_RES; r++) row.la_estimate_x[r - 2] = est[r];
        }
        // NodeNUMAResource PreFilter (plugin.go:219-269): PodRequestsAndLimits requests; skip when all zero
        {
            kg_resource_list nreq, nlim;
            requests_and_limits(pv, nreq, nlim);
            bool all_zero = true;
            for (int r = 0; r < KG_NUM_RES; r++) {
                row.numa_request[r] = val(nreq, r);
                if (row.numa_request[r] != 0) all_zero = false;
            }
            row.numa_request_present = nreq.present;
            if (all_zero) row.flags |= KG_POD_NUMA_SKIP;
        }
        const int pc = priority_class_of(pv);
        // PreFilter's cpuset decision (plugin.go:232-262) for AllowUseCPUSet pods (util.go:43-50: raw QoS
        // label LSE / LSR and koord-prod): the preferred policy falls back to DefaultCPUBindPolicy when
        // unset or Default, a required Default means DefaultCPUBindPolicy, and a required policy wins
        if (!(row.flags & KG_POD_NUMA_SKIP) && (pv.p.label_qos == KG_QOS_LSE || pv.p.label_qos == KG_QOS_LSR) &&
            pc == KG_PRIO_PROD) {
            const int32_t dflt = cfg->numa_default_cpu_bind_policy;
            int32_t bind = pv.p.cpu_bind_preferred;
            if (bind == KG_CPU_BIND_UNSET || bind == KG_CPU_BIND_DEFAULT) bind = dflt;
            int32_t required = pv.p.cpu_bind_required;
            if (required == KG_CPU_BIND_DEFAULT) required = dflt;
            if (required != KG_CPU_BIND_UNSET) bind = required;
            if (required < 0 || required > KG_CPU_BIND_OTHER || bind < 0 || bind > KG_CPU_BIND_OTHER ||
                pv.p.cpu_exclusive < 0 || pv.p.cpu_exclusive > KG_CPU_EXCL_NUMA_NODE_LEVEL)
                return KG_ERR_INVALID_ARG;
            const int64_t cpu = row.numa_request[KG_RES_CPU];
            if (bind == KG_CPU_BIND_FULL_PCPUS || bind == KG_CPU_BIND_SPREAD_BY_PCPUS) {
                if (cpu % 1000 != 0) {
                    row.flags |= KG_POD_NUMA_BIND_INVALID;   // ErrInvalidRequestedCPUs
                } else if (cpu > 0) {
                    row.flags |= KG_POD_NUMA_CPU_BIND;
                    row.cpu_bind = (uint32_t)required | (uint32_t)bind << 4 | (uint32_t)pv.p.cpu_exclusive << 8;
                }
            }
        }
        if (pc == KG_PRIO_PROD) row.flags |= KG_POD_PROD;
        if (pc == KG_PRIO_PROD && cfg->la_score_according_prod_usage) row.flags |= KG_POD_LA_PROD_SCORE;
        if (pv.p.is_daemonset) row.flags |= KG_POD_DAEMONSET;
        if (pv.p.non_preemptible) row.flags |= KG_POD_NON_PREEMPTIBLE;
        row.rsv_owner_class = pv.p.rsv_owner_class;
        row.rsv_affinity_class = pv.p.rsv_affinity_class;
        row.quota = pv.p.quota;
        row.flags |= KG_POD_VALID;
    }
    return KG_OK;
}

kg_status kg_build_node_rows(const kg_config *cfg, const kg_cluster_view *view, const int32_t *node_index, int32_t n,
                             kg_node_row *out) {
    if (!cfg || !view || (!node_index && n > 0) || (!out && n > 0) || n < 0) return KG_ERR_INVALID_ARG;
    for (int32_t k = 0; k < n; k++) {
        const int32_t ni = node_index[k];
        if (ni < 0 || ni >= view->n_nodes) return KG_ERR_RANGE;
        const kg_node_spec &ns = view->nodes[ni];
        kg_node_row &row = out[k];
        memset(&row, 0, sizeof(row));
        for (int r = 0; r < KG_NUM_RES; r++) {
            row.alloc[r] = val(ns.allocatable, r);
            row.requested[r] = val(ns.requested, r);
        }
        row.alloc_present = ns.allocatable.present & KG_SCALAR_RES_MASK;
        row.nonzero_requested[0] = ns.nonzero_requested[0];
        row.nonzero_requested[1] = ns.nonzero_requested[1];
        row.pod_count = ns.pod_count;
        row.allowed_pods = ns.allowed_pods;
        row.flags = KG_NODE_VALID;
        kg_resource_list est;
        estimate_node(ns, est);
        row.la_alloc[0] = val(est, KG_RES_CPU);
        row.la_alloc[1] = val(est, KG_RES_MEMORY);
        for (int r = 2; r < KG_NUM_RES; r++) row.la_alloc_x[r - 2] = val(est, r);
        if (ns.has_node_metric) {
            row.flags |= KG_NODE_HAS_METRIC;
            if (ns.has_update_time) {
                row.flags |= KG_NODE_HAS_UPDATE_TIME;
                row.metric_update_ns = ns.update_time_ns;
            }
            // LoadAware.Filter threshold checks (daemonset / expiry handled in-kernel)
            const Thresholds t = thresholds_of(*cfg, ns);
            bool pass_np = true;
            const kg_resource_list &thr = t.agg ? t.agg_thr : t.usage;
            if (nkeys(thr) > 0 && ns.has_node_metric_info) {
                const kg_resource_list *used = t.agg ? aggregated_usage(*view, ns, t.agg_dur, t.agg_type) : &ns.node_usage;
                pass_np = !exceeds(thr, est, used);
            }
            bool pass_p = pass_np;
            if (nkeys(t.prod) > 0) {
                pass_p = true;
                if (ns.n_pod_metric > 0) {
                    const MetricIndex pm = pod_metric_map(*view, ns, true);
                    kg_resource_list prod_used{};
                    for (int64_t name : pm.order) {
                        const kg_resource_list *u = pm.usage.at(name);
                        for (int r = 0; r < KG_NUM_RES; r++)
                            if (bit(u->present, r)) set_thr(prod_used, r, val(prod_used, r) + u->v[r]);
                    }
                    pass_p = !exceeds(t.prod, est, &prod_used);
                }
            }
            if (pass_np) row.flags |= KG_NODE_LA_PASS_NONPROD;
            if (pass_p) row.flags |= KG_NODE_LA_PASS_PROD;
            for (int v = 0; v < 2; v++) {
                int64_t used[KG_NUM_RES];
                loadaware_node_term(*cfg, *view, ns, v, used);
                row.la_used[v][0] = used[KG_RES_CPU];
                row.la_used[v][1] = used[KG_RES_MEMORY];
                for (int r = 2; r < KG_NUM_RES; r++) row.la_used_x[v][r - 2] = used[r];
            }
        }
        // NodeNUMAResource topology options (topology_options.go) with amplified zone cpu
        // (util.go:62-85 amplifyNUMANodeResources) and the plugin's zone allocations
        row.cpu_amplification_ratio = 1.0;
        if (ns.numa >= 0) {
            if (ns.numa >= view->n_numa) return KG_ERR_RANGE;
            const kg_numa_spec &nm = view->numa[ns.numa];
            if (nm.n_zones < 0 || nm.n_zones > KG_MAX_ZONES) return KG_ERR_RANGE;
            row.flags |= KG_NODE_NUMA_OPTIONS;
            if (nm.cpu_topology_valid < -1 || nm.cpu_topology_valid > 1) return KG_ERR_INVALID_ARG;
            if (nm.cpu_topology_valid == 1) row.flags |= KG_NODE_NUMA_TOPO_VALID;
            if (nm.cpu_topology_valid == 0) row.flags |= KG_NODE_NUMA_TOPO_INVALID;
            // cpuset allocations are recorded only on a valid topology (resourceManager.Update)
            if (nm.cpuset_cpus < 0 || (nm.cpuset_cpus > 0 && nm.cpu_topology_valid != 1)) return KG_ERR_INVALID_ARG;
            const double ratio = nm.cpu_amplification_ratio;
            const auto amplify = [ratio](int64_t x) { return ratio > 1.0 ? (int64_t)ceil((double)x * ratio) : x; };
            row.cpuset_milli = (int64_t)nm.cpuset_cpus * 1000;
            row.cpuset_amp_milli = amplify(row.cpuset_milli);
            for (int z = 0; z < KG_MAX_ZONES; z++) {
                const int32_t zc = z < nm.n_zones ? nm.zone_cpuset_cpus[z] : 0;
                if (zc < 0 || zc > nm.cpuset_cpus || (z >= nm.n_zones && nm.zone_cpuset_cpus[z] != 0))
                    return KG_ERR_INVALID_ARG;
                row.zone_cpuset_amp[z] = amplify((int64_t)zc * 1000) - (int64_t)zc * 1000;
            }
            // cpuset binding inputs: the node's CPU bind policy and, from the logical CPUs, the counts the
            // Filter's Allocate reduces to on a node without a NUMA topology policy
            if (nm.node_cpu_bind_policy < KG_NODE_CPU_BIND_NONE || nm.node_cpu_bind_policy > KG_NODE_CPU_BIND_SPREAD_BY_PCPUS ||
                nm.n_cpus < 0 || nm.max_ref_count < 0)
                return KG_ERR_INVALID_ARG;
            row.node_cpu_bind = nm.node_cpu_bind_policy;
            if (nm.numa_allocate_strategy < KG_NUMA_ALLOC_DEFAULT || nm.numa_allocate_strategy > KG_NUMA_ALLOC_DISTRIBUTE_EVENLY)
                return KG_ERR_INVALID_ARG;
            row.numa_policy = nm.policy;
            row.n_zones = nm.n_zones;
            row.cpu_amplification_ratio = nm.cpu_amplification_ratio;
            for (int z = 0; z < nm.n_zones; z++) {
                if (nm.zone_id[z] < 0 || nm.zone_id[z] >= 64) return KG_ERR_RANGE;
                // the engine's zones carry cpu and memory only
                if ((nm.zone_total[z].present | nm.zone_allocated[z].present) & ~0x3u) return KG_ERR_UNSUPPORTED;
                row.zone_id[z] = nm.zone_id[z];
                for (int r = 0; r < 2; r++) {
                    int64_t t = val(nm.zone_total[z], r);
                    if (r == KG_RES_CPU && nm.cpu_amplification_ratio > 1.0 && t != 0)
                        t = (int64_t)ceil((double)t * nm.cpu_amplification_ratio);
                    row.zone_total[z][r] = t;
                    row.zone_allocated[z][r] = val(nm.zone_allocated[z], r);
                    if (bit(nm.zone_total[z].present, r)) row.zone_keys |= 1u << (2 * z + r);
                    if (bit(nm.zone_allocated[z].present, r)) row.zone_alloc_keys |= 1u << (2 * z + r);
                }
            }
            // the CPU detail's counts (kg_cpuset_row_fields, the derivation a cpuset Reserve repeats); the
            // count fields of the spec must agree with it
            if (nm.n_cpus > 0) {
                if (nm.first_cpu < 0 || nm.first_cpu + (int64_t)nm.n_cpus > view->n_cpus || !view->cpus) return KG_ERR_RANGE;
                if (nm.n_cpus > KG_MAX_NODE_CPUS) return KG_ERR_UNSUPPORTED;
                const int32_t max_ref = nm.max_ref_count > 0 ? nm.max_ref_count : 1;
                if (kg_cpuset_row_fields(row, view->cpus + nm.first_cpu, nm.n_cpus, max_ref) != nm.cpuset_cpus)
                    return KG_ERR_INVALID_ARG;
                // … and so must the per-zone counts (the rows of nodes with and without CPU detail take the zones'
                // cpuset CPUs from the same facts)
                for (int z = 0; z < nm.n_zones; z++) {
                    int32_t held = 0;
                    for (int32_t c = 0; c < nm.n_cpus; c++) {
                        const kg_cpu_info &ci = view->cpus[nm.first_cpu + c];
                        if (ci.refcount > 0 && ci.node == nm.zone_id[z]) held++;
                    }
                    if (held != nm.zone_cpuset_cpus[z]) return KG_ERR_INVALID_ARG;
                }
            }
        }
    }
    return KG_OK;
}

// whether NodeNUMAResource binds a cpuset for the pair (requestCPUBind, util.go:105-122), and whether the
// engine answers it (with CPU detail when the topology is valid)
static bool row_binds(const kg_config &cfg, const kg_node_row &node, const kg_pod_row &pod, bool &answered) {
    answered = true;
    if (!(cfg.enabled_plugins & KG_PLUGIN_NUMA) || (pod.flags & KG_POD_NUMA_SKIP)) return false;
    const bool opts = (node.flags & KG_NODE_NUMA_OPTIONS) != 0;
    const bool bind = (pod.flags & KG_POD_NUMA_CPU_BIND) ||
                      (opts && node.node_cpu_bind != KG_NODE_CPU_BIND_NONE && pod.numa_request[KG_RES_CPU] != 0);
    if (bind) answered = !((node.flags & KG_NODE_NUMA_TOPO_VALID) && node.cpus_per_core <= 0);
    return bind;
}

kg_status kg_row_commit(const kg_config *cfg, kg_node_row *node, const kg_pod_row *pod) {
    if (!cfg || !node || !pod) return KG_ERR_INVALID_ARG;
    bool answered;
    if (row_binds(*cfg, *node, *pod, answered)) return KG_ERR_UNSUPPORTED;   // Reserve takes a cpuset: kg_row_reserve
    kg_pod_dev pd;
    kg_pod_dev_from_row(*cfg, *pod, pd);
    kg_consts k;
    kg_consts_from_config(*cfg, k);
    kg_numa_commit(k, *node, pd);   // zone allocations first: they see the pre-Reserve node
    kg_apply_commit(*node, pd);
    return KG_OK;
}

kg_status kg_row_reserve(const kg_config *cfg, kg_node_row *node, const kg_pod_row *pod, kg_cpu_info *cpus,
                         int32_t n_cpus, int32_t max_ref_count, int32_t numa_allocate_strategy, uint8_t *taken) {
    if (!cfg || !node || !pod || n_cpus < 0 || n_cpus > KG_MAX_NODE_CPUS || (n_cpus > 0 && (!cpus || !taken)) ||
        numa_allocate_strategy < KG_NUMA_ALLOC_DEFAULT || numa_allocate_strategy > KG_NUMA_ALLOC_DISTRIBUTE_EVENLY)
        return KG_ERR_INVALID_ARG;
    kg_pod_dev pd;
    kg_pod_dev_from_row(*cfg, *pod, pd);
    kg_consts k;
    kg_consts_from_config(*cfg, k);
    if (n_cpus > 0) memset(taken, 0, (size_t)n_cpus);
    int required, take;
    const bool bind = (k.plugins & KG_PLUGIN_NUMA) && kg_numa_binds(*node, pd, required, take);
    if (bind) {   // NodeNUMAResource.Reserve → Allocate: the cpuset comes first, a failure changes nothing
        if (!(node->flags & KG_NODE_NUMA_TOPO_VALID)) return KG_NOT_FOUND;   // ErrInvalidCPUTopology
        if (n_cpus == 0) return KG_ERR_UNSUPPORTED;   // a valid topology without CPU detail
        if (kg_cpuset_allocate(k, *node, pd, required, take, cpus, n_cpus, max_ref_count,
                               kg_cpuset_strategy(*cfg, numa_allocate_strategy), taken) != 0)
            return KG_NOT_FOUND;
    }
    kg_numa_commit(k, *node, pd);   // zone allocations first: they see the pre-Reserve node
    kg_apply_commit(*node, pd);
    if (bind) {   // Update: the cpuset into the node allocation, and the row's counts from it
        kg_cpuset_apply(pd, cpus, n_cpus, taken);
        kg_cpuset_row_fields(*node, cpus, n_cpus, max_ref_count);
    }
    return KG_OK;
}

kg_status kg_row_eval(const kg_config *cfg, const kg_node_row *node, const kg_pod_row *pod, int64_t now_ns,
                      int32_t *feasible, int32_t *fit_score, int32_t *la_score, int32_t *numa_score) {
    if (!cfg || !node || !pod || !feasible) return KG_ERR_INVALID_ARG;
    bool answered;
    if (row_binds(*cfg, *node, *pod, answered) && !answered) return KG_ERR_UNSUPPORTED;
    kg_consts k;
    kg_consts_from_config(*cfg, k);
    kg_pod_dev pd;
    kg_pod_dev_from_row(*cfg, *pod, pd);
    // one-node planes, only for the derived flags
    kg_node_row row = *node;
    int64_t free_[KG_NUM_RES], metric_ns;
    double fit_R[KG_NUM_RES], fit_F[KG_NUM_RES], la_R[2], la_F[4];
    uint32_t dflags, fmask;
    kg_planes pl{&row, free_, fit_R, fit_F, la_R, la_F, &metric_ns, &dflags, &fmask, 1};
    kg_finalize_node(k, pl, 0);
    bool ok;
    uint32_t fit, la, numa = 0;
    kg_pair_exact(k, row, dflags, pd, now_ns, ok, fit, la);
    if (pd.flags & KGP_RSV_REQUIRED) ok = false;  // no reservation on this node can match
    if (k.plugins & KG_PLUGIN_NUMA) {
        // through the zone-table provider of k_eval_numa2 (the table filled by one lane), so the CPU
        // row tests pin that path too; kg_row_commit keeps k_resolve's per-call zone sums
        kg_zone_tab_data zt;
        if (row.n_zones > 0) kg_zone_tab_fill(row, 0, 1, zt, [] {});
        kg_numa_out o;
        kg_numa_pair_z(k, row, pd, o, kg_zone_tab{zt});
        ok = ok && o.feasible;
        numa = o.score;
    }
    *feasible = ok ? 1 : 0;
    if (fit_score) *fit_score = (int32_t)fit;
    if (la_score) *la_score = (int32_t)la;
    if (numa_score) *numa_score = (int32_t)numa;
    return KG_OK;
}

kg_status kg_row_eval_rsv(const kg_config *cfg, const kg_node_row *node, const kg_reservation *rsv, int32_t n_rsv,
                          const kg_pod_row *pod, int64_t now_ns, int32_t *feasible, int32_t *fit_score,
                          int32_t *la_score, int32_t *numa_score, int32_t *rsv_raw, int64_t *order,
                          int32_t *nominated) {
    if (!cfg || !node || !pod || !feasible || n_rsv < 0 || n_rsv > KG_MAX_RSV_PER_NODE || (n_rsv > 0 && !rsv))
        return KG_ERR_INVALID_ARG;
    kg_consts k;
    kg_consts_from_config(*cfg, k);
    kg_pod_dev pd;
    kg_pod_dev_from_row(*cfg, *pod, pd);
    kg_node_row row = *node;
    int64_t free_[KG_NUM_RES], metric_ns;
    double fit_R[KG_NUM_RES], fit_F[KG_NUM_RES], la_R[2], la_F[4];
    uint32_t dflags, fmask;
    kg_planes pl{&row, free_, fit_R, fit_F, la_R, la_F, &metric_ns, &dflags, &fmask, 1};
    kg_finalize_node(k, pl, 0);
    kg_rsv_out o;
    kg_rsv_pair(k, row, dflags, rsv, n_rsv, pd, now_ns, o);
    *feasible = o.feasible ? 1 : 0;
    if (fit_score) *fit_score = (int32_t)o.fit;
    if (la_score) *la_score = (int32_t)o.la;
    if (numa_score) *numa_score = (int32_t)o.numa;
    if (rsv_raw) *rsv_raw = (int32_t)o.raw;
    if (order) *order = o.order;
    if (nominated) *nominated = o.nominated;
    return KG_OK;
}

kg_status kg_row_rsv_restore(const kg_config *cfg, const kg_node_row *node, const kg_reservation *rsv, int32_t n_rsv,
                             const kg_pod_row *pod, kg_rsv_restored *out) {
    if (!cfg || !node || !pod || !out || n_rsv < 0 || n_rsv > KG_MAX_RSV_PER_NODE || (n_rsv > 0 && !rsv))
        return KG_ERR_INVALID_ARG;
    kg_pod_dev pd;
    kg_pod_dev_from_row(*cfg, *pod, pd);
    kg_rsv_view v;
    kg_rsv_restore(*node, rsv, n_rsv, pd, v);
    memset(out, 0, sizeof(*out));
    for (int r = 0; r < KG_NUM_RES; r++) {
        out->requested[r] = v.requested[r];
        out->pod_requested[r] = v.pod_requested[r];
        out->r_allocated[r] = v.r_allocated[r];
    }
    out->nonzero[0] = v.nonzero[0];
    out->nonzero[1] = v.nonzero[1];
    out->pod_count = (int32_t)v.pod_count;
    out->n_matched = v.n_matched;
    out->has_state = v.has_state ? 1 : 0;
    return KG_OK;
}

}  // extern "C"

// ---- engine-internal helpers shared with kg_engine.hip ------------------------------------

void kg_consts_from_config(const kg_config &c, kg_consts &k) {
    memset(&k, 0, sizeof(k));
    k.plugins = c.enabled_plugins;
    k.weight_fit = c.weight_fit;
    k.weight_la = c.weight_loadaware;
    k.fit_most = c.fit_strategy == KG_STRATEGY_MOST_ALLOCATED;
    for (int r = 0; r < KG_NUM_RES; r++) k.fit_w[r] = (int32_t)c.fit_resource_weight[r];
    k.la_w[0] = (int32_t)c.la_resource_weight[0];
    k.la_w[1] = (int32_t)c.la_resource_weight[1];
    k.la_wsum = k.la_w[0] + k.la_w[1];
    for (int r = 2; r < KG_NUM_RES; r++) {
        k.la_wx[r - 2] = (int32_t)c.la_resource_weight[r];
        k.la_wsum += k.la_wx[r - 2];
        if (k.la_wx[r - 2] != 0) k.la_extra = 1;
    }
    k.la_magic = k.la_wsum ? (uint32_t)((0x80000000ULL + (uint64_t)k.la_wsum - 1) / (uint64_t)k.la_wsum) : 0;
    k.la_shift = 0xFF;
    if (k.la_wsum > 0 && (k.la_wsum & (k.la_wsum - 1)) == 0) k.la_shift = __builtin_ctz((unsigned)k.la_wsum);
    k.la_rcp = k.la_wsum ? 1.0f / (float)k.la_wsum : 0.0f;
    k.la_filter_expired = c.la_filter_expired_node_metrics;
    k.la_has_exp = c.la_has_expiration;
    k.la_exp_ns = c.la_has_expiration ? c.la_expiration_seconds * 1000000000LL : 0;
    k.weight_numa = c.weight_numa;
    k.numa_most = c.numa_strategy == KG_STRATEGY_MOST_ALLOCATED;
    k.numa_hint_most = c.numa_hint_strategy == KG_STRATEGY_MOST_ALLOCATED;
    for (int r = 0; r < KG_NUM_RES; r++) k.numa_w[r] = (int32_t)c.numa_resource_weight[r];
    k.weight_rsv = (c.enabled_plugins & KG_PLUGIN_RESERVATION) ? c.weight_reservation : 0;
    int8_t order[KG_NUM_RES];
    kg_res_sorted_order(c, order);
    for (int i = 0; i < KG_NUM_RES; i++) k.res_rank[order[i]] = (int8_t)i;
}

void kg_pod_dev_from_row(const kg_config &c, const kg_pod_row &row, kg_pod_dev &d) {
    memset(&d, 0, sizeof(d));
    for (int r = 0; r < KG_NUM_RES; r++) {
        d.req[r] = row.request[r];
        d.fit_pr_i[r] = row.fit_score_request[r];
        const double pr = (double)row.fit_score_request[r];
        d.fit_pr[r] = c.fit_strategy == KG_STRATEGY_MOST_ALLOCATED ? pr : -pr;
    }
    d.la_est[0] = -(double)row.la_estimate[0];
    d.la_est[1] = -(double)row.la_estimate[1];
    d.flags = row.flags;
    d.request_present = row.request_present;
    uint32_t cmp = 0, zero = 0;
    if (row.flags & KG_POD_HAS_REQUEST) {
        for (int r = 0; r < 3; r++) (row.request[r] != 0 ? cmp : zero) |= 1u << r;
        cmp |= row.request_present & KG_SCALAR_RES_MASK;
    }
    d.cmp_mask = cmp;
    d.zero_native_mask = zero;
    uint32_t fm = 0, w = 0;
    for (int r = 0; r < KG_NUM_RES; r++) {
        if (c.fit_resource_weight[r] <= 0) continue;
        if (scalar_res(r) && row.fit_score_request[r] == 0) continue;
        fm |= 1u << r;
        w += (uint32_t)c.fit_resource_weight[r];
    }
    d.fit_mask = fm;
    d.fit_w = w;
    d.fit_magic = w ? (uint32_t)((0x80000000ULL + w - 1) / w) : 0;
    d.nonzero[0] = row.nonzero_request[0];
    d.nonzero[1] = row.nonzero_request[1];
    d.la_est_i[0] = row.la_estimate[0];
    d.la_est_i[1] = row.la_estimate[1];
    for (int r = 0; r < KG_NUM_RES - 2; r++) d.la_est_x[r] = row.la_estimate_x[r];
    for (int r = 0; r < KG_NUM_RES; r++) d.numa_req[r] = row.numa_request[r];
    d.numa_present = row.numa_request_present;
    d.cpu_bind = row.cpu_bind;
    d.rsv_owner = row.rsv_owner_class;
    d.rsv_aff = row.rsv_affinity_class;
    d.quota = (c.enabled_plugins & KG_PLUGIN_ELASTICQUOTA) ? row.quota : -1;
    if ((c.enabled_plugins & KG_PLUGIN_RESERVATION) && row.rsv_affinity_class >= 0) d.flags |= KGP_RSV_REQUIRED;
}

int kg_numa_list_count(const kg_pod_row &row) {
    // hint lists a pod can produce: cpu / memory (zone resources) and every zero-valued request key
    int n = 0;
    for (int r = 0; r < KG_NUM_RES; r++)
        if (((row.numa_request_present >> r) & 1u) && (r <= KG_RES_MEMORY || row.numa_request[r] == 0)) n++;
    return n;
}

template <int S>
uint32_t kg_pod_hot_from_row(const kg_config &c, const kg_pod_row &row, const int32_t *slot_res, kg_pod_hot_t<S> &h) {
    memset(&h, 0, sizeof(h));
    const bool hr = (row.flags & KG_POD_HAS_REQUEST) != 0;
    const bool fit_on = (c.enabled_plugins & KG_PLUGIN_FIT) != 0;
    // resources that need a slot: natives with a non-zero request and scalar keys (a zero native
    // request only fails an overcommitted node, which the kernel folds into the node filter bits),
    // and every resource the pod scores
    uint32_t need = 0, fit_mask = 0, w = 0;
    if (fit_on && hr) {
        for (int r = 0; r < 3; r++)
            if (row.request[r] != 0) need |= 1u << r;
        need |= row.request_present & KG_SCALAR_RES_MASK;
    }
    for (int r = 0; fit_on && r < KG_NUM_RES; r++) {
        if (c.fit_resource_weight[r] <= 0) continue;
        if (scalar_res(r) && row.fit_score_request[r] == 0) continue;
        fit_mask |= 1u << r;
        w += (uint32_t)c.fit_resource_weight[r];
    }
    need |= fit_mask;
    uint32_t flags = (row.flags & KG_POD_LA_PROD_SCORE) ? KG_HOT_PROD : 0u;
    for (int s = 0; s < S; s++) {
        const int r = slot_res[s];
        h.req[s] = KG_NEUTRAL_REQ;
        if (r < 0) continue;
        // natives are compared once the pod requests anything; scalars only when the key is present
        if (fit_on && hr && (r < 3 || bit(row.request_present, r))) {
            h.req[s] = row.request[r];
            flags |= 1u << (KG_HOT_CMP_SHIFT + s);
        }
        if (bit(fit_mask, r)) {
            h.fit_w[s] = (uint32_t)c.fit_resource_weight[r];
            const double pr = (double)row.fit_score_request[r];
            h.fit_pr[s] = c.fit_strategy == KG_STRATEGY_MOST_ALLOCATED ? pr : -pr;
            flags |= 1u << (KG_HOT_FIT_SHIFT + s);
        }
    }
    h.fit_shift = (w > 0 && (w & (w - 1)) == 0) ? (uint32_t)__builtin_ctz(w) : (w == 0 ? 0u : 0xFFu);
    h.fit_rcp = w ? 1.0f / (float)w : 0.0f;
    h.la_est[0] = -(double)row.la_estimate[0];
    h.la_est[1] = -(double)row.la_estimate[1];
    const uint32_t variant = (row.flags & KG_POD_DAEMONSET) ? 2u : (row.flags & KG_POD_PROD) ? 1u : 0u;
    h.okshift = variant + (hr && fit_on ? 3u : 0u);
    h.flags = flags;
    return need;
}
template uint32_t kg_pod_hot_from_row<2>(const kg_config &, const kg_pod_row &, const int32_t *, kg_pod_hot_t<2> &);
template uint32_t kg_pod_hot_from_row<4>(const kg_config &, const kg_pod_row &, const int32_t *, kg_pod_hot_t<4> &);
template uint32_t kg_pod_hot_from_row<8>(const kg_config &, const kg_pod_row &, const int32_t *, kg_pod_hot_t<8> &);

bool kg_pod_row_in_bounds(const kg_pod_row &row) {
    for (int r = 0; r < KG_NUM_RES; r++)
        if (row.request[r] < 0 || row.request[r] >= KG_VAL_LIMIT || row.fit_score_request[r] < 0 ||
            row.fit_score_request[r] >= KG_VAL_LIMIT || row.numa_request[r] < 0 || row.numa_request[r] >= KG_VAL_LIMIT)
            return false;
    return row.la_estimate[0] >= 0 && row.la_estimate[0] < KG_VAL_LIMIT && row.la_estimate[1] >= 0 &&
           row.la_estimate[1] < KG_VAL_LIMIT;
}
