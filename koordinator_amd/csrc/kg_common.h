// kg_common.h — engine internals shared by the host library and the HIP kernels.
//
// The node snapshot lives in HBM as
//   * canonical rows   kg_node_row[cap]            (what kg_snapshot_upsert / kg_commit mutate)
//   * derived planes   struct-of-arrays per node   (what the hot kernels read; rebuilt from the
//                                                   canonical row by kg_finalize_node)
// kg_finalize_node() is __host__ __device__ so the host ingest path and the device commit path
// (placement mode) derive bit-identical planes.
//
// Integer-exact scores with one fp64 FMA per resource.  The plugins' least-requested score is
//   LR(req, cap) = cap == 0 || req > cap ? 0 : (cap - req) * 100 / cap          (Go int64 division)
// (load_aware.go:388-397; upstream least_allocated.go, mirrored at nodenumaresource/least_allocated.go:49-58)
// with req = base(node) + pr(pod).  Per node we store R = RN(100/cap) and
// F = RN(100*(cap-base)/cap + 2^-42) (computed from an exact int64 quotient/remainder), and per pair
//   q = max((int)fma(-pr, R, F), 0)
// The summed rounding error is below 2^-44.7 whenever the true value lies in [-1, 101], so
// adding 2^-42 keeps exact integers from rounding down, and the gap 1/cap > 2^-41.8 keeps
// non-integers from rounding up, for every cap <= 2^41.  Nodes outside those bounds get
// KGD_SLOW and take the exact int64 path (kg_pair_exact).  MostAllocated is the same with
// F = RN(100*base/cap + 2^-42), q = min(q, 100).
#pragma once
#include <stdint.h>

#include "../../include/koord_gpu.h"

#if defined(__HIPCC__)
#define KG_HD __host__ __device__ __forceinline__
#else
#define KG_HD inline
#endif

#define KG_TILE 1024                // nodes per eval workgroup / per-pod partial key (two nodes per lane)
#define KG_TILE_SHIFT 10            // log2 KG_TILE: partial key = ((total + 1) << 10) | (1023 − local node)
#define KG_BLOCK 512                // threads per eval workgroup
#define KG_EPS 0x1p-42
#define KG_CAP_LIMIT (1LL << 41)    // fast-path bound on every divisor
#define KG_VAL_LIMIT (1LL << 50)    // fast-path bound on every numerator term

// derived node flags
#define KGD_VALID 0x1u
#define KGD_PODS_FULL 0x2u          // len(Pods)+1 > AllowedPodNumber
#define KGD_OVER_CPU 0x4u           // Allocatable - Requested < 0  (fails even a zero request)
#define KGD_OVER_MEM 0x8u
#define KGD_OVER_EPH 0x10u
#define KGD_SLOW 0x20u              // outside the fp64 exactness bounds → kg_pair_exact
#define KGD_HAS_METRIC 0x40u
#define KGD_HAS_UPDATE 0x80u
#define KGD_LA_PASS_NP 0x100u
#define KGD_LA_PASS_P 0x200u

// per-pod derived data the kernels read (uniform → scalar loads)
struct kg_pod_dev {
    int64_t req[KG_NUM_RES];     // Fit filter request
    double fit_pr[KG_NUM_RES];   // Fit score pod request, negated for LeastAllocated (fma operand)
    double la_est[2];            // −EstimatePod (fma operand)
    int64_t fit_pr_i[KG_NUM_RES];// Fit score pod request (exact path)
    uint32_t flags;              // KG_POD_*
    uint32_t cmp_mask;           // resources compared by the Fit filter (request != 0 or scalar key)
    uint32_t zero_native_mask;   // native resources with request == 0 (checked via KGD_OVER_*)
    uint32_t fit_mask;           // Fit score resources the pod contributes (weight > 0, not (scalar && pr == 0))
    uint32_t fit_magic;          // ceil(2^31 / W) for W = Σ weight over fit_mask: s / W = umulhi(2s, magic)
    uint32_t fit_w;              // W
    uint32_t request_present;
    uint32_t _pad;
    int64_t nonzero[2];
    int64_t la_est_i[2];
};

// config-derived constants passed by value to every kernel
struct kg_consts {
    uint32_t plugins;            // KG_PLUGIN_*
    int32_t weight_fit, weight_la;
    int32_t fit_most;            // MostAllocated
    int32_t fit_w[KG_NUM_RES];   // NodeResourcesFit resource weights
    int32_t la_w[2];             // LoadAware weights (cpu, memory)
    uint32_t la_magic;           // ceil(2^31 / Σ la_w)
    int32_t la_wsum;
    int32_t la_filter_expired;
    int32_t la_has_exp;
    int32_t la_shift;            // log2 Σ la_w when a power of two, else 0xFF
    float la_rcp;                // 1 / Σ la_w
    int64_t la_exp_ns;
};

#define KG_NEUTRAL_REQ INT64_MIN  // request that passes every Fit compare

// per-pod data of the hot kernel (k_eval2), over S resource "slots" (the launch's resource
// profile maps slot s → resource id).  Read as whole 64-byte blocks with s_load_dwordx16.
#define KG_HOT_PROD 0x1u             // flags: LoadAware prod-usage variant
#define KG_HOT_CMP_SHIFT 8           // flags bits 8..15: slot s is compared by the Fit filter
#define KG_HOT_FIT_SHIFT 16          // flags bits 16..23: slot s is scored by NodeResourcesFit
template <int S>
struct alignas(64) kg_pod_hot_t {
    int64_t req[S];        // Fit filter request; KG_NEUTRAL_REQ where the slot is not compared
    double fit_pr[S];      // signed fma operand (−pr LeastAllocated, +pr MostAllocated); 0 if not scored
    double la_est[2];      // −EstimatePod (cpu, memory)
    uint32_t fit_w[S];     // Fit weight of the slot for this pod (0 ⇔ not scored)
    uint32_t okshift;      // node filter bit: variant (0 non-prod, 1 prod, 2 daemonset) + 3·has_request
    uint32_t fit_shift;    // log2 W when W is a power of two (W = Σ fit_w), else 0xFF
    float fit_rcp;         // 1 / W
    uint32_t flags;        // KG_HOT_*
};

// ---- class-specialised matrix mode (k_eval3) ---------------------------------------------
// Pods of a batch that compare the same resources in the Fit filter, score the same resources,
// take the same node-filter variant and the same LoadAware usage variant form a class.  Within a
// class every per-pair branch is a compile-time constant: NC compared resources (int64), NF scored
// resources (fp64 fma), padded to 2 or 4.  Rows are stored class after class (queue order inside a
// class) and carry their output offsets.
#define KG_CLS_MAX 16                // classes per batch on the specialised path
template <int NC, int NF>
struct alignas(64) kg_pod_cls_t {
    int64_t req[NC];       // Fit filter request of the compared resources (INT64_MIN pads)
    double pr[NF];         // signed Fit pod request of the scored resources (0 pads)
    double la[2];          // −EstimatePod (cpu, memory)
    int64_t score_off;     // output row × score stride (elements)
    int32_t mask_off;      // output row × mask words
    int32_t row;           // output row (partial keys)
};

struct kg_cls_desc {
    int32_t kind;          // 0: (2,2)  1: (2,4)  2: (4,2)  3: (4,4)   (NC, NF)
    int32_t first;         // first row of the class in the class-sorted pod array
    int32_t count;
    int32_t cmp_res[4];    // resource of each compared slot (−1 pad)
    int32_t fit_res[4];    // resource of each scored slot (−1 pad)
    uint32_t fit_w[4];     // Fit weight of each scored slot (0 pad)
    uint32_t fit_shift;    // log2 Σ fit_w (a power of two on this path)
    uint32_t node_ok_sel;  // node filter bit: variant (0 non-prod, 1 prod, 2 daemonset) + 3·has_request
    uint32_t la_variant;   // 0 non-prod usage, 1 prod usage (ScoreAccordingProdUsage)
    uint32_t over_mask;    // natives with a zero request on a pod with requests: fail an overcommitted node
    int64_t row_bytes;     // sizeof(kg_pod_cls_t<NC, NF>)
    int64_t rows_offset;   // byte offset of the class's rows in the row buffer
};

// one workgroup row of the launch grid: a pod range of one class
struct kg_cls_work {
    int32_t cls;
    int32_t begin;         // [begin, end) within the class
    int32_t end;
    int32_t _pad;
};

struct kg_planes {
    kg_node_row *rows;   // [cap]
    int64_t *free_;      // [KG_NUM_RES][cap]   Allocatable − Requested
    double *fit_R;       // [KG_NUM_RES][cap]
    double *fit_F;       // [KG_NUM_RES][cap]
    double *la_R;        // [2][cap]
    double *la_F;        // [2 variants][2 resources][cap]
    int64_t *metric_ns;  // [cap]
    uint32_t *dflags;    // [cap]
    uint32_t *fit_mask;  // [cap] resources the node contributes to the Fit score
    int64_t cap;
};

KG_HD int64_t kg_abs64(int64_t x) { return x < 0 ? -x : x; }

// RN(100*num/den + eps) from an exact int64 quotient and remainder (|100*num| < 2^63)
KG_HD double kg_scaled_ratio(int64_t num, int64_t den) {
    int64_t n100 = num * 100;
    int64_t q = n100 / den;
    int64_t r = n100 % den;
    return (double)q + ((double)r / (double)den + KG_EPS);
}

// Derived planes of node i from its canonical row (host ingest and device commit share this).
KG_HD void kg_finalize_node(const kg_consts &c, const kg_planes &pl, int64_t i) {
    const kg_node_row &row = pl.rows[i];
    const int64_t cap = pl.cap;
    uint32_t df = 0;
    if (row.flags & KG_NODE_VALID) df |= KGD_VALID;
    if ((int64_t)row.pod_count + 1 > (int64_t)row.allowed_pods) df |= KGD_PODS_FULL;
    bool slow = false;
    uint32_t fmask = 0;
    for (int r = 0; r < KG_NUM_RES; r++) {
        int64_t fr = row.alloc[r] - row.requested[r];
        pl.free_[r * cap + i] = fr;
        if (r == KG_RES_CPU && fr < 0) df |= KGD_OVER_CPU;
        if (r == KG_RES_MEMORY && fr < 0) df |= KGD_OVER_MEM;
        if (r == KG_RES_EPHEMERAL_STORAGE && fr < 0) df |= KGD_OVER_EPH;
        double R = 0.0, F = 0.0;
        int64_t a = row.alloc[r];
        bool present = r < 3 || ((row.alloc_present >> r) & 1u);
        if (c.fit_w[r] > 0 && present && a != 0) {
            fmask |= 1u << r;
            int64_t base = r < 2 ? row.nonzero_requested[r] : row.requested[r];
            if (a < 0 || a >= KG_CAP_LIMIT || kg_abs64(base) >= KG_VAL_LIMIT) {
                slow = true;
            } else {
                R = 100.0 / (double)a;
                F = c.fit_most ? kg_scaled_ratio(base, a) : kg_scaled_ratio(a - base, a);
            }
        }
        pl.fit_R[r * cap + i] = R;
        pl.fit_F[r * cap + i] = F;
    }
    for (int r = 0; r < 2; r++) {
        int64_t a = row.la_alloc[r];
        double R = 0.0, F0 = 0.0, F1 = 0.0;
        if (a != 0) {
            if (a < 0 || a >= KG_CAP_LIMIT || kg_abs64(row.la_used[0][r]) >= KG_VAL_LIMIT ||
                kg_abs64(row.la_used[1][r]) >= KG_VAL_LIMIT) {
                slow = true;
            } else {
                R = 100.0 / (double)a;
                F0 = kg_scaled_ratio(a - row.la_used[0][r], a);
                F1 = kg_scaled_ratio(a - row.la_used[1][r], a);
            }
        }
        pl.la_R[r * cap + i] = R;
        pl.la_F[(0 * 2 + r) * cap + i] = F0;
        pl.la_F[(1 * 2 + r) * cap + i] = F1;
    }
    if (slow) df |= KGD_SLOW;
    if (row.flags & KG_NODE_HAS_METRIC) df |= KGD_HAS_METRIC;
    if (row.flags & KG_NODE_HAS_UPDATE_TIME) df |= KGD_HAS_UPDATE;
    if (row.flags & KG_NODE_LA_PASS_NONPROD) df |= KGD_LA_PASS_NP;
    if (row.flags & KG_NODE_LA_PASS_PROD) df |= KGD_LA_PASS_P;
    pl.metric_ns[i] = row.metric_update_ns;
    pl.fit_mask[i] = fmask;
    pl.dflags[i] = df;
}

// Reserve delta: NodeInfo.AddPod (requested += request, nonzero += nonzero, pods += 1;
// mirror reservation/transformer.go:293-306) + LoadAware.Reserve → podAssignCache.assign: the new
// pod has no PodMetric yet, so it is always "estimated" and adds EstimatePod(pod) to the
// non-prod term and, if the pod is prod, to the prod term (load_aware.go:348-373).
KG_HD void kg_apply_commit(kg_node_row &row, const kg_pod_dev &p) {
    for (int r = 0; r < KG_NUM_RES; r++) row.requested[r] += p.req[r];
    row.nonzero_requested[0] += p.nonzero[0];
    row.nonzero_requested[1] += p.nonzero[1];
    row.pod_count += 1;
    row.la_used[0][0] += p.la_est_i[0];
    row.la_used[0][1] += p.la_est_i[1];
    if (p.flags & KG_POD_PROD) {
        row.la_used[1][0] += p.la_est_i[0];
        row.la_used[1][1] += p.la_est_i[1];
    }
}

// LoadAware time checks (helper.go:36-41) evaluated per node at `now`.
KG_HD bool kg_metric_expired(const kg_consts &c, uint32_t df, int64_t upd_ns, int64_t now_ns) {
    return !(df & KGD_HAS_UPDATE) || (c.la_exp_ns > 0 && now_ns - upd_ns >= c.la_exp_ns);
}
// LoadAware.Filter outcome for a non-prod (variant 0) / prod (variant 1) pod, daemonset aside.
KG_HD bool kg_la_pass(const kg_consts &c, uint32_t df, bool expired, int variant) {
    if (!(df & KGD_HAS_METRIC)) return true;
    if (c.la_filter_expired && c.la_has_exp && expired) return true;
    return variant ? (df & KGD_LA_PASS_P) != 0 : (df & KGD_LA_PASS_NP) != 0;
}
KG_HD bool kg_la_valid(const kg_consts &c, uint32_t df, bool expired) {
    return (df & KGD_HAS_METRIC) && !(c.la_has_exp && expired);
}

// Exact int64 evaluation of one (pod, node) pair straight from the canonical row (slow path).
KG_HD void kg_pair_exact(const kg_consts &c, const kg_node_row &row, uint32_t df, const kg_pod_dev &p,
                         int64_t now_ns, bool &feasible, uint32_t &fit, uint32_t &la) {
    bool expired = kg_metric_expired(c, df, row.metric_update_ns, now_ns);
    bool ok = (df & KGD_VALID) != 0;
    if (c.plugins & KG_PLUGIN_FIT) {
        if (df & KGD_PODS_FULL) ok = false;
        if (p.flags & KG_POD_HAS_REQUEST) {
            for (int r = 0; r < KG_NUM_RES; r++) {
                bool chk = r < 3 || ((p.request_present >> r) & 1u);
                if (chk && p.req[r] > row.alloc[r] - row.requested[r]) ok = false;
            }
        }
    }
    if (c.plugins & KG_PLUGIN_LOADAWARE) {
        if (!(p.flags & KG_POD_DAEMONSET) && !kg_la_pass(c, df, expired, (p.flags & KG_POD_PROD) ? 1 : 0)) ok = false;
    }
    feasible = ok;
    fit = 0;
    la = 0;
    if (c.plugins & KG_PLUGIN_FIT) {
        int64_t s = 0, w = 0;
        for (int r = 0; r < KG_NUM_RES; r++) {
            if (!((p.fit_mask >> r) & 1u)) continue;
            bool present = r < 3 || ((row.alloc_present >> r) & 1u);
            int64_t a = row.alloc[r];
            if (!present || a == 0) continue;
            int64_t base = r < 2 ? row.nonzero_requested[r] : row.requested[r];
            int64_t req = base + p.fit_pr_i[r];
            int64_t q;
            if (c.fit_most) q = (req > a ? a : req) * 100 / a;
            else q = req > a ? 0 : (a - req) * 100 / a;
            s += q * c.fit_w[r];
            w += c.fit_w[r];
        }
        fit = w ? (uint32_t)(s / w) : 0;
    }
    if ((c.plugins & KG_PLUGIN_LOADAWARE) && kg_la_valid(c, df, expired)) {
        int v = (p.flags & KG_POD_LA_PROD_SCORE) ? 1 : 0;
        int64_t s = 0;
        for (int r = 0; r < 2; r++) {
            if (c.la_w[r] == 0) continue;
            int64_t a = row.la_alloc[r];
            int64_t req = p.la_est_i[r] + row.la_used[v][r];
            int64_t q = (a == 0 || req > a) ? 0 : (a - req) * 100 / a;
            s += q * c.la_w[r];
        }
        la = c.la_wsum ? (uint32_t)(s / c.la_wsum) : 0;
    }
}
