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
#include <math.h>
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
#define KGD_RSV 0x400u              // carries reservation slots: only the exact Reservation path evaluates it
#define KGD_XSLOW 0x800u            // outside the fp64 bounds of a plane the batch reads, LoadAware extra resources
                                    // included: under LoadAware weights beyond cpu / memory every node carries
                                    // KGD_SLOW (the paths without extra-resource planes take kg_pair_exact), and the
                                    // matrix kernel with those planes takes the exact path only for KGD_XSLOW nodes

// engine-internal pod flag: Reservation is enabled and the pod has a required reservation affinity,
// so every node without a matching reservation fails Reservation.Filter (plugin.go:354-357)
#define KGP_RSV_REQUIRED 0x40000000u

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
    uint32_t cpu_bind;           // kg_pod_row.cpu_bind: required | preferred << 4 | exclusive << 8
    int64_t nonzero[2];
    int64_t la_est_i[2];
    int64_t numa_req[KG_NUM_RES];// NodeNUMAResource PreFilter requests (PodRequestsAndLimits)
    uint32_t numa_present;       // their key set
    int32_t rsv_owner;           // Reservation owner class (−1 none)
    int32_t rsv_aff;             // required reservation-affinity class (−1 none)
    int32_t quota;               // ElasticQuota group (−1 none)
    uint32_t _pad2;
    int64_t la_est_x[KG_NUM_RES - 2]; // EstimatePod of resources 2..7 (LoadAware weights beyond cpu / memory)
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
    int32_t weight_numa;
    int32_t numa_most;           // ScoringStrategy MostAllocated
    int32_t numa_hint_most;      // NUMAScoringStrategy MostAllocated
    int32_t numa_w[KG_NUM_RES];  // ScoringStrategy.Resources weights
    int32_t weight_rsv;          // Reservation profile weight
    int32_t la_extra;            // LoadAware weights beyond cpu / memory: every node takes kg_pair_exact
    int32_t la_wx[KG_NUM_RES - 2]; // their weights (resources 2..11; included in la_wsum)
    int8_t res_rank[KG_NUM_RES];   // each resource's rank in sorted resource-name order (kg_res_sorted_order: the fixed
                                   // names and kg_config.ext_resource_names), the order the topology merge walks the lists
    int32_t numa_bz;             // placement of a batch that binds cpusets on NUMA-policy nodes: the chunk and
                                 // resolve kernels answer those pairs (kg_numa_pair_bz) instead of leaving them out
};

#define KG_NEUTRAL_REQ INT64_MIN  // request that passes every Fit compare

// The fast per-pair paths keep resources 0 .. KG_FAST_RES − 1 (the fixed ones and the first named slot) in registers;
// the later named slots are read from memory where a pod uses them (kg_pair_view) or take the exact path (eval_pair)
#define KG_FAST_RES 8

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
// class); the output row of each is in a parallel int32 array (kg_cls_desc::ids_first).
#define KG_CLS_MAX 32                // class parts per batch on the specialised path (a class: plain + duplicate-row part)
template <int NC, int NF>
struct alignas(16) kg_pod_cls_t {
    int64_t req[NC];       // Fit filter request of the compared resources (INT64_MIN pads)
    double pr[NF];         // signed Fit pod request of the scored resources (0 pads)
    double la[2];          // −EstimatePod (cpu, memory)
};

struct kg_cls_desc {
    int32_t kind;          // 0: (2,2)  1: (2,4)  2: (4,2)  3: (4,4)   (NC, NF)
    int32_t ids_first;     // the class's first entry in the output-row array
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
    // scored resources whose Fit request is the same for every pod of the class (e.g. the NonZero cpu /
    // memory defaults of batch pods): their least-requested terms depend on the node only and are summed
    // once per node (ClsNode::cq) instead of per pair; the class's rows carry only the other slots
    int32_t uni_res[4];    // resource of each uniform slot (−1 pad)
    uint32_t uni_w[4];     // its Fit weight
    double uni_pr[4];      // its request, signed like kg_pod_cls_t::pr
    // pods [0, la_uni_end) of the class come in whole k_eval3 chunks of one EstimatePod each (cls_order_la)
    int32_t la_uni_end;
    // duplicate-row part of a class (k_eval3<DUP>): the rows are the distinct rows of the class's pods whose row
    // occurs more than once, `count` counts their pods, whose output rows (ids_first) are grouped by row and
    // whose row indices are at ux_first in the same int32 array; −1 for the plain part
    int32_t ux_first;
};

// one workgroup row of the launch grid: a pod range of one class
struct kg_cls_work {
    int32_t cls;
    int32_t begin;         // [begin, end) within the class (a duplicate-row part: its pods, grouped by row)
    int32_t end;
    int32_t tile;          // duplicate-row part: the item's tile (its 1-D grid is ordered XCD by XCD); else 0
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
    int32_t *rsv_of;     // [cap] index of the node in the reservation node list, −1 none (nullptr: no list)
    double *la_Rx;       // [KG_NUM_RES − 2][cap] LoadAware planes of resources 2..7 (nullptr: not kept)
    double *la_Fx;       // [2 variants][KG_NUM_RES − 2][cap]
};

KG_HD int64_t kg_abs64(int64_t x) { return x < 0 ? -x : x; }

// Exact truncating int64 quotient and remainder of n / d (d > 0) — the device has no int64 divide
// instruction: an fp64 estimate n · RN(1/d) (relative error ≤ 3·2^-53, so off by < |n/d|·2^-51.4 + 1 ≤ 49) is
// corrected with exact int64 arithmetic, the residual's own estimate r0 · RN(1/d) (off from r0/d by < 2^-45.8,
// less than 1/d: its truncation is exact but at exact integers, where it is low by one) and a final ±1 step.
// One fp64 division (the reciprocal) instead of two: the placement resolve's Reserve derives its planes through
// this chain (r05: the LoadAware part 4.0k → Fit part 3.9k cycles per pod were mostly fp64 divisions).
// Valid for |n| < 2^57 and 0 < d < 2^41 (the finalize operands: |100·(a − base)| < 2^57, a < KG_CAP_LIMIT).
KG_HD void kg_divmod64_fp(int64_t n, int64_t d, int64_t &q, int64_t &r) {
    const double inv = 1.0 / (double)d;
    int64_t q0 = (int64_t)((double)n * inv);
    int64_t r0 = n - q0 * d;
    const int64_t q1 = (int64_t)((double)r0 * inv);
    q0 += q1;
    r0 -= q1 * d;
    // C truncation: the remainder takes the sign of n and |r| < d
    if (n >= 0) {
        if (r0 < 0) { q0 -= 1; r0 += d; }
        else if (r0 >= d) { q0 += 1; r0 -= d; }
    } else {
        if (r0 > 0) { q0 += 1; r0 -= d; }
        else if (r0 <= -d) { q0 -= 1; r0 += d; }
    }
    q = q0;
    r = r0;
}
KG_HD void kg_divmod64(int64_t n, int64_t d, int64_t &q, int64_t &r) {
#if defined(__HIP_DEVICE_COMPILE__)
    kg_divmod64_fp(n, d, q, r);
#else
    q = n / d;
    r = n % d;
#endif
}

// RN(100*num/den + eps) from an exact int64 quotient and remainder (|100*num| < 2^63)
KG_HD double kg_scaled_ratio(int64_t num, int64_t den) {
    int64_t n100 = num * 100;
    int64_t q, r;
    kg_divmod64(n100, den, q, r);
    return (double)q + ((double)r / (double)den + KG_EPS);
}

// Derived planes of node i from its canonical row (host ingest and device commit share this).
// Split in parts so the placement resolve can derive them with one thread per part:
//   kg_finalize_fit(r)  Fit planes and free_ of resource r (r < KG_NUM_RES) → bit 0: slow, bit 1: in fit_mask
//   kg_finalize_la(r)   LoadAware planes of resource r (r < 2)             → slow
//   kg_finalize_flags   dflags / fit_mask / metric from the parts' results
// (free / R / F out: optional copies of the written plane values, for the resolve kernel's node cache)
// (the _r forms take the canonical row by reference: the placement resolve passes its LDS copy)
KG_HD uint32_t kg_finalize_fit_r(const kg_consts &c, const kg_planes &pl, int64_t i, const kg_node_row &row, int r,
                                 int64_t *free_out = nullptr, double *R_out = nullptr, double *F_out = nullptr) {
    const int64_t cap = pl.cap;
    uint32_t out = 0;
    const int64_t fr = row.alloc[r] - row.requested[r];
    pl.free_[r * cap + i] = fr;
    if (free_out) *free_out = fr;
    double R = 0.0, F = 0.0;
    int64_t a = row.alloc[r];
    bool present = r < 3 || ((row.alloc_present >> r) & 1u);
    if (c.fit_w[r] > 0 && present && a != 0) {
        out |= 2u;
        int64_t base = r < 2 ? row.nonzero_requested[r] : row.requested[r];
        if (a < 0 || a >= KG_CAP_LIMIT || kg_abs64(base) >= KG_VAL_LIMIT) {
            out |= 1u;
        } else {
            R = 100.0 / (double)a;
            F = c.fit_most ? kg_scaled_ratio(base, a) : kg_scaled_ratio(a - base, a);
        }
    }
    pl.fit_R[r * cap + i] = R;
    pl.fit_F[r * cap + i] = F;
    if (R_out) *R_out = R;
    if (F_out) *F_out = F;
    return out;
}
KG_HD uint32_t kg_finalize_fit(const kg_consts &c, const kg_planes &pl, int64_t i, int r, int64_t *free_out = nullptr,
                               double *R_out = nullptr, double *F_out = nullptr) {
    return kg_finalize_fit_r(c, pl, i, pl.rows[i], r, free_out, R_out, F_out);
}
// bit 0: slow (KGD_SLOW: outside the bounds, or LoadAware weights beyond cpu / memory, whose planes only the
// matrix kernel's extra-resource form reads); bit 1: outside the bounds (KGD_XSLOW)
KG_HD uint32_t kg_finalize_la_r(const kg_consts &c, const kg_planes &pl, int64_t i, const kg_node_row &row, int r,
                                double *R_out = nullptr, double *F0_out = nullptr, double *F1_out = nullptr) {
    const int64_t cap = pl.cap;
    uint32_t slow = c.la_extra != 0 ? 1u : 0u;
    int64_t a = row.la_alloc[r];
    double R = 0.0, F0 = 0.0, F1 = 0.0;
    if (a != 0) {
        if (a < 0 || a >= KG_CAP_LIMIT || kg_abs64(row.la_used[0][r]) >= KG_VAL_LIMIT ||
            kg_abs64(row.la_used[1][r]) >= KG_VAL_LIMIT) {
            slow = 3u;
        } else {
            R = 100.0 / (double)a;
            F0 = kg_scaled_ratio(a - row.la_used[0][r], a);
            F1 = kg_scaled_ratio(a - row.la_used[1][r], a);
        }
    }
    pl.la_R[r * cap + i] = R;
    pl.la_F[(0 * 2 + r) * cap + i] = F0;
    pl.la_F[(1 * 2 + r) * cap + i] = F1;
    if (R_out) {
        *R_out = R;
        *F0_out = F0;
        *F1_out = F1;
    }
    return slow;
}
KG_HD uint32_t kg_finalize_la(const kg_consts &c, const kg_planes &pl, int64_t i, int r, double *R_out = nullptr,
                              double *F0_out = nullptr, double *F1_out = nullptr) {
    return kg_finalize_la_r(c, pl, i, pl.rows[i], r, R_out, F0_out, F1_out);
}
// LoadAware planes of extra resource x (resource 2 + x), both usage variants, when LoadAware weighs it; true when
// outside the fp64 bounds.  The same operands as the cpu / memory planes: R = RN(100/a), F_v = RN(100·(a − used_v)/a
// + 2^-42), so the pair score cvt_sat(fma(−EstimatePod, R, F_v)) is the exact least-requested integer.
KG_HD bool kg_finalize_lax_r(const kg_consts &c, const kg_planes &pl, int64_t i, const kg_node_row &row, int x,
                             double *R_out = nullptr, double *F0_out = nullptr, double *F1_out = nullptr) {
    const int64_t cap = pl.cap;
    bool slow = false;
    const int64_t a = row.la_alloc_x[x];
    double R = 0.0, F0 = 0.0, F1 = 0.0;
    if (c.la_wx[x] > 0 && a != 0) {
        if (a < 0 || a >= KG_CAP_LIMIT || kg_abs64(row.la_used_x[0][x]) >= KG_VAL_LIMIT ||
            kg_abs64(row.la_used_x[1][x]) >= KG_VAL_LIMIT) {
            slow = true;
        } else {
            R = 100.0 / (double)a;
            F0 = kg_scaled_ratio(a - row.la_used_x[0][x], a);
            F1 = kg_scaled_ratio(a - row.la_used_x[1][x], a);
        }
    }
    if (pl.la_Rx) {
        pl.la_Rx[x * cap + i] = R;
        pl.la_Fx[(0 * (KG_NUM_RES - 2) + x) * cap + i] = F0;
        pl.la_Fx[(1 * (KG_NUM_RES - 2) + x) * cap + i] = F1;
    }
    if (R_out) {
        *R_out = R;
        *F0_out = F0;
        *F1_out = F1;
    }
    return slow;
}
// the bits of dflags a Reserve can change, from the committed row values
#define KGD_DYNAMIC (KGD_PODS_FULL | KGD_OVER_CPU | KGD_OVER_MEM | KGD_OVER_EPH | KGD_SLOW | KGD_XSLOW)
KG_HD uint32_t kg_dflags_dynamic(bool pods_full, const bool over[3], bool slow, bool xslow) {
    return (pods_full ? KGD_PODS_FULL : 0u) | (over[0] ? KGD_OVER_CPU : 0u) | (over[1] ? KGD_OVER_MEM : 0u) |
           (over[2] ? KGD_OVER_EPH : 0u) | (slow ? KGD_SLOW : 0u) | (xslow ? KGD_XSLOW : 0u);
}
KG_HD void kg_finalize_flags(const kg_planes &pl, int64_t i, bool slow, uint32_t fmask, bool xslow = false) {
    const kg_node_row &row = pl.rows[i];
    uint32_t df = 0;
    if (row.flags & KG_NODE_VALID) df |= KGD_VALID;
    if ((int64_t)row.pod_count + 1 > (int64_t)row.allowed_pods) df |= KGD_PODS_FULL;
    if (row.alloc[KG_RES_CPU] - row.requested[KG_RES_CPU] < 0) df |= KGD_OVER_CPU;
    if (row.alloc[KG_RES_MEMORY] - row.requested[KG_RES_MEMORY] < 0) df |= KGD_OVER_MEM;
    if (row.alloc[KG_RES_EPHEMERAL_STORAGE] - row.requested[KG_RES_EPHEMERAL_STORAGE] < 0) df |= KGD_OVER_EPH;
    if (slow) df |= KGD_SLOW;
    if (xslow) df |= KGD_XSLOW;
    if (row.flags & KG_NODE_HAS_METRIC) df |= KGD_HAS_METRIC;
    if (row.flags & KG_NODE_HAS_UPDATE_TIME) df |= KGD_HAS_UPDATE;
    if (row.flags & KG_NODE_LA_PASS_NONPROD) df |= KGD_LA_PASS_NP;
    if (row.flags & KG_NODE_LA_PASS_PROD) df |= KGD_LA_PASS_P;
    if (pl.rsv_of && pl.rsv_of[i] >= 0) df = (df & ~(KGD_VALID | KGD_SLOW | KGD_XSLOW)) | KGD_RSV;  // kg_rsv_pair owns it
    pl.metric_ns[i] = row.metric_update_ns;
    pl.fit_mask[i] = fmask;
    pl.dflags[i] = df;
}
KG_HD void kg_finalize_node(const kg_consts &c, const kg_planes &pl, int64_t i) {
    bool slow = false, xslow = false;
    uint32_t fmask = 0;
    for (int r = 0; r < KG_NUM_RES; r++) {
        const uint32_t f = kg_finalize_fit(c, pl, i, r);
        slow = slow || (f & 1u);
        if (f & 2u) fmask |= 1u << r;
    }
    xslow = slow;
    for (int r = 0; r < 2; r++) {
        const uint32_t f = kg_finalize_la(c, pl, i, r);
        slow = slow || (f & 1u);
        xslow = xslow || (f & 2u);
    }
    if (c.la_extra)
        for (int x = 0; x < KG_NUM_RES - 2; x++) xslow = kg_finalize_lax_r(c, pl, i, pl.rows[i], x) || xslow;
    kg_finalize_flags(pl, i, slow, fmask, xslow);
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
    for (int r = 0; r < KG_NUM_RES - 2; r++) {   // zero unless LoadAware weights name the resource
        row.la_used_x[0][r] += p.la_est_x[r];
        if (p.flags & KG_POD_PROD) row.la_used_x[1][r] += p.la_est_x[r];
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


// ---- NodeNUMAResource (no cpuset binding) on engine rows -----------------------------------
// Restates nodenumaresource/{plugin.go:264-373, scoring.go:55-226, resource_manager.go:195-250,
// 418-532} and topologymanager/{policy.go:94-185, policy_*.go} (the oracle's numa_pair) for zones
// holding cpu and memory.  Zones are handled in index space (bit i = zone i of the row, i < 8);
// hint masks become affinity-id masks only where the merge compares them.
//
// A hint list exists per requested resource in sorted-name order (cpu, ephemeral-storage,
// example.com/gpu, batch-cpu, batch-memory, mid-cpu, mid-memory, memory — the reference walks a Go
// map).  Zone sums are non-negative, so "total ≥ request" and "available ≥ request" are
// monotone in the mask: the list's minimum affinity size is the first prefix of the descending
// zone totals that covers the request, and the list is non-empty iff the whole-node mask fits.
// A preferred merged hint always beats a non-preferred one (policy.go:158-169), so the merge folds
// only preferred × preferred permutations when one exists; the full fold over every permutation is
// needed only for a BestEffort node without any.  kg_pods_set bounds a pod to 2 hint lists.
#define KG_NUMA_MAX_LISTS 2

struct kg_numa_out {
    bool feasible;
    uint32_t score;
    int32_t n_alloc;                  // zones with a non-zero allocation (Reserve)
    int32_t zone[KG_MAX_ZONES];       // their row zone index
    int64_t alloc[KG_MAX_ZONES][2];   // allocated cpu, memory
};

// n / d (Go int64 division) for the score quotients: when 0 ≤ n < 128·d and d < 2^46 (device; 2^40 host) the quotient
// is < 128; on the device one correctly rounded fp64 division gives it (below), on the host one fp32
// estimate (relative error < 2^-21, absolute < 2^-14) is off by at most one and a single exact int64
// multiply-compare settles it; every other operand takes the division
// Go int64 division kept out of line on the device: the kernels reach it only on the rare operands the
// fast quotients exclude, and one shared body keeps its long expansion out of every inlined caller
#if defined(__HIP_DEVICE_COMPILE__) && !defined(KG_DIV_INLINE)
__device__ __attribute__((noinline)) int64_t kg_div_slow(int64_t n, int64_t d) { return n / d; }
#else
KG_HD int64_t kg_div_slow(int64_t n, int64_t d) { return n / d; }
#endif

KG_HD int64_t kg_qdiv(int64_t n, int64_t d) {
#if !defined(KG_QDIV_F32) && defined(__HIP_DEVICE_COMPILE__)
    if (n < 0 || d <= 0 || d >= (1LL << 46) || n >= (d << 7)) return kg_div_slow(n, d);
#else
    if (n < 0 || d <= 0 || d >= (1LL << 40) || n >= (d << 7)) return kg_div_slow(n, d);
#endif
#if !defined(KG_QDIV_F32) && defined(__HIP_DEVICE_COMPILE__)
    // n < 2^53 and d < 2^46 convert to double exactly; the quotient (< 128) has an ulp ≤ 2^-46, so the
    // correctly rounded division is within 2^-47 of n / d, while a non-integer n / d lies ≥ 1 / d > 2^-46
    // below the next integer: the rounded value never reaches it and truncation gives the floor
    return (int64_t)((double)n / (double)d);
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    const float r = __builtin_amdgcn_rcpf((float)d);
#else
    const float r = 1.0f / (float)d;
#endif
    int64_t q = (int64_t)((float)n * r);
    const int64_t t = q * d;
    if (t > n) q--;
    else if (t + d <= n) q++;
    return q;
}
KG_HD int64_t kg_lr_i(int64_t req, int64_t cap) { return (cap == 0 || req > cap) ? 0 : kg_qdiv((cap - req) * 100, cap); }
KG_HD int64_t kg_mr_i(int64_t req, int64_t cap) { return cap == 0 ? 0 : kg_qdiv((req > cap ? cap : req) * 100, cap); }

// resourceAllocationScorer.score (scoring.go:187-226) where only cpu / memory can be allocatable
// (zone sums): every other resource is either native with allocatable 0 or a missing scalar key.
KG_HD uint32_t kg_numa_score_zones(const kg_consts &c, bool most, const int64_t used[2], const int64_t total[2],
                                   const kg_pod_dev &p, int64_t pod_cpu = -1) {
    int64_t s = 0, w = 0;
    for (int r = 0; r < 2; r++) {
        if (c.numa_w[r] <= 0 || total[r] == 0) continue;
        const int64_t rq = used[r] + ((r == KG_RES_CPU && pod_cpu >= 0) ? pod_cpu : p.numa_req[r]);
        s += (most ? kg_mr_i(rq, total[r]) : kg_lr_i(rq, total[r])) * c.numa_w[r];
        w += c.numa_w[r];
    }
    return w ? (uint32_t)kg_qdiv(s, w) : 0u;
}

// the same over the node's Requested / Allocatable (policy None, or nothing allocated in zones)
// `amplified`: scoreWithAmplifiedCPUs (scoring.go:99-116), the node's cpuset CPUs counted amplified
// `pod_cpu` ≥ 0 replaces the pod's cpu request (a cpuset-bound pod's amplified request, plugin.go:458-462)
KG_HD uint32_t kg_numa_score_node(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p,
                                  bool amplified = false, const int64_t *requested = nullptr, int64_t pod_cpu = -1) {
    if (!requested) requested = row.requested;
    int64_t s = 0, w = 0;
#pragma unroll   // constant indices into the pod row (a private copy in k_eval_numa2)
    for (int r = 0; r < KG_NUM_RES; r++) {
        if (c.numa_w[r] <= 0) continue;
        const bool scalar = (KG_SCALAR_RES_MASK >> r) & 1u;
        const int64_t pr = (r == KG_RES_CPU && pod_cpu >= 0) ? pod_cpu : p.numa_req[r];
        if (scalar && (pr == 0 || !((row.alloc_present >> r) & 1u))) continue;
        const int64_t a = row.alloc[r];
        if (a == 0) continue;
        int64_t rq = requested[r] + pr;
        if (amplified && r == KG_RES_CPU) rq += row.cpuset_amp_milli - row.cpuset_milli;
        s += (c.numa_most ? kg_mr_i(rq, a) : kg_lr_i(rq, a)) * c.numa_w[r];
        w += c.numa_w[r];
    }
    return w ? (uint32_t)kg_qdiv(s, w) : 0u;
}

// zone total / available of resource r ∈ {cpu, memory} for zone i (available = max(total − allocated, 0))
KG_HD int64_t kg_zone_total(const kg_node_row &row, int i, int r) {
    return ((row.zone_keys >> (2 * i + r)) & 1u) ? row.zone_total[i][r] : 0;
}
// allocated resource r of zone i as getAvailableNUMANodeResources reads it (node_allocation.go:155-177):
// with a cpu amplification ratio > 1, a zone with an allocation entry counts its cpuset CPUs amplified
KG_HD int64_t kg_zone_alloc(const kg_node_row &row, int i, int r) {
    int64_t a = row.zone_allocated[i][r];
    if (r == KG_RES_CPU && row.cpu_amplification_ratio > 1.0 && ((row.zone_alloc_keys >> (2 * i)) & 3u))
        a += row.zone_cpuset_amp[i];
    return a;
}
// key set of those allocations: the amplified entry always carries a cpu quantity
KG_HD uint32_t kg_zone_alloc_keys(const kg_node_row &row) {
    const uint32_t k = row.zone_alloc_keys;
    return row.cpu_amplification_ratio > 1.0 ? k | ((k | (k >> 1)) & 0x5555u) : k;
}
KG_HD int64_t kg_zone_avail(const kg_node_row &row, int i, int r) {
    const int64_t a = kg_zone_total(row, i, r) - kg_zone_alloc(row, i, r);
    return a > 0 ? a : 0;
}

KG_HD void kg_mask_sums(const kg_node_row &row, uint32_t m, int64_t tot[2], int64_t av[2]) {
    tot[0] = tot[1] = av[0] = av[1] = 0;
    for (int i = 0; i < KG_MAX_ZONES; i++) {
        if (!((m >> i) & 1u)) continue;
        for (int r = 0; r < 2; r++) {
            tot[r] += kg_zone_total(row, i, r);
            av[r] += kg_zone_avail(row, i, r);
        }
    }
}

KG_HD uint64_t kg_id_mask(const kg_node_row &row, uint32_t m) {
    uint64_t out = 0;
    for (int i = 0; i < KG_MAX_ZONES; i++)
        if ((m >> i) & 1u) out |= 1ull << row.zone_id[i];
    return out;
}

// lexicographic successor of a k-combination of {0..Z-1} held as an index bitmask (0 when done):
// bitmask.IterateBitMasks order within one size
KG_HD uint32_t kg_combo_next(uint32_t m, int Z) {
    int cnt = 0, t = Z - 1;
    while (t >= 0 && ((m >> t) & 1u)) { cnt++; t--; }
    int b = t;
    while (b >= 0 && !((m >> b) & 1u)) b--;
    if (b < 0) return 0;
    return (m & ((1u << b) - 1u)) | (((1u << (cnt + 1)) - 1u) << (b + 1));
}

// Zone-sum providers for the hint enumeration.  kg_zone_calc sums the canonical row's zones per
// call (host, placement kernels); kg_zone_tab reads a per-node table of every index mask's sums, id
// mask and the descending-total prefix sums, built once per node by kg_zone_tab_fill (k_eval_numa2
// keeps it in LDS, so the per-pair enumeration over a wave's pods does table lookups).  Both derive
// every value with the same functions, so the pair results are identical.
struct kg_zone_calc {
    const kg_node_row &row;
    KG_HD void sums(uint32_t m, int64_t tot[2], int64_t av[2]) const { kg_mask_sums(row, m, tot, av); }
    KG_HD uint64_t idmask(uint32_t m) const { return kg_id_mask(row, m); }
    KG_HD uint32_t next(uint32_t m, int Z) const { return kg_combo_next(m, Z); }
    // minimum affinity of resource r ∈ {cpu, memory}: fewest zones whose largest totals cover q
    KG_HD int min_k(int r, int64_t q, int Z) const {
        int64_t t[KG_MAX_ZONES];
        for (int i = 0; i < Z; i++) t[i] = kg_zone_total(row, i, r);
        int64_t acc = 0;
        for (int k = 1; k <= Z; k++) {
            int best_i = 0;
            for (int i = 1; i < Z; i++)
                if (t[i] > t[best_i]) best_i = i;
            acc += t[best_i];
            t[best_i] = -1;
            if (acc >= q) return k;
        }
        return Z;
    }
};

#define KG_ZTAB_MASKS (1 << KG_MAX_ZONES)
struct kg_zone_tab_data {
    int64_t tot[2][KG_ZTAB_MASKS], av[2][KG_ZTAB_MASKS];
    uint64_t idm[KG_ZTAB_MASKS];
    uint8_t succ[KG_ZTAB_MASKS];         // kg_combo_next(m, n_zones)
    int64_t pref[2][KG_MAX_ZONES + 1];   // pref[r][k]: the acc of kg_zone_calc::min_k after k picks
    int64_t srt[2][KG_MAX_ZONES];        // the zone totals of resource r in descending order (fill scratch)
};

struct kg_zone_tab {
    const kg_zone_tab_data &d;
    KG_HD void sums(uint32_t m, int64_t tot[2], int64_t av[2]) const {
        tot[0] = d.tot[0][m];
        tot[1] = d.tot[1][m];
        av[0] = d.av[0][m];
        av[1] = d.av[1][m];
    }
    KG_HD uint64_t idmask(uint32_t m) const { return d.idm[m]; }
    KG_HD uint32_t next(uint32_t m, int) const { return d.succ[m]; }
    KG_HD int min_k(int r, int64_t q, int Z) const {
        for (int k = 1; k <= Z; k++)
            if (d.pref[r][k] >= q) return k;
        return Z;
    }
};

// the table of one node, filled by `nlanes` cooperating lanes (1 on the host) in two rounds, `sync` (a wave
// barrier on the device) between them and after:
//  1. the sums and id masks of the masks inside one half (zones 0-3: m < 16; zones 4-7: m = h << 4) by
//     adding their zones; the descending-total order of the zones (rank, the first largest first — the
//     picks of kg_zone_calc::min_k) and each total at its rank;
//  2. every other mask as its low half + its high half (int64 sums: the order of the adds is immaterial);
//     the prefix sums of the ranked totals; the combination successors when `succ` (they depend on Z only:
//     the caller skips them while consecutive nodes keep the same zone count)
template <class Sync>
KG_HD void kg_zone_tab_fill(const kg_node_row &row, int lane, int nlanes, kg_zone_tab_data &d, Sync sync,
                            bool succ = true) {
    static_assert(KG_MAX_ZONES == 8, "the table splits masks into two 4-zone halves");
    const int Z = row.n_zones;
    const int n_masks = 1 << Z;
    for (int x = lane; x < 48; x += nlanes) {
        if (x < 32) {   // round 1a: half masks (x < 16: m = x; 16 ≤ x < 31: m = (x − 15) << 4)
            if (x == 31) continue;
            const uint32_t m = x < 16 ? (uint32_t)x : (uint32_t)(x - 15) << 4;
            if ((int)m >= n_masks) continue;
            int64_t t0 = 0, t1 = 0, a0 = 0, a1 = 0;
            uint64_t id = 0;
            for (int i = 0; i < KG_MAX_ZONES; i++) {
                if (!((m >> i) & 1u)) continue;
                t0 += kg_zone_total(row, i, 0);
                t1 += kg_zone_total(row, i, 1);
                a0 += kg_zone_avail(row, i, 0);
                a1 += kg_zone_avail(row, i, 1);
                id |= 1ull << row.zone_id[i];
            }
            d.tot[0][m] = t0;
            d.tot[1][m] = t1;
            d.av[0][m] = a0;
            d.av[1][m] = a1;
            d.idm[m] = id;
        } else {        // round 1b: the rank of zone i's total of resource r, the total stored at its rank
            const int r = (x - 32) >> 3, i = (x - 32) & 7;
            if (i >= Z) continue;
            const int64_t t = kg_zone_total(row, i, r);
            int rank = 0;
            for (int j = 0; j < Z; j++) {
                const int64_t u = kg_zone_total(row, j, r);
                rank += (u > t || (u == t && j < i)) ? 1 : 0;
            }
            d.srt[r][rank] = t;
        }
    }
    sync();
    for (int m = lane; m < n_masks; m += nlanes) {   // round 2
        const uint32_t lo = (uint32_t)m & 15u, hi = (uint32_t)m & 0xF0u;
        if (lo && hi) {
            d.tot[0][m] = d.tot[0][lo] + d.tot[0][hi];
            d.tot[1][m] = d.tot[1][lo] + d.tot[1][hi];
            d.av[0][m] = d.av[0][lo] + d.av[0][hi];
            d.av[1][m] = d.av[1][lo] + d.av[1][hi];
            d.idm[m] = d.idm[lo] | d.idm[hi];
        }
        if (succ) d.succ[m] = (uint8_t)kg_combo_next((uint32_t)m, Z);
    }
    for (int x = lane; x < 2 * (KG_MAX_ZONES + 1); x += nlanes) {
        const int r = x / (KG_MAX_ZONES + 1), k = x % (KG_MAX_ZONES + 1);
        if (k > Z) continue;
        int64_t acc = 0;
        for (int j = 0; j < k; j++) acc += d.srt[r][j];
        d.pref[r][k] = acc;
    }
}

struct kg_numa_list {
    int32_t res;       // resource id; zone resources are cpu (0) and memory (1)
    int32_t k;         // minimum affinity size: hints of this size are preferred
    bool any;          // the list holds at least one hint
    int64_t req;
};

template <class ZS>
KG_HD bool kg_list_fits(const ZS &zs, const kg_numa_list &l, uint32_t m) {
    if (l.req == 0) return true;
    if (l.res > 1) return false;
    int64_t tot[2], av[2];
    zs.sums(m, tot, av);
    return tot[l.res] >= l.req && av[l.res] >= l.req;
}

struct kg_numa_best {
    uint64_t mask;     // affinity-id mask
    bool pref;
    uint32_t score;
};

// mergeFilteredHints: one permutation's merged hint against the running best (policy.go:140-182)
KG_HD void kg_numa_fold(kg_numa_best &b, uint64_t m, bool pref, uint32_t score) {
    if (pref && !b.pref) { b = kg_numa_best{m, pref, score}; return; }
    if (!pref && b.pref) return;
    const int cm = __builtin_popcountll(m), cb = __builtin_popcountll(b.mask);
    const bool narrower = cm == cb ? m < b.mask : cm < cb;
    if (narrower || (cm == cb && score > b.score)) b = kg_numa_best{m, pref, score};
}

// score of a hint mask (generateResourceHints: the NUMA scorer over requested = total − available)
template <class ZS>
KG_HD uint32_t kg_hint_score(const kg_consts &c, const ZS &zs, const kg_pod_dev &p, uint32_t m, int64_t pod_cpu) {
    int64_t tot[2], av[2];
    zs.sums(m, tot, av);
    const int64_t used[2] = {tot[0] - av[0], tot[1] - av[1]};
    return kg_numa_score_zones(c, c.numa_hint_most != 0, used, tot, p, pod_cpu);
}

// one permutation (masks a, b in index space; `full` stands for a nil hint of an empty list)
template <class ZS>
KG_HD void kg_numa_visit(const kg_consts &c, const ZS &zs, const kg_pod_dev &p, kg_numa_best &best,
                         uint32_t a, bool a_hint, uint32_t b, bool b_hint, bool pref, int64_t pod_cpu) {
    const uint32_t m = a & b;
    if (m == 0) return;
    const bool member = (a_hint && a == m) || (b_hint && b == m);
    kg_numa_fold(best, zs.idmask(m), pref, member ? kg_hint_score(c, zs, p, m, pod_cpu) : 0u);
}

// a cpuset request on a node with a NUMA topology policy (plugin.go:297-331 → FilterByNUMANode → Allocate)
struct kg_numa_bind {
    int64_t need;        // numCPUsNeeded
    int required;        // the effective required bind policy (kg_cpu_bind_policy; UNSET ⇔ not required)
};

// trimNUMANodeResources (resource_manager.go:141-169) for a required bind policy: a zone's available cpu
// is capped by its available CPUs — after the policy's filter (whole available cores / one CPU per core)
// when those are at least the quantity — in milli-CPUs.  Hint totals are untouched.
struct kg_zone_trim {
    const kg_node_row &row;
    int64_t cap[KG_MAX_ZONES];
    KG_HD kg_zone_trim(const kg_node_row &r, int required) : row(r) {
        for (int i = 0; i < KG_MAX_ZONES; i++) {
            int64_t q = i < r.n_zones ? kg_zone_avail(r, i, KG_RES_CPU) : 0;
            if (q != 0 && required != KG_CPU_BIND_UNSET) {
                int64_t n = r.zone_cpus_avail[i];
                if (n * 1000 >= q)
                    n = required == KG_CPU_BIND_FULL_PCPUS ? r.zone_cpus_full[i]
                      : required == KG_CPU_BIND_SPREAD_BY_PCPUS ? r.zone_cores_free[i] : n;
                if (n * 1000 < q) q = n * 1000;
            }
            cap[i] = q;
        }
    }
    KG_HD void sums(uint32_t m, int64_t tot[2], int64_t av[2]) const {
        kg_mask_sums(row, m, tot, av);
        av[0] = 0;
        for (int i = 0; i < KG_MAX_ZONES; i++)
            if ((m >> i) & 1u) av[0] += cap[i];
    }
    KG_HD uint64_t idmask(uint32_t m) const { return kg_id_mask(row, m); }
    KG_HD uint32_t next(uint32_t m, int Z) const { return kg_combo_next(m, Z); }
    KG_HD int min_k(int r, int64_t q, int Z) const { return kg_zone_calc{row}.min_k(r, q, Z); }
};

template <class ZS, bool REC = true>
KG_HD void kg_numa_zoned(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o,
                         const ZS &zs, const int64_t *requested, int policy, int64_t pcpu, const kg_numa_bind *bd);
template <class ZS, bool REC = false>
KG_HD void kg_numa_zoned_one(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o,
                             const ZS &zs, const int64_t *requested, int64_t pcpu);

// the cpuset path with its own (trimmed) zone provider, out of line on the device: the hint enumeration
// of k_eval_numa2 keeps its register budget for the common, unbound pods
#if defined(__HIPCC__)
static __host__ __device__ __noinline__
#else
inline
#endif
void kg_numa_bind_zoned(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o,
                        const int64_t *requested, int policy, int64_t pcpu_eff, int required) {
    const kg_numa_bind bd{p.numa_req[KG_RES_CPU] / 1000, required};
    kg_numa_zoned(c, row, p, o, kg_zone_trim(row, required), requested, policy, pcpu_eff, &bd);
}

// Filter + Score of NodeNUMAResource for one pair; o.zone / o.alloc are what Reserve records.
// `requested`: NodeInfo.Requested the plugin sees (default the row's; the Reservation restore's view on a
// node with reservations, transformer.go:49-291 restores the snapshot NodeInfo every plugin reads).
// `reserve`: the Reserve path (Allocate on the stored hint, plugin.go:406-416) — no Filter-only checks.
// BZ: answer cpusets on NUMA-policy nodes here (host, k_numa_bind_fix); the hot device kernels pass false
// and leave those pairs infeasible for the fix-up kernel, so they carry no call into the cpuset path.
// REC: record the allocation (o.zone / o.alloc, what Reserve needs); Filter / Score callers pass false and
// get o.feasible, o.score and o.n_alloc only (no per-lane arrays written at a run-time index)
// `one`: the pair meets kg_numa_one_node, kg_numa_one_pod and kg_numa_one_pair, so the zoned part takes
// kg_numa_zoned_one (the single-zone hints only, recording the allocation when REC) instead of the whole enumeration
template <class ZS, bool BZ = true, bool REC = true>
KG_HD void kg_numa_pair_z(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o,
                          const ZS &zs, const int64_t *requested = nullptr, bool reserve = false, bool one = false) {
    if (!requested) requested = row.requested;
    o.feasible = true;
    o.score = 0;
    o.n_alloc = 0;
    if (p.flags & KG_POD_NUMA_SKIP) return;
    if (p.flags & KG_POD_NUMA_BIND_INVALID) {   // PreFilter: cpuset request not in whole cores
        o.feasible = false;
        return;
    }
    const bool opts = (row.flags & KG_NODE_NUMA_OPTIONS) != 0;
    const int policy = opts ? row.numa_policy : KG_NUMA_NONE;
    const double ratio = opts ? row.cpu_amplification_ratio : 0.0;
    const int64_t pcpu = p.numa_req[KG_RES_CPU];
    // requestCPUBind (util.go:105-122): the pod's own decision, or a node CPU bind policy for any cpu request
    bool bind = (p.flags & KG_POD_NUMA_CPU_BIND) != 0;
    const int node_bind = opts ? row.node_cpu_bind : KG_NODE_CPU_BIND_NONE;
    if (!bind && pcpu != 0 && node_bind != KG_NODE_CPU_BIND_NONE) {
        if (pcpu % 1000 != 0) {   // ErrInvalidRequestedCPUs
            o.feasible = false;
            return;
        }
        bind = true;
    }
    const bool amplified = pcpu != 0 && ratio > 1.0;
    // a cpuset-bound pod's cpu request is amplified (plugin.go:354-356, getResourceOptions :458-462)
    const int64_t pcpu_eff = bind && amplified ? (int64_t)ceil((double)pcpu * ratio) : pcpu;
    if (amplified && !reserve) {   // filterAmplifiedCPUs (plugin.go:340-373)
        if (row.flags & KG_NODE_NUMA_TOPO_INVALID) {   // GetAvailableCPUs: invalid CPU topology
            o.feasible = false;
            return;
        }
        int64_t rq = requested[KG_RES_CPU];
        const int64_t am = row.cpuset_milli;
        if (rq >= am && am > 0) rq += row.cpuset_amp_milli - am;
        if (pcpu_eff > row.alloc[KG_RES_CPU] - rq) {
            o.feasible = false;
            return;
        }
    }
    if (bind && !reserve) {   // Filter's cpuset branch (plugin.go:297-331)
        if (!(row.flags & KG_NODE_NUMA_TOPO_VALID)) {   // ErrInvalidCPUTopology (nil or invalid)
            o.feasible = false;
            return;
        }
        const int own = (int)(p.cpu_bind & 15u);
        int required = own;
        if (node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = KG_CPU_BIND_FULL_PCPUS;
        else if (node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = KG_CPU_BIND_SPREAD_BY_PCPUS;
        const int64_t ncpus = pcpu / 1000;   // numCPUsNeeded
        if ((own != KG_CPU_BIND_UNSET && own != required) ||   // ErrCPUBindPolicyConflict
            (required == KG_CPU_BIND_FULL_PCPUS && (row.cpus_per_core <= 0 || ncpus % row.cpus_per_core != 0))) {
            o.feasible = false;   // (or ErrSMTAlignmentError)
            return;
        }
        // Allocate without a NUMA hint: available CPUs after the required policy's filter (whole free cores /
        // one CPU per core), then takeCPUs, which succeeds whenever they are enough
        if (required != KG_CPU_BIND_UNSET && policy == KG_NUMA_NONE) {
            const int64_t avail = required == KG_CPU_BIND_FULL_PCPUS ? row.cpuset_full_free_cpus
                                : required == KG_CPU_BIND_SPREAD_BY_PCPUS ? row.cpuset_free_cores : 0;
            if (avail < ncpus) {
                o.feasible = false;
                return;
            }
        }
    }
    if (policy == KG_NUMA_NONE) {
        o.score = kg_numa_score_node(c, row, p, amplified, requested, pcpu_eff);
        return;
    }
    if (bind) {   // FilterByNUMANode with the cpuset options: trimmed hints, then the zone-wise take
        const int own = (int)(p.cpu_bind & 15u);
        int required = own;
        if (node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = KG_CPU_BIND_FULL_PCPUS;
        else if (node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = KG_CPU_BIND_SPREAD_BY_PCPUS;
        if constexpr (BZ) kg_numa_bind_zoned(c, row, p, o, requested, policy, pcpu_eff, required);
        else o.feasible = false;   // the caller re-evaluates these pairs (k_numa_bind_fix)
        return;
    }
    if (one) kg_numa_zoned_one<ZS, REC>(c, row, p, o, zs, requested, pcpu);
    else kg_numa_zoned<ZS, REC>(c, row, p, o, zs, requested, policy, pcpu, (const kg_numa_bind *)nullptr);
}

// hint generation, merge, Admit, allocateResourcesByHint and the zone score (the part of Filter / Score
// that depends on the zone provider); `pcpu`: the cpu request (a cpuset-bound pod's amplified one)
template <class ZS, bool REC>
KG_HD void kg_numa_zoned(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o,
                         const ZS &zs, const int64_t *requested, int policy, int64_t pcpu, const kg_numa_bind *bd) {
    const int Z = row.n_zones;
    if (Z <= 0) {
        o.feasible = false;
        return;
    }
    const uint32_t full = (1u << Z) - 1u;
    // hint lists (generateResourceHints), ordered by resource name: the resources are visited in slot order with
    // constant indices into the pod row (a run-time resource index would move the row to scratch memory) and each
    // list takes its place by the name rank of its resource (kg_consts.res_rank; at most two lists)
    kg_numa_list L[KG_NUMA_MAX_LISTS];
    int nl = 0, rank0 = 0;
#pragma unroll
    for (int r = 0; r < KG_NUM_RES; r++) {
        if (!((p.numa_present >> r) & 1u)) continue;
        const int64_t q = r == KG_RES_CPU ? pcpu : p.numa_req[r];
        kg_numa_list l{r, Z, false, q};
        bool keyed = false;   // some zone's total has the resource (totalResourceNames)
        if (r <= KG_RES_MEMORY) {
            int64_t tot_all[2], av_all[2];
            zs.sums(full, tot_all, av_all);
            keyed = (row.zone_keys & (0x5555u << r) & ((1u << (2 * Z)) - 1u)) != 0;
            l.k = zs.min_k(r, q, Z);   // minimum affinity: fewest zones whose largest totals cover q
            l.any = tot_all[r] >= q && av_all[r] >= q;
        } else if (q == 0) {
            l.k = 1;       // a zero request fits every mask
            l.any = true;
        }
        if (!l.any && !keyed) continue;   // no list for the resource
        if (nl == KG_NUMA_MAX_LISTS) {    // excluded by kg_pods_set
            o.feasible = false;
            return;
        }
        // constant indices only: the two lists stay in registers
        const int rk = c.res_rank[r];
        if (nl == 0) {
            L[0] = l;
            rank0 = rk;
        } else if (rk < rank0) {
            L[1] = L[0];
            L[0] = l;
        } else {
            L[1] = l;
        }
        nl++;
    }
    const bool single = policy == KG_NUMA_SINGLE_NUMA_NODE;
    const uint64_t dflt = zs.idmask(full);
    kg_numa_best best{dflt, false, 0u};
    if (nl == 0) {
        best = kg_numa_best{dflt, true, 0u};   // no provider hints: any affinity, preferred
    } else {
        static_assert(KG_NUMA_MAX_LISTS == 2, "the enumeration below is written for two lists");
        bool can_pref = L[0].any && !(single && L[0].k != 1);
        if (nl > 1 && (!L[1].any || (single && L[1].k != 1))) can_pref = false;
        if (can_pref) {
            for (uint32_t a = (1u << L[0].k) - 1u; a; a = zs.next(a, Z)) {
                if (!kg_list_fits(zs, L[0], a)) continue;
                if (nl == 1) {
                    kg_numa_visit(c, zs, p, best, a, true, full, false, true, pcpu);
                    continue;
                }
                if (L[0].k == 1) {
                    // a = {i}: every b it meets merges to m = a with a's own score, and repeating a
                    // candidate right after folding it is a no-op, so one visit iff some fitting b ⊇ a
                    bool hit = false;
                    if (L[1].k == 1) {
                        hit = kg_list_fits(zs, L[1], a);
                    } else {
                        for (uint32_t b = (1u << L[1].k) - 1u; b && !hit; b = zs.next(b, Z))
                            hit = (a & b) && kg_list_fits(zs, L[1], b);
                    }
                    if (hit) kg_numa_visit(c, zs, p, best, a, true, a, true, true, pcpu);
                    continue;
                }
                // a permutation with a & b == 0 is skipped by kg_numa_visit: test that before the
                // (zone-sum) fit of b, so disjoint hints cost a bit test, not a zone sum
                for (uint32_t b = (1u << L[1].k) - 1u; b; b = zs.next(b, Z))
                    if ((a & b) && kg_list_fits(zs, L[1], b)) kg_numa_visit(c, zs, p, best, a, true, b, true, true, pcpu);
            }
        }
        if (!best.pref && policy == KG_NUMA_BEST_EFFORT) {
            // no preferred permutation: the full fold, hints of every size in IterateBitMasks order
            const int ka0 = L[0].any ? 1 : 0, ka1 = L[0].any ? Z : 0;
            for (int ka = ka0; ka <= ka1; ka++) {
                for (uint32_t a = ka ? (1u << ka) - 1u : full; a; a = ka ? zs.next(a, Z) : 0u) {
                    if (ka && !kg_list_fits(zs, L[0], a)) continue;
                    const bool pa = ka == L[0].k;
                    if (nl == 1) {
                        kg_numa_visit(c, zs, p, best, a, ka != 0, full, false, pa && ka != 0, pcpu);
                        continue;
                    }
                    const int kb0 = L[1].any ? 1 : 0, kb1 = L[1].any ? Z : 0;
                    for (int kb = kb0; kb <= kb1; kb++) {
                        for (uint32_t b = kb ? (1u << kb) - 1u : full; b; b = kb ? zs.next(b, Z) : 0u) {
                            if (!(a & b) || (kb && !kg_list_fits(zs, L[1], b))) continue;
                            const bool pb = kb == L[1].k;
                            kg_numa_visit(c, zs, p, best, a, ka != 0, b, kb != 0, pa && ka != 0 && pb && kb != 0, pcpu);
                        }
                    }
                }
            }
        }
    }
    // Admit (manager.go:58-80)
    if (policy != KG_NUMA_BEST_EFFORT && !best.pref) {
        o.feasible = false;
        return;
    }
    // per allocated zone, as it is allocated: calculateAllocatableAndRequested's sums (scoring.go:118-164) and
    // allocateCPUSet's per-zone CPUs (below)
    int64_t z_tot[2] = {0, 0}, z_used[2] = {0, 0}, bd_sum = 0;
    bool bd_whole = true;
    const int req_pol = bd ? bd->required : KG_CPU_BIND_UNSET;
    if (!(single && best.mask == dflt)) {   // SingleNUMANode: the all-zones hint is nil
        // allocateResourcesByHint: zones of the hint in ascending affinity id, greedily
        // allocateResourcesByHint takes a cpuset request's original (unamplified) requests
        int64_t req[2] = {p.numa_req[0], p.numa_req[1]};
        bool want[2] = {(p.numa_present & 1u) != 0, ((p.numa_present >> 1) & 1u) != 0};
        bool inter[2] = {false, false};
        uint32_t left = 0;
        for (int i = 0; i < Z; i++)
            if ((best.mask >> row.zone_id[i]) & 1ull) left |= 1u << i;
        while (left) {
            int zi = -1;
            for (int i = 0; i < Z; i++)
                if (((left >> i) & 1u) && (zi < 0 || row.zone_id[i] < row.zone_id[zi])) zi = i;
            left &= ~(1u << zi);
            int64_t got[2] = {0, 0};
            for (int r = 0; r < 2; r++) {
                if (!want[r] || !(((row.zone_keys | kg_zone_alloc_keys(row)) >> (2 * zi + r)) & 1u)) continue;
                inter[r] = true;
                const int64_t a = kg_zone_avail(row, zi, r);
                got[r] = a < req[r] ? a : req[r];
                req[r] -= got[r];
            }
            if (got[0] != 0 || got[1] != 0) {
                if constexpr (REC) {
                    o.zone[o.n_alloc] = zi;
                    o.alloc[o.n_alloc][0] = got[0];
                    o.alloc[o.n_alloc][1] = got[1];
                }
                o.n_alloc++;
                for (int r = 0; r < 2; r++) {
                    z_tot[r] += kg_zone_total(row, zi, r);
                    const int64_t u = kg_zone_alloc(row, zi, r);
                    z_used[r] += u > 0 ? u : 0;
                }
                if (bd) {
                    const int64_t zav = req_pol == KG_CPU_BIND_FULL_PCPUS ? row.zone_cpus_full[zi]
                                      : req_pol == KG_CPU_BIND_SPREAD_BY_PCPUS ? row.zone_cores_free[zi] : row.zone_cpus_avail[zi];
                    int64_t n = got[0] / 1000;
                    if (zav < n) n = zav;
                    if (req_pol == KG_CPU_BIND_FULL_PCPUS && (row.cpus_per_core <= 0 || n % row.cpus_per_core != 0))
                        bd_whole = false;
                    bd_sum += n;
                }
            }
        }
        if ((inter[0] && req[0] != 0) || (inter[1] && req[1] != 0)) {
            o.feasible = false;
            o.n_alloc = 0;
            return;
        }
    }
    if (bd) {
        // allocateCPUSet (resource_manager.go:273-360): the available CPUs (filtered by a required policy)
        // must cover the request; each allocated zone gives min(its available CPUs, its cpu / 1000), which
        // takeCPUs always finds, and those must add up to the request exactly; a required FullPCPUs
        // policy needs whole cores from every zone (satisfiedRequiredCPUBindPolicy)
        const int64_t node_av = req_pol == KG_CPU_BIND_FULL_PCPUS ? row.cpuset_full_free_cpus
                              : req_pol == KG_CPU_BIND_SPREAD_BY_PCPUS ? row.cpuset_free_cores : row.cpuset_avail_cpus;
        bool ok = node_av >= bd->need;
        if (ok && o.n_alloc > 0) ok = bd_whole && bd_sum == bd->need;
        if (!ok) {
            o.feasible = false;
            o.n_alloc = 0;
            return;
        }
    }
    if (o.n_alloc > 0) {
        // calculateAllocatableAndRequested (scoring.go:118-164) over the allocated zones; with a cpuset the
        // requested cpu is the node's amplified cpuset CPUs
        if (bd) z_used[KG_RES_CPU] = row.cpuset_amp_milli;
        o.score = kg_numa_score_zones(c, c.numa_most != 0, z_used, z_tot, p, pcpu);
    } else if (bd) {
        int64_t rq[KG_NUM_RES];
        #pragma unroll
        for (int r = 0; r < KG_NUM_RES; r++) rq[r] = requested[r];
        rq[KG_RES_CPU] = row.cpuset_amp_milli;
        o.score = kg_numa_score_node(c, row, p, false, rq, pcpu);
    } else {
        o.score = kg_numa_score_node(c, row, p, false, requested);
    }
}

// The common NodeNUMAResource pair, answered without the hint enumeration: the node has ≥ 2 zones with distinct
// affinity ids, every zone carries cpu and memory totals, and its policy is SingleNUMANode or Restricted
// (kg_numa_one_node); the pod's hint lists are at most cpu and memory (no zero request of another resource makes a
// list of its own) and each list's minimum affinity is one zone (kg_numa_one_pair: the request is within the largest
// zone total).  Then kg_numa_zoned's preferred pass visits exactly the single zones that fit every list, in index
// order, each merging to itself with its own hint score (the k = 1 branch: visit(a, a) / visit(a, full)); the fold
// keeps the first of the narrowest, replaced by a smaller id mask or a higher score; no fitting zone is a
// non-preferred merge, which Admit rejects under both policies; the allocation takes the chosen zone alone.
KG_HD bool kg_numa_one_node(const kg_node_row &row) {
    const int Z = row.n_zones;
    if (Z < 2 || Z > KG_MAX_ZONES || (row.numa_policy != KG_NUMA_SINGLE_NUMA_NODE && row.numa_policy != KG_NUMA_RESTRICTED))
        return false;
    uint64_t ids = 0;
    for (int i = 0; i < KG_MAX_ZONES; i++)
        if (i < Z) ids |= 1ull << (row.zone_id[i] & 63);
    const uint32_t keys = row.zone_keys & ((1u << (2 * Z)) - 1u);
    return __builtin_popcountll(ids) == Z && keys == ((1u << (2 * Z)) - 1u);
}
// the pod side that does not depend on the node (once per pod): no resource beyond cpu / memory makes a hint list
KG_HD bool kg_numa_one_pod(const kg_pod_dev &p) {
    bool ok = true;
#pragma unroll
    for (int r = 2; r < KG_NUM_RES; r++) ok = ok && !(((p.numa_present >> r) & 1u) && p.numa_req[r] == 0);
    return ok;
}
// `mx[r]`: the node's largest zone total of cpu / memory (kg_zone_total)
KG_HD bool kg_numa_one_pair(const kg_pod_dev &p, const int64_t mx[2]) {
    return (!(p.numa_present & 1u) || p.numa_req[KG_RES_CPU] <= mx[0]) &&
           (!(p.numa_present & 2u) || p.numa_req[KG_RES_MEMORY] <= mx[1]);
}

// the three conditions for one pair on its own (the per-pair kernels: k_resolve's re-scores, the cache refresh, the
// placement chunks), the largest zone totals taken from the row
KG_HD bool kg_numa_one(const kg_node_row &row, const kg_pod_dev &p) {
    if (!(row.flags & KG_NODE_NUMA_OPTIONS) || !kg_numa_one_node(row) || !kg_numa_one_pod(p)) return false;
    int64_t mx[2] = {0, 0};
    for (int i = 0; i < KG_MAX_ZONES; i++) {
        if (i >= row.n_zones) break;
        const int64_t t0 = kg_zone_total(row, i, 0), t1 = kg_zone_total(row, i, 1);
        mx[0] = t0 > mx[0] ? t0 : mx[0];
        mx[1] = t1 > mx[1] ? t1 : mx[1];
    }
    return kg_numa_one_pair(p, mx);
}

template <class ZS, bool REC>
KG_HD void kg_numa_zoned_one(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o,
                             const ZS &zs, const int64_t *requested, int64_t pcpu) {
    const int Z = row.n_zones;
    const bool hc = (p.numa_present & 1u) != 0, hm = (p.numa_present & 2u) != 0;
    if (!hc && !hm) {   // no hint lists: any affinity, preferred; nothing to allocate in zones
        o.score = kg_numa_score_node(c, row, p, false, requested);
        return;
    }
    const int64_t qc = pcpu, qm = p.numa_req[KG_RES_MEMORY];
    bool pref = false;
    uint64_t bmask = 0;
    uint32_t bscore = 0;
    int bi = 0;
    for (int i = 0; i < KG_MAX_ZONES; i++) {
        if (i >= Z) break;
        int64_t tot[2], av[2];
        zs.sums(1u << i, tot, av);
        const bool fit = (!hc || qc == 0 || (tot[0] >= qc && av[0] >= qc)) && (!hm || qm == 0 || (tot[1] >= qm && av[1] >= qm));
        if (!fit) continue;
        const int64_t used[2] = {tot[0] - av[0], tot[1] - av[1]};
        const uint32_t sc = kg_numa_score_zones(c, c.numa_hint_most != 0, used, tot, p, pcpu);
        const uint64_t m = zs.idmask(1u << i);
        if (!pref || m < bmask || sc > bscore) {   // kg_numa_fold between preferred single-zone masks
            pref = true;
            bmask = m;
            bscore = sc;
            bi = i;
        }
    }
    if (!pref) {   // Admit (SingleNUMANode / Restricted)
        o.feasible = false;
        return;
    }
    // allocateResourcesByHint on the one zone (kg_numa_zoned's allocation loop)
    const uint32_t keys = row.zone_keys | kg_zone_alloc_keys(row);
    int64_t got[2] = {0, 0};
    bool short_ = false;
    const int64_t req[2] = {p.numa_req[0], p.numa_req[1]};
    const bool want[2] = {hc, hm};
    for (int r = 0; r < 2; r++) {
        if (!want[r] || !((keys >> (2 * bi + r)) & 1u)) continue;
        const int64_t a = kg_zone_avail(row, bi, r);
        got[r] = a < req[r] ? a : req[r];
        short_ = short_ || req[r] - got[r] != 0;
    }
    if (short_) {
        o.feasible = false;
        return;
    }
    if (got[0] != 0 || got[1] != 0) {
        if constexpr (REC) {   // what Reserve records (kg_numa_apply)
            o.zone[0] = bi;
            o.alloc[0][0] = got[0];
            o.alloc[0][1] = got[1];
        }
        o.n_alloc = 1;
        int64_t z_tot[2], z_used[2];
        for (int r = 0; r < 2; r++) {
            z_tot[r] = kg_zone_total(row, bi, r);
            const int64_t u = kg_zone_alloc(row, bi, r);
            z_used[r] = u > 0 ? u : 0;
        }
        o.score = kg_numa_score_zones(c, c.numa_most != 0, z_used, z_tot, p, pcpu);
    } else {
        o.score = kg_numa_score_node(c, row, p, false, requested);
    }
}

// Out of line on the device: the sequential k_resolve and the placement-chunk kernel keep their own
// register budget instead of inheriting the hint enumeration's
#if defined(__HIPCC__)
static __host__ __device__ __noinline__
#else
inline
#endif
void kg_numa_pair(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o,
                  const int64_t *requested = nullptr, bool reserve = false) {
#if defined(__HIP_DEVICE_COMPILE__)
    kg_numa_pair_z<kg_zone_calc, false>(c, row, p, o, kg_zone_calc{row}, requested, reserve, kg_numa_one(row, p));
#else
    kg_numa_pair_z(c, row, p, o, kg_zone_calc{row}, requested, reserve);
#endif
}

// kg_numa_pair with the cpuset-on-NUMA-policy path answered (the placement kernels of a binding batch call
// it behind kg_consts.numa_bz; out of line like kg_numa_pair)
#if defined(__HIPCC__)
static __host__ __device__ __noinline__
#else
inline
#endif
void kg_numa_pair_bz(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o) {
    kg_numa_pair_z<kg_zone_calc, true>(c, row, p, o, kg_zone_calc{row});
}
KG_HD void kg_numa_pair_any(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, kg_numa_out &o) {
    if (c.numa_bz) kg_numa_pair_bz(c, row, p, o);
    else kg_numa_pair(c, row, p, o);
}

// Filter + Score only (no allocation record), by value: feasible << 32 | score (the chunk and resolve kernels'
// per-pair calls, out of line like kg_numa_pair)
#if defined(__HIPCC__)
static __host__ __device__ __noinline__
#else
inline
#endif
uint64_t kg_numa_eval_any(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p) {
    kg_numa_out o;
    const bool one = kg_numa_one(row, p);
    if (c.numa_bz) kg_numa_pair_z<kg_zone_calc, true, false>(c, row, p, o, kg_zone_calc{row}, nullptr, false, one);
    else kg_numa_pair_z<kg_zone_calc, false, false>(c, row, p, o, kg_zone_calc{row}, nullptr, false, one);
    return ((uint64_t)(o.feasible ? 1u : 0u) << 32) | o.score;
}

// Reserve's cpuset decision for a pair (plugin.go:375-404): requestCPUBind (util.go:105-122) and
// getCPUBindPolicy (util.go:85-103) — *required: the required bind policy (the pod's own, else the node's CPU
// bind policy; UNSET ⇔ none), *take: the policy the accumulator takes with (required, else the pod's
// preferred).  A pod skipped by PreFilter or with an invalid cpu request never reaches Reserve.
KG_HD bool kg_numa_binds(const kg_node_row &row, const kg_pod_dev &p, int &required, int &take) {
    required = take = KG_CPU_BIND_UNSET;
    if (p.flags & (KG_POD_NUMA_SKIP | KG_POD_NUMA_BIND_INVALID)) return false;
    const bool opts = (row.flags & KG_NODE_NUMA_OPTIONS) != 0;
    const int node_bind = opts ? row.node_cpu_bind : KG_NODE_CPU_BIND_NONE;
    const int64_t pcpu = p.numa_req[KG_RES_CPU];
    const bool own = (p.flags & KG_POD_NUMA_CPU_BIND) != 0;
    if (!own && (pcpu == 0 || node_bind == KG_NODE_CPU_BIND_NONE || pcpu % 1000 != 0)) return false;
    required = own ? (int)(p.cpu_bind & 15u) : KG_CPU_BIND_UNSET;
    if (required == KG_CPU_BIND_UNSET) {
        if (node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = KG_CPU_BIND_FULL_PCPUS;
        else if (node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = KG_CPU_BIND_SPREAD_BY_PCPUS;
    }
    take = required != KG_CPU_BIND_UNSET ? required : (int)((p.cpu_bind >> 4) & 15u);
    return true;
}

// the zone allocations of a feasible Reserve hint into the row
KG_HD void kg_numa_apply(kg_node_row &row, const kg_numa_out &o) {
    if (!o.feasible) return;
    for (int j = 0; j < o.n_alloc; j++) {
        const int zi = o.zone[j];
        for (int r = 0; r < 2; r++) {
            if (o.alloc[j][r] == 0) continue;
            row.zone_allocated[zi][r] += o.alloc[j][r];
            row.zone_alloc_keys |= 1u << (2 * zi + r);
        }
    }
}

// Reserve of NodeNUMAResource (plugin.go:375-419): record the zone allocations of the chosen node — the
// hint of its Filter (for a cpuset, the trimmed hint of FilterByNUMANode with the cpuset options) and
// allocateResourcesByHint on the original requests.  The cpuset itself is taken on the host (kg_cpuset.cpp).
KG_HD void kg_numa_commit(const kg_consts &c, kg_node_row &row, const kg_pod_dev &p) {
    if (!(c.plugins & KG_PLUGIN_NUMA) || !(row.flags & KG_NODE_NUMA_OPTIONS) || row.numa_policy == KG_NUMA_NONE ||
        !(row.flags & KG_NODE_NUMA_TOPO_VALID))
        return;
    kg_numa_out o;
    int required, take;
    if (kg_numa_binds(row, p, required, take)) {
        const int64_t pcpu = p.numa_req[KG_RES_CPU];
        const double ratio = row.cpu_amplification_ratio;
        const int64_t pcpu_eff = pcpu != 0 && ratio > 1.0 ? (int64_t)ceil((double)pcpu * ratio) : pcpu;
        o.feasible = true;
        o.score = 0;
        o.n_alloc = 0;
        kg_numa_bind_zoned(c, row, p, o, row.requested, row.numa_policy, pcpu_eff, required);
    } else {
        kg_numa_pair(c, row, p, o, nullptr, true);
    }
    kg_numa_apply(row, o);
}

// kg_numa_commit over a prebuilt zone table of the (pre-commit) row (k_resolve: built by one wave in LDS, so the
// hint enumeration of the Reserve does table lookups instead of summing zones per mask); the cpuset path keeps
// its trimmed provider.  Same allocation as kg_numa_commit.  Out of line on the device (the resolve keeps its
// register budget).
#if defined(__HIPCC__)
static __host__ __device__ __noinline__
#else
inline
#endif
void kg_numa_commit_tab(const kg_consts &c, kg_node_row &row, const kg_pod_dev &p, const kg_zone_tab_data &zt) {
    if (!(c.plugins & KG_PLUGIN_NUMA) || !(row.flags & KG_NODE_NUMA_OPTIONS) || row.numa_policy == KG_NUMA_NONE ||
        !(row.flags & KG_NODE_NUMA_TOPO_VALID))
        return;
    int required, take;
    if (kg_numa_binds(row, p, required, take)) {
        kg_numa_commit(c, row, p);
        return;
    }
    kg_numa_out o;
    kg_numa_pair_z<kg_zone_tab, false, true>(c, row, p, o, kg_zone_tab{zt}, nullptr, true, kg_numa_one(row, p));
    kg_numa_apply(row, o);
}

// Exact int64 evaluation of one (pod, node) pair from the canonical row with NodeInfo's Requested /
// NonZeroRequested / pod count given separately (the row's own, or the Reservation restore's view).
KG_HD void kg_pair_view(const kg_consts &c, const kg_node_row &row, const int64_t *requested, const int64_t *nonzero,
                        int64_t pod_count, uint32_t df, const kg_pod_dev &p, int64_t now_ns, bool &feasible,
                        uint32_t &fit, uint32_t &la) {
    // every row field first, as independent loads (on the device the row is in global memory: loads
    // interleaved with the compares below would each wait for the previous one); the later named slots
    // (KG_FAST_RES.., rare) are read where a pod uses them, so they cost the common pairs no registers
    int64_t al[KG_FAST_RES], rq[KG_FAST_RES];
#pragma unroll
    for (int r = 0; r < KG_FAST_RES; r++) {
        al[r] = row.alloc[r];
        rq[r] = requested[r];
    }
    const int64_t nz[2] = {nonzero[0], nonzero[1]};
    const int v = (p.flags & KG_POD_LA_PROD_SCORE) ? 1 : 0;
    const int64_t la_a[2] = {row.la_alloc[0], row.la_alloc[1]};
    const int64_t la_u[2] = {row.la_used[v][0], row.la_used[v][1]};
    const uint32_t rflags = row.flags, apresent = row.alloc_present;
    const int64_t allowed = (int64_t)row.allowed_pods;
    bool expired = kg_metric_expired(c, df, row.metric_update_ns, now_ns);
    bool ok = (rflags & KG_NODE_VALID) != 0;
    if (c.plugins & KG_PLUGIN_FIT) {
        if (pod_count + 1 > allowed) ok = false;
        if (p.flags & KG_POD_HAS_REQUEST) {
#pragma unroll
            for (int r = 0; r < KG_FAST_RES; r++) {
                bool chk = r < 3 || ((p.request_present >> r) & 1u);
                if (chk && p.req[r] > al[r] - rq[r]) ok = false;
            }
#pragma unroll   // (constant indices: the pod row may be a private copy)
            for (int r = KG_FAST_RES; r < KG_NUM_RES; r++)
                if (((p.request_present >> r) & 1u) && p.req[r] > row.alloc[r] - requested[r]) ok = false;
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
#pragma unroll
        for (int r = 0; r < KG_NUM_RES; r++) {
            if (!((p.fit_mask >> r) & 1u)) continue;
            bool present = r < 3 || ((apresent >> r) & 1u);
            int64_t a = r < KG_FAST_RES ? al[r] : row.alloc[r];
            if (!present || a == 0) continue;
            int64_t base = r < 2 ? nz[r] : r < KG_FAST_RES ? rq[r] : requested[r];
            int64_t req = base + p.fit_pr_i[r];
            int64_t q;
            // kg_qdiv: the exact quotient by one fp64 division on the device (a software int64 division otherwise)
            if (c.fit_most) q = kg_qdiv((req > a ? a : req) * 100, a);
            else q = req > a ? 0 : kg_qdiv((a - req) * 100, a);
            s += q * c.fit_w[r];
            w += c.fit_w[r];
        }
        fit = w ? (uint32_t)kg_qdiv(s, w) : 0;
    }
    if ((c.plugins & KG_PLUGIN_LOADAWARE) && kg_la_valid(c, df, expired)) {
        int64_t s = 0;
        for (int r = 0; r < 2; r++) {
            if (c.la_w[r] == 0) continue;
            int64_t a = la_a[r];
            int64_t req = p.la_est_i[r] + la_u[r];
            int64_t q = (a == 0 || req > a) ? 0 : kg_qdiv((a - req) * 100, a);
            s += q * c.la_w[r];
        }
        if (c.la_extra) {
            for (int r = 0; r < KG_NUM_RES - 2; r++) {
                if (c.la_wx[r] == 0) continue;
                const int64_t a = row.la_alloc_x[r];
                const int64_t req = p.la_est_x[r] + row.la_used_x[v][r];
                s += ((a == 0 || req > a) ? 0 : kg_qdiv((a - req) * 100, a)) * c.la_wx[r];
            }
        }
        la = c.la_wsum ? (uint32_t)kg_qdiv(s, c.la_wsum) : 0;
    }
}

// Exact int64 evaluation of one (pod, node) pair straight from the canonical row (slow path).
KG_HD void kg_pair_exact(const kg_consts &c, const kg_node_row &row, uint32_t df, const kg_pod_dev &p,
                         int64_t now_ns, bool &feasible, uint32_t &fit, uint32_t &la) {
    kg_pair_view(c, row, row.requested, row.nonzero_requested, row.pod_count, df, p, now_ns, feasible, fit, la);
}

// ---- Reservation on engine rows ------------------------------------------------------------
// Restates reservation/{transformer.go:49-346 (restore), plugin.go:311-476 (Filter, fitsNode),
// scoring.go:42-203 (PreScore order preference, scoreReservation), nominator.go:76-135} and
// ReservationInfo.AddAssignedPod (reservation_info.go:379-388) per (pod, node) — the oracle's
// rsv_* functions.  A node's slots are walked in kg_rsv_set order (the reservation cache walks a Go
// map, cache.go:256).  Pod requests are PodRequestsAndLimits (kg_pod_dev.numa_req / numa_present).
#define KG_MIB200 (200LL * 1024 * 1024)

KG_HD int64_t kg_rl_get(const kg_resource_list &l, int r) { return ((l.present >> r) & 1u) ? l.v[r] : 0; }

struct kg_rsv_view {
    bool has_state;                        // nodeReservationStates[node] exists
    int32_t n_matched;
    uint32_t matched;                      // bit i ⇔ slot i of the node matches (ascending = the slot order)
    int64_t requested[KG_NUM_RES];         // NodeInfo.Requested after the restore
    int64_t nonzero[2];                    // NodeInfo.NonZeroRequested after the restore
    int64_t pod_count;                     // len(NodeInfo.Pods) after the restore
    int64_t pod_requested[KG_NUM_RES];     // nodeRState.podRequested
    int64_t r_allocated[KG_NUM_RES];       // nodeRState.rAllocated
};

// updateNodeInfoRequested / NodeInfo.RemovePod of a pod requesting `l` (calculateResource with
// GetNonzeroRequests' 100m / 200Mi defaults for absent cpu / memory keys)
KG_HD void kg_rsv_update(kg_rsv_view &v, const kg_resource_list &l, int64_t sign) {
    #pragma unroll
    for (int r = 0; r < KG_NUM_RES; r++) v.requested[r] += sign * kg_rl_get(l, r);
    v.nonzero[0] += sign * ((l.present & 1u) ? l.v[0] : 100);
    v.nonzero[1] += sign * ((l.present & 2u) ? l.v[1] : KG_MIB200);
}
KG_HD bool kg_rsv_usable(const kg_reservation &r) {
    return (r.flags & KG_RSV_AVAILABLE) && !((r.flags & KG_RSV_ALLOCATE_ONCE) && r.n_assigned > 0);
}
KG_HD bool kg_rsv_match(const kg_pod_dev &p, const kg_reservation &r) {
    if (p.rsv_owner < 0 || p.rsv_owner > 31 || !((r.owner_classes >> p.rsv_owner) & 1u)) return false;
    if (p.rsv_aff >= 0 && (p.rsv_aff > 31 || !((r.affinity_classes >> p.rsv_aff) & 1u))) return false;
    return true;
}
// quotav1.SubtractWithNonNegativeResult(a, b)[q]
KG_HD int64_t kg_rsv_remained(const kg_reservation &r, int q) {
    int64_t x = kg_rl_get(r.allocatable, q) - kg_rl_get(r.allocated, q);
    return x > 0 ? x : 0;
}

KG_HD void kg_rsv_restore(const kg_node_row &row, const kg_reservation *rs, int nr, const kg_pod_dev &p, kg_rsv_view &v) {
    v.has_state = false;
    v.n_matched = 0;
    v.matched = 0;
    #pragma unroll
    for (int r = 0; r < KG_NUM_RES; r++) {
        v.requested[r] = row.requested[r];
        v.pod_requested[r] = row.requested[r];
        v.r_allocated[r] = 0;
    }
    v.nonzero[0] = row.nonzero_requested[0];
    v.nonzero[1] = row.nonzero_requested[1];
    v.pod_count = row.pod_count;
    // slot sets as bitmasks (KG_MAX_RSV_PER_NODE ≤ 32), walked in ascending slot order: no per-lane arrays at
    // run-time indices (on the device those live in scratch memory)
    static_assert(KG_MAX_RSV_PER_NODE <= 32, "slot sets are 32-bit masks");
    uint32_t unm = 0;
    for (int i = 0; i < nr; i++) {
        const kg_reservation &r = rs[i];
        if (!kg_rsv_usable(r)) continue;
        if (!(r.flags & KG_RSV_UNSCHEDULABLE) && kg_rsv_match(p, r)) v.matched |= 1u << i;
        else if (r.n_assigned > 0) unm |= 1u << i;
    }
    v.n_matched = __builtin_popcount(v.matched);
    if (v.n_matched == 0 && unm == 0) return;
    if (p.rsv_aff >= 0 && v.n_matched == 0) return;  // the affinity needs a match: node left alone
    v.has_state = true;
    for (uint32_t m = unm; m; m &= m - 1u) {  // restoreUnmatchedReservations
        const kg_reservation &r = rs[__builtin_ctz(m)];
        kg_rsv_update(v, r.allocatable, -1);
        kg_resource_list rem;
        rem.present = r.allocatable.present | r.allocated.present;
        rem._pad = 0;
        bool zero = true;
        #pragma unroll
        for (int q = 0; q < KG_NUM_RES; q++) {
            rem.v[q] = ((rem.present >> q) & 1u) ? kg_rsv_remained(r, q) : 0;
            if (rem.v[q] != 0) zero = false;
        }
        if (!zero) kg_rsv_update(v, rem, +1);
    }
    #pragma unroll
    for (int q = 0; q < KG_NUM_RES; q++) v.pod_requested[q] = v.requested[q];
    for (uint32_t m = v.matched; m; m &= m - 1u) {  // restoreMatchedReservation → RemovePod(reserve pod)
        const kg_reservation &r = rs[__builtin_ctz(m)];
        kg_rsv_update(v, r.allocatable, -1);
        v.pod_count -= 1;
        #pragma unroll
        for (int q = 0; q < KG_NUM_RES; q++) v.r_allocated[q] += kg_rl_get(r.allocated, q);
    }
}

// fitsNode(podRequests, nodeInfo, nodeRState, rInfo, preemptible = nil) (plugin.go:427-476)
KG_HD bool kg_rsv_fits_node(const kg_node_row &row, const kg_rsv_view &v, const kg_reservation &r, const kg_pod_dev &p) {
    if (v.pod_count - v.n_matched + 1 > (int64_t)row.allowed_pods) return false;
    const uint32_t scal = p.numa_present & KG_SCALAR_RES_MASK;
    if (p.numa_req[0] == 0 && p.numa_req[1] == 0 && p.numa_req[2] == 0 && scal == 0) return true;
    #pragma unroll
    for (int q = 0; q < KG_NUM_RES; q++) {
        if (q >= 3 && !((scal >> q) & 1u)) continue;
        const int64_t free_q = row.alloc[q] - (v.pod_requested[q] - kg_rsv_remained(r, q) - v.r_allocated[q]);
        if (p.numa_req[q] > free_q) return false;
    }
    return true;
}

// filterWithReservations over the slots of `set` (bit i ⇔ slot i, ascending) (plugin.go:377-425)
KG_HD bool kg_rsv_filter_with(const kg_node_row &row, const kg_rsv_view &v, const kg_reservation *rs, uint32_t set,
                              bool required, const kg_pod_dev &p) {
    bool ok = false;
    for (uint32_t m = set; m && !ok; m &= m - 1u) {
        const kg_reservation &r = rs[__builtin_ctz(m)];
        if ((r.allocatable.present & p.numa_present) == 0) continue;
        const bool node_fits = kg_rsv_fits_node(row, v, r, p);
        if (r.policy == KG_RSV_POLICY_DEFAULT || r.policy == KG_RSV_POLICY_ALIGNED) {
            ok = node_fits;
        } else if (r.policy == KG_RSV_POLICY_RESTRICTED) {
            bool fits = true;  // Mask(podRequests, names) ≤ Allocatable − Mask(Allocated, names)
            #pragma unroll
            for (int q = 0; q < KG_NUM_RES; q++) {
                if (!((r.allocatable.present >> q) & 1u) || !((p.numa_present >> q) & 1u)) continue;
                const int64_t rem = r.allocatable.v[q] - kg_rl_get(r.allocated, q);
                if (p.numa_req[q] > (rem > 0 ? rem : 0)) fits = false;
            }
            ok = fits && node_fits;
        }
    }
    return ok || !required;
}

// findMostPreferredReservationByOrder (scoring.go:162-181) over the slots of `set` (ascending): the slot or −1;
// *order
KG_HD int kg_rsv_most_preferred(const kg_reservation *rs, uint32_t set, int64_t &order) {
    order = INT64_MAX;
    int hi = -1;
    for (uint32_t m = set; m; m &= m - 1u) {
        const int i = __builtin_ctz(m);
        const int64_t o = rs[i].order;
        if (o != 0 && order > o) {
            order = o;
            hi = i;
        }
    }
    return hi;
}

// scoreReservation (scoring.go:183-203): MostAllocated over RemoveZeros(Allocatable) in MilliValue
KG_HD uint32_t kg_rsv_score(const kg_reservation &r, const kg_pod_dev &p) {
    int64_t w = 0, s = 0;
    #pragma unroll
    for (int q = 0; q < KG_NUM_RES; q++) {
        if (!((r.allocatable.present >> q) & 1u) || r.allocatable.v[q] == 0) continue;
        w++;
        const int64_t cap = r.allocatable.v[q];
        const int64_t req = (((p.numa_present >> q) & 1u) ? p.numa_req[q] : 0) + kg_rl_get(r.allocated, q);
        const int64_t m = q == KG_RES_CPU ? 1 : 1000;  // Quantity.MilliValue of the stored unit
        if (req <= cap) s += kg_qdiv(100 * (req * m), cap * m);
    }
    return w <= 0 ? 0u : (uint32_t)kg_qdiv(s, w);
}

// NominateReservation (nominator.go:76-135): slot index or −1
KG_HD int kg_rsv_nominate(const kg_node_row &row, const kg_rsv_view &v, const kg_reservation *rs, const kg_pod_dev &p) {
    uint32_t cand = 0;
    for (uint32_t m = v.matched; m; m &= m - 1u) {
        const uint32_t bit = m & (~m + 1u);
        if (kg_rsv_filter_with(row, v, rs, bit, true, p)) cand |= bit;
    }
    if (cand == 0) return -1;
    int64_t order;
    const int hi = kg_rsv_most_preferred(rs, cand, order);
    if (hi >= 0) return hi;
    int best = -1;  // sort.Slice by score descending: insertion sort (≤ 12 items) keeps the first
    uint32_t bs = 0;
    for (uint32_t m = cand; m; m &= m - 1u) {
        const int i = __builtin_ctz(m);
        const uint32_t sc = kg_rsv_score(rs[i], p);
        if (best < 0 || sc > bs) {
            bs = sc;
            best = i;
        }
    }
    return best;
}

struct kg_rsv_out {
    bool feasible;
    uint32_t fit, la, numa; // plugin scores on the restored NodeInfo
    uint32_t raw;           // Reservation.Score before the preferred-node override and NormalizeScore
    int64_t order;          // PreScore node order (INT64_MAX: none)
    int32_t nominated;      // slot of the nominated reservation, −1 none
};

// Filter + Score of one (pod, node-with-reservations) pair.  NUMA = false: a form without the NodeNUMAResource call
// (the device kernels of a profile without that plugin: its call frame would otherwise cost them scratch memory).
template <bool NUMA = true>
KG_HD void kg_rsv_pair(const kg_consts &c, const kg_node_row &row, uint32_t df, const kg_reservation *rs, int nr,
                       const kg_pod_dev &p, int64_t now_ns, kg_rsv_out &o) {
    kg_rsv_view v;
    kg_rsv_restore(row, rs, nr, p, v);
    bool feas;
    kg_pair_view(c, row, v.requested, v.nonzero, v.pod_count, df, p, now_ns, feas, o.fit, o.la);
    o.numa = 0;
    if (NUMA && (c.plugins & KG_PLUGIN_NUMA)) {
        // NodeNUMAResource on the restored NodeInfo; its own RestoreReservation hands back only the
        // reservations' cpusets (reservation.go:68-122), which reservations of non-binding pods do not hold
        kg_numa_out no;
        kg_numa_pair(c, row, p, no, v.requested);
        feas = feas && no.feasible;
        o.numa = no.score;
    }
    if (v.n_matched == 0) feas = feas && p.rsv_aff < 0;  // Reservation.Filter (plugin.go:351-369)
    else feas = feas && kg_rsv_filter_with(row, v, rs, v.matched, p.rsv_aff >= 0, p);
    o.feasible = feas;
    o.raw = 0;
    o.order = INT64_MAX;
    o.nominated = -1;
    if (feas && v.n_matched > 0) {
        kg_rsv_most_preferred(rs, v.matched, o.order);
        o.nominated = kg_rsv_nominate(row, v, rs, p);
        if (o.nominated >= 0) o.raw = kg_rsv_score(rs[o.nominated], p);
    }
}

// Reservation.Reserve → ReservationInfo.AddAssignedPod: Allocated += Mask(requests, ResourceNames)
KG_HD void kg_rsv_commit(kg_reservation &r, const kg_pod_dev &p) {
    const uint32_t m = p.numa_present & r.allocatable.present;
    for (int q = 0; q < KG_NUM_RES; q++)
        if ((m >> q) & 1u) r.allocated.v[q] = kg_rl_get(r.allocated, q) + p.numa_req[q];
    r.allocated.present |= m;
    r.n_assigned += 1;
}

// ---- ElasticQuota (plugin.go:210-255 PreFilter, :323-337 Reserve) ----------------------------
KG_HD bool kg_quota_leq(const kg_pod_dev &p, const kg_resource_list &used, const kg_resource_list &limit) {
    for (int q = 0; q < KG_NUM_RES; q++)
        if (((limit.present >> q) & 1u) && ((p.numa_present >> q) & 1u) && p.numa_req[q] + kg_rl_get(used, q) > limit.v[q])
            return false;
    return true;
}
// the pod's group g; with EnableCheckParentQuota also checkQuotaRecursive (plugin_helper.go:281-297):
// every ancestor below the root passes used + request ≤ usedLimit (kg_quota_set bounds the chains)
KG_HD bool kg_quota_pass(const kg_quota *qs, int32_t g, const kg_pod_dev &p, bool check_parent) {
    const kg_quota &q = qs[g];
    if (!kg_quota_leq(p, q.used, q.used_limit)) return false;
    if ((p.flags & KG_POD_NON_PREEMPTIBLE) && !kg_quota_leq(p, q.non_preemptible_used, q.min)) return false;
    if (check_parent)
        for (int32_t a = q.parent, d = 0; a >= 0 && d < KG_QUOTA_MAX_DEPTH; a = qs[a].parent, d++)
            if (!kg_quota_leq(p, qs[a].used, qs[a].used_limit)) return false;
    return true;
}
KG_HD void kg_rl_add_pod(kg_resource_list &l, const kg_pod_dev &p) {
    for (int q = 0; q < KG_NUM_RES; q++)
        if ((p.numa_present >> q) & 1u) l.v[q] = kg_rl_get(l, q) + p.numa_req[q];
    l.present |= p.numa_present;
}
// ReservePod → updateGroupDeltaUsedNoLock: the group and all its ancestors (group_quota_manager.go:227-238)
KG_HD void kg_quota_commit(kg_quota *qs, int32_t g, const kg_pod_dev &p) {
    for (int32_t a = g, d = 0; a >= 0 && d <= KG_QUOTA_MAX_DEPTH; a = qs[a].parent, d++) {
        kg_rl_add_pod(qs[a].used, p);
        if (p.flags & KG_POD_NON_PREEMPTIBLE) kg_rl_add_pod(qs[a].non_preemptible_used, p);
    }
}
