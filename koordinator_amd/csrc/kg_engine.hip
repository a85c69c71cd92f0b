// kg_engine.hip — HBM-resident node snapshot + CDNA4 Filter/Score kernels behind the C-ABI.
//
// Hot kernel k_eval (matrix mode, reference hot loops #1 Filter and #2 Score of
// upstream findNodesThatPassFilters / prioritizeNodes over LoadAwareScheduling
// load_aware.go:123-335 and NodeResourcesFit):
//   * one node per thread, a 512-node tile per workgroup (8 waves); the node's derived
//     planes are loaded once into registers and reused for every pod of the workgroup's
//     pod range (node bytes are read once per pod range, not once per pair);
//   * the pod row is wave-uniform → scalar loads (SMEM) and scalar branches on its masks;
//   * per pair: the Fit filter as int64 compares, LoadAware filter as precomputed node bits,
//     each LR score as one fp64 FMA + cvt (exactness argument in kg_common.h);
//   * outputs: a feasibility bit plane written from the wave ballot (one 8-B word per
//     64 nodes), the u8 score pair {Fit, LoadAware} per pair as one u16 store per lane
//     (128 B contiguous per wave), and per (pod, tile) the best (total, lowest node) key
//     from a DPP wave max + an LDS combine across the 8 waves.
// No MFMA: nothing here is a dense contraction; the roofline is HBM bytes (or VALU issue).
//
// Placement mode (sequential scheduling cycle, upstream scheduleOne → selectHost → Reserve):
// pods are processed in chunks; k_eval writes per-(pod, tile) partial keys against the
// snapshot at chunk start, then one workgroup (k_resolve) walks the chunk in queue order:
// a tile's partial is still exact if its best node was not touched by an earlier pod of the
// chunk; touched nodes are re-scored; tiles whose best node was touched are re-scanned; the
// winner is committed to the canonical row and its planes re-derived on the device.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <unordered_map>
#include <utility>
#include <string>
#include <vector>

#include "kg_comm.h"
#include "kg_common.h"
#include "kg_host.h"

#define KG_POD_CHUNK 64          // pods between two LDS partial combines in k_eval
#define KG_RESOLVE_THREADS 512
#define KG_RESOLVE_LA_T0 448     // k_resolve's LoadAware Reserve threads (wave 7)
#define KG_CLS_ITEM_MAX 512         // pods per k_eval3 work item (one output-row entry per thread)
#define KG_MAX_CHUNK KG_PLACE_CHUNK_MAX   // max pods per resolve call (touched-list capacity)
#define KG_MAX_TILES 4096        // max tiles per snapshot in k_resolve (2M nodes)
#define KG_LAX 4                 // LoadAware extra resources k_eval2's LAX form carries (more: k_eval_exact)
#define KG_XCDS 8                // workgroup b of a 1-D grid runs on XCD b % 8 (each XCD has its own L2)

// Bounds-checked build (-DKG_BOUNDS_CHECK, koordinator_amd/build.py build_bounds → lib/libkoordgpu_bounds.so): the
// indices of the pipelined placement's shared buffers (previous-chunk lists, pvkeys, the outcome cache, the touched
// lists, the partial keys) are checked before use; a violation is recorded (count, first site / index / bound) and
// the access skipped, and the next kg_place / kg_eval returns KG_ERR_STATE naming it — a test reads the violation
// instead of faulting the GPU.  The product build compiles every check to `true`.
#ifdef KG_BOUNDS_CHECK
__device__ unsigned long long g_kg_oob[4];   // count, first site, first index, first bound
__device__ __noinline__ bool kg_oob_ok(int site, int64_t idx, int64_t bound) {
    if (idx >= 0 && idx < bound) return true;
    if (atomicAdd(&g_kg_oob[0], 1ull) == 0ull) {
        g_kg_oob[1] = (unsigned long long)site;
        g_kg_oob[2] = (unsigned long long)idx;
        g_kg_oob[3] = (unsigned long long)bound;
    }
    return false;
}
#define KG_IN(site, idx, bound) kg_oob_ok((site), (int64_t)(idx), (int64_t)(bound))
#else
#define KG_IN(site, idx, bound) true
#endif

// ---------------------------------------------------------------------------------------
// wave reductions
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dpp_max_step(uint32_t v, int ctrl_sel) {
    uint32_t o;
    switch (ctrl_sel) {  // old = 0 is the identity of unsigned max
        case 0: o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false); break;  // row_shr:1
        case 1: o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false); break;  // row_shr:2
        case 2: o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false); break;  // row_shr:4
        case 3: o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false); break;  // row_shr:8
        case 4: o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); break;  // row_bcast:15
        default: o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); break; // row_bcast:31
    }
    return v > o ? v : o;
}

// max over the 64 lanes, result valid in lane 63 (returned as a wave-uniform value)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = dpp_max_step(v, 0);
    v = dpp_max_step(v, 1);
    v = dpp_max_step(v, 2);
    v = dpp_max_step(v, 3);
    v = dpp_max_step(v, 4);
    v = dpp_max_step(v, 5);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// the same DPP ladder on 64-bit keys (each half moved by its own v_mov_dpp; old = 0 is the identity of unsigned
// max): no LDS round trips (the ds_bpermute butterfly it replaces sat on the placement resolve's critical path)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ unsigned long long dpp_max64_step(unsigned long long v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROW_MASK, 0xf, false);
    const unsigned long long o = ((unsigned long long)hi << 32) | lo;
    return v > o ? v : o;
}
// max over the 64 lanes, returned wave-uniform
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
    v = dpp_max64_step<0x111, 0xf>(v);   // row_shr:1
    v = dpp_max64_step<0x112, 0xf>(v);   // row_shr:2
    v = dpp_max64_step<0x114, 0xf>(v);   // row_shr:4
    v = dpp_max64_step<0x118, 0xf>(v);   // row_shr:8
    v = dpp_max64_step<0x142, 0xa>(v);   // row_bcast:15
    v = dpp_max64_step<0x143, 0xc>(v);   // row_bcast:31
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}

// ---------------------------------------------------------------------------------------
// per-lane node registers and the pair evaluation
// ---------------------------------------------------------------------------------------
// The fast per-pair path keeps the planes of resources 0 .. KG_FAST_RES − 1 in registers (the fixed resources and
// the first named slot); a pod that compares or scores a later named slot takes the exact int64 path on the node's
// canonical row (kg_pair_exact), so those slots cost the common batches no registers (eval_pair, pair_key_cached).
static_assert(KG_FAST_RES <= KG_NUM_RES, "fast resources are a prefix of the resource slots");
struct NodeRegs {
    int64_t free_[KG_FAST_RES];
    double fit_R[KG_FAST_RES];
    double fit_F[KG_FAST_RES];
    double la_R[2];
    double la_F0[2];           // LoadAware offset, non-prod usage variant
    double la_F1[2];           // LoadAware offset, prod usage variant
    uint32_t fit_mask;
    uint32_t df;
    uint32_t ok_bits;          // bit 0: non-prod pod passes node-only filters, bit 1: prod pod, bit 2: daemonset
    bool la_valid;
};
// pods select their node-only filter bit with a uniform shift: no per-lane select of addresses
#define KG_OKBIT_SHIFT(pf) (((pf) & KG_POD_DAEMONSET) ? 2u : (((pf) & KG_POD_PROD) ? 1u : 0u))

// batch-level union masks: which planes the pods of this launch need
struct BatchMasks {
    uint32_t cmp;   // Fit filter compares
    uint32_t fit;   // Fit score resources
};

// node-only filter bits and LoadAware validity from dflags (and the NodeMetric expiry at `now`)
__device__ __forceinline__ void node_regs_status(const kg_consts &c, uint32_t df, bool expired, NodeRegs &n) {
    bool base = (df & KGD_VALID) != 0;
    if (c.plugins & KG_PLUGIN_FIT) base = base && !(df & KGD_PODS_FULL);
    uint32_t ok = base ? 4u : 0u;
    if (c.plugins & KG_PLUGIN_LOADAWARE) {
        ok |= (base && kg_la_pass(c, df, expired, 0)) ? 1u : 0u;
        ok |= (base && kg_la_pass(c, df, expired, 1)) ? 2u : 0u;
        n.la_valid = kg_la_valid(c, df, expired);
    } else {
        ok |= base ? 3u : 0u;
        n.la_valid = false;
    }
    n.ok_bits = ok;
}

__device__ __forceinline__ void load_node(const kg_consts &c, const kg_planes &pl, int64_t i, bool in_range,
                                          const BatchMasks &bm, int64_t now_ns, NodeRegs &n) {
    const int64_t cap = pl.cap;
    uint32_t df = in_range ? pl.dflags[i] : 0u;
    n.df = df;
#pragma unroll
    for (int r = 0; r < KG_FAST_RES; r++) {
        n.free_[r] = 0;
        n.fit_R[r] = 0.0;
        n.fit_F[r] = 0.0;
        if (in_range && ((bm.cmp >> r) & 1u)) n.free_[r] = pl.free_[r * cap + i];
        if (in_range && ((bm.fit >> r) & 1u)) {
            n.fit_R[r] = pl.fit_R[r * cap + i];
            n.fit_F[r] = pl.fit_F[r * cap + i];
        }
    }
    n.fit_mask = in_range ? pl.fit_mask[i] : 0u;
    bool expired = false;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        n.la_R[r] = 0.0;
        n.la_F0[r] = 0.0;
        n.la_F1[r] = 0.0;
    }
    if (c.plugins & KG_PLUGIN_LOADAWARE) {
        int64_t upd = in_range ? pl.metric_ns[i] : 0;
        expired = kg_metric_expired(c, df, upd, now_ns);
        if (in_range) {
#pragma unroll
            for (int r = 0; r < 2; r++) {
                n.la_R[r] = pl.la_R[r * cap + i];
                n.la_F0[r] = pl.la_F[(0 * 2 + r) * cap + i];
                n.la_F1[r] = pl.la_F[(1 * 2 + r) * cap + i];
            }
        }
    }
    node_regs_status(c, df, expired, n);
}

__device__ __forceinline__ int lr_q(double neg_pr, double R, double F) {
    int q = (int)__builtin_fma(neg_pr, R, F);
    return q > 0 ? q : 0;
}

// Fast-path evaluation of one pair. Returns feasibility; fit/la scores in [0,100].
__device__ __forceinline__ bool eval_fast(const kg_consts &c, const kg_pod_dev &p, const NodeRegs &n, uint32_t &fit,
                                          uint32_t &la) {
    const uint32_t pf = p.flags;
    bool ok = (n.ok_bits >> KG_OKBIT_SHIFT(pf)) & 1u;
    fit = 0;
    la = 0;
    if (c.plugins & KG_PLUGIN_FIT) {
        const uint32_t over = ((p.zero_native_mask & 1u) ? KGD_OVER_CPU : 0u) |
                              ((p.zero_native_mask & 2u) ? KGD_OVER_MEM : 0u) |
                              ((p.zero_native_mask & 4u) ? KGD_OVER_EPH : 0u);
        ok = ok && !(n.df & over);
#pragma unroll
        for (int r = 0; r < KG_FAST_RES; r++)
            if ((p.cmp_mask >> r) & 1u) ok = ok && (p.req[r] <= n.free_[r]);
        uint32_t s = 0;
#pragma unroll
        for (int r = 0; r < KG_FAST_RES; r++) {
            if ((p.fit_mask >> r) & 1u) {
                int q = lr_q(p.fit_pr[r], n.fit_R[r], n.fit_F[r]);
                if (c.fit_most) q = q < 100 ? q : 100;
                s += (uint32_t)(c.fit_w[r] * q);
            }
        }
        if ((n.fit_mask & p.fit_mask) == p.fit_mask) {
            fit = __umulhi(s << 1, p.fit_magic);
        } else {
            uint32_t w = 0;
#pragma unroll
            for (int r = 0; r < KG_FAST_RES; r++)
                if (((n.fit_mask & p.fit_mask) >> r) & 1u) w += (uint32_t)c.fit_w[r];
            fit = w ? s / w : 0u;
        }
    }
    if (c.plugins & KG_PLUGIN_LOADAWARE) {
        // the variant is pod-uniform: select with a ternary (a runtime index would push NodeRegs to scratch)
        const bool prod = (pf & KG_POD_LA_PROD_SCORE) != 0;
        const int q0 = lr_q(p.la_est[0], n.la_R[0], prod ? n.la_F1[0] : n.la_F0[0]);
        const int q1 = lr_q(p.la_est[1], n.la_R[1], prod ? n.la_F1[1] : n.la_F0[1]);
        const uint32_t s = (uint32_t)(c.la_w[0] * q0 + c.la_w[1] * q1);
        la = n.la_valid ? __umulhi(s << 1, c.la_magic) : 0u;
    }
    return ok;
}

__device__ __forceinline__ bool eval_pair(const kg_consts &c, const kg_planes &pl, const kg_pod_dev &p,
                                          const NodeRegs &n, int64_t node, int64_t now_ns, uint32_t &fit, uint32_t &la) {
    if ((n.df & KGD_SLOW) || ((p.cmp_mask | p.fit_mask) >> KG_FAST_RES)) {   // (a later named slot: exact path)
        bool feas;
        kg_pair_exact(c, pl.rows[node], n.df, p, now_ns, feas, fit, la);
        return feas;
    }
    return eval_fast(c, p, n, fit, la);
}

__device__ __forceinline__ uint32_t total_of(const kg_consts &c, uint32_t fit, uint32_t la, uint32_t numa = 0u) {
    return (uint32_t)c.weight_fit * fit + (uint32_t)c.weight_la * la + (uint32_t)c.weight_numa * numa;
}

// ---------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------
__global__ void k_upsert(kg_consts c, kg_planes pl, const kg_node_row *__restrict__ staged,
                         const int32_t *__restrict__ idx, int32_t n) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int64_t i = idx[k];
    pl.rows[i] = staged[k];
    kg_finalize_node(c, pl, i);
}

__global__ void k_finalize_range(kg_consts c, kg_planes pl, int64_t begin, int64_t end) {
    int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= end) return;
    kg_finalize_node(c, pl, i);
}

// ---------------------------------------------------------------------------------------
// hot kernel: S resource slots per launch, branch-free per pair
// ---------------------------------------------------------------------------------------
// The host maps slot s → resource id per pod batch (KG_PROF_*: cpu+memory, + batch-cpu/memory,
// or all 8) and builds kg_pod_hot_t<S> rows.  Per pair and slot: one int64 compare (Fit filter)
// and one fp64 FMA + cvt (least-requested score); node-only filter outcomes are six wave
// lane-masks selected per pod by a scalar index.
typedef uint32_t kg_u32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t cvt_u32_sat(double x) {
    uint32_t r;  // v_cvt_u32_f64 clamps negatives to 0 (and truncates toward zero)
    asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// s / W, exact for s < 2^16 and W ≤ 2^11: a shift when every W of the launch is a power of two
// (POW2), else fma with 1/W + 2^-12 (|s·RN(1/W) − s/W| ≤ 100·2^-23 ≪ 2^-12 < 1/W − 2^-12)
template <bool POW2>
__device__ __forceinline__ uint32_t div_w(uint32_t s, uint32_t shift, float rcp) {
    if (POW2) return s >> shift;
    return (uint32_t)__builtin_fmaf((float)s, rcp, 0x1p-12f);
}

// whole-row scalar load: the row is wave-uniform and read-only → s_load_dwordx16 per 64 B
template <int S>
__device__ __forceinline__ kg_pod_hot_t<S> load_pod(const kg_pod_hot_t<S> *__restrict__ p) {
    constexpr int NB = sizeof(kg_pod_hot_t<S>) / 64;
    union U {
        kg_u32x16 v[NB];
        kg_pod_hot_t<S> h;
        __device__ U() {}
    } u;
    const kg_u32x16 *src = reinterpret_cast<const kg_u32x16 *>(p);
#pragma unroll
    for (int i = 0; i < NB; i++) u.v[i] = src[i];
    return u.h;
}

struct HotArgs {
    int32_t n_pods;
    int32_t pods_per_block;
    int32_t tile_begin;
    int32_t tiles_total;
    int64_t node_end;
    int64_t col_begin;
    int64_t score_stride;
    int32_t mask_words;
    uint32_t fit_cap;        // 100 for MostAllocated (clamp), 0xFFFFFFFF for LeastAllocated (no-op)
    int32_t slot_res[8];     // resource id of each slot (−1 unused)
    int64_t now_ns;
    // LoadAware weights beyond cpu / memory (k_eval2's LAX form): the weighted extra resources (index x into the
    // LoadAware extra planes, resource 2 + x), their weights, and the pods' −EstimatePod of each ([pod][KG_LAX])
    int32_t lax_n;
    int32_t lax_x[KG_LAX];
    uint32_t lax_w[KG_LAX];
    const double *lax_est;
};

// ---------------------------------------------------------------------------------------
// v2: two nodes per lane (a 1024-node tile per 512-thread workgroup)
// ---------------------------------------------------------------------------------------
// per-lane registers of one node
template <int S, bool LA_PROD, bool LAX = false>
struct HotNode {
    int64_t fr[S];          // Allocatable − Requested per slot (Fit filter)
    double R[S], F[S];      // Fit least/most-requested fma operands per slot
    double laR[2], laF0[2], laF1[2];
    double lxR[LAX ? KG_LAX : 1], lxF0[LAX ? KG_LAX : 1], lxF1[LAX ? KG_LAX : 1];   // the LoadAware extra resources
    uint32_t okbits;        // node-only filter outcome per pod variant (bit variant + 3·has_request)
    uint32_t slot_mask;     // slots the node contributes to the Fit score
};

template <int S, bool LA_PROD, bool LAX = false>
__device__ __forceinline__ void load_hot_node(const kg_consts &c, const kg_planes &pl, const HotArgs &a, int64_t node,
                                              uint32_t slot_natives, HotNode<S, LA_PROD, LAX> &n) {
    const int64_t cap = pl.cap;
    const bool in_range = node < a.node_end;   // nodes past the shard end are never feasible
    const uint32_t df = in_range ? pl.dflags[node] : 0u;
    // LAX: the extra-resource planes are read, so only nodes outside the fp64 bounds are slow
    const bool slow = (df & (LAX ? KGD_XSLOW : KGD_SLOW)) != 0;
    const uint32_t nfm = in_range ? pl.fit_mask[node] : 0u;
    n.slot_mask = 0;
#pragma unroll
    for (int s = 0; s < S; s++) {
        const int r = a.slot_res[s];
        n.fr[s] = 0;
        n.R[s] = 0.0;
        n.F[s] = 0.0;
        if (r >= 0) {
            if (in_range) n.fr[s] = pl.free_[r * cap + node];
            if (in_range && !slow) {
                n.R[s] = pl.fit_R[r * cap + node];
                n.F[s] = pl.fit_F[r * cap + node];
            }
            if ((nfm >> r) & 1u) n.slot_mask |= 1u << s;
        }
    }
#pragma unroll
    for (int r = 0; r < 2; r++) n.laR[r] = n.laF0[r] = n.laF1[r] = 0.0;
    bool expired = false;
    if (c.plugins & KG_PLUGIN_LOADAWARE) {
        expired = kg_metric_expired(c, df, in_range ? pl.metric_ns[node] : 0, a.now_ns);
        if (in_range && !slow && kg_la_valid(c, df, expired)) {  // invalid NodeMetric ⇒ score 0 via R = F = 0
#pragma unroll
            for (int r = 0; r < 2; r++) {
                n.laR[r] = pl.la_R[r * cap + node];
                n.laF0[r] = pl.la_F[(0 * 2 + r) * cap + node];
                if (LA_PROD) n.laF1[r] = pl.la_F[(1 * 2 + r) * cap + node];
            }
        }
    }
    if constexpr (LAX) {
        const bool use = in_range && !slow && (c.plugins & KG_PLUGIN_LOADAWARE) && kg_la_valid(c, df, expired);
#pragma unroll
        for (int k = 0; k < KG_LAX; k++) {
            const int x = k < a.lax_n ? a.lax_x[k] : 0;
            const bool on = use && k < a.lax_n;
            n.lxR[k] = on ? pl.la_Rx[x * cap + node] : 0.0;
            n.lxF0[k] = on ? pl.la_Fx[(0 * (KG_NUM_RES - 2) + x) * cap + node] : 0.0;
            n.lxF1[k] = (on && LA_PROD) ? pl.la_Fx[(1 * (KG_NUM_RES - 2) + x) * cap + node] : 0.0;
        }
    }
    bool base = (df & KGD_VALID) && !slow;
    if (c.plugins & KG_PLUGIN_FIT) base = base && !(df & KGD_PODS_FULL);
    bool over = false;  // a zero request of a native resource without a slot still fails an overcommitted node
    if (c.plugins & KG_PLUGIN_FIT) {
        if (!(slot_natives & 1u)) over |= (df & KGD_OVER_CPU) != 0;
        if (!(slot_natives & 2u)) over |= (df & KGD_OVER_MEM) != 0;
        if (!(slot_natives & 4u)) over |= (df & KGD_OVER_EPH) != 0;
    }
    uint32_t okbits = 0;
#pragma unroll
    for (int v = 0; v < 3; v++) {
        bool okv = base;
        if ((c.plugins & KG_PLUGIN_LOADAWARE) && v < 2) okv = okv && kg_la_pass(c, df, expired, v);
        okbits |= (okv ? 1u : 0u) << v;
        okbits |= (okv && !over ? 1u : 0u) << (v + 3);
    }
    n.okbits = okbits;
}

// One (pod, node) pair on the fast path: feasibility, Fit and LoadAware scores.
template <int S, bool FAST, bool LA_PROD, bool FULL, bool LAX = false>
__device__ __forceinline__ bool eval_hot(const kg_consts &c, const HotArgs &a, const kg_pod_hot_t<S> &pd,
                                         const HotNode<S, LA_PROD, LAX> &n, uint32_t &fit, uint32_t &la,
                                         const double *lax_est = nullptr) {
    bool ok = (n.okbits >> pd.okshift) & 1u;
    fit = 0;
    if (FAST || (c.plugins & KG_PLUGIN_FIT)) {
#pragma unroll
        for (int s = 0; s < S; s++) {
            if (s >= 2 && !((pd.flags >> (KG_HOT_CMP_SHIFT + s)) & 1u)) continue;  // uniform
            ok &= pd.req[s] <= n.fr[s];
        }
        uint32_t sum = 0;
#pragma unroll
        for (int s = 0; s < S; s++) {
            if (s >= 2 && !((pd.flags >> (KG_HOT_FIT_SHIFT + s)) & 1u)) continue;  // uniform
            uint32_t q = cvt_u32_sat(__builtin_fma(pd.fit_pr[s], n.R[s], n.F[s]));
            if (!FAST) q = q < a.fit_cap ? q : a.fit_cap;  // MostAllocated clamp
            sum = __umul24(pd.fit_w[s], q) + sum;
        }
        const uint32_t pmask = (pd.flags >> KG_HOT_FIT_SHIFT) & 0xFFu;
        if (FULL || (n.slot_mask & pmask) == pmask) {
            fit = FAST ? sum >> pd.fit_shift : div_w<false>(sum, pd.fit_shift, pd.fit_rcp);
        } else {  // the node lacks a resource the pod scores (no allocatable): its weight drops out
            uint32_t w = 0;
#pragma unroll
            for (int s = 0; s < S; s++) w += ((n.slot_mask & pmask) >> s & 1u) ? pd.fit_w[s] : 0u;
            fit = w ? sum / w : 0u;
        }
    }
    la = 0;
    if (FAST || (c.plugins & KG_PLUGIN_LOADAWARE)) {
        const bool prod = LA_PROD && (pd.flags & KG_HOT_PROD);
        const uint32_t q0 = cvt_u32_sat(__builtin_fma(pd.la_est[0], n.laR[0], prod ? n.laF1[0] : n.laF0[0]));
        const uint32_t q1 = cvt_u32_sat(__builtin_fma(pd.la_est[1], n.laR[1], prod ? n.laF1[1] : n.laF0[1]));
        uint32_t sum = __umul24((uint32_t)c.la_w[0], q0) + __umul24((uint32_t)c.la_w[1], q1);
        if constexpr (LAX) {
#pragma unroll
            for (int k = 0; k < KG_LAX; k++) {
                if (k >= a.lax_n) break;   // uniform
                const uint32_t q = cvt_u32_sat(__builtin_fma(lax_est[k], n.lxR[k], prod ? n.lxF1[k] : n.lxF0[k]));
                sum = __umul24(a.lax_w[k], q) + sum;
            }
        }
        la = FAST ? sum >> c.la_shift : div_w<false>(sum, (uint32_t)c.la_shift, c.la_rcp);
    }
    return ok;
}

// Pods [p0, p1) against the lane's two nodes (n0 = wave base + lane, n1 = n0 + 64).
// seg0 / seg1: the wave's two 64-node segments lie inside the output rows (wave-uniform).
template <int S, bool FAST, bool LA_PROD, bool FULL, bool OUT, bool TOPK, bool LAX = false>
__device__ __forceinline__ void hot_loop2(const kg_consts &c, const HotArgs &a, const kg_pod_hot_t<S> *__restrict__ pods,
                                          uint64_t *__restrict__ mrow, uint16_t *__restrict__ srow,
                                          const HotNode<S, LA_PROD, LAX> &n0, const HotNode<S, LA_PROD, LAX> &n1,
                                          uint32_t kb0, uint32_t kb1, int mask_lanes, bool seg0, bool seg1, int p0,
                                          int p1, uint32_t *kbuf) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    for (int p = p0; p < p1; p++) {
        const kg_pod_hot_t<S> pd = load_pod<S>(pods + p);
        double lx[LAX ? KG_LAX : 1];
        if constexpr (LAX) {
#pragma unroll
            for (int k = 0; k < KG_LAX; k++) lx[k] = a.lax_est[(int64_t)p * KG_LAX + k];   // scalar loads
        }
        uint32_t fit0, la0, fit1, la1;
        const bool ok0 = eval_hot<S, FAST, LA_PROD, FULL, LAX>(c, a, pd, n0, fit0, la0, lx);
        const bool ok1 = eval_hot<S, FAST, LA_PROD, FULL, LAX>(c, a, pd, n1, fit1, la1, lx);
        if (OUT) {
            uint16_t *s = srow + (int64_t)p * a.score_stride;
            if (seg0) s[0] = (uint16_t)(fit0 | (la0 << 8));
            if (seg1) s[64] = (uint16_t)(fit1 | (la1 << 8));
            const unsigned long long b0 = __ballot(ok0), b1 = __ballot(ok1);
            if (lane < mask_lanes) mrow[(int64_t)p * a.mask_words + lane] = lane ? b1 : b0;
        }
        uint32_t tot0, tot1;
        if (FAST) {
            tot0 = fit0 + la0;
            tot1 = fit1 + la1;
        } else {
            tot0 = __umul24((uint32_t)c.weight_fit, fit0) + __umul24((uint32_t)c.weight_la, la0);
            tot1 = __umul24((uint32_t)c.weight_fit, fit1) + __umul24((uint32_t)c.weight_la, la1);
        }
        const uint32_t k0 = ok0 ? (tot0 << KG_TILE_SHIFT) + kb0 : 0u;
        const uint32_t k1 = ok1 ? (tot1 << KG_TILE_SHIFT) + kb1 : 0u;
        if (TOPK) {   // every key of the tile: [pod][1024], node-local order irrelevant
            kbuf[(p - p0) * 2 * KG_BLOCK + tid] = k0;
            kbuf[(p - p0) * 2 * KG_BLOCK + KG_BLOCK + tid] = k1;
        } else {
            kbuf[(p - p0) * KG_BLOCK + tid] = k0 > k1 ? k0 : k1;
        }
    }
}

#define KG_TOPK KG_PARTIAL_SLOTS   // best keys per (pod, tile) in placement chunks

// Placement chunks: the KG_TOPK best keys of one pod's 1024 tile keys, by one wave, in descending order
// into lanes 0..KG_TOPK−1 of the result (0 where the tile has fewer feasible nodes).  Keys are unique
// (they carry the local node), so each round removes exactly one.
__device__ __forceinline__ uint32_t tile_topk(const uint32_t *keys) {
    const int lane = threadIdx.x & 63;
    uint32_t v[KG_TILE / 64];
#pragma unroll
    for (int i = 0; i < KG_TILE / 64; i++) v[i] = keys[lane + 64 * i];
    uint32_t out = 0;
    for (int r = 0; r < KG_TOPK; r++) {
        uint32_t m = v[0];
#pragma unroll
        for (int i = 1; i < KG_TILE / 64; i++) m = m > v[i] ? m : v[i];
        m = wave_max_u32(m);
        if (m == 0) break;   // wave-uniform
        out = lane == r ? m : out;
#pragma unroll
        for (int i = 0; i < KG_TILE / 64; i++) v[i] = v[i] == m ? 0u : v[i];
    }
    return out;
}

#define KG_KCHUNK 16   // pods per LDS key buffer

// TOPK (placement chunks, no planes): the partials hold KG_TOPK best keys per (pod, tile) instead of one
template <int S, bool FAST, bool LA_PROD, bool OUT, bool TOPK, bool LAX = false>
__global__ __launch_bounds__(KG_BLOCK) void k_eval2(kg_consts c, kg_planes pl, HotArgs a,
                                                    const kg_pod_hot_t<S> *__restrict__ pods,
                                                    uint64_t *__restrict__ mask, uint16_t *__restrict__ scores,
                                                    uint32_t *__restrict__ partials) {
    static_assert(!(TOPK && OUT), "top-k partials are a placement-chunk mode");
    __shared__ __attribute__((aligned(16))) uint32_t kbuf[KG_KCHUNK * KG_BLOCK * (TOPK ? 2 : 1)];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = a.tile_begin + blockIdx.x;
    const int64_t wave_base = (int64_t)tile * KG_TILE + wave * 128;   // first node of the wave
    const int64_t node0 = wave_base + lane, node1 = node0 + 64;
    uint32_t slot_natives = 0, all_slots = 0;
#pragma unroll
    for (int s = 0; s < S; s++) {
        const int r = a.slot_res[s];
        if (r >= 0 && r < 3) slot_natives |= 1u << r;
        all_slots |= (r >= 0) ? (1u << s) : 0u;
    }
    HotNode<S, LA_PROD, LAX> n0, n1;
    load_hot_node<S, LA_PROD, LAX>(c, pl, a, node0, slot_natives, n0);
    load_hot_node<S, LA_PROD, LAX>(c, pl, a, node1, slot_natives, n1);
    const bool full = __all(((n0.slot_mask & all_slots) == all_slots || node0 >= a.node_end) &&
                            ((n1.slot_mask & all_slots) == all_slots || node1 >= a.node_end));
    // output columns: a 64-node segment is written iff it lies inside the padded row (wave-uniform)
    const int64_t col0 = wave_base - a.col_begin;
    const bool seg0 = col0 < a.score_stride, seg1 = col0 + 64 < a.score_stride;
    const int mask_lanes = seg1 ? 2 : seg0 ? 1 : 0;
    uint16_t *srow = scores + col0 + lane;
    uint64_t *mrow = mask + (col0 >> 6);
    // key = ((tot + 1) << 10) | (1023 − local node) ⇒ max = best total, then lowest node
    const uint32_t local0 = (uint32_t)(wave * 128 + lane);
    const uint32_t kb0 = (1u << KG_TILE_SHIFT) + (KG_TILE - 1) - local0, kb1 = kb0 - 64;
    const int pb = blockIdx.y * a.pods_per_block;
    const int pe = min(pb + a.pods_per_block, a.n_pods);
    const int rj = tid >> 5, rg = tid & 31;
    for (int p0 = pb; p0 < pe; p0 += KG_KCHUNK) {
        const int p1 = min(p0 + KG_KCHUNK, pe);
        if (full)
            hot_loop2<S, FAST, LA_PROD, true, OUT, TOPK, LAX>(c, a, pods, mrow, srow, n0, n1, kb0, kb1, mask_lanes, seg0,
                                                              seg1, p0, p1, kbuf);
        else
            hot_loop2<S, FAST, LA_PROD, false, OUT, TOPK, LAX>(c, a, pods, mrow, srow, n0, n1, kb0, kb1, mask_lanes, seg0,
                                                               seg1, p0, p1, kbuf);
        __syncthreads();
        if (TOPK) {
            for (int pp = wave; pp < p1 - p0; pp += KG_BLOCK / 64) {
                const uint32_t t = tile_topk(kbuf + pp * 2 * KG_BLOCK);
                if (lane < KG_TOPK) partials[((int64_t)(p0 + pp) * a.tiles_total + tile) * KG_PARTIAL_SLOTS + lane] = t;
            }
            __syncthreads();
            continue;
        }
        const uint4 *src = reinterpret_cast<const uint4 *>(kbuf + rj * KG_BLOCK + rg * 16);
        uint32_t mx = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 v = src[k];
            const uint32_t a0 = v.x > v.y ? v.x : v.y, a1 = v.z > v.w ? v.z : v.w;
            const uint32_t a2 = a0 > a1 ? a0 : a1;
            mx = mx > a2 ? mx : a2;
        }
        mx = dpp_max_step(mx, 0);
        mx = dpp_max_step(mx, 1);
        mx = dpp_max_step(mx, 2);
        mx = dpp_max_step(mx, 3);
        mx = dpp_max_step(mx, 4);
        if (rg == 31 && rj < p1 - p0) partials[(int64_t)(p0 + rj) * a.tiles_total + tile] = mx;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------
// k_eval3: class-specialised matrix mode (each workgroup = one 1024-node tile × a pod range of ONE class, so
// every per-pair branch is resolved at compile time or per workgroup)
// ---------------------------------------------------------------------------------------
template <int NC, int NF>
struct ClsNode {
    int64_t fr[NC];        // Allocatable − Requested of the compared resources
    double R[NF], F[NF];   // Fit fma operands of the scored resources
    uint32_t w;            // Σ Fit weights of the scored resources the node has
    uint32_t cq;           // Σ weight · score of the class's uniform slots (kg_cls_desc::uni_res) on this node
    bool ok;               // node-only filters for the class (valid, pods, overcommit, LoadAware thresholds)
    bool la_use;           // the node's LoadAware planes are valid for this class (else every LoadAware term is 0)
};
struct ClsLa {
    double laR[2], laF[2]; // LoadAware fma operands (the class's usage variant); 0 where !la_use
};

template <int NC, int NF, bool MOST, bool FIT_ON, bool LA_ON>
__device__ __forceinline__ void load_cls_node(const kg_consts &c, const kg_planes &pl, const kg_cls_desc &d,
                                              int64_t node, int64_t node_end, int64_t now_ns, ClsNode<NC, NF> &n) {
    const int64_t cap = pl.cap;
    const bool in_range = node < node_end;
    const uint32_t df = in_range ? pl.dflags[node] : 0u;
    const bool slow = (df & KGD_SLOW) != 0;
    const uint32_t nfm = in_range ? pl.fit_mask[node] : 0u;
#pragma unroll
    for (int k = 0; k < NC; k++) {
        const int r = d.cmp_res[k];
        n.fr[k] = (r >= 0 && in_range) ? pl.free_[r * cap + node] : 0;
    }
    n.w = 0;
#pragma unroll
    for (int f = 0; f < NF; f++) {
        const int r = d.fit_res[f];
        const bool use = FIT_ON && r >= 0 && in_range && !slow;
        n.R[f] = use ? pl.fit_R[r * cap + node] : 0.0;
        n.F[f] = use ? pl.fit_F[r * cap + node] : 0.0;
        if (FIT_ON && r >= 0 && ((nfm >> r) & 1u)) n.w += d.fit_w[f];
    }
    n.cq = 0;
    if (FIT_ON) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int r = d.uni_res[u];   // workgroup-uniform: a scalar branch
            if (r < 0) continue;
            const bool use = in_range && !slow;
            const double R = use ? pl.fit_R[r * cap + node] : 0.0, F = use ? pl.fit_F[r * cap + node] : 0.0;
            uint32_t q = cvt_u32_sat(__builtin_fma(d.uni_pr[u], R, F));
            if (MOST) q = q < 100u ? q : 100u;
            n.cq += d.uni_w[u] * q;
            if ((nfm >> r) & 1u) n.w += d.uni_w[u];
        }
    }
    bool expired = false;
    n.la_use = false;
    if (LA_ON) {
        expired = kg_metric_expired(c, df, in_range ? pl.metric_ns[node] : 0, now_ns);
        n.la_use = in_range && !slow && kg_la_valid(c, df, expired);   // invalid NodeMetric ⇒ score 0 via R = F = 0
    }
    const uint32_t variant = d.node_ok_sel % 3u;
    bool ok = (df & KGD_VALID) && !slow;
    if (FIT_ON) {
        ok = ok && !(df & KGD_PODS_FULL);
        const uint32_t over = ((d.over_mask & 1u) ? KGD_OVER_CPU : 0u) | ((d.over_mask & 2u) ? KGD_OVER_MEM : 0u) |
                              ((d.over_mask & 4u) ? KGD_OVER_EPH : 0u);
        ok = ok && !(df & over);
    }
    if (LA_ON && variant < 2) ok = ok && kg_la_pass(c, df, expired, (int)variant);
    n.ok = ok;
}

template <bool LA_ON>
__device__ __forceinline__ void load_cls_la(const kg_planes &pl, const kg_cls_desc &d, int64_t node, bool use, ClsLa &l) {
    const int64_t cap = pl.cap;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        l.laR[r] = (LA_ON && use) ? pl.la_R[r * cap + node] : 0.0;
        l.laF[r] = (LA_ON && use) ? pl.la_F[(d.la_variant * 2 + r) * cap + node] : 0.0;
    }
}

// Fit compares of one pod against the lane's node as a wave lane mask: each int64 compare writes an
// SGPR pair and the masks are ANDed on the scalar unit (no per-lane booleans in VGPRs)
template <int NC, int NF>
__device__ __forceinline__ unsigned long long cls_ok_mask(const kg_pod_cls_t<NC, NF> &pd, const ClsNode<NC, NF> &n,
                                                          unsigned long long okm) {
    unsigned long long m = okm;
#pragma unroll
    for (int k = 0; k < NC; k++) m &= __builtin_amdgcn_ballot_w64(pd.req[k] <= n.fr[k]);
    return m;
}

// LoadAware weighted least-requested sum (before the weight-sum shift) of one EstimatePod (la0, la1 =
// −estimate) on the node
template <bool LA_ON, bool UNIT>
__device__ __forceinline__ uint32_t cls_la_sum(const kg_consts &c, double la0, double la1, const ClsLa &l) {
    if (!LA_ON) return 0u;
    const uint32_t q0 = cvt_u32_sat(__builtin_fma(la0, l.laR[0], l.laF[0]));
    const uint32_t q1 = cvt_u32_sat(__builtin_fma(la1, l.laR[1], l.laF[1]));
    return UNIT ? q0 + q1 : __umul24((uint32_t)c.la_w[0], q0) + __umul24((uint32_t)c.la_w[1], q1);
}

// Fit score of one pair (sum >> shift when the node has every scored resource, else ÷ its own weight sum)
template <int NC, int NF, bool MOST, bool FIT_ON, bool FULL, bool UNIT>
__device__ __forceinline__ uint32_t cls_fit(const kg_cls_desc &d, const kg_pod_cls_t<NC, NF> &pd, const ClsNode<NC, NF> &n) {
    if (!FIT_ON) return 0u;
    uint32_t sum = n.cq;
#pragma unroll
    for (int f = 0; f < NF; f++) {
        uint32_t q = cvt_u32_sat(__builtin_fma(pd.pr[f], n.R[f], n.F[f]));
        if (MOST) q = q < 100u ? q : 100u;
        sum = UNIT ? sum + q : __umul24(d.fit_w[f], q) + sum;
    }
    if (FULL) return sum >> d.fit_shift;
    return n.w ? sum / n.w : 0u;  // the node lacks a scored resource: its weight drops out
}

typedef uint16_t kg_u16x2 __attribute__((ext_vector_type(2)));

// Packed pair scores (FULL + unit weights): H = fit | la << 16 in u16 halves.  The Fit sum and the
// LoadAware sum << 16 meet in one v_add3 (every term ≤ 100, so each half holds its sum without carry) and
// one v_pk_lshrrev_b16 applies both plugins' weight-sum shifts.  `base` is the node's per-node part of the
// sums: the class's uniform Fit slots (ClsNode::cq) and, in a chunk whose pods share one EstimatePod, the
// LoadAware sum << 16 (evaluated once per node and estimate).
template <int NC, int NF, bool MOST, bool FIT_ON>
__device__ __forceinline__ uint32_t cls_fit_sum(const kg_pod_cls_t<NC, NF> &pd, const ClsNode<NC, NF> &n, uint32_t base) {
    uint32_t s = base;
    if (FIT_ON) {
#pragma unroll
        for (int f = 0; f < NF; f++) {
            uint32_t q = cvt_u32_sat(__builtin_fma(pd.pr[f], n.R[f], n.F[f]));
            if (MOST) q = q < 100u ? q : 100u;
            s += q;
        }
    }
    return s;
}

// v_cndmask_b32 with a wave lane mask as the condition: v where the lane's bit is set, else 0
__device__ __forceinline__ uint32_t sel_lanes(unsigned long long m, uint32_t v) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(v), "s"(m));
    return r;
}

// max(m0 ? k0 : 0, m1 ? k1 : 0) in two VALU instructions: the v_max runs under EXEC = m1, so lanes outside
// m1 keep the first value.  EXEC is restored from its copy (lanes outside the incoming EXEC are don't-care).
__device__ __forceinline__ uint32_t key_max2(unsigned long long m0, unsigned long long m1, uint32_t k0, uint32_t k1) {
    uint32_t r = sel_lanes(m0, k0);
    unsigned long long sv;
    asm("s_mov_b64 %1, exec\n\ts_mov_b64 exec, %2\n\tv_max_u32 %0, %0, %3\n\ts_mov_b64 exec, %1"
        : "+v"(r), "=&s"(sv)
        : "s"(m1), "v"(k1));
    return r;
}

// lane i of the 64-bit VGPR pairs w0 / w1 := the wave-uniform words b0 / b1 (lanebit = 1 << i): two
// v_mov_b64 under a one-lane EXEC, the feasibility words of pod i gathered for one coalesced store per chunk
__device__ __forceinline__ void put_lane2(unsigned long long &w0, unsigned long long &w1, unsigned long long lanebit,
                                          unsigned long long b0, unsigned long long b1) {
    unsigned long long sv;
    asm("s_mov_b64 %2, exec\n\ts_mov_b64 exec, %3\n\tv_mov_b64 %0, %4\n\tv_mov_b64 %1, %5\n\ts_mov_b64 exec, %2"
        : "+v"(w0), "+v"(w1), "=&s"(sv)
        : "s"(lanebit), "s"(b0), "s"(b1));
}

// f(integral_constant<int, I>) for I = 0, 1, …: a fully unrolled loop whose index is a constant expression
template <int... I, class F>
__device__ __forceinline__ void unroll_seq(std::integer_sequence<int, I...>, F &&f) {
    (f(std::integral_constant<int, I>{}), ...);
}

// key_max2 and put_lane2 of pod I in one EXEC window (the lane select an immediate):
//   kmax (= m0 ? k0 : 0) := max(kmax, k1) on the lanes of m1;  lane I of w0 / w1 := m0 / m1
template <int I>
__device__ __forceinline__ void key_max_put(uint32_t &kmax, unsigned long long &w0, unsigned long long &w1,
                                            unsigned long long m0, unsigned long long m1, uint32_t k1) {
    unsigned long long sv;
    asm("s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m1]\n\tv_max_u32 %[k], %[k], %[k1]\n\t"
        "s_mov_b64 exec, %[lb]\n\tv_mov_b64 %[w0], %[m0]\n\tv_mov_b64 %[w1], %[m1]\n\ts_mov_b64 exec, %[sv]"
        : [k] "+v"(kmax), [w0] "+v"(w0), [w1] "+v"(w1), [sv] "=&s"(sv)
        : [m0] "s"(m0), [m1] "s"(m1), [k1] "v"(k1), [lb] "n"(1ull << I));
}

// Workgroup barrier that orders LDS only.  __syncthreads() is also a release of global memory, so it waits
// for every outstanding vector-memory operation of the wave (s_waitcnt vmcnt(0)) — including the score
// stores, which then stall each chunk for the HBM write latency.  The pod loops share only LDS between
// waves, so their barriers wait for lgkmcnt alone.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// k_eval3's key buffer: pod i of a chunk at kg_kofs(i) (dwords) — even pods in the first 2048 dwords, odd pods
// 32 dwords (half the banks) further on, so the reducing wave's 16-lane read groups (two pods each) never
// share a bank
__device__ __forceinline__ int kg_kofs(int i) { return (i >> 1) * 512 + (i & 1) * (2048 + 32); }
#define KG_KBUF_DW (4096 + 32)

#define KG_EVAL3_CC 8    // pods per chunk (LDS key reduction, score staging, LoadAware-uniform chunks)
#define KG_EVAL3_WPE0 6  // waves per SIMD k_eval3's (2, 2) kind is register-allocated for (r03 A/B: 5 / 6 / 8)

// Pods [p0, p0 + np) of one class against the lane's two nodes (columns lane and 64 + lane of the wave's
// 128-column segment).  Pod rows are wave-uniform scalar loads.  UNR: a whole chunk, unrolled, so every
// LDS address and lane select is an immediate.  LAU: the chunk's pods share one EstimatePod, whose LoadAware
// sums are lsum[] (per node); otherwise they are evaluated per pair from la[].
template <int NC, int NF, bool MOST, bool FIT_ON, bool LA_ON, bool OUT, bool FULL, bool W1, bool UNR, bool LAU>
__device__ __forceinline__ void cls_pods(const kg_consts &c, const kg_cls_desc &d, const ClsNode<NC, NF> (&n)[2],
                                         const ClsLa (&la)[2], const unsigned long long (&okm)[2],
                                         const uint32_t (&lsum)[2], int np_rt, const uint32_t (&kb)[2], uint32_t *kbuf,
                                         unsigned long long (&mb)[2], uint16_t *sst,
                                         const kg_pod_cls_t<NC, NF> *__restrict__ grows) {
    constexpr int CC = KG_EVAL3_CC;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int np = UNR ? CC : np_rt;
    const kg_u16x2 shifts = {(uint16_t)d.fit_shift, (uint16_t)c.la_shift};
    // ic: std::integral_constant<int, I> in the unrolled chunk (immediate lane selects), else the runtime index
    auto pod = [&](auto ic) {
        constexpr bool CT = !std::is_same<decltype(ic), int>::value;
        const int i = (int)ic;
        const kg_pod_cls_t<NC, NF> pd = grows[i];   // s_load into SGPRs
        unsigned long long m[2];
#pragma unroll
        for (int j = 0; j < 2; j++) m[j] = cls_ok_mask<NC, NF>(pd, n[j], okm[j]);
        uint32_t kmax, s01;
        if (FULL && W1) {
            // key = (fit + la) << 10 + kb in one v_dot2_u32_u16 of H; the staged u16 pair of both nodes is one
            // v_perm of the two H: {fit0, la0, fit1, la1}
            const kg_u16x2 kw = {(uint16_t)(1u << KG_TILE_SHIFT), (uint16_t)(1u << KG_TILE_SHIFT)};
            uint32_t h[2], k[2];
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t ls = LAU ? lsum[j] : cls_la_sum<LA_ON, true>(c, pd.la[0], pd.la[1], la[j]);
                const uint32_t s = cls_fit_sum<NC, NF, MOST, FIT_ON>(pd, n[j], n[j].cq + (ls << 16));
                h[j] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(kg_u16x2, s) >> shifts);
                k[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(kg_u16x2, h[j]), kw, kb[j], false);
            }
            if constexpr (CT && OUT) {
                kmax = sel_lanes(m[0], k[0]);
                key_max_put<decltype(ic)::value>(kmax, mb[0], mb[1], m[0], m[1], k[1]);
            } else {
                kmax = key_max2(m[0], m[1], k[0], k[1]);
                if (OUT) put_lane2(mb[0], mb[1], 1ull << i, m[0], m[1]);
            }
            s01 = __builtin_amdgcn_perm(h[1], h[0], 0x06040200u);
        } else {
            uint32_t s[2];
            kmax = 0;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t fit = cls_fit<NC, NF, MOST, FIT_ON, FULL, W1>(d, pd, n[j]);
                const uint32_t ls = LAU ? lsum[j] : cls_la_sum<LA_ON, W1>(c, pd.la[0], pd.la[1], la[j]);
                const uint32_t lv = LA_ON ? ls >> c.la_shift : 0u;
                const uint32_t tot = W1 ? fit + lv : __umul24((uint32_t)c.weight_fit, fit) + __umul24((uint32_t)c.weight_la, lv);
                const uint32_t k = sel_lanes(m[j], (tot << KG_TILE_SHIFT) + kb[j]);
                kmax = kmax > k ? kmax : k;
                s[j] = fit | (lv << 8);
            }
            s01 = s[0] | (s[1] << 16);
            if (OUT) put_lane2(mb[0], mb[1], 1ull << i, m[0], m[1]);
        }
        kbuf[kg_kofs(i) + tid] = kmax;
        if (OUT) {
            // the wave's 128-column score segment of this pod, written out per chunk
            sst[i * 128 + lane] = (uint16_t)s01;
            sst[i * 128 + 64 + lane] = (uint16_t)(s01 >> 16);
        }
    };
    if constexpr (UNR) {
        unroll_seq(std::make_integer_sequence<int, CC>{}, pod);
    } else {
        for (int i = 0; i < np; i++) pod(i);
    }
}

// One workgroup = one 1024-node tile (two nodes per lane, 8 waves) × a pod range of one class, walked in
// KG_EVAL3_CC-pod chunks: per chunk the pods' keys go to LDS and one wave (rotating) reduces them to one key per
// (pod, tile) while the others go on; the scores are staged in LDS and written as wave-wide 16-B-per-lane
// stores, the feasibility words as one u64 pair per pod.  LAU: a work item of LoadAware-uniform chunks (the
// host puts whole chunks of one EstimatePod first in each class, kg_cls_desc::la_uni_end): the LoadAware sums
// are per node, evaluated when the estimate changes from one chunk to the next, with the LoadAware planes
// loaded just for that (no registers held for them across the pod loops).
template <int NC, int NF, bool MOST, bool FIT_ON, bool LA_ON, bool OUT, bool W1, bool LAU>
__device__ __forceinline__ void cls_block(const kg_consts &c, const kg_planes &pl, const HotArgs &a, const kg_cls_desc &d,
                                          const kg_cls_work &w, const char *__restrict__ rows_base,
                                          const int32_t *__restrict__ ids, uint64_t *__restrict__ mask,
                                          uint16_t *__restrict__ scores, uint32_t *__restrict__ partials,
                                          uint32_t *kbuf, int32_t *lid, uint16_t *sstage) {
    constexpr int CC = KG_EVAL3_CC;
    constexpr int BT = KG_TILE / 2;                       // threads of the workgroup
    constexpr int SEGW = 128;                             // score columns of one wave
    static_assert(CC == 8 && BT == 512, "the key reduction maps one wave's lanes to 8 pods × 8 lanes");
    static_assert(KG_CLS_ITEM_MAX <= BT, "one output-row entry per thread");
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = a.tile_begin + blockIdx.x;
    const int64_t wave_base = (int64_t)tile * KG_TILE + wave * SEGW;
    ClsNode<NC, NF> n[2];
    ClsLa la[2];
    unsigned long long okm[2];
    bool full_l = true;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        load_cls_node<NC, NF, MOST, FIT_ON, LA_ON>(c, pl, d, wave_base + 64 * j + lane, a.node_end, a.now_ns, n[j]);
        if (!LAU) load_cls_la<LA_ON>(pl, d, wave_base + 64 * j + lane, n[j].la_use, la[j]);
        okm[j] = __builtin_amdgcn_ballot_w64(n[j].ok);
        full_l = full_l && (n[j].w == (1u << d.fit_shift) || wave_base + 64 * j + lane >= a.node_end);
    }
    const bool full = !FIT_ON || __all(full_l);
    const int64_t col0 = wave_base - a.col_begin;
    bool seg[2];
    uint32_t kb[2];
    const uint32_t local0 = (uint32_t)(wave * SEGW + lane);
#pragma unroll
    for (int j = 0; j < 2; j++) {
        seg[j] = col0 + 64 * j < a.score_stride;
        kb[j] = (1u << KG_TILE_SHIFT) + (KG_TILE - 1) - local0 - 64u * j;
    }
    // the work item's output rows (for the stores and the partial keys) go to LDS once: the chunk loop issues no
    // vector loads, so nothing in it waits on vmcnt — i.e. on its own score stores
    const kg_pod_cls_t<NC, NF> *grows = reinterpret_cast<const kg_pod_cls_t<NC, NF> *>(rows_base + d.rows_offset);
    if (tid < w.end - w.begin) lid[tid] = ids[d.ids_first + w.begin + tid];
    // every node-plane load has landed before the pod loop: the loop itself then never waits on
    // vector memory (its stores included)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    uint16_t *sst = sstage + wave * (CC * SEGW);
    // LAU: the estimate (bit patterns) whose LoadAware sums lsum holds
    uint64_t la_prev0 = 0, la_prev1 = 0;
    bool la_have = false;
    uint32_t lsum[2] = {0u, 0u};
    int ci = 0;
    for (int p0 = w.begin; p0 < w.end; p0 += CC, ci++) {
        const int p1 = min(p0 + CC, w.end);
        const int kslot = ci & 1;
        const int32_t *cur = lid + (p0 - w.begin);   // output rows of the chunk's pods
        uint32_t *kcur = kbuf + kslot * KG_KBUF_DW;
        unsigned long long mb[2] = {0ull, 0ull};
        if (LAU) {
            const uint64_t e0 = __builtin_bit_cast(uint64_t, grows[p0].la[0]), e1 = __builtin_bit_cast(uint64_t, grows[p0].la[1]);
            if (!la_have || e0 != la_prev0 || e1 != la_prev1) {
                ClsLa l[2];
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    load_cls_la<LA_ON>(pl, d, wave_base + 64 * j + lane, n[j].la_use, l[j]);
                    lsum[j] = cls_la_sum<LA_ON, W1>(c, __builtin_bit_cast(double, e0), __builtin_bit_cast(double, e1), l[j]);
                }
                la_prev0 = e0;
                la_prev1 = e1;
                la_have = true;
            }
        }
#define KG_CLS_PODS(FULL_, UNR_)                                                                              \
    cls_pods<NC, NF, MOST, FIT_ON, LA_ON, OUT, FULL_, W1, UNR_, LAU>(c, d, n, la, okm, lsum, p1 - p0, kb, kcur, mb, sst, \
                                                                     grows + p0)
        if (full && p1 - p0 == CC) KG_CLS_PODS(true, true);
        else if (full) KG_CLS_PODS(true, false);
        else KG_CLS_PODS(false, false);
#undef KG_CLS_PODS
        if (OUT) {
            // 16 lanes × 16 B cover one pod's 128 columns: 4 pods per wave-wide 1 KiB store.  The reads see
            // the other lanes' ds_writes: a wave's LDS operations complete in order.
            constexpr int LP = SEGW / 8, PPS = 64 / LP;
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const int np = p1 - p0, s8 = lane % LP;
            const bool segs = s8 < 8 ? seg[0] : seg[1];
            const bool whole = np == CC && seg[1];   // wave-uniform: every lane stores
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int it = 0; it < CC / PPS; it++) {
                const int pp = it * PPS + lane / LP;
                if (whole || (pp < np && segs)) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(sst + pp * SEGW + s8 * 8);
                    const int64_t off = (int64_t)cur[pp] * a.score_stride;
                    // non-temporal (a write-once stream): plain stores of the same data measured 0.94 vs 0.67 ms per pass
                    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4 *>(scores + off + col0 + s8 * 8));
                }
            }
            if (lane < np && seg[0]) {
                // lane l writes the two feasibility words of pod p0 + l
                uint64_t *mw = mask + (int64_t)cur[lane] * a.mask_words + (col0 >> 6);
                mw[0] = mb[0];
                if (seg[1]) mw[1] = mb[1];
            }
        }
        // one barrier per chunk: after it, one wave (rotating) reduces the chunk's keys while the others go on
        // with the next chunk, whose keys go to the other key buffer.  A key buffer is written again two chunks
        // later, after the next barrier, which the reducing wave reaches only after its reduction.
        lds_barrier();
        if (wave == ci % (BT / 64)) {
            // lane (p, q) = (l / 8, l % 8) takes 64 of pod p's 512 keys (16-B reads: each 16-lane group reads
            // two pods' 128 B at disjoint banks), then the 8 lanes of a pod meet by DPP
            const int p = lane >> 3, q = lane & 7;
            const uint4 *src = reinterpret_cast<const uint4 *>(kcur + kg_kofs(p)) + q;
            uint32_t mx = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint4 v = src[8 * k];
                mx = max(mx, max(max(v.x, v.y), max(v.z, v.w)));
            }
            mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x141, 0xf, 0xf, false));  // row_half_mirror
            mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x4e, 0xf, 0xf, false));   // quad_perm 2,3,0,1
            mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0xb1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
            if (q == 0 && p < p1 - p0) {
                partials[(int64_t)cur[p] * a.tiles_total + tile] = mx;
            }
        }
    }
}

// The duplicate-row part of a class (the equivalence-class idea of the old kube-scheduler equivalence cache): pods
// whose class rows are equal have equal output rows on every node, so a work item evaluates each distinct row
// once against its tile and writes the result to every pod of that row.  One workgroup = one 1024-node tile ×
// a run of the part's pods, grouped by row (w.begin..w.end); its distinct rows are walked in chunks of
// KG_EVAL3_CC through cls_pods' mixed form, then each wave writes its 128-column score segment of every pod of
// the chunk's rows from the LDS stage (16 lanes × 16 B per pod, 4 pods per wave store), the feasibility words by
// lane permutes of the rows' ballot words, and the reducing wave the (pod, tile) key of every pod.  The work is
// store-bound: per pod and tile 2 KiB of scores + 128 B of mask + 4 B of key against ~1/60 of a pod's compute.
template <int NC, int NF, bool MOST, bool FIT_ON, bool LA_ON, bool OUT, bool W1>
__device__ __forceinline__ void cls_block_dup(const kg_consts &c, const kg_planes &pl, const HotArgs &a, const kg_cls_desc &d,
                                              const kg_cls_work &w, const char *__restrict__ rows_base,
                                              const int32_t *__restrict__ ids, uint64_t *__restrict__ mask,
                                              uint16_t *__restrict__ scores, uint32_t *__restrict__ partials,
                                              uint32_t *kbuf, int32_t *lid, uint16_t *lux, int32_t *cst, uint16_t *sstage,
                                              uint4 *mstage) {
    constexpr int CC = KG_EVAL3_CC;
    constexpr int BT = KG_TILE / 2;
    constexpr int SEGW = 128;
    static_assert(CC == 8 && BT == 512, "the key reduction maps one wave's lanes to 8 rows × 8 lanes");
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = a.tile_begin + w.tile;
    const int64_t wave_base = (int64_t)tile * KG_TILE + wave * SEGW;
    ClsNode<NC, NF> n[2];
    ClsLa la[2];
    unsigned long long okm[2];
    bool full_l = true;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        load_cls_node<NC, NF, MOST, FIT_ON, LA_ON>(c, pl, d, wave_base + 64 * j + lane, a.node_end, a.now_ns, n[j]);
        load_cls_la<LA_ON>(pl, d, wave_base + 64 * j + lane, n[j].la_use, la[j]);
        okm[j] = __builtin_amdgcn_ballot_w64(n[j].ok);
        full_l = full_l && (n[j].w == (1u << d.fit_shift) || wave_base + 64 * j + lane >= a.node_end);
    }
    const bool full = !FIT_ON || __all(full_l);
    const int64_t col0 = wave_base - a.col_begin;
    bool seg[2];
    uint32_t kb[2];
    const uint32_t local0 = (uint32_t)(wave * SEGW + lane);
#pragma unroll
    for (int j = 0; j < 2; j++) {
        seg[j] = col0 + 64 * j < a.score_stride;
        kb[j] = (1u << KG_TILE_SHIFT) + (KG_TILE - 1) - local0 - 64u * j;
    }
    // the item's pods (output rows) and their row indices relative to the item's first row go to LDS
    const int nm = w.end - w.begin;
    const int32_t *uxs = ids + d.ux_first + w.begin;
    const int32_t u_first = uxs[0];
    if (tid < nm) {
        lid[tid] = ids[d.ids_first + w.begin + tid];
        lux[tid] = (uint16_t)(uxs[tid] - u_first);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the pod loops then never wait on vector memory
    __syncthreads();
    const int nu = lux[nm - 1] + 1;   // distinct rows of the item
    // cst[k]: the item's first pod whose row is in chunk k (pods are grouped by row, so chunks are pod runs)
    if (tid < nm) {
        const int ch = lux[tid] / CC;
        if (tid == 0 || lux[tid - 1] / CC != ch) cst[ch] = tid;
    }
    if (tid == 0) cst[(nu + CC - 1) / CC] = nm;
    __syncthreads();
    const kg_pod_cls_t<NC, NF> *grows = reinterpret_cast<const kg_pod_cls_t<NC, NF> *>(rows_base + d.rows_offset) + u_first;
    uint16_t *sst = sstage + wave * (CC * SEGW);
    const uint32_t lsum[2] = {0u, 0u};
    int ci = 0;
    for (int u0 = 0; u0 < nu; u0 += CC, ci++) {
        const int np = min(CC, nu - u0);
        uint32_t *kcur = kbuf + (ci & 1) * KG_KBUF_DW;
        unsigned long long mb[2] = {0ull, 0ull};
#define KG_CLS_PODS(FULL_, UNR_)                                                                                \
    cls_pods<NC, NF, MOST, FIT_ON, LA_ON, OUT, FULL_, W1, UNR_, false>(c, d, n, la, okm, lsum, np, kb, kcur, mb, sst, \
                                                                       grows + u0)
        if (full && np == CC) KG_CLS_PODS(true, true);
        else if (full) KG_CLS_PODS(true, false);
        else KG_CLS_PODS(false, false);
#undef KG_CLS_PODS
        const int m0 = cst[ci], m1 = cst[ci + 1];
        if (OUT) {
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const int s8 = lane & 15;
            const bool segs = s8 < 8 ? seg[0] : seg[1];
            // 16 lanes × 16 B = one pod's 128 columns: 4 pods per wave store
            for (int m = m0; m < m1; m += 4) {
                const int mm = m + (lane >> 4);
                if (mm < m1 && segs) {
                    const int u = lux[mm] - u0;
                    const uint4 v = *reinterpret_cast<const uint4 *>(sst + u * SEGW + s8 * 8);
                    const int64_t off = (int64_t)lid[mm] * a.score_stride;
                    // non-temporal: whole 256-B segments stream past L2 (plain stores: 0.65 vs 0.42 ms per pass, r05)
                    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4 *>(scores + off + col0 + s8 * 8));
                }
            }
            // the chunk rows' ballot words, [buffer][row][wave]: each pod's 128-B feasibility line is written whole
            // after the barrier
            if (lane < CC) mstage[((ci & 1) * CC + lane) * 8 + wave] = uint4{(uint32_t)mb[0], (uint32_t)(mb[0] >> 32),
                                                                            (uint32_t)mb[1], (uint32_t)(mb[1] >> 32)};
        }
        // as cls_block: one barrier per chunk, a rotating reducer wave, double-buffered keys
        lds_barrier();
        if (OUT) {
            // each pod's 128-B feasibility line of the tile (8 lanes × 16 B), 8 pods per wave store, the groups of 8
            // pods dealt to the waves; plain stores: the lines merge in L2 (non-temporal 128-B lines: 0.57 vs 0.41 ms
            // per pass, r05; 16-B pieces per wave and pod: 0.41 vs 0.407 ms)
            const int sub = lane >> 3, wl = lane & 7;   // pod of the group, wave segment of the line
            const int64_t c0 = (wave_base - wave * SEGW - a.col_begin) + wl * SEGW;   // tile column of segment wl
            for (int m = m0 + wave * 8; m < m1; m += 64) {
                const int mm = m + sub;
                if (mm < m1 && c0 < a.score_stride) {
                    const uint4 v = mstage[((ci & 1) * CC + (lux[mm] - u0)) * 8 + wl];
                    uint64_t *mw = mask + (int64_t)lid[mm] * a.mask_words + (c0 >> 6);
                    if (c0 + 64 < a.score_stride) {
                        *reinterpret_cast<uint4 *>(mw) = v;
                    } else {
                        mw[0] = (uint64_t)v.x | ((uint64_t)v.y << 32);
                    }
                }
            }
        }
        if (wave == ci % (BT / 64)) {
            const int p = lane >> 3, q = lane & 7;
            const uint4 *src = reinterpret_cast<const uint4 *>(kcur + kg_kofs(p)) + q;
            uint32_t mx = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint4 v = src[8 * k];
                mx = max(mx, max(max(v.x, v.y), max(v.z, v.w)));
            }
            mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x141, 0xf, 0xf, false));  // row_half_mirror
            mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x4e, 0xf, 0xf, false));   // quad_perm 2,3,0,1
            mx = max(mx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0xb1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
            // every lane of row p's group holds its key; pod m + l takes lane 8u's
            for (int m = m0; m < m1; m += 64) {
                const int mm = m + lane;
                const int u = mm < m1 ? lux[mm] - u0 : 0;
                const uint32_t k = (uint32_t)__builtin_amdgcn_ds_bpermute(u << 5, (int)mx);
                if (mm < m1) partials[(int64_t)lid[mm] * a.tiles_total + tile] = k;
            }
        }
    }
}

// k_eval3's duplicate-row form: one launch per class kind over a 1-D grid of (tile, pod run) items ordered tile by
// tile, dealt to the XCDs in contiguous ranges (workgroup b runs on XCD b % 8 and takes item (b % 8) · per + b / 8),
// so the items of one tile run on one XCD and its L2 serves the tile's node planes to all of them.
template <bool MOST, bool FIT_ON, bool LA_ON, bool OUT, bool W1, int KIND>
__global__ __launch_bounds__(KG_TILE / 2) __attribute__((amdgpu_waves_per_eu(KIND == 0 ? KG_EVAL3_WPE0 : KIND == 2 ? 5 : 4))) void k_eval3_dup(kg_consts c, kg_planes pl, HotArgs a,
                                                        const kg_cls_desc *__restrict__ descs,
                                                        const kg_cls_work *__restrict__ work, int32_t n_items,
                                                        const char *__restrict__ rows, const int32_t *__restrict__ ids,
                                                        uint64_t *__restrict__ mask, uint16_t *__restrict__ scores,
                                                        uint32_t *__restrict__ partials) {
    constexpr int CC = KG_EVAL3_CC, BT = KG_TILE / 2;
    __shared__ __attribute__((aligned(16))) uint32_t kbuf[2 * KG_KBUF_DW];
    static_assert(CC * BT <= 4096, "a chunk's keys fit the key buffer");
    __shared__ int32_t lid[KG_CLS_ITEM_MAX];
    __shared__ uint16_t lux[KG_CLS_ITEM_MAX];
    __shared__ int32_t cst[KG_CLS_ITEM_MAX / CC + 1];
    __shared__ __attribute__((aligned(16))) uint16_t sstage[OUT ? (BT / 64) * CC * 128 : 8];
    __shared__ uint4 mstage[2 * CC * 8];
    const int per = (int)(gridDim.x / KG_XCDS);
    const int item = (int)(blockIdx.x % KG_XCDS) * per + (int)(blockIdx.x / KG_XCDS);
    if (item >= n_items) return;   // grid padded to a multiple of 8; block-uniform
    const kg_cls_work w = work[item];
    const kg_cls_desc d = descs[w.cls];
#define KG_CLS_ARGS c, pl, a, d, w, rows, ids, mask, scores, partials, kbuf, lid, lux, cst, sstage, mstage
    if constexpr (KIND == 0) cls_block_dup<2, 2, MOST, FIT_ON, LA_ON, OUT, W1>(KG_CLS_ARGS);
    else if constexpr (KIND == 1) cls_block_dup<2, 4, MOST, FIT_ON, LA_ON, OUT, W1>(KG_CLS_ARGS);
    else if constexpr (KIND == 2) cls_block_dup<4, 2, MOST, FIT_ON, LA_ON, OUT, W1>(KG_CLS_ARGS);
    else cls_block_dup<4, 4, MOST, FIT_ON, LA_ON, OUT, W1>(KG_CLS_ARGS);
#undef KG_CLS_ARGS
}

// One launch per (class kind, LAU) (the work table is grouped that way): each kernel is register-allocated for
// its own kind.  OUT: the feasibility words and score planes are written (else per-(pod, tile) keys only).
template <bool MOST, bool FIT_ON, bool LA_ON, bool OUT, bool W1, int KIND, bool LAU>
__global__ __launch_bounds__(KG_TILE / 2) __attribute__((amdgpu_waves_per_eu(KIND == 0 ? KG_EVAL3_WPE0 : KIND == 2 ? 5 : 4))) void k_eval3(kg_consts c, kg_planes pl, HotArgs a,
                                                    const kg_cls_desc *__restrict__ descs,
                                                    const kg_cls_work *__restrict__ work,
                                                    const char *__restrict__ rows, const int32_t *__restrict__ ids,
                                                    uint64_t *__restrict__ mask, uint16_t *__restrict__ scores,
                                                    uint32_t *__restrict__ partials) {
    constexpr int CC = KG_EVAL3_CC, BT = KG_TILE / 2;
    __shared__ __attribute__((aligned(16))) uint32_t kbuf[2 * KG_KBUF_DW];
    static_assert(CC * BT <= 4096, "a chunk's keys fit the key buffer");
    __shared__ int32_t lid[KG_CLS_ITEM_MAX];
    __shared__ __attribute__((aligned(16))) uint16_t sstage[OUT ? (BT / 64) * CC * 128 : 8];
    const kg_cls_work w = work[blockIdx.y];
    const kg_cls_desc d = descs[w.cls];
#define KG_CLS_ARGS c, pl, a, d, w, rows, ids, mask, scores, partials, kbuf, lid, sstage
    if constexpr (KIND == 0) cls_block<2, 2, MOST, FIT_ON, LA_ON, OUT, W1, LAU>(KG_CLS_ARGS);
    else if constexpr (KIND == 1) cls_block<2, 4, MOST, FIT_ON, LA_ON, OUT, W1, LAU>(KG_CLS_ARGS);
    else if constexpr (KIND == 2) cls_block<4, 2, MOST, FIT_ON, LA_ON, OUT, W1, LAU>(KG_CLS_ARGS);
    else cls_block<4, 4, MOST, FIT_ON, LA_ON, OUT, W1, LAU>(KG_CLS_ARGS);
#undef KG_CLS_ARGS
}

// Pod equivalence (kg_engine::eq_on): row p of an output plane := row of[p] of the distinct batch's plane.  VB-byte
// vectors, non-temporal stores (a write-once stream); the distinct rows stay in L2 / MALL across their pods.
template <int VB>
__global__ __launch_bounds__(256) void k_eq_rows(const int32_t *__restrict__ of, int32_t P, const char *__restrict__ src,
                                                 char *__restrict__ dst, int64_t row_bytes) {
    typedef uint32_t vec_t __attribute__((ext_vector_type(VB / 4)));
    const int64_t nv = row_bytes / VB;
    for (int32_t p = blockIdx.y; p < P; p += gridDim.y) {
        const vec_t *s = reinterpret_cast<const vec_t *>(src + (int64_t)of[p] * row_bytes);
        vec_t *d = reinterpret_cast<vec_t *>(dst + (int64_t)p * row_bytes);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x)
            __builtin_nontemporal_store(s[i], d + i);
    }
}

// Slow nodes (outside the fp64 exactness bounds) come out of k_eval2 as infeasible with
// zero scores; k_slow_list collects them and k_fix_slow re-evaluates those pairs exactly.
__global__ void k_slow_list(const uint32_t *__restrict__ dflags, int64_t begin, int64_t end, int32_t *__restrict__ list,
                            int32_t *__restrict__ count, uint32_t bit = KGD_SLOW) {
    const int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < end && (dflags[i] & bit) && (dflags[i] & KGD_VALID)) list[atomicAdd(count, 1)] = (int32_t)i;
}

// (the list covers the whole snapshot; columns outside the evaluated range [col_begin, col_end) are skipped)
__global__ void k_fix_slow(kg_consts c, kg_planes pl, const kg_pod_dev *__restrict__ pods, int32_t n_pods,
                           const int32_t *__restrict__ list, const int32_t *__restrict__ count, int64_t col_begin,
                           int64_t col_end, int32_t mask_words, int64_t score_stride, int32_t tiles_total,
                           int64_t now_ns, unsigned long long *mask, uint16_t *scores, uint32_t *partials) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    const int32_t n = *count;
    for (int32_t k = 0; k < n; k++) {
        const int64_t node = list[k];
        if (node < col_begin || node >= col_end) continue;
        bool feas;
        uint32_t fit, la;
        kg_pair_exact(c, pl.rows[node], pl.dflags[node], pods[p], now_ns, feas, fit, la);
        const int64_t col = node - col_begin;
        if (scores) scores[(int64_t)p * score_stride + col] = (uint16_t)(fit | (la << 8));
        if (feas) {
            if (mask) atomicOr(&mask[(int64_t)p * mask_words + (col >> 6)], 1ull << (col & 63));
            const uint32_t tot = (uint32_t)c.weight_fit * fit + (uint32_t)c.weight_la * la;
            const uint32_t key = ((tot + 1u) << KG_TILE_SHIFT) | (uint32_t)(KG_TILE - 1 - (node % KG_TILE));
            atomicMax(&partials[(int64_t)p * tiles_total + node / KG_TILE], key);
        }
    }
}

// Matrix mode when every node takes the exact int64 pair path (LoadAware resourceWeights beyond cpu /
// memory, which the fp64 planes do not carry): one thread per (pod, node); a wave covers 64 columns
// of one pod row, so the feasibility word is its ballot.  Reservation nodes are left to k_rsv_eval.
__global__ __launch_bounds__(256) void k_eval_exact(kg_consts c, kg_planes pl, const kg_pod_dev *__restrict__ pods,
                                                    int32_t n_pods, int64_t begin, int64_t end, int32_t mask_words,
                                                    int64_t score_stride, int32_t tiles_total, int64_t now_ns,
                                                    unsigned long long *mask, uint16_t *scores, uint32_t *partials) {
    const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t node = begin + col;
    const bool in = node < end;
    const uint32_t df = in ? pl.dflags[node] : 0u;
    const bool own = in && !(df & KGD_RSV);
    for (int p = blockIdx.y; p < n_pods; p += gridDim.y) {
        bool feas = false;
        uint32_t fit = 0, la = 0;
        if (own) kg_pair_exact(c, pl.rows[node], df, pods[p], now_ns, feas, fit, la);
        if (own && scores) scores[(int64_t)p * score_stride + col] = (uint16_t)(fit | (la << 8));
        const unsigned long long word = __builtin_amdgcn_ballot_w64(feas);
        if (mask && (threadIdx.x & 63) == 0 && (col >> 6) < mask_words && in) mask[(int64_t)p * mask_words + (col >> 6)] = word;
        uint32_t key = 0;
        if (feas) {
            const uint32_t tot = (uint32_t)c.weight_fit * fit + (uint32_t)c.weight_la * la;
            key = ((tot + 1u) << KG_TILE_SHIFT) | (uint32_t)(KG_TILE - 1 - (node % KG_TILE));
        }
        key = wave_max_u32(key);
        if ((threadIdx.x & 63) == 0 && key) atomicMax(&partials[(int64_t)p * tiles_total + node / KG_TILE], key);
    }
}

// NodeNUMAResource pairs that bind a cpuset on a node with a NUMA topology policy (the trimmed-hint and
// zone-wise-take path): k_eval_numa2 leaves them infeasible; one thread per (pod, node) re-evaluates them in
// full and patches the mask bit, the score planes and the tile key.  Launched only when the batch or the
// snapshot can bind cpusets and the snapshot has NUMA-policy nodes.
__global__ __launch_bounds__(256) void k_numa_bind_fix(kg_consts c, kg_planes pl, HotArgs a, const kg_pod_dev *__restrict__ pods,
                                                       unsigned long long *mask, uint16_t *scores, uint8_t *numa_scores,
                                                       uint32_t *partials) {
    const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t node = a.col_begin + col;
    if (node >= a.node_end) return;
    const kg_node_row &row = pl.rows[node];
    if (!(row.flags & KG_NODE_NUMA_OPTIONS) || row.numa_policy == KG_NUMA_NONE || row.n_zones <= 0 ||
        !(row.flags & KG_NODE_NUMA_TOPO_VALID))
        return;
    const BatchMasks bm{0xFFu, 0xFFu};
    for (int p = blockIdx.y; p < a.n_pods; p += gridDim.y) {
        const kg_pod_dev &pd = pods[p];
        if (pd.flags & (KG_POD_NUMA_SKIP | KG_POD_NUMA_BIND_INVALID)) continue;
        const bool bind = (pd.flags & KG_POD_NUMA_CPU_BIND) ||
                          (row.node_cpu_bind != KG_NODE_CPU_BIND_NONE && pd.numa_req[KG_RES_CPU] != 0);
        if (!bind) continue;
        NodeRegs n;
        load_node(c, pl, node, true, bm, a.now_ns, n);
        uint32_t fit = 0, la = 0;
        bool ok = eval_pair(c, pl, pd, n, node, a.now_ns, fit, la);
        kg_numa_out o;
        kg_numa_pair_z<kg_zone_calc, true>(c, row, pd, o, kg_zone_calc{row});
        ok = ok && o.feasible;
        if (scores) scores[(int64_t)p * a.score_stride + col] = (uint16_t)(fit | (la << 8));
        if (numa_scores) numa_scores[(int64_t)p * a.score_stride + col] = (uint8_t)o.score;
        if (ok) {
            if (mask) atomicOr(&mask[(int64_t)p * a.mask_words + (col >> 6)], 1ull << (col & 63));
            const uint32_t key = ((total_of(c, fit, la, o.score) + 1u) << KG_TILE_SHIFT) | (uint32_t)(KG_TILE - 1 - (node % KG_TILE));
            atomicMax(&partials[(int64_t)p * a.tiles_total + node / KG_TILE], key);
        }
    }
}

// NodeNUMAResource enabled (config 3; matrix mode and placement chunks), pod per lane: a wave holds 64 pods and walks 256 nodes of a tile one
// node at a time, so every node-side value (derived planes, canonical row with its zones) is
// wave-uniform (one cache line per load, served to all 64 pods) and the NUMA hint enumeration runs
// on the node's structure for 64 requests at once.  Outputs accumulate per lane along the pod's own
// row: 64 feasibility bits per u64 word, 8 score pairs per 16-byte store, 16 NUMA scores per 16-byte
// store, the per-(pod, tile) key as a lane-private max (one atomicMax per wave).
#define KG_NUMA2_NODES 256
#define KG_NUMA2_SEG 32   // nodes per work item of the queued form (whole 32-bit halves of the mask words)
#define KG_NUMA2_SEG_TOPK 8   // ... of a placement chunk (keys only: no mask or score planes)
#ifndef KG_NUMA2_WPE
#define KG_NUMA2_WPE 3   // waves per SIMD the register budget is sized for (r02 A/B; r06: 2 is slower, 6.9 vs 5.9 ms)
#endif
typedef uint32_t kg_u32x4 __attribute__((ext_vector_type(4)));
#ifndef KG_NUMA2_FLUSH
#define KG_NUMA2_FLUSH 32   // nodes per output flush of k_eval_numa2 (a multiple of 16; r6 A/B against 16)
#endif
// one wave's run of `npw` nodes from `base` (inside tile `tile`) for the 64 pods of its lanes; npw is a
// multiple of 32, runs start on a 32-node boundary
#ifndef KG_NUMA2_PREFETCH
#define KG_NUMA2_PREFETCH 1
#endif
// one 16-byte LDS-DMA piece per lane into `slot` + lane·16 (a wave-uniform LDS address): issued from inline assembly,
// so the compiler adds no wait of its own before the wave's next LDS reads (it cannot tell the slots apart); the
// reader waits vmcnt(0) for the piece before it reads the slot
__device__ __forceinline__ void kg_glds16(const uint4 *src, uint4 *slot) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)slot);
    int keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
// COMBINE: the Fit + LoadAware planes (mask bits, score pairs) of the lane's pod row are already written (the class /
// slot kernels' pass); the run reads them per 32-node segment, adds the NodeNUMAResource term to the mask and keys and
// writes the NodeNUMAResource plane, without touching the score pairs
template <bool COMBINE>
__device__ __forceinline__ void numa2_run(const kg_consts &c, const kg_planes &pl, const HotArgs &a,
                                          const kg_pod_dev &pd,
                                          int p, bool live, int64_t tile, int64_t base, int npw,
                                          const kg_node_row *__restrict__ rows, unsigned long long *__restrict__ mask,
                                          uint16_t *__restrict__ scores, uint8_t *__restrict__ numa_scores,
                                          uint32_t *__restrict__ partials, const BatchMasks &bm,
                                          kg_zone_tab_data &zt, uint4 *__restrict__ lrow_w) {
    const int lane = threadIdx.x & 63;
    uint32_t best = 0;
    uint64_t mword = 0;
    // output segments of KG_NUMA2_FLUSH nodes per pod, held in registers and written by back-to-back stores: each
    // lane writes its own pod's row, so a store instruction touches 64 rows; one 16-byte piece every 8 nodes left
    // partial lines in L2 that reached HBM as partial writes (r6 PMC: 5.4 GB written for 0.31 GB of planes on a
    // 1k-pod pass); whole 64-byte (scores) / 32-byte (NodeNUMAResource) segments per flush
    constexpr int FL = KG_NUMA2_FLUSH;
    static_assert(FL % 16 == 0 && KG_NUMA2_SEG % FL == 0, "flush segments are whole 16-byte pieces of a run");
    uint32_t sacc[FL / 2], nacc[FL / 4];
#pragma unroll
    for (int i = 0; i < FL / 2; i++) sacc[i] = 0u;
#pragma unroll
    for (int i = 0; i < FL / 4; i++) nacc[i] = 0u;
    constexpr int ROW_U4 = (int)(sizeof(kg_node_row) / 16);
    int succ_z = -1;   // the zone count the wave's table holds combination successors for
    uint32_t sin[COMBINE ? FL / 2 : 1], min32 = 0;   // COMBINE: the segment's score pairs and feasibility bits
    const bool pod_one = kg_numa_one_pod(pd);
#if KG_NUMA2_PREFETCH
    // the canonical rows reach LDS by LDS-DMA one node ahead (two 1 KiB slots per wave): node k + 1's row is in
    // flight while node k's hint enumeration runs, instead of a load → LDS → read chain at the head of every node
    const int src_u4 = lane < ROW_U4 ? lane : ROW_U4 - 1;   // lanes past the row re-read its last piece into the pad
    if (base < a.node_end) kg_glds16(reinterpret_cast<const uint4 *>(rows + base) + src_u4, lrow_w);
#endif
    for (int k = 0; k < npw; k++) {
        const int64_t node = base + k;
        const bool in_range = node < a.node_end;
        uint32_t fit = 0, la = 0, nsc = 0;
        bool ok = false;
        if (COMBINE && (k & (FL - 1)) == 0) {   // (runs start on a 32-node boundary: k = 0 begins a segment)
            const int64_t c0 = node - a.col_begin;
            const bool have = live && in_range && c0 < a.score_stride;
            const kg_u32x4 *src = reinterpret_cast<const kg_u32x4 *>(scores + (int64_t)p * a.score_stride + c0);
#pragma unroll
            for (int i = 0; i < FL / 8; i++) {
                const kg_u32x4 v = have ? src[i] : kg_u32x4{0u, 0u, 0u, 0u};
                sin[4 * i] = v.x;
                sin[4 * i + 1] = v.y;
                sin[4 * i + 2] = v.z;
                sin[4 * i + 3] = v.w;
            }
        }
        if (COMBINE && (k & 31) == 0) {
            const int64_t c0 = node - a.col_begin;
            min32 = live && in_range && c0 < (int64_t)a.mask_words * 64
                        ? reinterpret_cast<const uint32_t *>(mask + (int64_t)p * a.mask_words)[c0 >> 5] : 0u;
        }
        if (in_range) {  // wave-uniform branch
#if defined(KG_NUMA2_ABLATE) && KG_NUMA2_ABLATE == 4   // measurement build: NodeNUMAResource term only
            ok = true;
            fit = la = 0;
#else
            if constexpr (COMBINE) {
                const int si = (k & (FL - 1)) >> 1;
                uint32_t w = 0;
#pragma unroll
                for (int i = 0; i < FL / 2; i++) w |= i == si ? sin[i] : 0u;
                const uint32_t sv = (w >> ((k & 1) * 16)) & 0xFFFFu;
                fit = sv & 0xFFu;
                la = sv >> 8;
                ok = (min32 >> (k & 31)) & 1u;
            } else {
                NodeRegs n;
                load_node(c, pl, node, true, bm, a.now_ns, n);
                ok = eval_pair(c, pl, pd, n, node, a.now_ns, fit, la);
            }
#endif
            // the node's canonical row, staged once into the wave's LDS: the hint enumeration re-reads
            // its zone fields in every loop of every lane
#if KG_NUMA2_PREFETCH
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this node's row has landed (and the last flush)
            __builtin_amdgcn_wave_barrier();
            if (k + 1 < npw && node + 1 < a.node_end)   // the other slot: its node's reads are done (in-order LDS)
                kg_glds16(reinterpret_cast<const uint4 *>(rows + node + 1) + src_u4, lrow_w + 64 * ((k + 1) & 1));
            const kg_node_row &row = *reinterpret_cast<const kg_node_row *>(lrow_w + 64 * (k & 1));
#else
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            if (lane < ROW_U4) lrow_w[lane] = reinterpret_cast<const uint4 *>(rows + node)[lane];
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const kg_node_row &row = *reinterpret_cast<const kg_node_row *>(lrow_w);
#endif
            const bool zoned = (row.flags & KG_NODE_NUMA_OPTIONS) && row.numa_policy != KG_NUMA_NONE &&
                               row.n_zones > 0;   // n_zones ≤ KG_MAX_ZONES (kg_build_node_rows)
            bool one = false;   // this lane's pair takes kg_numa_zoned_one
#if defined(KG_NUMA2_ABLATE) && KG_NUMA2_ABLATE >= 1 && KG_NUMA2_ABLATE <= 2   // measurement builds (the cost split of a node-wave)
            if (KG_NUMA2_ABLATE == 1 && zoned) {
                kg_zone_tab_fill(row, lane, 64, zt, [] { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); },
                                 row.n_zones != succ_z);
                succ_z = row.n_zones;
            }
            nsc = (uint32_t)zt.succ[lane & 255] & 1u;
            if (false)
#endif
            if (zoned) {  // wave-uniform; the previous node's reads precede these writes (in-order LDS per wave)
                const auto wsync = [] {
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                };
                wsync();
                // the single-zone entries of the table (what kg_numa_zoned_one reads); the whole table only when some
                // lane's pair takes the full enumeration
                const int Z = row.n_zones;
                if (lane < 2 * KG_MAX_ZONES) {
                    const int i = lane & (KG_MAX_ZONES - 1), r = lane >> 3;
                    if (i < Z) {
                        zt.tot[r][1u << i] = kg_zone_total(row, i, r);
                        zt.av[r][1u << i] = kg_zone_avail(row, i, r);
                    }
                } else if (lane < 3 * KG_MAX_ZONES) {
                    const int i = lane - 2 * KG_MAX_ZONES;
                    if (i < Z) zt.idm[1u << i] = 1ull << row.zone_id[i];
                }
                int64_t mx[2] = {0, 0};
#pragma unroll
                for (int i = 0; i < KG_MAX_ZONES; i++) {
                    if (i >= Z) break;
                    const int64_t t0 = kg_zone_total(row, i, 0), t1 = kg_zone_total(row, i, 1);
                    mx[0] = t0 > mx[0] ? t0 : mx[0];
                    mx[1] = t1 > mx[1] ? t1 : mx[1];
                }
                one = pod_one && kg_numa_one_node(row) && kg_numa_one_pair(pd, mx);
#if defined(KG_NUMA2_ABLATE) && KG_NUMA2_ABLATE == 3   // measurement build: every pair on the single-zone path
                one = true;
#endif
                wsync();
                if (__builtin_amdgcn_ballot_w64(!one)) {
                    kg_zone_tab_fill(row, lane, 64, zt, wsync, row.n_zones != succ_z);
                    succ_z = row.n_zones;
                    wsync();
                }
            }
#if !defined(KG_NUMA2_ABLATE) || KG_NUMA2_ABLATE == 0 || KG_NUMA2_ABLATE >= 3
            kg_numa_out o;   // a node without zones returns before the hint enumeration reads the table
            kg_numa_pair_z<kg_zone_tab, false, false>(c, row, pd, o, kg_zone_tab{zt}, nullptr, false, one);
            ok = ok && o.feasible;
            nsc = o.score;
#endif
        }
        const uint32_t local = (uint32_t)(node - tile * KG_TILE);
        if (ok) {
            const uint32_t key = ((total_of(c, fit, la, nsc) + 1u) << KG_TILE_SHIFT) | (KG_TILE - 1u - local);
            best = best > key ? best : key;
        }
        mword |= (uint64_t)ok << (k & 63);
        {   // (selects with constant indices: the segments stay in registers)
            const int si = (k & (FL - 1)) >> 1, ni = (k & (FL - 1)) >> 2;
            const uint32_t sv = (fit | (la << 8)) << ((k & 1) * 16), nv = nsc << ((k & 3) * 8);
            if constexpr (!COMBINE) {
#pragma unroll
                for (int i = 0; i < FL / 2; i++) sacc[i] |= i == si ? sv : 0u;
            }
#pragma unroll
            for (int i = 0; i < FL / 4; i++) nacc[i] |= i == ni ? nv : 0u;
        }
        const int64_t col = node - a.col_begin;
        if ((k & (FL - 1)) == FL - 1) {
            const int64_t c0 = col - (FL - 1);
            if (!COMBINE && live && scores && c0 < a.score_stride) {
                kg_u32x4 *d = reinterpret_cast<kg_u32x4 *>(scores + (int64_t)p * a.score_stride + c0);
#pragma unroll
                for (int i = 0; i < FL / 8; i++)
                    __builtin_nontemporal_store(kg_u32x4{sacc[4 * i], sacc[4 * i + 1], sacc[4 * i + 2], sacc[4 * i + 3]}, d + i);
            }
            if (live && numa_scores && c0 < a.score_stride) {
                kg_u32x4 *d = reinterpret_cast<kg_u32x4 *>(numa_scores + (int64_t)p * a.score_stride + c0);
#pragma unroll
                for (int i = 0; i < FL / 16; i++)
                    __builtin_nontemporal_store(kg_u32x4{nacc[4 * i], nacc[4 * i + 1], nacc[4 * i + 2], nacc[4 * i + 3]}, d + i);
            }
#pragma unroll
            for (int i = 0; i < FL / 2; i++) sacc[i] = 0u;
#pragma unroll
            for (int i = 0; i < FL / 4; i++) nacc[i] = 0u;
        }
        if ((k & 63) == 63) {
            const int64_t c0 = col - 63;
            if (live && mask && c0 < (int64_t)a.mask_words * 64) mask[(int64_t)p * a.mask_words + (c0 >> 6)] = mword;
            mword = 0;
        }
    }
    if (npw & 63) {  // a 32-node run: its half of the mask word (little-endian: low half = first 32 nodes)
        const int64_t c0 = base + npw - 32 - a.col_begin;
        if (live && mask && c0 < (int64_t)a.mask_words * 64)
            reinterpret_cast<uint32_t *>(mask + (int64_t)p * a.mask_words)[c0 >> 5] = (uint32_t)mword;
    }
    if (live && best) atomicMax(&partials[(int64_t)p * a.tiles_total + tile], best);
}

// NodeNUMAResource enabled (config 3; matrix mode and placement chunks), pod per lane: a wave holds 64 pods and
// walks a run of nodes one node at a time, so every node-side value (derived planes, canonical row with its
// zones) is wave-uniform (one cache line per load, served to all 64 pods) and the NUMA hint enumeration runs
// on the node's structure for 64 requests at once.  Outputs accumulate per lane along the pod's own row: 64
// feasibility bits per u64 word (32 per half), 8 score pairs per 16-byte store, 16 NUMA scores per 16-byte
// store, the per-(pod, tile) key as a lane-private max (one atomicMax per run).
// Two launch forms:
//  * grid (tiles, pod blocks, z): wave w of a workgroup takes nodes [w·256, w·256 + 256) of its tile, split
//    z ways (small placement chunks: one pod block still puts ≥ 1.5 waves on every SIMD);
//  * queued (queue != nullptr): a resident grid whose waves take 32-node work items
//    (tile, 32-node run, pod block), pod block fastest, from a device counter until `n_items` are taken —
//    the whole-workgroup grid of the first form leaves a last partial round of workgroups on a few CUs
//    (1568 workgroups over 768 resident slots is 3 rounds for 2.04 rounds of work).
template <bool COMBINE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KG_NUMA2_WPE))) void k_eval_numa2(kg_consts c, kg_planes pl, HotArgs a,
                                                    const kg_pod_dev *__restrict__ pods,
                                                    const kg_node_row *__restrict__ rows,
                                                    unsigned long long *__restrict__ mask,
                                                    uint16_t *__restrict__ scores, uint8_t *__restrict__ numa_scores,
                                                    uint32_t *__restrict__ partials, const int32_t *__restrict__ perm,
                                                    BatchMasks bm, int32_t *queue, int32_t n_items, int32_t seg) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // per-wave zone table of the current node (every index mask's sums and id mask, prefix sums of
    // the descending totals): filled by the wave's 64 lanes, read by the hint enumeration of its pods
    __shared__ kg_zone_tab_data ztab[256 / 64];
    // each wave's row slots: 64 × 16 B (one LDS-DMA wave-instruction) per slot, two slots with KG_NUMA2_PREFETCH
    __shared__ __attribute__((aligned(16))) uint4 lrow_s[256 / 64][KG_NUMA2_PREFETCH ? 2 : 1][64];
    static_assert(sizeof(kg_node_row) % 16 == 0 && sizeof(kg_node_row) <= 64 * 16, "rows are staged as 16-byte words");
    const int n_pb = (a.n_pods + 63) / 64;
    for (int it = 0;; it++) {   // grid form: one pass; queued: every wave leaves once the counter passes n_items
        int64_t tile, base;
        int npw, pb;
        if (queue == nullptr) {
            if (it > 0) break;
            tile = (int64_t)a.tile_begin + blockIdx.x;
            pb = blockIdx.y;
            npw = KG_NUMA2_NODES / (int)gridDim.z;
            base = tile * KG_TILE + wave * KG_NUMA2_NODES + (int64_t)blockIdx.z * npw;
        } else {
            int item = 0;
            if (lane == 0) item = atomicAdd(queue, 1);
            item = __builtin_amdgcn_readfirstlane(item);
            if (item >= n_items) break;
            pb = item % n_pb;
            const int run = item / n_pb;   // 32-node run of the launch's node range, from tile_begin · KG_TILE
            tile = (int64_t)a.tile_begin + run / (KG_TILE / seg);
            base = (int64_t)a.tile_begin * KG_TILE + (int64_t)run * seg;
            npw = seg;
        }
        const int slot = pb * 64 + lane;
        const bool live = slot < a.n_pods;
        const int p = live && perm ? perm[slot] : slot;   // the pod row this lane evaluates and writes
        const kg_pod_dev pd = pods[live ? p : 0];
        numa2_run<COMBINE>(c, pl, a, pd, p, live, tile, base, npw, rows, mask, scores, numa_scores, partials, bm, ztab[wave],
                  &lrow_s[wave][0][0]);
    }
}

__device__ __forceinline__ unsigned long long decode_partial(uint32_t k, int tile) {
    if (k == 0) return 0ull;
    const uint32_t node = (uint32_t)tile * KG_TILE + (KG_TILE - 1) - (k & (KG_TILE - 1));
    return ((unsigned long long)(k >> KG_TILE_SHIFT) << 32) | (0xFFFFFFFFull - node);
}

// per-pod max over the tile partials → (total+1) << 32 | (0xFFFFFFFF − node)
__global__ void k_top1(const uint32_t *__restrict__ partials, int32_t tiles, int32_t n_pods,
                       unsigned long long *__restrict__ out) {
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave >= n_pods) return;
    unsigned long long best = 0;
    for (int t = lane; t < tiles; t += 64) {
        unsigned long long k = decode_partial(partials[(int64_t)wave * tiles + t], t);
        best = best > k ? best : k;
    }
    best = wave_max_u64(best);
    if (lane == 0) out[wave] = best;
}

// NUMA: the resolve instantiation may meet NodeNUMAResource (the plain one carries no NUMA code)
template <bool NUMA>
__device__ unsigned long long pair_key(const kg_consts &c, const kg_planes &pl, const kg_pod_dev &p, int64_t node,
                                       int64_t n_nodes, int64_t now_ns) {
    if (node < 0 || node >= n_nodes) return 0ull;
    NodeRegs n;
    BatchMasks bm{0xFFu, 0xFFu};
    load_node(c, pl, node, true, bm, now_ns, n);
    uint32_t fit, la, numa = 0;
    if (!eval_pair(c, pl, p, n, node, now_ns, fit, la)) return 0ull;
    if (NUMA && (c.plugins & KG_PLUGIN_NUMA)) {
        const uint64_t ns = kg_numa_eval_any(c, pl.rows[node], p);
        if (!(ns >> 32)) return 0ull;
        numa = (uint32_t)ns;
    }
    return ((unsigned long long)(total_of(c, fit, la, numa) + 1u) << 32) | (0xFFFFFFFFull - (unsigned long long)node);
}

// NodeNUMAResource placement chunks (≤ KG_NUMA_CHUNK_PODS pods): node per lane, so all 64 lanes work
// on a small pod chunk (the matrix kernel's pod-per-lane layout would leave most lanes idle).  One
// workgroup per (tile, pod): each thread holds 4 nodes of the 1024-node tile, the tile's keys sit in
// LDS and wave 0 writes the pod's top-k list of the tile (k_eval2's partial layout).  The hint
// enumeration reads each lane's own canonical row (kg_zone_calc).  XCD-aware order: hardware hands
// workgroup b to XCD b % 8, so the n pods of one tile are consecutive workgroups of ONE XCD and its
// L2 serves the tile's rows to all of them.
#define KG_NUMA_CHUNK_PODS 16
// BZ (kg_consts.numa_bz): the launch answers cpusets on NUMA-policy nodes (a call into the cpuset path); the
// common BZ = false form inlines the whole pair and carries no call, so its register budget is its own
// (a call would charge it the callee's full-ABI budget: 254 VGPRs + 132 AGPRs, one wave per SIMD)
#define KG_CHUNK_WPE 3   // r03 A/B: 9.5k pods/s at 3, 8.5k at 2 (config-3 placement)
template <bool BZ>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KG_CHUNK_WPE))) void k_eval_numa_chunk(kg_consts c, kg_planes pl, HotArgs a,
                                                         const kg_pod_dev *__restrict__ pods, int32_t shard_tiles,
                                                         uint32_t *__restrict__ partials) {
    __shared__ __attribute__((aligned(16))) kg_pod_dev lp;
    __shared__ __attribute__((aligned(16))) uint32_t kbuf[KG_TILE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int n = a.n_pods;   // 1..KG_NUMA_CHUNK_PODS (host-checked)
    const int b = blockIdx.x, xcd = b % KG_XCDS, r = b / KG_XCDS;
    const int tile_rel = (r / n) * KG_XCDS + xcd, p = r % n;
    if (tile_rel >= shard_tiles) return;   // grid padded to a multiple of 8 tiles; block-uniform
    constexpr int POD_DW = (int)(sizeof(kg_pod_dev) / 4);
    for (int k = tid; k < POD_DW; k += 256)
        reinterpret_cast<uint32_t *>(&lp)[k] = reinterpret_cast<const uint32_t *>(pods + p)[k];
    __syncthreads();
    const int tile = a.tile_begin + tile_rel;
    const BatchMasks bm{0xFFu, 0xFFu};
#pragma unroll 1
    for (int v = 0; v < KG_TILE / 256; v++) {
        const int local = v * 256 + tid;
        const int64_t node = (int64_t)tile * KG_TILE + local;
        const bool in_range = node < a.node_end;
        NodeRegs nr;
        load_node(c, pl, node, in_range, bm, a.now_ns, nr);
        uint32_t key = 0;
        uint32_t fit, la;
        if (in_range && eval_pair(c, pl, lp, nr, node, a.now_ns, fit, la)) {
            kg_numa_out o;
            const kg_node_row &row = pl.rows[node];
            kg_numa_pair_z<kg_zone_calc, BZ, false>(c, row, lp, o, kg_zone_calc{row}, nullptr, false, kg_numa_one(row, lp));
            if (o.feasible)
                key = ((total_of(c, fit, la, o.score) + 1u) << KG_TILE_SHIFT) | (uint32_t)(KG_TILE - 1 - local);
        }
        kbuf[local] = key;
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = tile_topk(kbuf);
        if (lane < KG_TOPK) partials[((int64_t)p * a.tiles_total + tile) * KG_PARTIAL_SLOTS + lane] = t;
    }
}

// NodeNUMAResource results per (distinct pod row, node) for the pipelined placement (kg_engine::ncache): a pod's
// Filter + NodeNUMAResource outcome on a node depends only on its device row and the node's state, so the batch's
// distinct rows (pod equivalence, eq_pods / eq_of) are evaluated over the shard once (k_eval_numa2, matrix mode) and
// each chunk's committed nodes are re-evaluated for every distinct row before the chunk two later is evaluated.
// One byte per entry: the NUMA score when the pair is feasible (eval_pair and the NUMA Filter), KG_NCACHE_NO else.
#define KG_NCACHE_NO 255u
// the matrix mask and NUMA planes of the distinct rows → the cache (one thread per entry)
__global__ __launch_bounds__(256) void k_ncache_init(const unsigned long long *__restrict__ mask,
                                                     const uint8_t *__restrict__ numa, int32_t U, int32_t words,
                                                     int64_t stride, int64_t width, uint8_t *__restrict__ cache) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)U * stride) return;
    const int64_t u = i / stride, col = i % stride;
    const bool ok = col < width && ((mask[u * words + (col >> 6)] >> (col & 63)) & 1ull);
    cache[i] = ok ? numa[i] : (uint8_t)KG_NCACHE_NO;
}

// the committed nodes of one chunk (nodes[0..n), −1 for an unplaced pod) re-evaluated for every distinct row: one
// single-wave workgroup per (row, node), every lane on that pair, its node and pod rows staged in LDS (k_prev_keys'
// form); the same pair functions as k_eval_numa2 (its zone-table provider derives every value with the functions
// kg_zone_calc calls, so the results are identical)
__global__ __launch_bounds__(64) void k_ncache_refresh(kg_consts c, kg_planes pl, const kg_pod_dev *__restrict__ rows,
                                                       int32_t U, const int32_t *__restrict__ nodes, int32_t n,
                                                       int64_t now_ns, uint8_t *__restrict__ cache, int64_t stride,
                                                       int64_t col_begin, int64_t col_end) {
    __shared__ __attribute__((aligned(16))) kg_node_row lrow;
    __shared__ __attribute__((aligned(16))) kg_pod_dev lpd;
    constexpr int ROW_U4 = (int)(sizeof(kg_node_row) / 16), POD_DW = (int)(sizeof(kg_pod_dev) / 4);
    const int64_t i = blockIdx.x;
    const int tid = threadIdx.x;
    if (n <= 0 || i >= (int64_t)U * n) return;   // block-uniform
    const int32_t u = (int32_t)(i / n), k = (int32_t)(i % n);
    const int64_t node = nodes[k];
    if (node < col_begin || node >= col_end) return;
    if (!KG_IN(20, (int64_t)u * stride + (node - col_begin), (int64_t)U * stride)) return;   // (block-uniform)
    for (int x = tid; x < ROW_U4; x += 64) reinterpret_cast<uint4 *>(&lrow)[x] = reinterpret_cast<const uint4 *>(pl.rows + node)[x];
    for (int x = tid; x < POD_DW; x += 64) reinterpret_cast<uint32_t *>(&lpd)[x] = reinterpret_cast<const uint32_t *>(rows + u)[x];
    __syncthreads();
    NodeRegs nr;
    load_node(c, pl, node, true, BatchMasks{0xFFu, 0xFFu}, now_ns, nr);
    uint32_t fit, la;
    bool ok = eval_pair(c, pl, lpd, nr, node, now_ns, fit, la);
    kg_numa_out o;
    kg_numa_pair_z<kg_zone_calc, false, false>(c, lrow, lpd, o, kg_zone_calc{lrow}, nullptr, false, kg_numa_one(lrow, lpd));
    ok = ok && o.feasible;
    if (tid == 0) cache[(int64_t)u * stride + (node - col_begin)] = ok ? (uint8_t)o.score : (uint8_t)KG_NCACHE_NO;
}

// k_eval_numa_chunk with the pair's Filter + NodeNUMAResource outcome read from the cache row of the pod's distinct
// row (cls_of: the chunk's pods' rows in the cache); Fit / LoadAware scores from the planes as in every fast path.
// The keys of nodes the previous chunk committed (not yet refreshed) are stale: the resolve re-scores those.
__global__ __launch_bounds__(256) void k_eval_numa_cached(kg_consts c, kg_planes pl, HotArgs a,
                                                          const kg_pod_dev *__restrict__ pods, int32_t shard_tiles,
                                                          uint32_t *__restrict__ partials, const uint8_t *__restrict__ cache,
                                                          const int32_t *__restrict__ cls_of, int64_t stride, int32_t U) {
    __shared__ __attribute__((aligned(16))) kg_pod_dev lp;
    __shared__ __attribute__((aligned(16))) uint32_t kbuf[KG_TILE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int n = a.n_pods;   // 1..KG_NUMA_CHUNK_PODS (host-checked)
    const int b = blockIdx.x, xcd = b % KG_XCDS, r = b / KG_XCDS;
    const int tile_rel = (r / n) * KG_XCDS + xcd, p = r % n;
    if (tile_rel >= shard_tiles) return;   // grid padded to a multiple of 8 tiles; block-uniform
    constexpr int POD_DW = (int)(sizeof(kg_pod_dev) / 4);
    for (int k = tid; k < POD_DW; k += 256)
        reinterpret_cast<uint32_t *>(&lp)[k] = reinterpret_cast<const uint32_t *>(pods + p)[k];
    __syncthreads();
    const int tile = a.tile_begin + tile_rel;
    if (!KG_IN(30, cls_of[p], U) || !KG_IN(31, (int64_t)tile * KG_TILE - a.col_begin, stride)) return;   // (block-uniform)
    const uint8_t *crow = cache + (int64_t)cls_of[p] * stride - a.col_begin;
    const BatchMasks bm{0xFFu, 0xFFu};
#pragma unroll 1
    for (int v = 0; v < KG_TILE / 256; v++) {
        const int local = v * 256 + tid;
        const int64_t node = (int64_t)tile * KG_TILE + local;
        const bool in_range = node < a.node_end;
        const uint32_t ns = in_range ? crow[node] : KG_NCACHE_NO;
        uint32_t key = 0;
        if (ns != KG_NCACHE_NO) {
            NodeRegs nr;
            load_node(c, pl, node, true, bm, a.now_ns, nr);
            uint32_t fit, la;
            if (eval_pair(c, pl, lp, nr, node, a.now_ns, fit, la))
                key = ((total_of(c, fit, la, ns) + 1u) << KG_TILE_SHIFT) | (uint32_t)(KG_TILE - 1 - local);
        }
        kbuf[local] = key;
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = tile_topk(kbuf);
        if (lane < KG_TOPK) partials[((int64_t)p * a.tiles_total + tile) * KG_PARTIAL_SLOTS + lane] = t;
    }
}

// ---------------------------------------------------------------------------------------
// Reservation + ElasticQuota (BASELINE config 5)
// ---------------------------------------------------------------------------------------
// Nodes carrying reservation slots (KGD_RSV) are dropped by every fast path (their derived VALID bit
// is cleared) and evaluated here, pair by pair, with kg_rsv_pair on the canonical row: the restore of
// transformer.go:49-291 depends on the pod's owner class, so these pairs have no pod-independent
// planes.  One entry per (pod, reservation node):
//   E = feasible ? (base + 1) << 32 | raw << 16 | (nominated + 1) : 0     base = Σ weight·score
//   O = PreScore order of the node (INT64_MAX: none or infeasible)
// The per-pod PreScore preferred node, Score override (1000) and DefaultNormalizeScore max
// are block reductions over the pod's entries (rsv_best_block).
struct kg_rsv_ment {   // one scored entry of a pod, as k_rsv_eval computed it
    int32_t k, node;
    unsigned long long e;
    int64_t o;
};
struct RsvArgs {
    kg_reservation *rsv;        // slots, grouped by node (nullptr: Reservation off)
    const int32_t *rfirst;      // [n_rn + 1] first slot of each reservation node
    const int32_t *rnode;       // [n_rn] node of each reservation node (ascending)
    int32_t n_rn;
    int32_t quota_parent;       // ElasticQuotaArgs.EnableCheckParentQuota
    unsigned long long *E;      // [pods][n_rn]
    int64_t *O;                 // [pods][n_rn]
    kg_quota *quota;            // ElasticQuota groups (nullptr: ElasticQuota off)
    // placement chunks (nullptr in matrix mode, or more groups than the resolve tracks): the entries split for
    // the resolve's reduction, written by k_rsv_eval beside E / O (rsv_best_resolve)
    struct kg_rsv_ment *M;      // [pods][n_rn] the entries that can take the preferred node or a raw score
    int32_t *Mn;                // [pods] their count
    unsigned long long *G;      // [pods][ngroups] per 64-entry group: the best key of its other feasible entries
    int32_t ngroups;
};
#define KG_RSV_GROUP 64
#define KG_RSV_MAX_GROUPS 2048   // the resolve's touched-group flags (LDS): up to 131072 reservation nodes

// an entry whose key depends on PreScore / NormalizeScore: a nominated reservation (raw score) or a
// reservation order (preferred-node candidate); every other feasible entry keys on its base total alone
__device__ __forceinline__ bool rsv_entry_scored(unsigned long long e, int64_t o) {
    return (e & 0xFFFFull) != 0 || (o != 0 && o != INT64_MAX);
}
__device__ __forceinline__ unsigned long long rsv_base_key(unsigned long long e, int32_t node) {
    return ((e >> 32) << 32) | (0xFFFFFFFFull - (unsigned long long)(uint32_t)node);
}

// `row` / `df`: the node's canonical row and dflags (global, or the resolve's LDS copies)
template <bool NUMA = true>
__device__ __forceinline__ void rsv_entry(const kg_consts &c, const kg_node_row &row, uint32_t df, const RsvArgs &ra,
                                          const kg_pod_dev &p, int32_t k, int64_t now_ns, kg_rsv_out *keep,
                                          unsigned long long &e, int64_t &o) {
    kg_rsv_out r;
    kg_rsv_pair<NUMA>(c, row, df, ra.rsv + ra.rfirst[k], ra.rfirst[k + 1] - ra.rfirst[k], p, now_ns, r);
    const uint32_t base = total_of(c, r.fit, r.la, r.numa);
    e = r.feasible ? ((unsigned long long)(base + 1u) << 32) | ((unsigned long long)r.raw << 16) |
                         (unsigned long long)(uint32_t)(r.nominated + 1)
                   : 0ull;
    o = r.feasible ? r.order : INT64_MAX;
    if (keep) *keep = r;
}

// PreScore / Score / NormalizeScore of one pod over its reservation-node entries, by a whole
// workgroup of NT threads; returns the best key (total + 1) << 32 | (0xFFFFFFFF − node) (all threads).
// `plane` (optional) receives the normalized Reservation score of columns [col_begin, col_end).
// Two passes: (1) the preferred node (the smallest non-zero order among feasible nodes, lowest node on ties)
// and the largest raw score; (2) totals and the best key.  DefaultNormalizeScore's maximum follows from pass 1:
// a raw score is ≤ 100 (kg_rsv_score: a mean of terms ≤ 100) and the preferred node scores 1000, so the
// maximum is 1000 when a preferred node exists and the largest raw score otherwise.  Entries are read
// RSV_UNR at a time (independent loads in flight: the passes are latency-bound at one workgroup per pod).
#define KG_RSV_UNR 8
template <int NT>
__device__ unsigned long long rsv_best_block(const kg_consts &c, const unsigned long long *E, const int64_t *O,
                                             const int32_t *rnode, int32_t n_rn, uint8_t *plane, int64_t col_begin,
                                             int64_t col_end, unsigned long long *red, int64_t *redo) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int NW = NT / 64;
    int64_t bo = INT64_MAX;
    int32_t bk = INT32_MAX;
    uint32_t mraw = 0;
    for (int32_t k0 = tid; k0 < n_rn; k0 += NT * KG_RSV_UNR) {
        unsigned long long e[KG_RSV_UNR];
        int64_t o[KG_RSV_UNR];
#pragma unroll
        for (int u = 0; u < KG_RSV_UNR; u++) {
            const int32_t k = k0 + u * NT;
            e[u] = k < n_rn ? E[k] : 0ull;
            o[u] = k < n_rn ? O[k] : INT64_MAX;
        }
#pragma unroll
        for (int u = 0; u < KG_RSV_UNR; u++) {
            if (!e[u]) continue;
            const uint32_t raw = (uint32_t)((e[u] >> 16) & 0xFFFFull);
            mraw = mraw > raw ? mraw : raw;
            if (o[u] != 0 && o[u] != INT64_MAX && o[u] < bo) {   // k ascends with u: the first of equal orders
                bo = o[u];
                bk = k0 + u * NT;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const int64_t o2 = __shfl_xor(bo, off, 64);
        const int32_t k2 = __shfl_xor(bk, off, 64);
        if (o2 < bo || (o2 == bo && k2 < bk)) {
            bo = o2;
            bk = k2;
        }
        const uint32_t m2 = __shfl_xor(mraw, off, 64);
        mraw = mraw > m2 ? mraw : m2;
    }
    if (lane == 0) {
        redo[wv] = bo;
        red[wv] = (unsigned long long)(uint32_t)bk | ((unsigned long long)mraw << 32);
    }
    __syncthreads();
    bo = redo[0];
    bk = (int32_t)(uint32_t)red[0];
    mraw = (uint32_t)(red[0] >> 32);
    for (int w = 1; w < NW; w++) {
        const int32_t k2 = (int32_t)(uint32_t)red[w];
        if (redo[w] < bo || (redo[w] == bo && k2 < bk)) {
            bo = redo[w];
            bk = k2;
        }
        const uint32_t m2 = (uint32_t)(red[w] >> 32);
        mraw = mraw > m2 ? mraw : m2;
    }
    const int32_t pref = bo == INT64_MAX ? -1 : bk;
    const unsigned long long mx = pref >= 0 ? 1000ull : mraw;
    __syncthreads();
    unsigned long long best = 0;
    for (int32_t k0 = tid; k0 < n_rn; k0 += NT * KG_RSV_UNR) {
        unsigned long long e[KG_RSV_UNR];
        int32_t nd[KG_RSV_UNR];
#pragma unroll
        for (int u = 0; u < KG_RSV_UNR; u++) {
            const int32_t k = k0 + u * NT;
            e[u] = k < n_rn ? E[k] : 0ull;
            nd[u] = k < n_rn ? rnode[k] : 0;
        }
#pragma unroll
        for (int u = 0; u < KG_RSV_UNR; u++) {
            const int32_t k = k0 + u * NT;
            if (k >= n_rn) continue;
            const int64_t node = nd[u];
            uint32_t sn = 0;
            if (e[u]) {
                const unsigned long long raw = k == pref ? 1000ull : ((e[u] >> 16) & 0xFFFFull);
                sn = mx ? 100u * (uint32_t)raw / (uint32_t)mx : 0u;   // (raw ≤ 0xFFFF, mx ≤ 0xFFFF: a 32-bit quotient)
                const unsigned long long total = (e[u] >> 32) - 1ull + (unsigned long long)c.weight_rsv * sn;
                const unsigned long long key = ((total + 1ull) << 32) | (0xFFFFFFFFull - (unsigned long long)node);
                best = best > key ? best : key;
            }
            if (plane && node >= col_begin && node < col_end) plane[node - col_begin] = (uint8_t)sn;
        }
    }
    best = wave_max_u64(best);
    if (lane == 0) red[wv] = best;
    __syncthreads();
    best = 0;
    for (int w = 0; w < NW; w++) best = best > red[w] ? best : red[w];
    __syncthreads();
    return best;
}

// The first KG_RSV_PF scored entries and the group keys of the resolve's next pod, loaded into LDS by the
// waves a Reserve leaves idle (rsv_prefetch) while the current pod is reserved.
#define KG_RSV_PF 1024
struct RsvPrefetch {
    int32_t k[KG_RSV_PF], node[KG_RSV_PF];
    unsigned long long e[KG_RSV_PF];
    int64_t o[KG_RSV_PF];
    unsigned long long g[KG_RSV_MAX_GROUPS];
    int32_t n, nm;   // entries held (≤ KG_RSV_PF), scored entries of the pod
};
// pod j's split into `pf` by threads [t0, t0 + nt) (the caller orders it against the readers with barriers)
__device__ __forceinline__ void rsv_prefetch(const RsvArgs &ra, int32_t j, RsvPrefetch &pf, int t, int nthr) {
    const int32_t nm = ra.Mn[j];
    const int32_t n = nm < KG_RSV_PF ? nm : KG_RSV_PF;
    const kg_rsv_ment *M = ra.M + (int64_t)j * ra.n_rn;
    for (int q = t; q < n; q += nthr) {
        const kg_rsv_ment m = M[q];
        pf.k[q] = m.k;
        pf.node[q] = m.node;
        pf.e[q] = m.e;
        pf.o[q] = m.o;
    }
    const unsigned long long *G = ra.G + (int64_t)j * ra.ngroups;
    for (int g = t; g < ra.ngroups; g += nthr) pf.g[g] = G[g];
    if (t == 0) {
        pf.n = n;
        pf.nm = nm;
    }
}

// rsv_best_block for pod j of a placement chunk, over the split k_rsv_eval wrote (prefetched into `pf`): pass 1
// (preferred node, largest raw score) and the scored part of pass 2 walk only the scored entries and the
// reservation nodes earlier pods of the chunk touched (their refreshed entries; duplicates are harmless under
// min / max); a scored entry in a group holding a touched node (`gflag`) is re-read from the refreshed E / O.
// The other feasible entries key on their base total whatever NormalizeScore's maximum, so their best is the
// max of the per-group keys — except in touched groups (listed in `glist`), which are rescanned from the
// refreshed entries.  The same keys as rsv_best_block over every entry.
template <int NT>
__device__ unsigned long long rsv_best_resolve(const kg_consts &c, const kg_planes &pl, const RsvArgs &ra, int32_t j,
                                               const RsvPrefetch &pf, const int32_t *touched, int nt,
                                               const uint8_t *gflag, const int32_t *glist, int ng,
                                               unsigned long long *red, int64_t *redo) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int NW = NT / 64;
    const unsigned long long *E = ra.E + (int64_t)j * ra.n_rn;
    const int64_t *O = ra.O + (int64_t)j * ra.n_rn;
    const kg_rsv_ment *M = ra.M + (int64_t)j * ra.n_rn;
    const int nm = pf.nm, nq = nm + nt;
    // entry q: a scored entry (prefetched, or from the list), else touched node q − nm; e = 0 ⇒ none
    auto get = [&](int q, int32_t &k, int32_t &node, unsigned long long &e, int64_t &o) {
        if (q < nm) {
            if (q < pf.n) {
                k = pf.k[q];
                node = pf.node[q];
                e = pf.e[q];
                o = pf.o[q];
            } else {
                const kg_rsv_ment m = M[q];
                k = m.k;
                node = m.node;
                e = m.e;
                o = m.o;
            }
            if (gflag[k / KG_RSV_GROUP]) {   // its group holds a touched node: the refreshed entry
                e = E[k];
                o = O[k];
            }
        } else {
            node = touched[q - nm];
            k = pl.rsv_of[node];
            e = k >= 0 ? E[k] : 0ull;
            o = k >= 0 ? O[k] : INT64_MAX;
        }
    };
    int64_t bo = INT64_MAX;
    int32_t bk = INT32_MAX;
    uint32_t mraw = 0;
    for (int q = tid; q < nq; q += NT) {
        int32_t k, node;
        unsigned long long e;
        int64_t o;
        get(q, k, node, e, o);
        if (!e) continue;
        const uint32_t raw = (uint32_t)((e >> 16) & 0xFFFFull);
        mraw = mraw > raw ? mraw : raw;
        if (o != 0 && o != INT64_MAX && (o < bo || (o == bo && k < bk))) {
            bo = o;
            bk = k;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const int64_t o2 = __shfl_xor(bo, off, 64);
        const int32_t k2 = __shfl_xor(bk, off, 64);
        if (o2 < bo || (o2 == bo && k2 < bk)) {
            bo = o2;
            bk = k2;
        }
        const uint32_t m2 = __shfl_xor(mraw, off, 64);
        mraw = mraw > m2 ? mraw : m2;
    }
    if (lane == 0) {
        redo[wv] = bo;
        red[wv] = (unsigned long long)(uint32_t)bk | ((unsigned long long)mraw << 32);
    }
    __syncthreads();
    bo = redo[0];
    bk = (int32_t)(uint32_t)red[0];
    mraw = (uint32_t)(red[0] >> 32);
    for (int w = 1; w < NW; w++) {
        const int32_t k2 = (int32_t)(uint32_t)red[w];
        if (redo[w] < bo || (redo[w] == bo && k2 < bk)) {
            bo = redo[w];
            bk = k2;
        }
        const uint32_t m2 = (uint32_t)(red[w] >> 32);
        mraw = mraw > m2 ? mraw : m2;
    }
    const int32_t pref = bo == INT64_MAX ? -1 : bk;
    const unsigned long long mx = pref >= 0 ? 1000ull : mraw;
    __syncthreads();
    unsigned long long best = 0;
    for (int q = tid; q < nq; q += NT) {   // the scored entries and the touched nodes
        int32_t k, node;
        unsigned long long e;
        int64_t o;
        get(q, k, node, e, o);
        if (!e) continue;
        const unsigned long long raw = k == pref ? 1000ull : ((e >> 16) & 0xFFFFull);
        const uint32_t sn = mx ? 100u * (uint32_t)raw / (uint32_t)mx : 0u;   // (raw ≤ 0xFFFF, mx ≤ 0xFFFF: a 32-bit quotient)
        const unsigned long long total = (e >> 32) - 1ull + (unsigned long long)c.weight_rsv * sn;
        const unsigned long long key = ((total + 1ull) << 32) | (0xFFFFFFFFull - (unsigned long long)(uint32_t)node);
        best = best > key ? best : key;
    }
    for (int g = tid; g < ra.ngroups; g += NT) {   // groups without a touched node: their best base key stands
        const unsigned long long key = gflag[g] ? 0ull : pf.g[g];
        best = best > key ? best : key;
    }
    for (int q = tid; q < ng * KG_RSV_GROUP; q += NT) {   // the others, from the refreshed entries
        const int32_t k = glist[q / KG_RSV_GROUP] * KG_RSV_GROUP + q % KG_RSV_GROUP;
        if (k >= ra.n_rn) continue;
        const unsigned long long e = E[k];
        if (!e || rsv_entry_scored(e, O[k])) continue;
        const unsigned long long key = rsv_base_key(e, ra.rnode[k]);
        best = best > key ? best : key;
    }
    best = wave_max_u64(best);
    if (lane == 0) red[wv] = best;
    __syncthreads();
    best = 0;
    for (int w = 0; w < NW; w++) best = best > red[w] ? best : red[w];
    __syncthreads();
    return best;
}

// entries of pods [0, P) × every reservation node; matrix mode also writes their planes
template <bool NUMA>
__global__ __launch_bounds__(256) void k_rsv_eval(kg_consts c, kg_planes pl, RsvArgs ra, const kg_pod_dev *pods,
                                                  int32_t P, int64_t now_ns, unsigned long long *mask,
                                                  uint16_t *scores, uint8_t *numa_scores, int64_t col_begin,
                                                  int64_t col_end, int32_t mask_words, int64_t score_stride) {
    const int32_t k = blockIdx.x * 256 + threadIdx.x;
    const int32_t p = blockIdx.y;
    if (p >= P) return;   // workgroup-uniform
    kg_rsv_out r;
    unsigned long long e = 0;
    int64_t o = INT64_MAX;
    const bool live = k < ra.n_rn;
    const int32_t nd = live ? ra.rnode[k] : 0;
    if (live) {
        rsv_entry<NUMA>(c, pl.rows[nd], pl.dflags[nd], ra, pods[p], k, now_ns, &r, e, o);
        ra.E[(int64_t)p * ra.n_rn + k] = e;
        ra.O[(int64_t)p * ra.n_rn + k] = o;
    }
    if (ra.M) {   // placement: the split for rsv_best_resolve (a wave is one 64-entry group)
        const bool scored = e && rsv_entry_scored(e, o);
        const unsigned long long bk = wave_max_u64(e && !scored ? rsv_base_key(e, nd) : 0ull);
        const unsigned long long bal = __ballot(scored);
        const int lane = threadIdx.x & 63;
        int32_t base = 0;
        if (lane == 0 && (k >> 6) < ra.ngroups) {   // (a wave past the last entry has no group)
            ra.G[(int64_t)p * ra.ngroups + (k >> 6)] = bk;
            if (bal) base = atomicAdd(&ra.Mn[p], (int32_t)__popcll(bal));
        }
        base = __shfl(base, 0, 64);
        if (scored) ra.M[(int64_t)p * ra.n_rn + base + (int32_t)__popcll(bal & ((1ull << lane) - 1ull))] = kg_rsv_ment{k, nd, e, o};
    }
    if (!live) return;
    const int64_t node = nd;
    if (scores && node >= col_begin && node < col_end) {
        const int64_t col = node - col_begin;
        scores[(int64_t)p * score_stride + col] = (uint16_t)(r.fit | (r.la << 8));
        if (numa_scores) numa_scores[(int64_t)p * score_stride + col] = (uint8_t)r.numa;
        if (r.feasible) atomicOr(&mask[(int64_t)p * mask_words + (col >> 6)], 1ull << (col & 63));
    }
}

// per pod: reservation-node best merged into top1; the normalized Reservation plane
__global__ __launch_bounds__(256) void k_rsv_reduce(kg_consts c, RsvArgs ra, int32_t P, unsigned long long *top1,
                                                    uint8_t *plane, int64_t col_begin, int64_t col_end,
                                                    int64_t plane_stride) {
    __shared__ unsigned long long red[4];
    __shared__ int64_t redo[4];
    const int32_t p = blockIdx.x;
    if (p >= P) return;
    const unsigned long long best = rsv_best_block<256>(c, ra.E + (int64_t)p * ra.n_rn, ra.O + (int64_t)p * ra.n_rn,
                                                        ra.rnode, ra.n_rn, plane ? plane + (int64_t)p * plane_stride : nullptr,
                                                        col_begin, col_end, red, redo);
    if (threadIdx.x == 0 && top1 && best > top1[p]) top1[p] = best;
}

// ElasticQuota PreFilter of pods [0, P) against the current quota state
// gate[p]: ElasticQuota PreFilter; gate[P + p]: the plain (reservation-less) nodes are open to the pod
__global__ void k_pod_gate(const kg_quota *__restrict__ quota, int32_t check_parent, const kg_pod_dev *__restrict__ pods,
                           int32_t P, uint8_t *__restrict__ gate) {
    const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const bool q = !quota || pods[p].quota < 0 || kg_quota_pass(quota, pods[p].quota, pods[p], check_parent != 0);
    gate[p] = q ? 1 : 0;
    gate[P + p] = (q && !(pods[p].flags & KGP_RSV_REQUIRED)) ? 1 : 0;
}

// pods failing the quota gate are infeasible everywhere: clear their mask rows and top1
__global__ void k_quota_apply(const uint8_t *__restrict__ gate, int32_t P, unsigned long long *mask, int32_t mask_words,
                              unsigned long long *top1, uint8_t *plane, int64_t plane_stride) {
    const int32_t p = blockIdx.x;
    if (p >= P || gate[p]) return;
    if (mask)
        for (int32_t w = threadIdx.x; w < mask_words; w += blockDim.x) mask[(int64_t)p * mask_words + w] = 0ull;
    if (plane)
        for (int64_t w = threadIdx.x; w < plane_stride; w += blockDim.x) plane[p * plane_stride + w] = 0;
    if (top1 && threadIdx.x == 0) top1[p] = 0ull;
}

// Reserve of the Reservation (nominated slot) and ElasticQuota (used) parts on `node`.
// Reservation.Reserve takes the nomination of PreScore, or runs NominateReservation itself when
// scheduleOne skipped scoring (plugin.go:525-560): on a feasible node both are kg_rsv_nominate
// over the same restored state (the pre-Reserve row: call before the AssumePod delta).
// `row`: the node's pre-Reserve canonical row (global, or a copy in LDS)
__device__ __forceinline__ void rsv_commit(const kg_planes &pl, const RsvArgs &ra, const kg_pod_dev &p, int32_t node,
                                           const kg_node_row &row) {
    if (ra.rsv && pl.rsv_of) {
        const int32_t k = pl.rsv_of[node];
        if (k >= 0) {
            const kg_reservation *rs = ra.rsv + ra.rfirst[k];
            kg_rsv_view v;
            kg_rsv_restore(row, rs, ra.rfirst[k + 1] - ra.rfirst[k], p, v);
            const int nom = kg_rsv_nominate(row, v, rs, p);
            if (nom >= 0) kg_rsv_commit(ra.rsv[ra.rfirst[k] + nom], p);
        }
    }
}
// rsv_commit in the resolve: the pod's entry of the node (E, refreshed when an earlier pod of the chunk touched
// it) holds the nomination PreScore made on the same restored state — Reserve's own NominateReservation
// (plugin.go:525-560) would recompute the same slot
__device__ __forceinline__ void rsv_commit_entry(const kg_planes &pl, const RsvArgs &ra, const kg_pod_dev &p,
                                                 int32_t node, const unsigned long long *E) {
    const int32_t k = pl.rsv_of[node];
    if (k < 0) return;
    const int nom = (int)(E[k] & 0xFFFFull) - 1;
    if (nom >= 0) kg_rsv_commit(ra.rsv[ra.rfirst[k] + nom], p);
}
__device__ __forceinline__ void rsv_quota_commit(const kg_planes &pl, const RsvArgs &ra, const kg_pod_dev &p,
                                                 int32_t node) {
    rsv_commit(pl, ra, p, node, pl.rows[node]);
    if (ra.quota && p.quota >= 0) kg_quota_commit(ra.quota, p.quota, p);
}

// Sequential commit of pods [pod_begin, pod_begin + n) given their per-tile partial keys.
// The resolve keeps the derived planes of the first KG_NCACHE nodes a chunk commits in LDS, written by
// the commit threads themselves, so later pods of the chunk re-score those nodes without a global round
// trip (the canonical row and the global planes are written as well).
#define KG_NCACHE 16
#define KG_TSLOTS 64    // touched tiles with a node bitmask in k_resolve (more: linear compares)
struct NodeCacheEntry {
    NodeRegs n;          // ok_bits / la_valid are derived at use (they depend on `now`)
    int64_t metric_ns;
};

template <bool NUMA>
__device__ __forceinline__ unsigned long long pair_key_cached(const kg_consts &c, const kg_planes &pl, const kg_pod_dev &p,
                                                              const NodeCacheEntry &ce, const kg_node_row &crow,
                                                              int64_t node, int64_t now_ns) {
    NodeRegs n = ce.n;
    const bool expired = (c.plugins & KG_PLUGIN_LOADAWARE) ? kg_metric_expired(c, n.df, ce.metric_ns, now_ns) : false;
    node_regs_status(c, n.df, expired, n);
    uint32_t fit, la, numa = 0;
    if ((n.df & KGD_SLOW) || ((p.cmp_mask | p.fit_mask) >> KG_FAST_RES)) {   // the exact pair path on the LDS copy of
        bool feas;   // the committed row (its global stores may still be in flight: the plain resolve orders pods by
                     // LDS-only barriers); a pod on a later named slot always takes it
        kg_pair_exact(c, crow, n.df, p, now_ns, feas, fit, la);
        if (!feas) return 0ull;
    } else if (!eval_fast(c, p, n, fit, la)) {
        return 0ull;
    }
    if (NUMA && (c.plugins & KG_PLUGIN_NUMA)) {
        const uint64_t ns = kg_numa_eval_any(c, crow, p);   // the LDS copy of the canonical row
        if (!(ns >> 32)) return 0ull;
        numa = (uint32_t)ns;
    }
    return ((unsigned long long)(total_of(c, fit, la, numa) + 1u) << 32) | (0xFFFFFFFFull - (unsigned long long)node);
}

// NodeNUMAResource, pipelined placement: the keys of every (chunk pod j, previous-chunk node q) pair, keys[j · n_prev + q],
// after the previous chunk's resolve and before this chunk's (k_resolve's pvkeys).  One single-wave workgroup per pair,
// every lane on the same pair (the node's row and the pod's row staged in LDS): lanes of one wave on different pairs
// ran the union of their hint enumerations (r05 PMC: ≈ 13k instructions per wave at ≈ 12 cycles each), the slowest
// wave setting the launch's length.
__global__ __launch_bounds__(64) void k_prev_keys(kg_consts c, kg_planes pl, const kg_pod_dev *__restrict__ pods, int32_t n,
                                                  const int32_t *__restrict__ prev_nodes, int32_t n_prev, int64_t n_nodes,
                                                  int64_t now_ns, unsigned long long *__restrict__ keys) {
    __shared__ __attribute__((aligned(16))) kg_node_row lrow;
    __shared__ __attribute__((aligned(16))) kg_pod_dev lpd;
    constexpr int ROW_U4 = (int)(sizeof(kg_node_row) / 16), POD_DW = (int)(sizeof(kg_pod_dev) / 4);
    const int i = blockIdx.x, tid = threadIdx.x;
    if (i >= n * n_prev) return;   // block-uniform
    const int j = i / n_prev, q = i - j * n_prev;
    if (!KG_IN(10, q, n_prev) || !KG_IN(11, j, n)) return;   // (block-uniform)
    const int64_t node = prev_nodes[q];
    const bool in = node >= 0 && node < n_nodes;
    for (int x = tid; in && x < ROW_U4; x += 64) reinterpret_cast<uint4 *>(&lrow)[x] = reinterpret_cast<const uint4 *>(pl.rows + node)[x];
    for (int x = tid; x < POD_DW; x += 64) reinterpret_cast<uint32_t *>(&lpd)[x] = reinterpret_cast<const uint32_t *>(pods + j)[x];
    __syncthreads();
    unsigned long long key = 0;
    if (in && !(lpd.flags & KGP_RSV_REQUIRED)) {
        NodeRegs nr;
        load_node(c, pl, node, true, BatchMasks{0xFFu, 0xFFu}, now_ns, nr);
        uint32_t fit, la;
        if (eval_pair(c, pl, lpd, nr, node, now_ns, fit, la)) {
            // inlined (kg_numa_eval_any is a call: its frame in scratch); placement pipelines carry no cpuset binds
            kg_numa_out o;
            kg_numa_pair_z<kg_zone_calc, false, false>(c, lrow, lpd, o, kg_zone_calc{lrow}, nullptr, false, kg_numa_one(lrow, lpd));
            if (o.feasible)
                key = ((unsigned long long)(total_of(c, fit, la, o.score) + 1u) << 32) | (0xFFFFFFFFull - (unsigned long long)node);
        }
    }
    if (tid == 0) keys[i] = key;
}

// Sequential commit of pods [pod_begin, pod_begin + n) given their per-tile partial keys (kslots per
// (pod, tile): 1 = the tile's best key, KG_PARTIAL_SLOTS = the top-KG_TOPK list + slow slot).
// One workgroup; per pod: (A) every tile's best untouched candidate and the re-scored touched nodes →
// block max; (B) Reserve, one thread per part, and the committed node's planes.  The next pod's row
// and tile keys are prefetched while the current pod is resolved.

#ifdef KG_RESOLVE_TIMING   // measurement build: per-pod phase timestamps of k_resolve (thread 0, shader clock)
__device__ unsigned long long g_rtimes[65536 * 16];
__device__ int g_rtimes_pod;
#define KG_RT_AT(t, k) do { if (threadIdx.x == (t)) { const int gp_ = rt_base + j; if (gp_ < 65536) g_rtimes[gp_ * 16 + (k)] = __builtin_amdgcn_s_memtime(); } } while (0)
#define KG_RT(k) KG_RT_AT(0, k)
#else
#define KG_RT_AT(t, k) do { } while (0)
#define KG_RT(k) do { } while (0)
#endif
// RSV: the batch has reservation nodes; NUMA: NodeNUMAResource is enabled (separate instantiations: the plain
// path keeps its register budget)
template <bool RSV, bool NUMA>
__global__ __launch_bounds__(KG_RESOLVE_THREADS) void k_resolve(kg_consts c, kg_planes pl,
                                                                const kg_pod_dev *__restrict__ pods, int32_t pod_begin,
                                                                int32_t n, const uint32_t *partials, int32_t tiles_total,
                                                                int64_t n_nodes, int64_t now_ns, int32_t *out_node,
                                                                int64_t *out_score, RsvArgs ra, int32_t kslots,
                                                                int32_t *slow_list, int32_t *slow_count,
                                                                int32_t rescore_slow, int32_t defer_last,
                                                                const int32_t *prev_nodes, int32_t n_prev,
                                                                const unsigned long long *pvkeys) {
    constexpr int POD_DW = (int)(sizeof(kg_pod_dev) / 4);
    static_assert(sizeof(kg_pod_dev) % 4 == 0 && POD_DW <= KG_RESOLVE_THREADS, "pod rows are staged one dword per thread");
    __shared__ int32_t touched[KG_MAX_CHUNK];
    // pipelined placement: the previous chunk's placements, committed while this chunk's keys were being
    // evaluated — treated as touched (their keys may predate the commit; re-scored like touched nodes)
    __shared__ int32_t prevt[KG_MAX_CHUNK];
    __shared__ int32_t prevq[KG_MAX_CHUNK];   // each one's index in prev_nodes (pvkeys' column)
    __shared__ int32_t n_prevt;
    // touched tiles (the key lists of the others are exact): ttile[t] = 0 none, s ∈ [1, KG_TSLOTS] the tile's slot in
    // tbits (a bit per node of the tile: "touched?" is one LDS read), 255 beyond KG_TSLOTS tiles (linear compares)
    __shared__ uint8_t ttile[KG_MAX_TILES];
    __shared__ uint32_t tbits[KG_TSLOTS][KG_TILE / 32];
    __shared__ int32_t n_tslots;
    __shared__ int32_t rescan[KG_MAX_TILES];
    __shared__ unsigned long long red[KG_RESOLVE_THREADS / 64];
    __shared__ int64_t redo[KG_RESOLVE_THREADS / 64];
    // the quota gate and the rescan counter alternate between two slots by pod parity: a pod that
    // commits nothing ends without a barrier, so the next pod must not overwrite what a slower wave of
    // this pod may still read
    __shared__ int32_t n_touched, n_rescan[2], gate_ok[2], slot_s;
    __shared__ uint32_t fin[KG_NUM_RES + 2 + (KG_NUM_RES - 2)];
    __shared__ int32_t fl_pods_full;
    __shared__ uint32_t fl_over[3];
    __shared__ uint32_t fl_old_df;
    __shared__ __attribute__((aligned(16))) kg_pod_dev lpod[2];
    __shared__ NodeCacheEntry ncache[KG_NCACHE];
    // NodeNUMAResource: canonical rows of the cached nodes (the hint enumeration of a re-score reads
    // LDS, not a chain of dependent global loads) and the committed node's row for the zone commit
    __shared__ __attribute__((aligned(16))) kg_node_row nrow[KG_NCACHE + 1];
    constexpr int ROW_U4 = (int)(sizeof(kg_node_row) / 16);
    static_assert(sizeof(kg_node_row) % 16 == 0 && ROW_U4 <= 64, "rows are staged as 16-byte words by one wave");
    const bool numa_on = NUMA && (c.plugins & KG_PLUGIN_NUMA) != 0;
    const bool rsv_on = RSV && ra.rsv && ra.n_rn > 0;
    constexpr bool LDSB = !RSV && !NUMA;   // the plain form's pods may end on LDS-only barriers (below)
#ifdef KG_RESOLVE_TIMING
    const int rt_base = g_rtimes_pod;
#endif
    __shared__ int32_t n_slow;
    // Reservation split (ra.M): the entry groups holding a touched reservation node (rsv_best_resolve)
    __shared__ uint8_t gflag[KG_RSV_MAX_GROUPS];
    __shared__ int32_t glist[KG_MAX_CHUNK];
    __shared__ int32_t n_glist;
    __shared__ RsvPrefetch rpf;   // the split of the pod whose reduction is next (rsv_prefetch)
    __shared__ kg_zone_tab_data czt;   // NodeNUMAResource: the zone table of the row being committed
    const int tid = threadIdx.x;
    // tile keys of the next pod, prefetched into registers by the thread owning the tile
    const bool key_prefetch = tiles_total <= KG_RESOLVE_THREADS;
    const int ks = kslots == 1 ? 1 : KG_PARTIAL_SLOTS;
    uint32_t kcur[KG_PARTIAL_SLOTS], knxt[KG_PARTIAL_SLOTS];
    auto load_keys = [&](int jj, uint32_t (&dst)[KG_PARTIAL_SLOTS]) {
        if (!key_prefetch || tid >= tiles_total || jj >= n) return;
        if (ks == 1) {
            dst[0] = partials[(int64_t)jj * tiles_total + tid];
        } else {
            const uint4 *src = reinterpret_cast<const uint4 *>(partials + ((int64_t)jj * tiles_total + tid) * KG_PARTIAL_SLOTS);
#pragma unroll
            for (int q = 0; q < KG_PARTIAL_SLOTS / 4; q++) {
                const uint4 v = src[q];
                dst[4 * q] = v.x;
                dst[4 * q + 1] = v.y;
                dst[4 * q + 2] = v.z;
                dst[4 * q + 3] = v.w;
            }
        }
    };
    if (tid == 0) {
        n_touched = 0;
        n_rescan[0] = n_rescan[1] = 0;
        n_slow = *slow_count;
        n_prevt = 0;
        n_tslots = 0;
        n_glist = 0;
    }
    for (int t = tid; t < tiles_total; t += KG_RESOLVE_THREADS) ttile[t] = 0;
    for (int q = tid; q < KG_TSLOTS * (KG_TILE / 32); q += KG_RESOLVE_THREADS) (&tbits[0][0])[q] = 0u;
    // node marked touched (one thread at a time: the slot allocation is not atomic)
    auto mark = [&](int32_t node) {
        const int t = node / KG_TILE;
        int sl = ttile[t];
        if (sl == 0) {
            sl = n_tslots < KG_TSLOTS ? ++n_tslots : 255;
            ttile[t] = (uint8_t)sl;
        }
        if (sl != 255) tbits[sl - 1][(node % KG_TILE) >> 5] |= 1u << (node & 31);
    };
    // was `node` (in a tile whose ttile entry is sl) touched by this chunk or the previous one?
    auto is_touched = [&](int sl, int32_t node, int nt_, int np_) {
        if (sl == 0) return false;
        if (sl != 255) return ((tbits[sl - 1][(node % KG_TILE) >> 5] >> (node & 31)) & 1u) != 0;
        bool hit = false;
        for (int q = 0; q < nt_; q++) hit |= touched[q] == node;
        for (int q = 0; q < np_; q++) hit |= prevt[q] == node;
        return hit;
    };
    if (rsv_on && ra.M) {
        for (int g = tid; g < ra.ngroups; g += KG_RESOLVE_THREADS) gflag[g] = 0;
        if (n > 0) rsv_prefetch(ra, 0, rpf, tid, KG_RESOLVE_THREADS);
    }
    if (tid < POD_DW && n > 0) reinterpret_cast<uint32_t *>(&lpod[0])[tid] = reinterpret_cast<const uint32_t *>(pods + pod_begin)[tid];
    load_keys(0, kcur);
    __syncthreads();
    if (n_prev > 0) {
        for (int q = tid; q < n_prev; q += KG_RESOLVE_THREADS) {
            const int32_t node = prev_nodes[q];
            if (node < 0) continue;
            const int slot = atomicAdd(&n_prevt, 1);
            if (!KG_IN(40, slot, KG_MAX_CHUNK) || !KG_IN(46, node, n_nodes)) continue;
            prevt[slot] = node;
            prevq[slot] = q;
        }
        __syncthreads();
        if (tid == 0)
            for (int q = 0; q < n_prevt; q++) mark(prevt[q]);
        __syncthreads();
    }
    const int np_prev = n_prevt;
    // NodeNUMAResource: the (pod, previous-chunk node) keys computed beforehand by k_prev_keys, all pairs at once (each
    // pod re-scored those nodes on its own: one single-lane NUMA pair chain per pod on the critical path); a pod takes
    // a node's key unless an earlier pod of this chunk touched the node again (the touched re-score then)
    const bool pv_pre = NUMA && pvkeys != nullptr;
    for (int j = 0; j < n; j++) {
        KG_RT(1);
        const int par = j & 1;
        const kg_pod_dev &pd = lpod[par];
        if (tid == 0)  // ElasticQuota PreFilter on the quota state after every earlier Reserve (read after the sync below)
            gate_ok[par] = !ra.quota || pd.quota < 0 || kg_quota_pass(ra.quota, pd.quota, pd, ra.quota_parent != 0);
        // prefetch pod j + 1 (its slot's last reader, pod j − 1, is past this pod's first barrier... see the
        // note above: a barrier-free pod j − 1 reads its row only before its own second barrier)
        if (j + 1 < n && tid >= KG_RESOLVE_THREADS - POD_DW)
            reinterpret_cast<uint32_t *>(&lpod[par ^ 1])[tid - (KG_RESOLVE_THREADS - POD_DW)] =
                reinterpret_cast<const uint32_t *>(pods + pod_begin + j + 1)[tid - (KG_RESOLVE_THREADS - POD_DW)];
        KG_RT_AT(KG_RESOLVE_THREADS - 1, 10);
        load_keys(j + 1, knxt);
        unsigned long long best = 0;
        const int nt = n_touched;
        if (rsv_on) {
            // nodes with reservations: this pod's entries of the nodes earlier pods of the chunk touched, refreshed
            // by the upper waves while the lower ones scan the tiles (the scan leaves them idle: ≤ 256 tiles)
            unsigned long long *E = ra.E + (int64_t)j * ra.n_rn;
            int64_t *O = ra.O + (int64_t)j * ra.n_rn;
            for (int q = tid - KG_RESOLVE_THREADS / 2; q >= 0 && q < nt; q += KG_RESOLVE_THREADS / 2) {
                const int32_t nd = touched[q];
                const int32_t k = pl.rsv_of[nd];
                if (k < 0) continue;
                if (q < KG_NCACHE)   // the committed row and flags cached in LDS
                    rsv_entry<NUMA>(c, nrow[q], ncache[q].n.df, ra, pd, k, now_ns, nullptr, E[k], O[k]);
                else
                    rsv_entry<NUMA>(c, pl.rows[nd], pl.dflags[nd], ra, pd, k, now_ns, nullptr, E[k], O[k]);
            }
        }
        // a pod that requires a reservation can only land on reservation nodes (rsv part below)
        const bool plain_ok = !(pd.flags & KGP_RSV_REQUIRED);
        for (int t = tid; t < tiles_total; t += KG_RESOLVE_THREADS) {
            if (!key_prefetch) {   // more tiles than threads: this thread's tiles straight from memory
                if (ks == 1) {
                    kcur[0] = partials[(int64_t)j * tiles_total + t];
                } else {
#pragma unroll
                    for (int q = 0; q < KG_PARTIAL_SLOTS; q++)
                        kcur[q] = partials[((int64_t)j * tiles_total + t) * KG_PARTIAL_SLOTS + q];
                }
            }
            if (ks == 1) {   // one key per tile: a touched best node forces a rescan of its tile
                const unsigned long long k = decode_partial(kcur[0], t);
                if (!k) continue;
                const int32_t node = (int32_t)(0xFFFFFFFFull - (k & 0xFFFFFFFFull));
                const bool hit = is_touched(ttile[t], node, nt, np_prev);
                if (hit) {
                    const int ri = atomicAdd(&n_rescan[par], 1);
                    if (KG_IN(42, ri, KG_MAX_TILES)) rescan[ri] = t;
                }
                else best = best > k ? best : k;
                continue;
            }
            // the tile's KG_TOPK best keys (descending, 0-padded): the first untouched key is the tile's
            // best untouched fast node; the tile is rescanned only when every key of a full list was touched
            // (fully unrolled: the list stays in registers)
            unsigned long long cand = 0;
            bool found = false, ended = false;
            const int tsl = ttile[t];
            if (!tsl) {   // no touched node in the tile: its best key stands
                cand = decode_partial(kcur[0], t);
                best = best > cand ? best : cand;
                continue;
            }
            if (tsl != 255) {
                // every entry's touched bit read at once (independent LDS reads, one latency), then the first
                // untouched entry taken; a partial key's low bits are 1023 − the node's tile offset
                uint32_t tw[KG_TOPK];
#pragma unroll
                for (int s = 0; s < KG_TOPK; s++) tw[s] = tbits[tsl - 1][(KG_TILE - 1 - (kcur[s] & (KG_TILE - 1))) >> 5];
#pragma unroll
                for (int s = 0; s < KG_TOPK; s++) {
                    const uint32_t loc = KG_TILE - 1 - (kcur[s] & (KG_TILE - 1));
                    ended = ended || kcur[s] == 0;
                    if (!found && !ended && !((tw[s] >> (loc & 31)) & 1u)) {
                        cand = decode_partial(kcur[s], t);
                        found = true;
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < KG_TOPK; s++) {
                    const unsigned long long k = decode_partial(kcur[s], t);
                    ended = ended || k == 0;
                    if (!found && !ended) {
                        const int32_t node = (int32_t)(0xFFFFFFFFull - (k & 0xFFFFFFFFull));
                        if (!is_touched(tsl, node, nt, np_prev)) {
                            cand = k;
                            found = true;
                        }
                    }
                }
            }
            const bool need = !found && !ended;
            if (need) {
                const int ri = atomicAdd(&n_rescan[par], 1);
                if (KG_IN(42, ri, KG_MAX_TILES)) rescan[ri] = t;
            }
            else best = best > cand ? best : cand;
        }
        KG_RT_AT(0, 9);
        KG_RT_AT(97, 11);
        if (!plain_ok) best = 0;
        // the touched nodes' re-scores on threads 128.. (beside the tile scan of the lower threads, not after it), the
        // pod row copied to registers first (its fields in LDS would be a chain of dependent reads)
        if (tid >= 128 && tid - 128 < nt && plain_ok) {
            for (int q = tid - 128; q < nt; q += KG_RESOLVE_THREADS - 128) {
                const unsigned long long k = q < KG_NCACHE ? pair_key_cached<NUMA>(c, pl, pd, ncache[q], nrow[q], touched[q], now_ns)
                                                           : pair_key<NUMA>(c, pl, pd, touched[q], n_nodes, now_ns);
                best = best > k ? best : k;
            }
        }
        KG_RT_AT(128, 8);
        // the previous chunk's nodes, on the upper half of the workgroup (the tile scan and the touched re-scores
        // run on the lower threads: each NodeNUMAResource re-score is a long single-lane chain)
        // A node an earlier pod of this chunk committed again is left to the touched re-score above: its key in pvkeys
        // predates that commit, and in the plain form (LDSB) its global row and planes may still be in flight behind
        // the LDS-only barriers (a global re-read would see the node before the commit, with more free capacity).
        for (int q = tid - KG_RESOLVE_THREADS / 2; q >= 0 && q < np_prev && plain_ok; q += KG_RESOLVE_THREADS / 2) {
            const int32_t nd = prevt[q];
            bool again = false;
            if (pv_pre || LDSB)
                for (int z = 0; z < nt; z++) again |= touched[z] == nd;
            unsigned long long k = 0ull;
            if (again) k = 0ull;
            else if (pv_pre && KG_IN(41, prevq[q], n_prev)) k = pvkeys[(int64_t)j * n_prev + prevq[q]];
            else k = pair_key<NUMA>(c, pl, pd, nd, n_nodes, now_ns);
            best = best > k ? best : k;
        }
        // nodes outside the fp64 bounds are not in the lists: re-scored exactly, every pod
        const int ns = (!rescore_slow || !plain_ok) ? 0 : n_slow;
        for (int q = tid; q < ns; q += KG_RESOLVE_THREADS) {
            const int32_t sn = slow_list[q];
            // a slow node the chunk touched is re-scored above (cached: from its LDS row)
            if (LDSB && sn >= 0 && sn < n_nodes && is_touched(ttile[sn / KG_TILE], sn, nt, 0)) continue;
            const unsigned long long k = pair_key<NUMA>(c, pl, pd, sn, n_nodes, now_ns);
            best = best > k ? best : k;
        }
        __syncthreads();
        KG_RT(2);
        const int nr = plain_ok ? n_rescan[par] : 0;
        for (int q = tid; q < nr * KG_TILE; q += KG_RESOLVE_THREADS) {
            const int64_t node = (int64_t)rescan[q / KG_TILE] * KG_TILE + (q % KG_TILE);
            // the chunk's touched nodes are re-scored above (cached: from their LDS rows, whose global stores the
            // plain form's LDS-only barriers leave unordered)
            if (LDSB && node < n_nodes && is_touched(ttile[rescan[q / KG_TILE]], (int32_t)node, nt, 0)) continue;
            const unsigned long long k = pair_key<NUMA>(c, pl, pd, node, n_nodes, now_ns);
            best = best > k ? best : k;
        }
        best = wave_max_u64(best);
        if ((tid & 63) == 0) red[tid >> 6] = best;
        __syncthreads();
        KG_RT(3);
        // every thread takes the block maximum itself (no broadcast barrier)
        unsigned long long wb = 0;
        for (int q = 0; q < KG_RESOLVE_THREADS / 64; q++) wb = wb > red[q] ? wb : red[q];
        if (tid == 0) n_rescan[par] = 0;   // pod j + 2's counter: every reader of it is past the sync above
#pragma unroll
        for (int q = 0; q < KG_PARTIAL_SLOTS; q++) kcur[q] = knxt[q];
        if (rsv_on) {
            __syncthreads();
            // PreScore / Score / NormalizeScore over every reservation node (the refreshed entries are ordered
            // by the barriers above)
            const unsigned long long *E = ra.E + (int64_t)j * ra.n_rn;
            const int64_t *O = ra.O + (int64_t)j * ra.n_rn;
            const unsigned long long rk =
                ra.M ? rsv_best_resolve<KG_RESOLVE_THREADS>(c, pl, ra, j, rpf, touched, nt, gflag, glist, n_glist, red, redo)
                     : rsv_best_block<KG_RESOLVE_THREADS>(c, E, O, ra.rnode, ra.n_rn, nullptr, 0, 0, red, redo);
            wb = wb > rk ? wb : rk;
        }
        const unsigned long long w = gate_ok[par] ? wb : 0ull;   // a pod failing the quota gate is unschedulable
        int32_t node = w ? (int32_t)(0xFFFFFFFFull - (w & 0xFFFFFFFFull)) : -1;
        if (w && !KG_IN(44, node, n_nodes)) node = -1;   // (every thread decodes the same w)
        if (node < 0 || (defer_last && j == n - 1)) {
            // no feasible node; or the chunk's last pod may bind a cpuset: it is selected here and reserved by
            // the host (the CPU accumulator) after the launch
            if (tid == 0) {
                out_node[j] = node;
                out_score[j] = w ? (int64_t)(w >> 32) - 1 : -1;
            }
            if (rsv_on && ra.M && j + 1 < n && tid >= KG_RESOLVE_THREADS / 2)   // (the reduction's reads are done)
                rsv_prefetch(ra, j + 1, rpf, tid - KG_RESOLVE_THREADS / 2, KG_RESOLVE_THREADS / 2);
            continue;   // nothing changed: the next pod's first barrier orders the outputs
        }
        // Reserve.  NodeNUMAResource's zone commit (its amplified-cpu filter) reads the pre-Reserve node, so it
        // goes first when enabled; the Reservation commit takes the nomination from the pod's entry.
        // the node's canonical row, staged into LDS by one wave (a single coalesced round trip): the
        // Reserve parts below update and re-derive from this copy and store their fields back
        kg_node_row &srow = nrow[KG_NCACHE];
        // the node's slot in the touched list (and node cache): its position, or the next one — found by wave 0 with
        // one ballot (a touched list of ≤ 64; longer lists are walked), handed to the other waves through LDS
        uint32_t old_df = 0;
        int64_t old_metric = 0;
        if (tid < 64) {
            int sl = nt;
            if (nt <= 64) {
                const unsigned long long hit = __ballot(tid < nt && touched[tid] == node);
                sl = hit ? __builtin_ctzll(hit) : nt;
            } else {
                for (int q = 0; q < nt; q++)
                    if (touched[q] == node) sl = q;
            }
            // a node an earlier pod of the chunk committed is staged from its LDS copy (the committed row, flags and
            // NodeMetric time), the others from global memory
            const bool cached = sl < nt && sl < KG_NCACHE;
            if (tid == 0) {   // the planes tid 0 needs, in flight with the row
                old_df = cached ? ncache[sl].n.df : pl.dflags[node];
                old_metric = cached ? ncache[sl].metric_ns : pl.metric_ns[node];
                slot_s = sl;
            }
            if (tid < ROW_U4)
                reinterpret_cast<uint4 *>(&srow)[tid] = cached ? reinterpret_cast<const uint4 *>(&nrow[sl])[tid]
                                                               : reinterpret_cast<const uint4 *>(pl.rows + node)[tid];
        }
        __syncthreads();
        const int slot = slot_s;
        KG_RT(4);
        if (numa_on) {
            // the zone table of the staged row (wave 0), then the zone commit's hint enumeration over it (tid 0)
            const bool zoned = (srow.flags & KG_NODE_NUMA_OPTIONS) && srow.numa_policy != KG_NUMA_NONE &&
                               srow.n_zones > 0;   // n_zones ≤ KG_MAX_ZONES (kg_build_node_rows)
            if (zoned && tid < 64) {
                kg_zone_tab_fill(srow, tid, 64, czt, [] {
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                });
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
            }
            if (tid == 0) {
                if (zoned) kg_numa_commit_tab(c, srow, pd, czt);
                else kg_numa_commit(c, srow, pd);
            }
            // the parts below read only srow (LDS)
            __syncthreads();
        }
        NodeCacheEntry *ce = slot < KG_NCACHE ? &ncache[slot] : nullptr;
        // AssumePod / LoadAware deltas and the committed node's derived planes, one thread per part:
        // thread 64 + r owns resource r's fields of the row and its Fit planes, 64 + 8 + r the LoadAware
        // terms of r; thread 192 the reservation nomination; thread 0 the quota Reserve, the pod count and the outputs
        kg_node_row &row = pl.rows[node];
        if (tid >= 64 && tid < 64 + KG_NUM_RES) {
            const int r = tid - 64;
            const int64_t req = srow.requested[r] + pd.req[r];
            srow.requested[r] = req;
            row.requested[r] = req;
            if (r < 2) {
                const int64_t nz = srow.nonzero_requested[r] + pd.nonzero[r];
                srow.nonzero_requested[r] = nz;
                row.nonzero_requested[r] = nz;
            }
            if (r < 3) fl_over[r] = srow.alloc[r] - req < 0 ? 1u : 0u;
            int64_t fr;
            double R, F;
            fin[r] = kg_finalize_fit_r(c, pl, node, srow, r, &fr, &R, &F);
            KG_RT_AT(64 + 1, 7);
            if (ce && r < KG_FAST_RES) {
                ce->n.free_[r] = fr;
                ce->n.fit_R[r] = R;
                ce->n.fit_F[r] = F;
            }
        } else if (tid >= KG_RESOLVE_LA_T0 && tid < KG_RESOLVE_LA_T0 + 4) {
            // LoadAware Reserve, one thread per (resource r, usage variant v), on a wave of their own (in the Fit
            // parts' wave they ran after them: 6.8k → the Fit part's 2.4k cycles per pod, r05): the term and its
            // planes (kg_finalize_la_r split by variant; the slow test reads both new terms, computed by each)
            const int r = (tid - KG_RESOLVE_LA_T0) >> 1, v = (tid - KG_RESOLVE_LA_T0) & 1;
            const int64_t est = pd.la_est_i[r];
            const bool prod = (pd.flags & KG_POD_PROD) != 0;
            const int64_t u0 = srow.la_used[0][r] + est, u1 = srow.la_used[1][r] + (prod ? est : 0);
            if (v == 0) {
                srow.la_used[0][r] = u0;
                row.la_used[0][r] = u0;
            } else if (prod) {
                srow.la_used[1][r] = u1;
                row.la_used[1][r] = u1;
            }
            const int64_t cap = pl.cap, a = srow.la_alloc[r], uv = v ? u1 : u0;
            bool bounds = false;
            double R = 0.0, F = 0.0;
            if (a != 0) {
                if (a < 0 || a >= KG_CAP_LIMIT || kg_abs64(u0) >= KG_VAL_LIMIT || kg_abs64(u1) >= KG_VAL_LIMIT) {
                    bounds = true;
                } else {
                    R = 100.0 / (double)a;
                    F = kg_scaled_ratio(a - uv, a);
                }
            }
            if (v == 0) pl.la_R[r * cap + node] = R;
            pl.la_F[(v * 2 + r) * cap + node] = F;
            // (kg_finalize_la_r's bits: 1 slow, LoadAware weights beyond cpu / memory included; 2 outside the bounds)
            if (v == 0) fin[KG_NUM_RES + r] = (bounds || c.la_extra ? 1u : 0u) | (bounds ? 2u : 0u);
            KG_RT_AT(KG_RESOLVE_LA_T0, 0);
            if (ce) {
                if (v == 0) {
                    ce->n.la_R[r] = R;
                    ce->n.la_F0[r] = F;
                } else {
                    ce->n.la_F1[r] = F;
                }
            }
        } else if (tid >= KG_RESOLVE_LA_T0 + 4 && tid < KG_RESOLVE_LA_T0 + 4 + (KG_NUM_RES - 2)) {
            // LoadAware weights beyond cpu / memory: extra resource x's terms and planes (kg_finalize_lax_r)
            const int x = tid - KG_RESOLVE_LA_T0 - 4;
            bool bounds = false;
            if (c.la_extra) {
                srow.la_used_x[0][x] += pd.la_est_x[x];
                row.la_used_x[0][x] = srow.la_used_x[0][x];
                if (pd.flags & KG_POD_PROD) {
                    srow.la_used_x[1][x] += pd.la_est_x[x];
                    row.la_used_x[1][x] = srow.la_used_x[1][x];
                }
                bounds = kg_finalize_lax_r(c, pl, node, srow, x);
            }
            fin[KG_NUM_RES + 2 + x] = bounds ? 1u : 0u;
        } else if (numa_on && tid >= 128 && tid < 128 + KG_MAX_ZONES) {   // the zone commit, back to the row
            const int zi = tid - 128;
            row.zone_allocated[zi][0] = srow.zone_allocated[zi][0];
            row.zone_allocated[zi][1] = srow.zone_allocated[zi][1];
            if (zi == 0) row.zone_alloc_keys = srow.zone_alloc_keys;
        } else if (rsv_on && tid == 192) {   // Reservation.Reserve (its global writes are ordered for the next pod
            rsv_commit_entry(pl, ra, pd, node, ra.E + (int64_t)j * ra.n_rn);   // by the barrier that ends this one)
        } else if (rsv_on && ra.M && tid >= KG_RESOLVE_THREADS / 2 && tid < KG_RESOLVE_LA_T0) {   // the idle upper
            // waves: the next pod's split
            if (j + 1 < n) rsv_prefetch(ra, j + 1, rpf, tid - KG_RESOLVE_THREADS / 2, KG_RESOLVE_LA_T0 - KG_RESOLVE_THREADS / 2);
        } else if (tid == 0) {
            if (ra.quota && pd.quota >= 0) kg_quota_commit(ra.quota, pd.quota, pd);
            const int32_t pc = srow.pod_count + 1;
            srow.pod_count = pc;
            row.pod_count = pc;
            fl_pods_full = (int64_t)pc + 1 > (int64_t)srow.allowed_pods ? 1 : 0;
            fl_old_df = old_df;
            if (ce) ce->metric_ns = old_metric;
            if (slot == nt && KG_IN(43, n_touched, KG_MAX_CHUNK)) {
                touched[n_touched++] = node;
                mark(node);
                const int32_t rk = rsv_on && ra.M ? pl.rsv_of[node] : -1;
                if (rk >= 0 && !gflag[rk / KG_RSV_GROUP]) {   // its entry group: rescanned by later pods
                    gflag[rk / KG_RSV_GROUP] = 1;
                    glist[n_glist++] = rk / KG_RSV_GROUP;
                }
            }
            out_node[j] = node;
            out_score[j] = (int64_t)(w >> 32) - 1;
        }
        // the flags step reads the parts' LDS results only.  Their global stores (row, planes) need to be complete
        // only for a later global read of this node in the kernel: with a node-cache slot (the plain resolve) every
        // later read of it is served from LDS (staging, re-scores, exact pairs) and the barriers order LDS only;
        // otherwise (no slot, or the Reservation / NodeNUMAResource forms) they are full barriers.
        const bool lds_only = LDSB && slot < KG_NCACHE;
        if (lds_only) lds_barrier();
        else __syncthreads();
        KG_RT(5);
        if (ce && tid >= 128 && tid < 128 + ROW_U4)   // the committed row into the node cache
            reinterpret_cast<uint4 *>(&nrow[slot])[tid - 128] = reinterpret_cast<const uint4 *>(&srow)[tid - 128];
        if (tid == 0) {   // kg_finalize_flags from the parts (metric and the static bits are unchanged)
            bool slow = false, xslow = false;
            uint32_t fmask = 0;
            for (int r = 0; r < KG_NUM_RES; r++) slow = slow || (fin[r] & 1u);
            xslow = slow;
            for (int r = KG_NUM_RES; r < KG_NUM_RES + 2; r++) {
                slow = slow || (fin[r] & 1u);
                xslow = xslow || (fin[r] & 2u);
            }
            for (int x = 0; x < KG_NUM_RES - 2; x++) xslow = xslow || (fin[KG_NUM_RES + 2 + x] & 1u);
            for (int r = 0; r < KG_NUM_RES; r++)
                if (fin[r] & 2u) fmask |= 1u << r;
            const bool over[3] = {fl_over[0] != 0, fl_over[1] != 0, fl_over[2] != 0};
            const uint32_t old = fl_old_df;
            uint32_t dyn = kg_dflags_dynamic(fl_pods_full != 0, over, slow, xslow);
            if (old & KGD_RSV) dyn &= ~(KGD_SLOW | KGD_XSLOW);   // kg_rsv_pair owns reservation nodes
            const uint32_t df = (old & ~KGD_DYNAMIC) | dyn;
            pl.dflags[node] = df;
            pl.fit_mask[node] = fmask;
            if ((df & KGD_SLOW) && !(old & KGD_SLOW) && KG_IN(45, n_slow, pl.cap)) {   // the node left the fast paths: list it
                slow_list[n_slow++] = node;
                *slow_count = n_slow;
                if (lds_only) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the list entry is read next pod
            }
            if (ce) {
                ce->n.df = df;
                ce->n.fit_mask = fmask;
            }
        }
        if (lds_only) lds_barrier();
        else __syncthreads();
        KG_RT(6);
    }
#ifdef KG_RESOLVE_TIMING
    if (threadIdx.x == 0) g_rtimes_pod += n;
#endif
}

__global__ void k_commit_one(kg_consts c, kg_planes pl, const kg_pod_dev *__restrict__ pods, int32_t pod, int32_t node,
                             RsvArgs ra) {
    rsv_quota_commit(pl, ra, pods[pod], node);
    kg_numa_commit(c, pl.rows[node], pods[pod]);
    kg_apply_commit(pl.rows[node], pods[pod]);
    kg_finalize_node(c, pl, node);
}

// ---------------------------------------------------------------------------------------
// engine
// ---------------------------------------------------------------------------------------
struct kg_engine {
    kg_config cfg;
    kg_consts consts;
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    kg_planes pl{};
    void *plane_mem = nullptr;
    int64_t n_nodes = 0;
    int64_t shard_begin = 0, shard_end = 0;
    kg_pod_dev *pods = nullptr;     // generic per-pod rows (exact path, placement resolve)
    void *hot = nullptr;            // hot-kernel per-pod rows: kg_pod_hot_t<nslot>[n]
    int32_t nslot = 2;              // resource slots of the batch's profile (2, 4 or 8)
    int32_t slot_res[8] = {0, 1, -1, -1, -1, -1, -1, -1};
    int32_t n_pods = 0, pods_cap = 0;
    size_t hot_bytes = 0;
    int32_t *numa_perm = nullptr;   // NodeNUMAResource matrix mode: pod rows grouped by hint-list shape
    bool numa_perm_on = false;
    // pod equivalence in matrix mode off the class path (NodeNUMAResource, LoadAware extra weights): every output
    // of a pod is a function of its device row, so kg_eval evaluates each distinct row once (a batch of the
    // distinct rows) and copies the rows of the planes to every pod of it (k_eq_rows)
    bool eq_on = false;
    int32_t eq_n = 0;                  // distinct rows
    kg_pod_dev *eq_pods = nullptr;     // [eq_n]
    void *eq_hot = nullptr;            // [eq_n] their hot rows (the batch's slot map), for the Fit + LoadAware pass
    bool reps_in = false;              // pods / hot hold the distinct rows (eval_eq, ncache_build)
    int32_t *eq_perm = nullptr;        // [eq_n] their NodeNUMAResource visiting order (as numa_perm)
    bool eq_perm_on = false;
    int32_t *eq_of = nullptr;          // [n_pods] the distinct row of each pod
    void *eq_mem = nullptr;            // the distinct batch's outputs, then the staging of host outputs
    size_t eq_mem_bytes = 0;
    // pipelined NodeNUMAResource placement over the distinct rows (k_ncache_*): the cache [eq_n][stride] and the
    // matrix outputs it is built from, in one buffer; ncache_live while place_pipelined runs on it
    void *ncache_mem = nullptr;
    size_t ncache_bytes = 0;
    uint8_t *ncache = nullptr;
    int64_t ncache_stride = 0;
    bool ncache_live = false;
    BatchMasks bm{0, 0};
    uint32_t forms = 0;             // kg_set_forms: size-chosen kernel forms forced (KG_FORM_*), 0 = by size
    int64_t numa_resident_wgs = 0;  // resident k_eval_numa2 workgroups of the device (queried at first use)
    int64_t numa_resident_wgs_c = 0;  // ... of its COMBINE form
    int32_t *numa_queue = nullptr;  // its work-item counter
    int32_t numa_chunk_pods = KG_NUMA_CHUNK_PODS;   // placement chunks up to this many pods take k_eval_numa_chunk
                                                    // (0 under KG_FORM_NUMA_CHUNK_TILE: k_eval_numa2 for every chunk)
    bool la_prod = false;           // some pod of the batch scores with the prod-usage variant
    bool pow2 = true;               // every Fit / LoadAware weight sum of the batch is a power of two
    // class-specialised matrix mode (k_eval3): built from the batch in kg_pods_set, laid out for
    // the current shard width on the first kg_eval that needs it
    bool cls_ok = false;                    // every pod of the batch belongs to a specialisable class
    bool cls_dirty = true;
    int64_t cls_width = -1, cls_tiles = -1;
    std::vector<kg_cls_desc> cls_desc;      // host copies, one per class part (plain / duplicate-row)
    std::vector<std::vector<int32_t>> cls_members;   // pod indices per class part (a duplicate-row part: grouped by row)
    std::vector<std::vector<int32_t>> cls_ux;        // duplicate-row part: each member's row index (else empty)
    std::vector<std::vector<int32_t>> cls_reps;      // duplicate-row part: a pod of each distinct row (else empty)
    std::vector<kg_pod_row> pod_rows_h;
    void *cls_mem = nullptr;                // device: descs | work | rows
    size_t cls_mem_bytes = 0;
    int32_t cls_nwork = 0;
    int32_t cls_kind_work[12][2] = {};  // [3 · kind + form] = (first work item, count); form 0 mixed, 1 LoadAware-
                                        // uniform, 2 duplicate-row (its items carry their tile)
    size_t cls_work_off = 0, cls_rows_off = 0, cls_ids_off = 0;
    int32_t *xslow_list = nullptr;  // [cap] LoadAware-extra batches: nodes outside the bounds of any plane (KGD_XSLOW)
    int32_t *xslow_count = nullptr;
    double *hot_lax = nullptr;      // [n_pods][KG_LAX] the pods' −EstimatePod of the weighted extra resources
    bool lax_ok = false;            // the batch takes k_eval2's LAX form in matrix mode (≤ KG_LAX weighted extras)
    int32_t lax_n = 0, lax_x[KG_LAX] = {};
    int32_t *slow_list = nullptr;   // [cap] nodes outside the fast-path bounds, whole snapshot
    int32_t *slow_count = nullptr;
    bool slow_valid = false;        // the list matches the planes (rebuilt lazily after host-side changes;
                                    // the placement resolve appends the nodes its commits make slow)
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    // SURVEY §5 error contract: every successful snapshot mutation (reset, upsert / remove, commit,
    // placement resolve) advances the generation; a HIP error marks the device state stale, and every
    // entry point but kg_snapshot_reset then fails with KG_ERR_STATE until the snapshot is reloaded
    uint64_t generation = 0;
    bool stale = false;
    // cpuset binding (matrix mode on nodes without a NUMA topology policy): per-node facts of the host rows
    // pushed by upsert, and whether the pod batch binds cpusets (KG_POD_NUMA_CPU_BIND)
    std::vector<uint8_t> node_bind_facts;   // bit 0: NUMA topology policy; bit 1: node CPU bind policy;
                                            // bit 2: valid CPU topology without CPU detail
    int64_t n_numa_policy_nodes = 0, n_node_bind_nodes = 0, n_no_detail_nodes = 0;
    bool batch_bind = false;
    // cpuset Reserve (kg_cpus_set): each node's logical CPUs as NodeAllocation holds them, its MaxRefCount and
    // accumulator strategy; pods that may bind a cpuset end their placement chunk (pod_may_bind)
    struct CpuTable {
        int32_t max_ref = 1, strategy = KG_STRATEGY_LEAST_ALLOCATED;
        std::vector<kg_cpu_info> cpus;
    };
    std::unordered_map<int32_t, CpuTable> cpu_tab;
    std::vector<uint8_t> pod_may_bind;   // bit 0: binds by its own PreFilter; bit 1: a cpu request (node policy)
    bool profiling = false;
    // k_eval3 work items per class part ≈ these / tiles: the plain form (r03 A/B: 1024 / 2048 / 3072 0.78 ms,
    // 4096 / 6144 0.80 ms), the duplicate-row form (r05 A/B: 4096 / 8192 0.407 ms, 2048 0.424, 1024 0.427)
    int64_t cls_target_blocks = 2048, cls_dup_target_blocks = 4096;
    // the class kinds' launches on two streams (the mixed form on stream2), so one grid's tail is filled by the
    // other's workgroups (r03 A/B: 0.84 vs 0.87 ms per config-2 pass)
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t ev_res[3] = {};          // kg_place's pipeline (place_pipelined)
    // Reservation / ElasticQuota (config 5)
    void *rsv_mem = nullptr;            // slots | rfirst | rnode | E | O | M | Mn | G
    kg_reservation *rsv = nullptr;      // slots grouped by node (stable)
    std::vector<int32_t> rsv_perm;      // device slot → caller index
    int32_t n_rsv = 0;
    int32_t *rfirst = nullptr, *rnode = nullptr;
    int32_t n_rn = 0;
    unsigned long long *rsv_e = nullptr;
    int64_t *rsv_o = nullptr;
    kg_rsv_ment *rsv_m = nullptr;                  // the placement split of the entries (RsvArgs::M / Mn / G)
    int32_t *rsv_mn = nullptr;
    unsigned long long *rsv_g = nullptr;
    kg_quota *quota = nullptr;
    int32_t n_quota = 0;
    int32_t max_pod_quota = -1;         // largest quota index of the batch
    uint8_t *gate = nullptr;            // [pods] ElasticQuota PreFilter outcome (matrix mode)
    kg_counters ctr{};                  // kg_counters_get
    int64_t ev_acc = 0;                 // profiled launches already summed into ctr.kernel_ns
    ncclComm_t comm = nullptr;          // kg_comm_init: this rank's RCCL communicator (kg_place_sharded)
    kg_shm_comm *shm = nullptr;         // kg_comm_init_loopback: the host shared-memory communicator (kg_comm.cpp)
    uint32_t *shm_stage = nullptr;      // its pinned staging buffer (the slot size)
    uint32_t *comm_word = nullptr;      // device word of the status all-reduce (comm_agree)
    int32_t comm_rank = 0, comm_world = 0;
    hipStream_t eval_stream = nullptr;  // kg_set_eval_stream (kg_place_chunk_eval), nullptr ⇒ stream
    // recorded on eval_stream after each kg_place_chunk_eval, one per partial buffer (keyed by its address): a chunk
    // resolve makes the engine stream wait for the evaluation that wrote the partials it reads, whatever the caller
    // enqueued on the eval stream since
    static constexpr int kEvalEvents = 4;
    hipEvent_t ev_eval[kEvalEvents] = {};
    const void *ev_eval_buf[kEvalEvents] = {};
    int32_t ev_eval_next = 0;
    static constexpr int kRing = 256;   // event pairs: one per profiled k_eval launch
    hipEvent_t ev0[kRing] = {}, ev1[kRing] = {};
    int64_t ev_count = 0;               // launches recorded since kg_set_profiling
    std::string err;
};

// RCCL, loaded on first use (kg_comm_*): the engine library does not depend on it otherwise
namespace {
struct Rccl {
    bool tried = false;
    void *h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};
Rccl &rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
        r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        if (r.h) break;
    }
    if (!r.h) return r;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
    r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
    if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy || !r.error_string) {
        dlclose(r.h);
        r.h = nullptr;
    }
    return r;
}
}  // namespace

namespace {

kg_status set_err(kg_engine *e, kg_status code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (e) {
        e->err = buf;
        if (code == KG_ERR_HIP) e->stale = true;
    }
    return code;
}

#define HIP_TRY(e, expr)                                                                         \
    do {                                                                                         \
        hipError_t _st = (expr);                                                                 \
        if (_st != hipSuccess) return set_err(e, KG_ERR_HIP, "%s: %s", #expr, hipGetErrorString(_st)); \
    } while (0)

// the bounds-checked build's verdict (KG_BOUNDS_CHECK): the violations the kernels recorded since the last call
kg_status bounds_verdict(kg_engine *e) {
#ifdef KG_BOUNDS_CHECK
    unsigned long long v[4] = {};
    HIP_TRY(e, hipDeviceSynchronize());
    HIP_TRY(e, hipMemcpyFromSymbol(v, HIP_SYMBOL(g_kg_oob), sizeof(v)));
    if (v[0]) {
        const unsigned long long z[4] = {};
        HIP_TRY(e, hipMemcpyToSymbol(HIP_SYMBOL(g_kg_oob), z, sizeof(z)));
        return set_err(e, KG_ERR_STATE, "bounds check: %llu violations, the first at site %llu: index %lld outside [0, %lld)",
                       v[0], v[1], (long long)v[2], (long long)v[3]);
    }
#endif
    (void)e;
    return KG_OK;
}

// host → device copies go through here (kg_counters.h2d_bytes)
hipError_t h2d(kg_engine *e, void *dst, const void *src, size_t bytes, hipStream_t s) {
    e->ctr.h2d_bytes += bytes;
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
}

// Profiled launches (kg_set_profiling): an event pair per launch in a ring of kRing; a slot about to be reused is
// summed into the counters first, so kg_counters_get's kernel_ns covers every timed launch
hipError_t prof_sum(kg_engine *e, int64_t k) {
    const int64_t slot = k % kg_engine::kRing;
    float ms = 0.f;
    hipError_t st = hipEventSynchronize(e->ev1[slot]);
    if (st == hipSuccess) st = hipEventElapsedTime(&ms, e->ev0[slot], e->ev1[slot]);
    if (st != hipSuccess) return st;
    e->ctr.kernel_ns += (uint64_t)((double)ms * 1e6);
    e->ctr.timed_launches++;
    return hipSuccess;
}
hipError_t prof_begin(kg_engine *e) {
    if (e->ev_count - e->ev_acc >= kg_engine::kRing) {
        const hipError_t st = prof_sum(e, e->ev_acc);
        if (st != hipSuccess) return st;
        e->ev_acc++;
    }
    return hipEventRecord(e->ev0[e->ev_count % kg_engine::kRing], e->stream);
}
hipError_t prof_end(kg_engine *e) {
    const hipError_t st = hipEventRecord(e->ev1[e->ev_count % kg_engine::kRing], e->stream);
    e->ev_count++;
    return st;
}

kg_status ensure_scratch(kg_engine *e, size_t bytes) {
    if (e->scratch_bytes >= bytes) return KG_OK;
    if (e->scratch) HIP_TRY(e, hipFree(e->scratch));
    e->scratch = nullptr;
    e->scratch_bytes = 0;
    HIP_TRY(e, hipMalloc(&e->scratch, bytes));
    e->scratch_bytes = bytes;
    return KG_OK;
}

int64_t tiles_total(const kg_engine *e) { return e->pl.cap / KG_TILE; }

int pods_per_block_for(int64_t n_pods, int64_t tiles, int64_t target_blocks = 2048) {
    int64_t ppb = (n_pods * tiles + target_blocks - 1) / target_blocks;
    ppb = (ppb + KG_POD_CHUNK - 1) / KG_POD_CHUNK * KG_POD_CHUNK;
    if (ppb < KG_POD_CHUNK) ppb = KG_POD_CHUNK;
    if (ppb > KG_CLS_ITEM_MAX) ppb = KG_CLS_ITEM_MAX;
    return (int)ppb;
}

template <int S, bool FAST, bool LA_PROD>
void launch_hot_div(kg_engine *e, dim3 grid, const HotArgs &a, int32_t pod_begin, uint64_t *mask, uint16_t *scores,
                    uint32_t *partials, bool topk) {
    const kg_pod_hot_t<S> *pods = reinterpret_cast<const kg_pod_hot_t<S> *>(e->hot) + pod_begin;
    if (mask)
        hipLaunchKernelGGL((k_eval2<S, FAST, LA_PROD, true, false>), grid, dim3(KG_BLOCK), 0, e->stream, e->consts,
                           e->pl, a, pods, mask, scores, partials);
    else if (topk)
        hipLaunchKernelGGL((k_eval2<S, FAST, LA_PROD, false, true>), grid, dim3(KG_BLOCK), 0, e->stream, e->consts,
                           e->pl, a, pods, mask, scores, partials);
    else
        hipLaunchKernelGGL((k_eval2<S, FAST, LA_PROD, false, false>), grid, dim3(KG_BLOCK), 0, e->stream, e->consts,
                           e->pl, a, pods, mask, scores, partials);
}

template <int S>
void launch_hot(kg_engine *e, dim3 grid, const HotArgs &a, int32_t pod_begin, uint64_t *mask, uint16_t *scores,
                uint32_t *partials, bool topk) {
    const kg_consts &c = e->consts;
    const bool fast = e->pow2 && !c.fit_most && c.weight_fit == 1 && c.weight_la == 1 &&
                      (c.plugins & (KG_PLUGIN_FIT | KG_PLUGIN_LOADAWARE)) == (KG_PLUGIN_FIT | KG_PLUGIN_LOADAWARE);
    if (e->la_prod) {
        if (fast) launch_hot_div<S, true, true>(e, grid, a, pod_begin, mask, scores, partials, topk);
        else launch_hot_div<S, false, true>(e, grid, a, pod_begin, mask, scores, partials, topk);
    } else {
        if (fast) launch_hot_div<S, true, false>(e, grid, a, pod_begin, mask, scores, partials, topk);
        else launch_hot_div<S, false, false>(e, grid, a, pod_begin, mask, scores, partials, topk);
    }
}

// ---- class-specialised path (k_eval3): host-side class building -------------------------------
struct ClsKey {
    uint32_t nzc, zc, fitm, sel, lav;
    bool operator<(const ClsKey &o) const {
        if (nzc != o.nzc) return nzc < o.nzc;
        if (zc != o.zc) return zc < o.zc;
        if (fitm != o.fitm) return fitm < o.fitm;
        if (sel != o.sel) return sel < o.sel;
        return lav < o.lav;
    }
};

// The class of a pod: which resources the Fit filter compares (nzc: per-pod values; zc: zero native
// requests, a node-only overcommit check), which it scores, its node-filter variant and LoadAware
// usage variant.  False when the pod needs the generic slot kernel.
bool pod_class(const kg_config &cfg, const kg_pod_row &row, ClsKey &key) {
    const bool fit_on = (cfg.enabled_plugins & KG_PLUGIN_FIT) != 0;
    const bool la_on = (cfg.enabled_plugins & KG_PLUGIN_LOADAWARE) != 0;
    const bool hr = fit_on && (row.flags & KG_POD_HAS_REQUEST);
    key = ClsKey{0, 0, 0, 0, 0};
    if (hr) {
        for (int r = 0; r < 3; r++) (row.request[r] != 0 ? key.nzc : key.zc) |= 1u << r;
        key.nzc |= row.request_present & KG_SCALAR_RES_MASK;
    }
    uint32_t w = 0;
    if (fit_on) {
        for (int r = 0; r < KG_NUM_RES; r++) {
            if (cfg.fit_resource_weight[r] <= 0) continue;
            if (((KG_SCALAR_RES_MASK >> r) & 1u) && row.fit_score_request[r] == 0) continue;
            key.fitm |= 1u << r;
            w += (uint32_t)cfg.fit_resource_weight[r];
        }
    }
    const uint32_t variant = (row.flags & KG_POD_DAEMONSET) ? 2u : (row.flags & KG_POD_PROD) ? 1u : 0u;
    key.sel = variant + (hr ? 3u : 0u);
    key.lav = (la_on && (row.flags & KG_POD_LA_PROD_SCORE)) ? 1u : 0u;
    if (__builtin_popcount(key.nzc) > 4 || __builtin_popcount(key.fitm) > 4) return false;
    if (w != 0 && (w & (w - 1)) != 0) return false;
    return true;
}

// LoadAware-uniform chunks: a class's pods regrouped by EstimatePod, the whole KG_EVAL3_CC-pod chunks of one
// estimate first (aligned to the class start, so every chunk k_eval3 walks there is one estimate: its LoadAware
// least-requested sums depend on the node only and are evaluated once per node and chunk, the way the uniform
// Fit slots fold into ClsNode::cq), the remainders after them.  Rows carry their own output offsets, so the
// order within a class is free.  Returns the end of the uniform region.
int32_t cls_order_la(const kg_engine *e, std::vector<int32_t> &mem) {
    const bool la_on = (e->cfg.enabled_plugins & KG_PLUGIN_LOADAWARE) != 0;
    if (!la_on) return 0;
    auto est = [&](int32_t i) { return std::make_pair(e->pod_rows_h[i].la_estimate[0], e->pod_rows_h[i].la_estimate[1]); };
    std::vector<int32_t> s = mem;
    std::stable_sort(s.begin(), s.end(), [&](int32_t x, int32_t y) { return est(x) < est(y); });
    std::vector<int32_t> head, tail;
    head.reserve(s.size());
    for (size_t a = 0; a < s.size();) {
        size_t b = a + 1;
        while (b < s.size() && est(s[b]) == est(s[a])) b++;
        const size_t whole = (b - a) / KG_EVAL3_CC * KG_EVAL3_CC;
        head.insert(head.end(), s.begin() + a, s.begin() + a + whole);
        tail.insert(tail.end(), s.begin() + a + whole, s.begin() + b);
        a = b;
    }
    const int32_t end = (int32_t)head.size();
    head.insert(head.end(), tail.begin(), tail.end());
    mem.swap(head);
    return end;
}

template <int NC, int NF>
void cls_fill_row(const kg_engine *e, const kg_cls_desc &d, const kg_pod_row &r, char *dst) {
    kg_pod_cls_t<NC, NF> h;
    memset(&h, 0, sizeof(h));
    const bool most = e->cfg.fit_strategy == KG_STRATEGY_MOST_ALLOCATED;
    for (int k = 0; k < NC; k++) h.req[k] = d.cmp_res[k] >= 0 ? r.request[d.cmp_res[k]] : KG_NEUTRAL_REQ;
    for (int f = 0; f < NF; f++) {
        const double pr = d.fit_res[f] >= 0 ? (double)r.fit_score_request[d.fit_res[f]] : 0.0;
        h.pr[f] = most ? pr : -pr;
    }
    h.la[0] = -(double)r.la_estimate[0];
    h.la[1] = -(double)r.la_estimate[1];
    memcpy(dst, &h, sizeof(h));
}

void cls_fill_any(const kg_engine *e, const kg_cls_desc &d, const kg_pod_row &r, char *dst) {
    if (d.kind == 0) cls_fill_row<2, 2>(e, d, r, dst);
    else if (d.kind == 1) cls_fill_row<2, 4>(e, d, r, dst);
    else if (d.kind == 2) cls_fill_row<4, 2>(e, d, r, dst);
    else cls_fill_row<4, 4>(e, d, r, dst);
}

// Classes of the batch, each split in two parts: the pods whose class row (the only per-pod input of k_eval3)
// occurs more than once in the class form its duplicate-row part (evaluated once per distinct row, written to
// every pod of it: k_eval3_dup), the rest its plain part.
void cls_prepare(kg_engine *e) {
    e->cls_ok = false;
    e->cls_dirty = true;
    e->cls_desc.clear();
    e->cls_members.clear();
    e->cls_ux.clear();
    e->cls_reps.clear();
    const bool la_on = (e->cfg.enabled_plugins & KG_PLUGIN_LOADAWARE) != 0;
    if (la_on && e->consts.la_shift == 0xFF) return;
    std::map<ClsKey, int> index;
    std::vector<ClsKey> keys;
    std::vector<std::vector<int32_t>> members;
    for (int32_t i = 0; i < (int32_t)e->pod_rows_h.size(); i++) {
        ClsKey k;
        if (!pod_class(e->cfg, e->pod_rows_h[i], k)) return;
        auto it = index.find(k);
        int c;
        if (it == index.end()) {
            if (2 * (int)keys.size() == KG_CLS_MAX) return;
            c = (int)keys.size();
            index.emplace(k, c);
            keys.push_back(k);
            members.emplace_back();
        } else {
            c = it->second;
        }
        members[c].push_back(i);
    }
    for (size_t c = 0; c < keys.size(); c++) {
        const ClsKey &k = keys[c];
        kg_cls_desc d;
        memset(&d, 0, sizeof(d));
        // scored resources whose request is one value over the whole class fold into a per-node term when
        // that leaves at most two per-pod slots (a four-slot class then runs as a two-slot kind)
        const std::vector<int32_t> &mem = members[c];
        uint32_t unim = 0;
        for (int r = 0; r < KG_NUM_RES; r++) {
            if (!((k.fitm >> r) & 1u)) continue;
            const int64_t v0 = e->pod_rows_h[mem[0]].fit_score_request[r];
            bool same = true;
            for (size_t j = 1; j < mem.size() && same; j++) same = e->pod_rows_h[mem[j]].fit_score_request[r] == v0;
            if (same) unim |= 1u << r;
        }
        if (__builtin_popcount(k.fitm) <= 2 || __builtin_popcount(k.fitm & ~unim) > 2) unim = 0;
        const uint32_t varm = k.fitm & ~unim;
        const int nc = __builtin_popcount(k.nzc) <= 2 ? 2 : 4, nf = __builtin_popcount(varm) <= 2 ? 2 : 4;
        d.kind = (nc == 2 ? 0 : 2) + (nf == 2 ? 0 : 1);
        int a = 0, b = 0, u = 0;
        uint32_t w = 0;
        const bool most = e->cfg.fit_strategy == KG_STRATEGY_MOST_ALLOCATED;
        for (int s = 0; s < 4; s++) d.cmp_res[s] = d.fit_res[s] = d.uni_res[s] = -1;
        for (int r = 0; r < KG_NUM_RES; r++) {
            if ((k.nzc >> r) & 1u) d.cmp_res[a++] = r;
            if ((varm >> r) & 1u) {
                d.fit_w[b] = (uint32_t)e->cfg.fit_resource_weight[r];
                w += d.fit_w[b];
                d.fit_res[b++] = r;
            }
            if ((unim >> r) & 1u) {
                d.uni_w[u] = (uint32_t)e->cfg.fit_resource_weight[r];
                w += d.uni_w[u];
                const double pr = (double)e->pod_rows_h[mem[0]].fit_score_request[r];
                d.uni_pr[u] = most ? pr : -pr;
                d.uni_res[u++] = r;
            }
        }
        d.fit_shift = w ? (uint32_t)__builtin_ctz(w) : 0u;
        d.node_ok_sel = k.sel;
        d.la_variant = k.lav;
        d.over_mask = k.zc;
        d.row_bytes = d.kind == 0 ? (int64_t)sizeof(kg_pod_cls_t<2, 2>) : d.kind == 1 ? (int64_t)sizeof(kg_pod_cls_t<2, 4>)
                      : d.kind == 2 ? (int64_t)sizeof(kg_pod_cls_t<4, 2>) : (int64_t)sizeof(kg_pod_cls_t<4, 4>);
        // the class rows, grouped: distinct rows in order of first occurrence, each with its pods in queue order
        std::map<std::string, int32_t> row_id;
        std::vector<std::vector<int32_t>> by_row;
        std::string buf((size_t)d.row_bytes, '\0');
        for (int32_t i : mem) {
            cls_fill_any(e, d, e->pod_rows_h[i], &buf[0]);
            auto it = row_id.emplace(buf, (int32_t)by_row.size());
            if (it.second) by_row.emplace_back();
            by_row[it.first->second].push_back(i);
        }
        std::vector<int32_t> plain, dup, ux, reps;
        for (const std::vector<int32_t> &g : by_row) {
            if (g.size() == 1) {
                plain.push_back(g[0]);
                continue;
            }
            reps.push_back(g[0]);
            for (int32_t i : g) {
                dup.push_back(i);
                ux.push_back((int32_t)reps.size() - 1);
            }
        }
        if (!plain.empty()) {
            kg_cls_desc dp = d;
            dp.la_uni_end = cls_order_la(e, plain);
            dp.count = (int32_t)plain.size();
            dp.ux_first = -1;
            e->cls_desc.push_back(dp);
            e->cls_members.push_back(std::move(plain));
            e->cls_ux.emplace_back();
            e->cls_reps.emplace_back();
        }
        if (!dup.empty()) {
            kg_cls_desc dd = d;
            dd.la_uni_end = 0;
            dd.count = (int32_t)dup.size();
            dd.ux_first = 0;   // laid out by cls_layout
            e->cls_desc.push_back(dd);
            e->cls_members.push_back(std::move(dup));
            e->cls_ux.push_back(std::move(ux));
            e->cls_reps.push_back(std::move(reps));
        }
    }
    e->cls_ok = true;
}

// Lay the class rows out for the shard width (output offsets) and the work table for its tiles.
kg_status cls_layout(kg_engine *e, int64_t width, int64_t shard_tiles) {
    if (!e->cls_dirty && e->cls_width == width && e->cls_tiles == shard_tiles) return KG_OK;
    const int64_t words = (width + 63) / 64;
    if ((int64_t)e->pod_rows_h.size() * words >= (1LL << 31)) return set_err(e, KG_ERR_RANGE, "mask too large");
    std::vector<kg_cls_desc> descs = e->cls_desc;
    std::vector<kg_cls_work> work;
    size_t rows_bytes = 0;
    int32_t n_ids = 0;
    for (size_t c = 0; c < descs.size(); c++) {
        const bool dup = !e->cls_reps[c].empty();
        descs[c].rows_offset = (int64_t)rows_bytes;
        rows_bytes += (size_t)descs[c].row_bytes * (dup ? e->cls_reps[c].size() : (size_t)descs[c].count);
        descs[c].ids_first = n_ids;
        n_ids += descs[c].count;
        if (dup) {
            descs[c].ux_first = n_ids;
            n_ids += descs[c].count;
        }
    }
    // the work table grouped by (kind, form): one launch each; a plain part's LoadAware-uniform region
    // [0, la_uni_end) and its tail are split into work items separately; a duplicate-row part is split into pod runs
    // of equal length per tile, tile by tile (k_eval3_dup's XCD order)
    for (int g = 0; g < 12; g++) {
        const int kind = g / 3, form = g % 3;
        e->cls_kind_work[g][0] = (int32_t)work.size();
        if (form < 2) {
            const bool lau = form == 1;
            for (size_t c = 0; c < descs.size(); c++) {
                if (descs[c].kind != kind || !e->cls_reps[c].empty()) continue;
                const int32_t b0 = lau ? 0 : descs[c].la_uni_end, b1 = lau ? descs[c].la_uni_end : descs[c].count;
                if (b1 <= b0) continue;
                const int32_t ppb = pods_per_block_for(b1 - b0, shard_tiles, e->cls_target_blocks);
                for (int32_t b = b0; b < b1; b += ppb) work.push_back(kg_cls_work{(int32_t)c, b, b + ppb < b1 ? b + ppb : b1, 0});
            }
        } else {
            std::vector<std::pair<int32_t, int32_t>> runs;   // (part, run length) of one tile
            for (size_t c = 0; c < descs.size(); c++) {
                if (descs[c].kind != kind || e->cls_reps[c].empty()) continue;
                const int32_t cnt = descs[c].count;
                const int32_t ppb = pods_per_block_for(cnt, shard_tiles, e->cls_dup_target_blocks);
                const int32_t n_it = (cnt + ppb - 1) / ppb;
                runs.emplace_back((int32_t)c, (cnt + n_it - 1) / n_it);
            }
            for (int32_t t = 0; t < (int32_t)shard_tiles; t++)
                for (const auto &r : runs) {
                    const int32_t cnt = descs[r.first].count;
                    for (int32_t b = 0; b < cnt; b += r.second)
                        work.push_back(kg_cls_work{r.first, b, b + r.second < cnt ? b + r.second : cnt, t});
                }
        }
        e->cls_kind_work[g][1] = (int32_t)work.size() - e->cls_kind_work[g][0];
    }
    std::vector<char> rows(rows_bytes, 0);
    std::vector<int32_t> ids((size_t)n_ids + 1, 0);
    for (size_t c = 0; c < descs.size(); c++) {
        const kg_cls_desc &d = descs[c];
        const std::vector<int32_t> &mem = e->cls_members[c];
        for (int32_t j = 0; j < d.count; j++) ids[(size_t)d.ids_first + (size_t)j] = mem[(size_t)j];
        const bool dup = !e->cls_reps[c].empty();
        if (dup)
            for (int32_t j = 0; j < d.count; j++) ids[(size_t)d.ux_first + (size_t)j] = e->cls_ux[c][(size_t)j];
        const std::vector<int32_t> &src = dup ? e->cls_reps[c] : mem;
        for (size_t j = 0; j < src.size(); j++)
            cls_fill_any(e, d, e->pod_rows_h[src[j]], rows.data() + d.rows_offset + j * (size_t)d.row_bytes);
    }
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t desc_b = sizeof(kg_cls_desc) * KG_CLS_MAX, work_b = sizeof(kg_cls_work) * (work.size() + 1);
    const size_t need = up(desc_b) + up(work_b) + up(rows.size()) + up(ids.size() * 4);
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    if (need > e->cls_mem_bytes) {
        if (e->cls_mem) HIP_TRY(e, hipFree(e->cls_mem));
        e->cls_mem = nullptr;
        e->cls_mem_bytes = 0;
        HIP_TRY(e, hipMalloc(&e->cls_mem, need));
        e->cls_mem_bytes = need;
    }
    e->cls_work_off = up(desc_b);
    e->cls_rows_off = up(desc_b) + up(work_b);
    char *m = (char *)e->cls_mem;
    HIP_TRY(e, h2d(e, m, descs.data(), sizeof(kg_cls_desc) * descs.size(), e->stream));
    if (!work.empty()) HIP_TRY(e, h2d(e, m + e->cls_work_off, work.data(), sizeof(kg_cls_work) * work.size(), e->stream));
    e->cls_ids_off = e->cls_rows_off + up(rows.size());
    if (!rows.empty()) HIP_TRY(e, h2d(e, m + e->cls_rows_off, rows.data(), rows.size(), e->stream));
    HIP_TRY(e, h2d(e, m + e->cls_ids_off, ids.data(), ids.size() * 4, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));   // the host vectors end with this call
    e->cls_nwork = (int32_t)work.size();
    e->cls_width = width;
    e->cls_tiles = shard_tiles;
    e->cls_dirty = false;
    return KG_OK;
}

template <bool MOST, bool FIT_ON, bool LA_ON, bool W1, int KIND, int FORM>
void launch_cls_kind(kg_engine *e, dim3 grid, const HotArgs &a, const kg_cls_desc *descs, const kg_cls_work *work,
                     const char *rows, const int32_t *ids, uint64_t *mask, uint16_t *scores, uint32_t *partials,
                     hipStream_t stream) {
    constexpr bool LAU = FORM == 1;
    const int32_t first = e->cls_kind_work[3 * KIND + FORM][0], count = e->cls_kind_work[3 * KIND + FORM][1];
    if (count == 0) return;
    if constexpr (LAU && !LA_ON) return;   // (no such work items: cls_order_la)
    else if constexpr (FORM == 2) {
        const dim3 g1((unsigned)((count + KG_XCDS - 1) / KG_XCDS * KG_XCDS));
        if (mask)
            hipLaunchKernelGGL((k_eval3_dup<MOST, FIT_ON, LA_ON, true, W1, KIND>), g1, dim3(KG_TILE / 2), 0, stream,
                               e->consts, e->pl, a, descs, work + first, count, rows, ids, mask, scores, partials);
        else
            hipLaunchKernelGGL((k_eval3_dup<MOST, FIT_ON, LA_ON, false, W1, KIND>), g1, dim3(KG_TILE / 2), 0, stream,
                               e->consts, e->pl, a, descs, work + first, count, rows, ids, mask, scores, partials);
    } else {
        grid.y = (unsigned)count;
        // matrix mode: 8-pod chunks, score segments staged in LDS and written as 1 KiB wave stores; two nodes per
        // lane (four: 92 VGPRs, 5 waves per SIMD, 1.98 vs 0.88 ms per config-2 pass, round 2)
        if (mask)
            hipLaunchKernelGGL((k_eval3<MOST, FIT_ON, LA_ON, true, W1, KIND, LAU>), grid, dim3(KG_TILE / 2), 0, stream,
                               e->consts, e->pl, a, descs, work + first, rows, ids, mask, scores, partials);
        else
            hipLaunchKernelGGL((k_eval3<MOST, FIT_ON, LA_ON, false, W1, KIND, LAU>), grid, dim3(KG_TILE / 2), 0, stream,
                               e->consts, e->pl, a, descs, work + first, rows, ids, mask, scores, partials);
    }
}

template <bool MOST, bool FIT_ON, bool LA_ON, bool W1>
void launch_cls4(kg_engine *e, dim3 grid, const HotArgs &a, uint64_t *mask, uint16_t *scores, uint32_t *partials) {
    const char *m = (const char *)e->cls_mem;
    const kg_cls_desc *descs = (const kg_cls_desc *)m;
    const kg_cls_work *work = (const kg_cls_work *)(m + e->cls_work_off);
    const char *rows = m + e->cls_rows_off;
    const int32_t *ids = (const int32_t *)(m + e->cls_ids_off);
    // fork: stream2 starts after everything already queued on the engine stream
    if (!e->stream2) {
        (void)hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking);
        (void)hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming);
    }
    (void)hipEventRecord(e->ev_fork, e->stream);
    (void)hipStreamWaitEvent(e->stream2, e->ev_fork, 0);
    hipStream_t s2 = e->stream2;
    // duplicate-row and LoadAware-uniform work on the engine stream, the mixed rest on stream2: one grid's tail is
    // filled by the other's workgroups
#define KG_LAUNCH_KIND(K)                                                                                              \
    launch_cls_kind<MOST, FIT_ON, LA_ON, W1, K, 2>(e, grid, a, descs, work, rows, ids, mask, scores, partials, e->stream); \
    launch_cls_kind<MOST, FIT_ON, LA_ON, W1, K, 1>(e, grid, a, descs, work, rows, ids, mask, scores, partials, e->stream); \
    launch_cls_kind<MOST, FIT_ON, LA_ON, W1, K, 0>(e, grid, a, descs, work, rows, ids, mask, scores, partials, s2)
    KG_LAUNCH_KIND(0);
    KG_LAUNCH_KIND(1);
    KG_LAUNCH_KIND(2);
    KG_LAUNCH_KIND(3);
#undef KG_LAUNCH_KIND
    // join: the engine stream continues after every kind
    (void)hipEventRecord(e->ev_join, s2);
    (void)hipStreamWaitEvent(e->stream, e->ev_join, 0);
}

template <bool MOST, bool FIT_ON, bool LA_ON>
void launch_cls3(kg_engine *e, dim3 grid, const HotArgs &a, uint64_t *mask, uint16_t *scores, uint32_t *partials) {
    // plugin weights 1 and every Fit / LoadAware resource weight 1 (the shipped profile): all weighted
    // sums are plain sums
    bool unit = e->consts.weight_fit == 1 && e->consts.weight_la == 1;
    if (LA_ON) unit = unit && e->consts.la_w[0] == 1 && e->consts.la_w[1] == 1;
    for (const kg_cls_desc &d : e->cls_desc)
        for (int f = 0; f < 4; f++) unit = unit && d.fit_w[f] <= 1u && d.uni_w[f] <= 1u;
    if (unit) launch_cls4<MOST, FIT_ON, LA_ON, true>(e, grid, a, mask, scores, partials);
    else launch_cls4<MOST, FIT_ON, LA_ON, false>(e, grid, a, mask, scores, partials);
}

void launch_cls(kg_engine *e, dim3 grid, const HotArgs &a, uint64_t *mask, uint16_t *scores, uint32_t *partials) {
    const bool most = e->consts.fit_most != 0;
    const bool fit = (e->consts.plugins & KG_PLUGIN_FIT) != 0, la = (e->consts.plugins & KG_PLUGIN_LOADAWARE) != 0;
    if (!fit) launch_cls3<false, false, true>(e, grid, a, mask, scores, partials);
    else if (most && la) launch_cls3<true, true, true>(e, grid, a, mask, scores, partials);
    else if (most) launch_cls3<true, true, false>(e, grid, a, mask, scores, partials);
    else if (la) launch_cls3<false, true, true>(e, grid, a, mask, scores, partials);
    else launch_cls3<false, true, false>(e, grid, a, mask, scores, partials);
}

// mask and scores are both produced or both omitted (the host path provides scratch for a missing one)
// the slow-node list of the whole snapshot, rebuilt when host-side changes invalidated it
kg_status slow_refresh(kg_engine *e) {
    if (e->slow_valid) return KG_OK;
    HIP_TRY(e, hipMemsetAsync(e->slow_count, 0, sizeof(int32_t), e->stream));
    if (e->n_nodes > 0)
        hipLaunchKernelGGL(k_slow_list, dim3((unsigned)((e->n_nodes + 255) / 256)), dim3(256), 0, e->stream, e->pl.dflags,
                           (int64_t)0, e->n_nodes, e->slow_list, e->slow_count);
    HIP_TRY(e, hipGetLastError());
    e->slow_valid = true;
    return KG_OK;
}

// topk: placement chunk (partials of KG_PARTIAL_SLOTS per (pod, tile) on the non-NUMA path; the NUMA
// kernel writes one key per (pod, tile), slot 0 of a dense [n][tiles] layout — see partial_slots)
// Fit + LoadAware over the launch's pods (every form but NodeNUMAResource's): the LAX / exact forms for LoadAware
// weights beyond cpu / memory, the class kernels, the slot kernels, then the slow-node fix-up
// `prof`: its own profiled interval (false inside the NodeNUMAResource launch's, which covers both passes)
kg_status launch_eval_plain(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n, uint64_t *mask, uint16_t *scores,
                            uint32_t *partials, bool use_cls, bool topk, HotArgs a, int64_t shard_tiles, bool prof = true) {
    if (e->consts.la_extra && !topk && e->lax_ok) {
        // LoadAware weights beyond cpu / memory, at most KG_LAX of them: k_eval2's LAX form reads their planes too;
        // the nodes outside the fp64 bounds of any plane (KGD_XSLOW) are re-evaluated exactly after it
        a.lax_n = e->lax_n;
        for (int k = 0; k < KG_LAX; k++) {
            a.lax_x[k] = k < e->lax_n ? e->lax_x[k] : 0;
            a.lax_w[k] = k < e->lax_n ? (uint32_t)e->consts.la_wx[e->lax_x[k]] : 0u;
        }
        a.lax_est = e->hot_lax + (int64_t)pod_begin * KG_LAX;
        if (prof && e->profiling) HIP_TRY(e, prof_begin(e));
        dim3 grid((unsigned)shard_tiles, (unsigned)((n + a.pods_per_block - 1) / a.pods_per_block));
        const bool prod = e->la_prod;
#define KG_LAX_LAUNCH(S_)                                                                                               \
        do {                                                                                                            \
            const kg_pod_hot_t<S_> *hp = reinterpret_cast<const kg_pod_hot_t<S_> *>(e->hot) + pod_begin;                \
            if (mask && prod)                                                                                          \
                hipLaunchKernelGGL((k_eval2<S_, false, true, true, false, true>), grid, dim3(KG_BLOCK), 0, e->stream,  \
                                   e->consts, e->pl, a, hp, mask, scores, partials);                                   \
            else if (mask)                                                                                             \
                hipLaunchKernelGGL((k_eval2<S_, false, false, true, false, true>), grid, dim3(KG_BLOCK), 0, e->stream, \
                                   e->consts, e->pl, a, hp, mask, scores, partials);                                   \
            else if (prod)                                                                                             \
                hipLaunchKernelGGL((k_eval2<S_, false, true, false, false, true>), grid, dim3(KG_BLOCK), 0, e->stream, \
                                   e->consts, e->pl, a, hp, mask, scores, partials);                                   \
            else                                                                                                       \
                hipLaunchKernelGGL((k_eval2<S_, false, false, false, false, true>), grid, dim3(KG_BLOCK), 0, e->stream,\
                                   e->consts, e->pl, a, hp, mask, scores, partials);                                   \
        } while (0)
        if (e->nslot == 2) KG_LAX_LAUNCH(2);
        else if (e->nslot == 4) KG_LAX_LAUNCH(4);
        else KG_LAX_LAUNCH(8);
#undef KG_LAX_LAUNCH
        HIP_TRY(e, hipGetLastError());
        if (prof && e->profiling) HIP_TRY(e, prof_end(e));
        HIP_TRY(e, hipMemsetAsync(e->xslow_count, 0, sizeof(int32_t), e->stream));
        if (e->n_nodes > 0)
            hipLaunchKernelGGL(k_slow_list, dim3((unsigned)((e->n_nodes + 255) / 256)), dim3(256), 0, e->stream, e->pl.dflags,
                               (int64_t)0, e->n_nodes, e->xslow_list, e->xslow_count, (uint32_t)KGD_XSLOW);
        hipLaunchKernelGGL(k_fix_slow, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, e->consts, e->pl,
                           e->pods + pod_begin, n, e->xslow_list, e->xslow_count, e->shard_begin, e->shard_end,
                           a.mask_words, a.score_stride, a.tiles_total, now_ns, (unsigned long long *)mask, scores,
                           partials);
        HIP_TRY(e, hipGetLastError());
        return KG_OK;
    }
    if (e->consts.la_extra && !topk) {   // every node is on the exact path: no fast kernel, no slow list
        if (prof && e->profiling) HIP_TRY(e, prof_begin(e));
        const int64_t width = e->shard_end - e->shard_begin;
        dim3 grid((unsigned)((width + 255) / 256), (unsigned)(n < 65535 ? n : 65535));
        hipLaunchKernelGGL(k_eval_exact, grid, dim3(256), 0, e->stream, e->consts, e->pl, e->pods + pod_begin, n,
                           e->shard_begin, e->shard_end, a.mask_words, a.score_stride, a.tiles_total, now_ns,
                           (unsigned long long *)mask, scores, partials);
        HIP_TRY(e, hipGetLastError());
        if (prof && e->profiling) HIP_TRY(e, prof_end(e));
        return KG_OK;
    }
    use_cls = use_cls && e->cls_ok && !e->reps_in && pod_begin == 0 && n == e->n_pods;
    if (use_cls) {
        kg_status st = cls_layout(e, e->shard_end - e->shard_begin, shard_tiles);
        if (st) return st;
    }
    dim3 grid((unsigned)shard_tiles, use_cls ? (unsigned)e->cls_nwork : (unsigned)((n + a.pods_per_block - 1) / a.pods_per_block));
    if (prof && e->profiling) HIP_TRY(e, prof_begin(e));
    if (use_cls) launch_cls(e, grid, a, mask, scores, partials);
    else if (e->nslot == 2) launch_hot<2>(e, grid, a, pod_begin, mask, scores, partials, topk);
    else if (e->nslot == 4) launch_hot<4>(e, grid, a, pod_begin, mask, scores, partials, topk);
    else launch_hot<8>(e, grid, a, pod_begin, mask, scores, partials, topk);
    HIP_TRY(e, hipGetLastError());
    if (prof && e->profiling) HIP_TRY(e, prof_end(e));
    // exact re-evaluation of the (rare) nodes outside the fp64 fast-path bounds; a placement chunk
    // leaves them to the resolve, which re-scores the slow-node list itself
    kg_status st = slow_refresh(e);
    if (st) return st;
    if (!topk) {
        hipLaunchKernelGGL(k_fix_slow, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, e->consts, e->pl,
                           e->pods + pod_begin, n, e->slow_list, e->slow_count, e->shard_begin, e->shard_end,
                           a.mask_words, a.score_stride, a.tiles_total, now_ns, (unsigned long long *)mask, scores,
                           partials);
        HIP_TRY(e, hipGetLastError());
    }
    return KG_OK;
}

kg_status launch_eval(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n, uint64_t *mask, uint16_t *scores,
                      uint32_t *partials, bool use_cls = false, uint8_t *numa_scores = nullptr, bool topk = false) {
    if (n <= 0) return KG_OK;
    if ((mask == nullptr) != (scores == nullptr)) return set_err(e, KG_ERR_INVALID_ARG, "mask and scores go together");
    const int64_t shard_tiles = (e->shard_end - e->shard_begin + KG_TILE - 1) / KG_TILE;
    if (shard_tiles <= 0) return KG_OK;
    HotArgs a;
    a.n_pods = n;
    a.pods_per_block = pods_per_block_for(n, shard_tiles);
    a.tile_begin = (int32_t)(e->shard_begin / KG_TILE);
    a.tiles_total = (int32_t)tiles_total(e);
    a.node_end = e->shard_end;
    a.col_begin = e->shard_begin;
    a.mask_words = (int32_t)((e->shard_end - e->shard_begin + 63) / 64);
    a.score_stride = (e->shard_end - e->shard_begin + 63) / 64 * 64;
    a.fit_cap = e->consts.fit_most ? 100u : 0xFFFFFFFFu;
    for (int s = 0; s < 8; s++) a.slot_res[s] = s < e->nslot ? e->slot_res[s] : -1;
    a.now_ns = now_ns;
    if ((e->consts.plugins & KG_PLUGIN_NUMA) && topk && n <= e->numa_chunk_pods) {
        if (e->profiling) HIP_TRY(e, prof_begin(e));
        const unsigned blocks = (unsigned)((shard_tiles + KG_XCDS - 1) / KG_XCDS * KG_XCDS * n);
        if (e->ncache_live && !e->consts.numa_bz)
            hipLaunchKernelGGL(k_eval_numa_cached, dim3(blocks), dim3(256), 0, e->stream, e->consts, e->pl, a,
                               e->pods + pod_begin, (int32_t)shard_tiles, partials, e->ncache, e->eq_of + pod_begin,
                               e->ncache_stride, e->eq_n);
        else if (e->consts.numa_bz)
            hipLaunchKernelGGL(k_eval_numa_chunk<true>, dim3(blocks), dim3(256), 0, e->stream, e->consts, e->pl, a,
                               e->pods + pod_begin, (int32_t)shard_tiles, partials);
        else
            hipLaunchKernelGGL(k_eval_numa_chunk<false>, dim3(blocks), dim3(256), 0, e->stream, e->consts, e->pl, a,
                               e->pods + pod_begin, (int32_t)shard_tiles, partials);
        HIP_TRY(e, hipGetLastError());
        if (e->profiling) HIP_TRY(e, prof_end(e));
        return KG_OK;
    }
    if (e->consts.plugins & KG_PLUGIN_NUMA) {
        // matrix launches with planes: Fit + LoadAware by the class / slot kernels first (node per lane, pods uniform:
        // the per-pair form costs 0.08 ms per 1e8 pairs), their tile keys cleared, then k_eval_numa2 reads the two
        // score bytes and the feasibility bit back and adds the NodeNUMAResource term — the pod-per-lane kernel then
        // carries no node planes and no Fit / LoadAware pair code
        const bool combine = mask && scores && partials && !topk && !(e->forms & KG_FORM_NUMA_FUSED) &&
                             !(e->reps_in && (e->consts.la_extra || !e->eq_hot));
        if (e->profiling) HIP_TRY(e, prof_begin(e));   // one profiled interval for both passes
        if (combine) {
            kg_status st = launch_eval_plain(e, now_ns, pod_begin, n, mask, scores, partials, use_cls, false, a, shard_tiles,
                                             false);
            if (st) return st;
            HIP_TRY(e, hipMemsetAsync(partials, 0, (size_t)n * (size_t)a.tiles_total * 4, e->stream));
        }
        {  // pod per lane; queued 32-node items when they fill every resident wave slot several times over,
           // else a grid where a single pod block splits each wave's node run 4 ways
            // segment: 32 nodes (half mask words); 8 for a placement chunk's keys-only launch
            const int32_t seg = mask == nullptr && scores == nullptr && numa_scores == nullptr ? KG_NUMA2_SEG_TOPK : KG_NUMA2_SEG;
            const int32_t *perm = e->numa_perm_on && pod_begin == 0 && n == e->n_pods ? e->numa_perm : nullptr;
            const BatchMasks bm = e->bm;
            if (e->numa_resident_wgs == 0) {
                int dev_cus = 0, per_cu = 0;
                HIP_TRY(e, hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, e->device));
                HIP_TRY(e, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_eval_numa2<false>, 256, 0));
                e->numa_resident_wgs = (int64_t)dev_cus * (per_cu > 0 ? per_cu : 1);
                per_cu = 0;
                HIP_TRY(e, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_eval_numa2<true>, 256, 0));
                e->numa_resident_wgs_c = (int64_t)dev_cus * (per_cu > 0 ? per_cu : 1);
                HIP_TRY(e, hipMalloc(&e->numa_queue, sizeof(int32_t)));
            }
            // queued when the items give every resident wave one at least; else the grid, each wave's 256-node run
            // split z ways so that the grid covers the resident slots twice (a 70-row distinct batch of config 3:
            // 98 tiles × 2 pod blocks would otherwise be 196 workgroups for 768 slots)
            const int64_t n_items = shard_tiles * (KG_TILE / seg) * ((n + 63) / 64);
            const bool queued = (e->forms & KG_FORM_NUMA_QUEUED) || topk || n_items >= 4 * e->numa_resident_wgs;
            if (queued && n_items < INT32_MAX) {
                HIP_TRY(e, hipMemsetAsync(e->numa_queue, 0, sizeof(int32_t), e->stream));
                const int64_t wgs = std::min<int64_t>(combine ? e->numa_resident_wgs_c : e->numa_resident_wgs, (n_items + 3) / 4);
                if (combine)
                    hipLaunchKernelGGL(k_eval_numa2<true>, dim3((unsigned)wgs), dim3(256), 0, e->stream, e->consts, e->pl, a,
                                       e->pods + pod_begin, e->pl.rows, (unsigned long long *)mask, scores, numa_scores,
                                       partials, perm, bm, e->numa_queue, (int32_t)n_items, seg);
                else
                    hipLaunchKernelGGL(k_eval_numa2<false>, dim3((unsigned)wgs), dim3(256), 0, e->stream, e->consts, e->pl, a,
                                       e->pods + pod_begin, e->pl.rows, (unsigned long long *)mask, scores, numa_scores,
                                       partials, perm, bm, e->numa_queue, (int32_t)n_items, seg);
            } else {
                const int64_t blocks = shard_tiles * ((n + 63) / 64);
                unsigned z = 1;
                while (z < KG_NUMA2_NODES / 32 && blocks * z < 2 * e->numa_resident_wgs) z *= 2;
                dim3 grid((unsigned)shard_tiles, (unsigned)((n + 63) / 64), z);
                if (combine)
                    hipLaunchKernelGGL(k_eval_numa2<true>, grid, dim3(256), 0, e->stream, e->consts, e->pl, a, e->pods + pod_begin,
                                       e->pl.rows, (unsigned long long *)mask, scores, numa_scores, partials, perm, bm,
                                       (int32_t *)nullptr, 0, 0);
                else
                    hipLaunchKernelGGL(k_eval_numa2<false>, grid, dim3(256), 0, e->stream, e->consts, e->pl, a, e->pods + pod_begin,
                                       e->pl.rows, (unsigned long long *)mask, scores, numa_scores, partials, perm, bm,
                                       (int32_t *)nullptr, 0, 0);
            }
        }
        HIP_TRY(e, hipGetLastError());
        // cpusets on NUMA-policy nodes: patched in after the hot kernel (matrix planes, or the one-key-per-tile
        // partials of a large placement chunk)
        if ((!topk || e->consts.numa_bz) && e->n_numa_policy_nodes > 0 && (e->batch_bind || e->n_node_bind_nodes > 0)) {
            const int64_t width = e->shard_end - e->shard_begin;
            dim3 grid((unsigned)((width + 255) / 256), (unsigned)(n < 65535 ? n : 65535));
            hipLaunchKernelGGL(k_numa_bind_fix, grid, dim3(256), 0, e->stream, e->consts, e->pl, a, e->pods + pod_begin,
                               (unsigned long long *)mask, scores, numa_scores, partials);
            HIP_TRY(e, hipGetLastError());
        }
        if (e->profiling) HIP_TRY(e, prof_end(e));
        return KG_OK;
    }
    return launch_eval_plain(e, now_ns, pod_begin, n, mask, scores, partials, use_cls, topk, a, shard_tiles);
}

#define KG_RSV_POD_CHUNK 1024   // pods per reservation-entry pass (E/O hold [chunk][n_rn])

RsvArgs rsv_args(const kg_engine *e) {
    RsvArgs ra{};
    if ((e->consts.plugins & KG_PLUGIN_RESERVATION) && e->n_rn > 0) {
        ra.rsv = e->rsv;
        ra.rfirst = e->rfirst;
        ra.rnode = e->rnode;
        ra.n_rn = e->n_rn;
        ra.E = e->rsv_e;
        ra.O = e->rsv_o;
        const int32_t ng = (e->n_rn + KG_RSV_GROUP - 1) / KG_RSV_GROUP;
        if (ng <= KG_RSV_MAX_GROUPS) {   // else the resolve reduces over every entry (rsv_best_block)
            ra.M = e->rsv_m;
            ra.Mn = e->rsv_mn;
            ra.G = e->rsv_g;
            ra.ngroups = ng;
        }
    }
    if (e->consts.plugins & KG_PLUGIN_ELASTICQUOTA) ra.quota = e->quota;
    ra.quota_parent = e->cfg.eq_check_parent_quota != 0;
    return ra;
}

// Cpuset binding (NodeNUMAResource for LSE / LSR pods, or any cpu request on a node with a CPU bind policy):
// the Filter's Allocate reduces to counts of free CPUs (node-wide without a NUMA topology policy, per allocated
// zone with one), which the rows carry; the Reserve takes the CPUs on the host from the kg_cpus_set tables
// (kg_place, kg_commit).  The sharded chunk API (no host Reserve step), nodes whose valid topology lacks CPU
// detail and reservation-reserved cpusets are refused explicitly instead of being answered wrongly.
kg_status bind_ready(kg_engine *e, bool placement, bool host_reserve = false) {
    if (!(e->cfg.enabled_plugins & KG_PLUGIN_NUMA)) return KG_OK;
    const bool any_bind = e->batch_bind || e->n_node_bind_nodes > 0;
    if (placement && any_bind && !host_reserve)
        return set_err(e, KG_ERR_UNSUPPORTED,
                       "cpuset Reserve runs in kg_place / kg_commit (the host takes the CPUs between chunks); the "
                       "chunk API does not bind cpusets");
    if (placement && any_bind) {   // every node a cpuset can land on needs its CPU table
        for (size_t i = 0; i < e->node_bind_facts.size(); i++)
            if ((e->node_bind_facts[i] & 8) && !e->cpu_tab.count((int32_t)i))
                return set_err(e, KG_ERR_STATE, "node %zu: cpuset Reserve needs the node's CPUs (kg_cpus_set)", i);
    }
    if (e->batch_bind && e->n_no_detail_nodes > 0)
        return set_err(e, KG_ERR_UNSUPPORTED,
                       "cpuset-bound pods need CPU detail on every node with a valid CPU topology (%lld without)",
                       (long long)e->n_no_detail_nodes);
    if (any_bind && (e->cfg.enabled_plugins & KG_PLUGIN_RESERVATION))
        return set_err(e, KG_ERR_UNSUPPORTED, "cpuset binding with Reservation (reserved cpusets) is not on the engine path");
    return KG_OK;
}

kg_status quota_ready(kg_engine *e) {
    if (!(e->consts.plugins & KG_PLUGIN_ELASTICQUOTA)) return KG_OK;
    if (e->max_pod_quota >= e->n_quota)
        return set_err(e, KG_ERR_STATE, "pod quota index %d without a kg_quota_set group (have %d)", e->max_pod_quota,
                       e->n_quota);
    return KG_OK;
}

// entries of pods [pod_begin, pod_begin + n) (n ≤ KG_RSV_POD_CHUNK) for every reservation node
// split: also the placement split of the entries (RsvArgs::M / Mn / G) for the resolve
kg_status rsv_eval_chunk(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n, uint64_t *mask, uint16_t *scores,
                         uint8_t *numa_scores, int32_t mask_words, int64_t score_stride, bool split = false) {
    RsvArgs ra = rsv_args(e);
    if (!ra.rsv || n <= 0) return KG_OK;
    if (!split) ra.M = nullptr;
    if (ra.M) HIP_TRY(e, hipMemsetAsync(ra.Mn, 0, 4 * (size_t)n, e->stream));
    dim3 grid((unsigned)((ra.n_rn + 255) / 256), (unsigned)n);
    auto *kre = (e->consts.plugins & KG_PLUGIN_NUMA) ? k_rsv_eval<true> : k_rsv_eval<false>;
    hipLaunchKernelGGL(kre, grid, dim3(256), 0, e->stream, e->consts, e->pl, ra, e->pods + pod_begin, n, now_ns,
                       (unsigned long long *)mask, scores, numa_scores, e->shard_begin, e->shard_end, mask_words,
                       score_stride);
    HIP_TRY(e, hipGetLastError());
    return KG_OK;
}

kg_status check_engine(kg_engine *e, bool reloading = false) {
    if (!e) return KG_ERR_INVALID_ARG;
    if (e->stale && !reloading)
        return set_err(e, KG_ERR_STATE, "device state is stale after a HIP error (%s): reload it with kg_snapshot_reset",
                       e->err.c_str());
    HIP_TRY(e, hipSetDevice(e->device));
    return KG_OK;
}

}  // namespace

namespace {
kg_status eval_eq(kg_engine *e, int64_t now_ns, const kg_eval_out *out);
}

extern "C" {

kg_status kg_engine_create(const kg_config *cfg, kg_engine **out) {
    if (!out) return KG_ERR_INVALID_ARG;
    *out = nullptr;
    char msg[256] = {0};
    kg_status st = kg_config_validate(cfg, msg, sizeof(msg));
    if (st != KG_OK) {
        fprintf(stderr, "kg_engine_create: %s\n", msg);
        return st;
    }
    kg_engine *e = new kg_engine();
    e->cfg = *cfg;
    kg_consts_from_config(*cfg, e->consts);
    e->device = cfg->device;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= e->device || e->device < 0) {
        fprintf(stderr, "kg_engine_create: no HIP device %d (found %d)\n", e->device, ndev);
        delete e;
        return KG_ERR_HIP;
    }
    if (hipSetDevice(e->device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return KG_ERR_HIP;
    }
    e->own_stream = true;
    *out = e;
    return KG_OK;
}

void kg_engine_destroy(kg_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->plane_mem) (void)hipFree(e->plane_mem);
    if (e->pods) (void)hipFree(e->pods);
    if (e->hot) (void)hipFree(e->hot);
    if (e->eq_hot) (void)hipFree(e->eq_hot);
    if (e->scratch) (void)hipFree(e->scratch);
    if (e->cls_mem) (void)hipFree(e->cls_mem);
    if (e->rsv_mem) (void)hipFree(e->rsv_mem);
    if (e->quota) (void)hipFree(e->quota);
    if (e->gate) (void)hipFree(e->gate);
    if (e->numa_perm) (void)hipFree(e->numa_perm);
    if (e->numa_queue) (void)hipFree(e->numa_queue);
    if (e->comm) (void)rccl().comm_destroy(e->comm);
    if (e->shm) kg_shm_comm_close(e->shm);
    if (e->shm_stage) (void)hipHostFree(e->shm_stage);
    if (e->comm_word) (void)hipFree(e->comm_word);
    if (e->hot_lax) (void)hipFree(e->hot_lax);
    if (e->eq_pods) (void)hipFree(e->eq_pods);
    if (e->eq_perm) (void)hipFree(e->eq_perm);
    if (e->eq_of) (void)hipFree(e->eq_of);
    if (e->eq_mem) (void)hipFree(e->eq_mem);
    if (e->ncache_mem) (void)hipFree(e->ncache_mem);
    if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
    if (e->stream2) (void)hipStreamDestroy(e->stream2);
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    for (int k = 0; k < kg_engine::kEvalEvents; k++)
        if (e->ev_eval[k]) (void)hipEventDestroy(e->ev_eval[k]);
    if (e->ev_join) (void)hipEventDestroy(e->ev_join);
    for (int k = 0; k < 3; k++)
        if (e->ev_res[k]) (void)hipEventDestroy(e->ev_res[k]);
    for (int k = 0; k < kg_engine::kRing; k++) {
        if (e->ev0[k]) (void)hipEventDestroy(e->ev0[k]);
        if (e->ev1[k]) (void)hipEventDestroy(e->ev1[k]);
    }
    delete e;
}

const char *kg_last_error(const kg_engine *e) { return e ? e->err.c_str() : "null engine"; }

kg_status kg_set_stream(kg_engine *e, void *s) {
    kg_status st = check_engine(e);
    if (st) return st;
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    if (e->own_stream) HIP_TRY(e, hipStreamDestroy(e->stream));
    if (s) {
        e->stream = (hipStream_t)s;
        e->own_stream = false;
    } else {
        HIP_TRY(e, hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
        e->own_stream = true;
    }
    return KG_OK;
}

kg_status kg_sync(kg_engine *e) {
    kg_status st = check_engine(e);
    if (st) return st;
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    return KG_OK;
}

kg_status kg_snapshot_reset(kg_engine *e, int32_t n_nodes) {
    kg_status st = check_engine(e, true);
    if (st) return st;
    if (n_nodes < 0) return set_err(e, KG_ERR_INVALID_ARG, "negative node count");
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    if (e->plane_mem) HIP_TRY(e, hipFree(e->plane_mem));
    e->plane_mem = nullptr;
    const int64_t cap = ((int64_t)n_nodes + KG_TILE - 1) / KG_TILE * KG_TILE + (n_nodes == 0 ? KG_TILE : 0);
    if (cap / KG_TILE > KG_MAX_TILES) return set_err(e, KG_ERR_RANGE, "too many nodes (max %d)", KG_MAX_TILES * KG_TILE);
    char *p = nullptr;
    auto carve = [&](size_t bytes) {
        char *r = p;
        p += (bytes + 255) / 256 * 256;
        return r;
    };
    size_t total = 0;
    const bool lax = e->consts.la_extra != 0;
    const size_t sizes[] = {sizeof(kg_node_row) * (size_t)cap, (size_t)KG_NUM_RES * 8 * cap, (size_t)KG_NUM_RES * 8 * cap,
                            (size_t)KG_NUM_RES * 8 * cap, 2 * 8 * (size_t)cap, 4 * 8 * (size_t)cap, 8 * (size_t)cap,
                            4 * (size_t)cap, 4 * (size_t)cap, 4 * (size_t)cap, 256, 4 * (size_t)cap,
                            // LoadAware weights beyond cpu / memory: their planes and the list of the nodes outside the
                            // fp64 bounds of any plane (KGD_XSLOW)
                            lax ? (size_t)(KG_NUM_RES - 2) * 8 * cap : 0, lax ? (size_t)2 * (KG_NUM_RES - 2) * 8 * cap : 0,
                            lax ? 4 * (size_t)cap : 0, lax ? (size_t)256 : 0};
    for (size_t s : sizes) total += (s + 255) / 256 * 256;
    HIP_TRY(e, hipMalloc(&e->plane_mem, total));
    HIP_TRY(e, hipMemsetAsync(e->plane_mem, 0, total, e->stream));
    p = (char *)e->plane_mem;
    e->pl.rows = (kg_node_row *)carve(sizes[0]);
    e->pl.free_ = (int64_t *)carve(sizes[1]);
    e->pl.fit_R = (double *)carve(sizes[2]);
    e->pl.fit_F = (double *)carve(sizes[3]);
    e->pl.la_R = (double *)carve(sizes[4]);
    e->pl.la_F = (double *)carve(sizes[5]);
    e->pl.metric_ns = (int64_t *)carve(sizes[6]);
    e->pl.dflags = (uint32_t *)carve(sizes[7]);
    e->pl.fit_mask = (uint32_t *)carve(sizes[8]);
    e->slow_list = (int32_t *)carve(sizes[9]);
    e->slow_count = (int32_t *)carve(sizes[10]);
    e->pl.rsv_of = (int32_t *)carve(sizes[11]);
    e->pl.la_Rx = lax ? (double *)carve(sizes[12]) : nullptr;
    e->pl.la_Fx = lax ? (double *)carve(sizes[13]) : nullptr;
    e->xslow_list = lax ? (int32_t *)carve(sizes[14]) : nullptr;
    e->xslow_count = lax ? (int32_t *)carve(sizes[15]) : nullptr;
    HIP_TRY(e, hipMemsetAsync(e->pl.rsv_of, 0xFF, sizes[11], e->stream));  // −1: no reservations
    if (e->rsv_mem) HIP_TRY(e, hipFree(e->rsv_mem));  // reservations refer to node indices: dropped
    e->rsv_mem = nullptr;
    e->rsv = nullptr;
    e->rfirst = e->rnode = nullptr;
    e->rsv_e = nullptr;
    e->rsv_o = nullptr;
    e->rsv_m = nullptr;
    e->rsv_mn = nullptr;
    e->rsv_g = nullptr;
    e->n_rsv = e->n_rn = 0;
    e->rsv_perm.clear();
    e->pl.cap = cap;
    e->n_nodes = n_nodes;
    e->node_bind_facts.assign((size_t)n_nodes, 0);
    e->cpu_tab.clear();   // CPU tables refer to node indices: dropped with the snapshot
    e->n_numa_policy_nodes = e->n_node_bind_nodes = e->n_no_detail_nodes = 0;
    e->shard_begin = 0;
    e->shard_end = n_nodes;
    hipLaunchKernelGGL(k_finalize_range, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, e->stream, e->consts, e->pl,
                       (int64_t)0, cap);
    HIP_TRY(e, hipGetLastError());
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->slow_valid = false;
    e->stale = false;
    e->generation++;
    return KG_OK;
}

kg_status kg_snapshot_generation(kg_engine *e, uint64_t *out) {
    if (!e || !out) return KG_ERR_INVALID_ARG;
    *out = e->generation;
    return e->stale ? KG_ERR_STATE : KG_OK;
}

kg_status kg_snapshot_upsert(kg_engine *e, const int32_t *node_index, const kg_node_row *rows, int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (n < 0 || (n > 0 && (!node_index || !rows))) return set_err(e, KG_ERR_INVALID_ARG, "bad upsert arguments");
    if (n == 0) return KG_OK;
    if (!e->plane_mem) return set_err(e, KG_ERR_STATE, "snapshot not initialised (kg_snapshot_reset)");
    for (int32_t k = 0; k < n; k++)
        if (node_index[k] < 0 || node_index[k] >= e->n_nodes) return set_err(e, KG_ERR_RANGE, "node index %d out of range", node_index[k]);
    // cpuset-binding facts of the rows (bind_ready); a node CPU bind policy turns every cpu request into a
    // cpuset request there, so it needs CPU detail
    std::vector<uint8_t> facts((size_t)n);
    for (int32_t k = 0; k < n; k++) {
        const kg_node_row &r = rows[k];
        const bool opts = (r.flags & KG_NODE_NUMA_OPTIONS) != 0;
        uint8_t f = 0;
        if (opts && r.numa_policy != KG_NUMA_NONE) f |= 1;
        if (opts && r.node_cpu_bind != KG_NODE_CPU_BIND_NONE) f |= 2;
        if ((r.flags & KG_NODE_NUMA_TOPO_VALID) && r.cpus_per_core <= 0) f |= 4;
        if ((r.flags & KG_NODE_NUMA_TOPO_VALID) && r.cpus_per_core > 0) f |= 8;   // CPU detail: a cpuset can land
        if ((f & 2) && (f & 4))
            return set_err(e, KG_ERR_UNSUPPORTED, "node %d: a CPU bind policy without CPU detail", node_index[k]);
        facts[k] = f;
    }
    for (int32_t k = 0; k < n; k++) {
        uint8_t &old = e->node_bind_facts[node_index[k]];
        e->n_numa_policy_nodes += (int)(facts[k] & 1) - (int)(old & 1);
        e->n_node_bind_nodes += (int)((facts[k] >> 1) & 1) - (int)((old >> 1) & 1);
        e->n_no_detail_nodes += (int)((facts[k] >> 2) & 1) - (int)((old >> 2) & 1);
        old = facts[k];
    }
    // a new row invalidates the node's CPU table: bind_ready then asks for the matching kg_cpus_set (the feeders
    // send both together), so a cpuset Reserve never runs the accumulator on CPUs of an older row
    for (int32_t k = 0; k < n; k++) e->cpu_tab.erase(node_index[k]);
    const size_t rb = sizeof(kg_node_row) * (size_t)n, ib = sizeof(int32_t) * (size_t)n;
    st = ensure_scratch(e, rb + ib + 256);
    if (st) return st;
    char *s = (char *)e->scratch;
    HIP_TRY(e, h2d(e, s, rows, rb, e->stream));
    HIP_TRY(e, h2d(e, s + (rb + 255) / 256 * 256, node_index, ib, e->stream));
    hipLaunchKernelGGL(k_upsert, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, e->consts, e->pl,
                       (const kg_node_row *)s, (const int32_t *)(s + (rb + 255) / 256 * 256), n);
    HIP_TRY(e, hipGetLastError());
    HIP_TRY(e, hipStreamSynchronize(e->stream));  // staging buffer reuse
    e->slow_valid = false;
    e->generation++;
    return KG_OK;
}

kg_status kg_snapshot_remove(kg_engine *e, int32_t node_index) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (node_index < 0 || node_index >= e->n_nodes) return set_err(e, KG_ERR_RANGE, "node index out of range");
    kg_node_row row;
    memset(&row, 0, sizeof(row));  // flags = 0 → invalid, never feasible
    e->cpu_tab.erase(node_index);
    return kg_snapshot_upsert(e, &node_index, &row, 1);
}

kg_status kg_snapshot_download(kg_engine *e, int32_t first, int32_t n, kg_node_row *out) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (first < 0 || n < 0 || first + (int64_t)n > e->n_nodes || (n > 0 && !out)) return set_err(e, KG_ERR_RANGE, "bad download range");
    if (n == 0) return KG_OK;
    HIP_TRY(e, hipMemcpyAsync(out, e->pl.rows + first, sizeof(kg_node_row) * (size_t)n, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    return KG_OK;
}

kg_status kg_set_shard(kg_engine *e, int32_t begin, int32_t end) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (begin < 0 || end < begin || end > e->n_nodes || (begin % KG_TILE && begin != end)) return set_err(e, KG_ERR_RANGE, "bad shard [%d,%d)", begin, end);
    e->shard_begin = begin;
    e->shard_end = end;
    return KG_OK;
}

int32_t kg_num_tiles(const kg_engine *e) { return e ? (int32_t)tiles_total(e) : 0; }

kg_status kg_pods_set(kg_engine *e, const kg_pod_row *rows, int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (n < 0 || (n > 0 && !rows)) return set_err(e, KG_ERR_INVALID_ARG, "bad pod batch");
    std::vector<kg_pod_dev> dev((size_t)n);
    BatchMasks bm{0, 0};
    bool la_prod = false, pow2 = true, batch_bind = false;
    uint32_t need = 0;
    int32_t max_quota = -1;
    for (int32_t i = 0; i < n; i++) {
        if (!kg_pod_row_in_bounds(rows[i])) return set_err(e, KG_ERR_RANGE, "pod %d: request outside the engine bounds", i);
        if ((e->cfg.enabled_plugins & KG_PLUGIN_NUMA) && !(rows[i].flags & KG_POD_NUMA_SKIP)) {
            if (rows[i].flags & KG_POD_NUMA_CPU_BIND) batch_bind = true;
            if (kg_numa_list_count(rows[i]) > KG_NUMA_MAX_LISTS)
                return set_err(e, KG_ERR_UNSUPPORTED, "pod %d: more than %d NUMA hint lists", i, KG_NUMA_MAX_LISTS);
        }
        kg_pod_dev_from_row(e->cfg, rows[i], dev[i]);
        if ((e->cfg.enabled_plugins & KG_PLUGIN_ELASTICQUOTA) && rows[i].quota > max_quota) max_quota = rows[i].quota;
        bm.cmp |= dev[i].cmp_mask;
        bm.fit |= dev[i].fit_mask;
        la_prod |= (rows[i].flags & KG_POD_LA_PROD_SCORE) != 0;
        pow2 &= dev[i].fit_w == 0 || (dev[i].fit_w & (dev[i].fit_w - 1)) == 0;
    }
    if (!(e->cfg.enabled_plugins & KG_PLUGIN_FIT)) bm.cmp = bm.fit = 0;
    if (!(e->cfg.enabled_plugins & KG_PLUGIN_LOADAWARE)) la_prod = false;
    pow2 &= e->consts.la_shift != 0xFF || !(e->cfg.enabled_plugins & KG_PLUGIN_LOADAWARE);
    // resource profile: the smallest slot set covering every resource the batch compares or scores
    int32_t nslot;
    int32_t slot_res[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    std::vector<char> hot;
    auto build = [&](auto tag, int ns, const int32_t *map) {
        using H = decltype(tag);
        nslot = ns;
        for (int s = 0; s < ns; s++) slot_res[s] = map[s];
        hot.assign(sizeof(H) * (size_t)n, 0);
        need = 0;
        for (int32_t i = 0; i < n; i++) need |= kg_pod_hot_from_row(e->cfg, rows[i], slot_res, ((H *)hot.data())[i]);
    };
    static const int32_t native_map[2] = {KG_RES_CPU, KG_RES_MEMORY};
    static const int32_t coloc_map[4] = {KG_RES_CPU, KG_RES_MEMORY, KG_RES_BATCH_CPU, KG_RES_BATCH_MEMORY};
    build(kg_pod_hot_t<2>(), 2, native_map);
    if (need & ~0x3u) build(kg_pod_hot_t<4>(), 4, coloc_map);
    if (need & ~0x1Bu) {   // 8 slots: cpu, memory and every other resource the batch compares or scores (≤ 6 more)
        int32_t map8[8] = {KG_RES_CPU, KG_RES_MEMORY, -1, -1, -1, -1, -1, -1};
        int ns8 = 2;
        for (int r = 2; r < KG_NUM_RES; r++) {
            if (!((need >> r) & 1u)) continue;
            if (ns8 == 8)
                return set_err(e, KG_ERR_UNSUPPORTED, "the batch compares or scores more than 8 resources (%d)",
                               __builtin_popcount(need | 3u));
            map8[ns8++] = r;
        }
        build(kg_pod_hot_t<8>(), 8, map8);
    }
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    if (n > e->pods_cap || hot.size() > e->hot_bytes) {
        if (e->pods) HIP_TRY(e, hipFree(e->pods));
        if (e->hot) HIP_TRY(e, hipFree(e->hot));
        if (e->gate) HIP_TRY(e, hipFree(e->gate));
        if (e->numa_perm) HIP_TRY(e, hipFree(e->numa_perm));
        e->pods = nullptr;
        e->hot = nullptr;
        e->gate = nullptr;
        e->numa_perm = nullptr;
        e->pods_cap = 0;
        e->hot_bytes = 0;
        HIP_TRY(e, hipMalloc(&e->pods, sizeof(kg_pod_dev) * (size_t)(n > 0 ? n : 1)));
        HIP_TRY(e, hipMalloc(&e->hot, sizeof(kg_pod_hot_t<8>) * (size_t)(n > 0 ? n : 1)));
        HIP_TRY(e, hipMalloc(&e->gate, 2 * (size_t)(n > 0 ? n : 1)));
        HIP_TRY(e, hipMalloc(&e->numa_perm, sizeof(int32_t) * (size_t)(n > 0 ? n : 1)));
        e->pods_cap = n;
        e->hot_bytes = sizeof(kg_pod_hot_t<8>) * (size_t)(n > 0 ? n : 1);
    }
    if (n) {
        HIP_TRY(e, h2d(e, e->pods, dev.data(), sizeof(kg_pod_dev) * (size_t)n, e->stream));
        HIP_TRY(e, h2d(e, e->hot, hot.data(), hot.size(), e->stream));
    }
    // k_eval_numa2 runs a wave's 64 pods in lockstep through the hint enumeration, whose trip counts
    // depend on the pod's hint lists: matrix mode visits the pods (of `ids`, as positions into ids) grouped by list count
    // and request size, so a wave's lanes mostly share one loop shape (outputs stay in pod-row order).  Within a list
    // count the key is the larger of the pod's cpu and memory request ranks: a wave takes the single-zone path on a
    // node only when every lane's requests fit its largest zone, so the pods large in either resource share waves
    auto numa_order = [&](const std::vector<int32_t> &ids) {
        const size_t m = ids.size();
        std::vector<int32_t> order(m);
        for (size_t i = 0; i < m; i++) order[i] = (int32_t)i;
        auto lists = [&](int32_t i) { return (rows[i].flags & KG_POD_NUMA_SKIP) ? 0 : kg_numa_list_count(rows[i]); };
        std::vector<int32_t> rank_max(m, 0), by(order);
        for (int r = 0; r < 2; r++) {   // dense rank of the request among the pods (equal requests share a rank)
            std::sort(by.begin(), by.end(), [&](int32_t a, int32_t b) {
                return dev[ids[(size_t)a]].numa_req[r] < dev[ids[(size_t)b]].numa_req[r];
            });
            int32_t rk = 0;
            for (size_t i = 0; i < m; i++) {
                if (i > 0 && dev[ids[(size_t)by[i]]].numa_req[r] != dev[ids[(size_t)by[i - 1]]].numa_req[r]) rk++;
                rank_max[(size_t)by[i]] = std::max(rank_max[(size_t)by[i]], rk);
            }
        }
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
            const int32_t x = ids[(size_t)a], y = ids[(size_t)b];
            const int lx = lists(x), ly = lists(y);
            if (lx != ly) return lx < ly;
            if (rank_max[(size_t)a] != rank_max[(size_t)b]) return rank_max[(size_t)a] < rank_max[(size_t)b];
            if (dev[x].numa_req[KG_RES_CPU] != dev[y].numa_req[KG_RES_CPU])
                return dev[x].numa_req[KG_RES_CPU] < dev[y].numa_req[KG_RES_CPU];
            return dev[x].numa_req[KG_RES_MEMORY] < dev[y].numa_req[KG_RES_MEMORY];
        });
        return order;
    };
    std::vector<int32_t> all((size_t)n);
    for (int32_t i = 0; i < n; i++) all[(size_t)i] = i;
    e->numa_perm_on = (e->cfg.enabled_plugins & KG_PLUGIN_NUMA) && n > 64;
    if (e->numa_perm_on) {
        const std::vector<int32_t> order = numa_order(all);
        HIP_TRY(e, h2d(e, e->numa_perm, order.data(), sizeof(int32_t) * (size_t)n, e->stream));
    }
    // LoadAware weights beyond cpu / memory: the pods' extra estimates for k_eval2's LAX form (exact in fp64:
    // within the value bound), when at most KG_LAX extra resources are weighted
    e->lax_ok = false;
    if (e->consts.la_extra && (e->cfg.enabled_plugins & KG_PLUGIN_LOADAWARE)) {
        int32_t nx = 0, xs[KG_NUM_RES - 2];
        for (int x = 0; x < KG_NUM_RES - 2; x++)
            if (e->consts.la_wx[x] > 0) xs[nx++] = x;
        bool ok = nx <= KG_LAX;
        for (int32_t i = 0; i < n && ok; i++)
            for (int k = 0; k < nx; k++) ok = ok && kg_abs64(dev[(size_t)i].la_est_x[xs[k]]) < KG_VAL_LIMIT;
        if (ok) {
            std::vector<double> est((size_t)(n > 0 ? n : 1) * KG_LAX, 0.0);
            for (int32_t i = 0; i < n; i++)
                for (int k = 0; k < nx; k++) est[(size_t)i * KG_LAX + k] = -(double)dev[(size_t)i].la_est_x[xs[k]];
            if (e->hot_lax) HIP_TRY(e, hipFree(e->hot_lax));
            e->hot_lax = nullptr;
            HIP_TRY(e, hipMalloc(&e->hot_lax, sizeof(double) * est.size()));
            HIP_TRY(e, h2d(e, e->hot_lax, est.data(), sizeof(double) * est.size(), e->stream));
            e->lax_n = nx;
            for (int k = 0; k < nx; k++) e->lax_x[k] = xs[k];
            e->lax_ok = true;
        }
    }
    // distinct device rows (pod equivalence, matrix mode off the class path): on when they are at most 3/4 of the
    // batch
    e->eq_on = false;
    if (((e->cfg.enabled_plugins & KG_PLUGIN_NUMA) || (e->consts.la_extra && !e->lax_ok)) && n >= 64) {
        std::unordered_map<std::string, int32_t> seen;
        std::vector<int32_t> of((size_t)n), reps;
        for (int32_t i = 0; i < n; i++) {
            auto it = seen.emplace(std::string(reinterpret_cast<const char *>(&dev[(size_t)i]), sizeof(kg_pod_dev)),
                                   (int32_t)reps.size());
            if (it.second) reps.push_back(i);
            of[(size_t)i] = it.first->second;
        }
        const int32_t u = (int32_t)reps.size();
        if (4 * (int64_t)u <= 3 * (int64_t)n) {
            if (e->eq_pods) HIP_TRY(e, hipFree(e->eq_pods));
            if (e->eq_perm) HIP_TRY(e, hipFree(e->eq_perm));
            if (e->eq_of) HIP_TRY(e, hipFree(e->eq_of));
            e->eq_pods = nullptr;
            e->eq_perm = nullptr;
            e->eq_of = nullptr;
            HIP_TRY(e, hipMalloc(&e->eq_pods, sizeof(kg_pod_dev) * (size_t)u));
            HIP_TRY(e, hipMalloc(&e->eq_perm, sizeof(int32_t) * (size_t)u));
            HIP_TRY(e, hipMalloc(&e->eq_of, sizeof(int32_t) * (size_t)n));
            std::vector<kg_pod_dev> udev((size_t)u);
            for (int32_t k = 0; k < u; k++) udev[(size_t)k] = dev[(size_t)reps[(size_t)k]];
            HIP_TRY(e, h2d(e, e->eq_pods, udev.data(), sizeof(kg_pod_dev) * (size_t)u, e->stream));
            HIP_TRY(e, h2d(e, e->eq_of, of.data(), sizeof(int32_t) * (size_t)n, e->stream));
            {   // the distinct rows' hot rows (the batch's slot map) for the Fit + LoadAware pass over them
                const size_t hs = hot.size() / (size_t)n;
                std::vector<char> uh(hs * (size_t)u);
                for (int32_t k = 0; k < u; k++) memcpy(uh.data() + hs * (size_t)k, hot.data() + hs * (size_t)reps[(size_t)k], hs);
                if (e->eq_hot) HIP_TRY(e, hipFree(e->eq_hot));
                e->eq_hot = nullptr;
                HIP_TRY(e, hipMalloc(&e->eq_hot, uh.size()));
                HIP_TRY(e, h2d(e, e->eq_hot, uh.data(), uh.size(), e->stream));
            }
            e->eq_perm_on = (e->cfg.enabled_plugins & KG_PLUGIN_NUMA) && u > 64;
            if (e->eq_perm_on) {
                const std::vector<int32_t> order = numa_order(reps);
                HIP_TRY(e, h2d(e, e->eq_perm, order.data(), sizeof(int32_t) * (size_t)u, e->stream));
            }
            e->eq_n = u;
            e->eq_on = true;
        }
    }
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->nslot = nslot;
    for (int s = 0; s < 8; s++) e->slot_res[s] = slot_res[s];
    e->n_pods = n;
    e->max_pod_quota = max_quota;
    e->bm = bm;
    e->la_prod = la_prod;
    e->pow2 = pow2;
    e->pod_rows_h.assign(rows, rows + n);
    e->batch_bind = batch_bind;
    e->pod_may_bind.assign((size_t)n, 0);
    if (e->cfg.enabled_plugins & KG_PLUGIN_NUMA)
        for (int32_t i = 0; i < n; i++) {
            if (rows[i].flags & (KG_POD_NUMA_SKIP | KG_POD_NUMA_BIND_INVALID)) continue;
            e->pod_may_bind[i] = (uint8_t)(((rows[i].flags & KG_POD_NUMA_CPU_BIND) ? 1 : 0) |
                                           (rows[i].numa_request[KG_RES_CPU] != 0 && rows[i].numa_request[KG_RES_CPU] % 1000 == 0 ? 2 : 0));
        }
    cls_prepare(e);
    return KG_OK;
}

kg_status kg_eval(kg_engine *e, int64_t now_ns, const kg_eval_out *out) {
    kg_status st = check_engine(e);
    if (st) return st;
    st = bind_ready(e, false);
    if (st) return st;
    if (!out) return set_err(e, KG_ERR_INVALID_ARG, "null output");
    if (!e->plane_mem) return set_err(e, KG_ERR_STATE, "snapshot not initialised");
    if (e->eq_on && e->n_pods > 0) return eval_eq(e, now_ns, out);
    const int32_t P = e->n_pods;
    const int64_t T = tiles_total(e);
    const int64_t width = e->shard_end - e->shard_begin;
    const size_t mask_b = (size_t)P * (size_t)((width + 63) / 64) * 8;
    const size_t score_b = (size_t)P * (size_t)((width + 63) / 64 * 64) * 2;
    const size_t part_b = (size_t)P * (size_t)T * 4;
    const size_t top_b = (size_t)P * 8;
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    const bool dev = out->out_on_device != 0;
    // the hot kernel writes the mask and the scores together: stage whichever is not a device output
    const bool planes = out->mask || out->scores;
    const bool stage_mask = planes && (!dev || !out->mask);
    const bool stage_scores = planes && (!dev || !out->scores);
    const size_t numa_b = (size_t)P * (size_t)((width + 63) / 64 * 64);
    const bool numa_on = (e->consts.plugins & KG_PLUGIN_NUMA) != 0;
    e->ctr.eval_calls++;
    e->ctr.evals += (uint64_t)P * (uint64_t)width;
    e->ctr.out_bytes += (out->mask ? mask_b : 0) + (out->scores ? score_b : 0) + (out->top1 ? top_b : 0) +
                        (out->numa_scores ? numa_b : 0) + (out->rsv_scores ? numa_b : 0);
    const bool stage_numa = out->numa_scores && !dev;
    const bool stage_rsv = out->rsv_scores && !dev;
    size_t need = up(part_b) + up(top_b) + (stage_mask ? up(mask_b) : 0) + (stage_scores ? up(score_b) : 0) +
                  (stage_numa ? up(numa_b) : 0) + (stage_rsv ? up(numa_b) : 0);
    st = ensure_scratch(e, need + 256);
    if (st) return st;
    char *s = (char *)e->scratch;
    uint32_t *part = (uint32_t *)s;
    unsigned long long *top = (unsigned long long *)(s + up(part_b));
    char *q = s + up(part_b) + up(top_b);
    uint64_t *mask = nullptr;
    uint16_t *scores = nullptr;
    if (planes) {
        if (stage_mask) { mask = (uint64_t *)q; q += up(mask_b); }
        else mask = out->mask;
        if (stage_scores) { scores = (uint16_t *)q; q += up(score_b); }
        else scores = (uint16_t *)out->scores;
    }
    uint8_t *numa = nullptr;
    if (out->numa_scores) {
        if (stage_numa) { numa = (uint8_t *)q; q += up(numa_b); }
        else numa = out->numa_scores;
        if (!numa_on && numa_b) HIP_TRY(e, hipMemsetAsync(numa, 0, numa_b, e->stream));
    }
    uint8_t *rsvp = nullptr;
    if (out->rsv_scores) {
        if (stage_rsv) { rsvp = (uint8_t *)q; q += up(numa_b); }
        else rsvp = out->rsv_scores;
        if (numa_b) HIP_TRY(e, hipMemsetAsync(rsvp, 0, numa_b, e->stream));
    }
    // reservation nodes are evaluated whole on every shard (replicated slots: the preferred reservation
    // and NormalizeScore's max are global); planes are written for the shard's columns only
    const RsvArgs ra = rsv_args(e);
    st = quota_ready(e);
    if (st) return st;
    const bool gated = (ra.quota || ra.rsv) && P > 0;
    if (gated) {
        hipLaunchKernelGGL(k_pod_gate, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, e->stream, ra.quota, ra.quota_parent, e->pods, P,
                           e->gate);
        HIP_TRY(e, hipGetLastError());
    }
    HIP_TRY(e, hipMemsetAsync(part, 0, part_b, e->stream));
    st = launch_eval(e, now_ns, 0, P, mask, scores, part, true, numa_on ? numa : nullptr);
    if (st) return st;
    unsigned long long *tdst = out->top1 ? (dev ? (unsigned long long *)out->top1 : top) : nullptr;
    if (tdst && P > 0) {
        hipLaunchKernelGGL(k_top1, dim3((unsigned)((P + 3) / 4)), dim3(256), 0, e->stream, part, (int32_t)T, P, tdst);
        HIP_TRY(e, hipGetLastError());
    }
    const int32_t mask_words = (int32_t)((width + 63) / 64);
    const int64_t stride = (width + 63) / 64 * 64;
    if (gated) {  // plain nodes closed to pods failing the quota or requiring a reservation
        hipLaunchKernelGGL(k_quota_apply, dim3((unsigned)P), dim3(256), 0, e->stream, e->gate + P, P,
                           (unsigned long long *)mask, mask_words, tdst, (uint8_t *)nullptr, stride);
        HIP_TRY(e, hipGetLastError());
    }
    if (ra.rsv) {
        for (int32_t b = 0; b < P; b += KG_RSV_POD_CHUNK) {
            const int32_t n = P - b < KG_RSV_POD_CHUNK ? P - b : KG_RSV_POD_CHUNK;
            st = rsv_eval_chunk(e, now_ns, b, n, mask ? mask + (int64_t)b * mask_words : nullptr,
                                scores ? scores + (int64_t)b * stride : nullptr,
                                numa_on && numa ? numa + (int64_t)b * stride : nullptr, mask_words, stride);
            if (st) return st;
            hipLaunchKernelGGL(k_rsv_reduce, dim3((unsigned)n), dim3(256), 0, e->stream, e->consts, ra, n,
                               tdst ? tdst + b : nullptr, rsvp ? rsvp + (int64_t)b * stride : nullptr, e->shard_begin,
                               e->shard_end, stride);
            HIP_TRY(e, hipGetLastError());
        }
    }
    if (ra.quota && P > 0) {
        hipLaunchKernelGGL(k_quota_apply, dim3((unsigned)P), dim3(256), 0, e->stream, e->gate, P,
                           (unsigned long long *)mask, mask_words, tdst, rsvp, stride);
        HIP_TRY(e, hipGetLastError());
    }
    if (!dev) {
        if (out->top1 && P > 0) HIP_TRY(e, hipMemcpyAsync(out->top1, top, top_b, hipMemcpyDeviceToHost, e->stream));
        if (out->mask && P > 0) HIP_TRY(e, hipMemcpyAsync(out->mask, mask, mask_b, hipMemcpyDeviceToHost, e->stream));
        if (out->scores && P > 0) HIP_TRY(e, hipMemcpyAsync(out->scores, scores, score_b, hipMemcpyDeviceToHost, e->stream));
        if (out->numa_scores && P > 0) HIP_TRY(e, hipMemcpyAsync(out->numa_scores, numa, numa_b, hipMemcpyDeviceToHost, e->stream));
        if (out->rsv_scores && P > 0) HIP_TRY(e, hipMemcpyAsync(out->rsv_scores, rsvp, numa_b, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(e, hipStreamSynchronize(e->stream));
    }
    return KG_OK;
}

}  // extern "C"

namespace {

// Matrix mode over the distinct rows of the batch (kg_engine::eq_on): the batch is swapped for its distinct rows,
// evaluated by kg_eval into device buffers, and every output row is copied to each pod of its distinct row.
kg_status eval_eq(kg_engine *e, int64_t now_ns, const kg_eval_out *out) {
    const int32_t P = e->n_pods, U = e->eq_n;
    const int64_t width = e->shard_end - e->shard_begin;
    const int64_t words = (width + 63) / 64, stride = words * 64;
    const size_t rb[5] = {(size_t)words * 8, (size_t)stride * 2, 8, (size_t)stride, (size_t)stride};   // mask scores top1 numa rsv
    void *const want[5] = {out->mask, out->scores, out->top1, out->numa_scores, out->rsv_scores};
    const bool dev = out->out_on_device != 0;
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    size_t need = 0, off_c[5] = {}, off_s[5] = {};
    for (int k = 0; k < 5; k++)
        if (want[k]) { off_c[k] = need; need += up(rb[k] * (size_t)U); }
    for (int k = 0; k < 5; k++)
        if (want[k] && !dev) { off_s[k] = need; need += up(rb[k] * (size_t)P); }
    if (need > e->eq_mem_bytes) {
        HIP_TRY(e, hipStreamSynchronize(e->stream));
        if (e->eq_mem) HIP_TRY(e, hipFree(e->eq_mem));
        e->eq_mem = nullptr;
        e->eq_mem_bytes = 0;
        HIP_TRY(e, hipMalloc(&e->eq_mem, need));
        e->eq_mem_bytes = need;
    }
    char *m = (char *)e->eq_mem;
    kg_eval_out cout;
    memset(&cout, 0, sizeof(cout));
    void **cptr[5] = {(void **)&cout.mask, (void **)&cout.scores, (void **)&cout.top1, (void **)&cout.numa_scores,
                      (void **)&cout.rsv_scores};
    for (int k = 0; k < 5; k++)
        if (want[k]) *cptr[k] = m + off_c[k];
    cout.out_on_device = 1;
    // the distinct batch in place of the batch for the inner call (restored on every path)
    const kg_counters ctr0 = e->ctr;
    std::swap(e->pods, e->eq_pods);
    std::swap(e->hot, e->eq_hot);
    std::swap(e->numa_perm, e->eq_perm);
    std::swap(e->numa_perm_on, e->eq_perm_on);
    e->n_pods = U;
    e->eq_on = false;
    e->reps_in = true;
    kg_status st = kg_eval(e, now_ns, &cout);
    e->reps_in = false;
    e->eq_on = true;
    e->n_pods = P;
    std::swap(e->pods, e->eq_pods);
    std::swap(e->hot, e->eq_hot);
    std::swap(e->numa_perm, e->eq_perm);
    std::swap(e->numa_perm_on, e->eq_perm_on);
    e->ctr = ctr0;   // counted as the whole batch below
    if (st) return st;
    e->ctr.eval_calls++;
    e->ctr.evals += (uint64_t)P * (uint64_t)width;
    for (int k = 0; k < 5; k++)
        if (want[k]) e->ctr.out_bytes += rb[k] * (size_t)P;
    for (int k = 0; k < 5; k++) {
        if (!want[k]) continue;
        char *dst = dev ? (char *)want[k] : m + off_s[k];
        const int64_t nvec = (int64_t)rb[k] / 8;
        const unsigned gx = (unsigned)std::min<int64_t>((nvec + 511) / 512, 1024);
        const dim3 grid(gx > 0 ? gx : 1, (unsigned)std::min<int32_t>(P, 65535));
        if (rb[k] % 16 == 0)
            hipLaunchKernelGGL(k_eq_rows<16>, grid, dim3(256), 0, e->stream, e->eq_of, P, (const char *)(m + off_c[k]), dst,
                               (int64_t)rb[k]);
        else
            hipLaunchKernelGGL(k_eq_rows<8>, grid, dim3(256), 0, e->stream, e->eq_of, P, (const char *)(m + off_c[k]), dst,
                               (int64_t)rb[k]);
        HIP_TRY(e, hipGetLastError());
    }
    if (!dev) {
        for (int k = 0; k < 5; k++)
            if (want[k]) HIP_TRY(e, hipMemcpyAsync(want[k], m + off_s[k], rb[k] * (size_t)P, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(e, hipStreamSynchronize(e->stream));
    }
    return KG_OK;
}

kg_status chunk_eval(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n, uint32_t *partial_dev) {
    if (pod_begin < 0 || n < 0 || pod_begin + (int64_t)n > e->n_pods || (n > 0 && !partial_dev))
        return set_err(e, KG_ERR_RANGE, "bad chunk");
    e->ctr.eval_calls++;
    e->ctr.evals += (uint64_t)n * (uint64_t)(e->shard_end - e->shard_begin);
    // the top-k kernel writes every slot of every tile of its shard; the NUMA kernel merges with atomics
    // and a shard leaves the other ranks' tiles to the merge: those start from zeros
    const bool whole = e->shard_begin == 0 && e->shard_end == e->n_nodes;
    if (((e->consts.plugins & KG_PLUGIN_NUMA) && n > e->numa_chunk_pods) || !whole)
        HIP_TRY(e, hipMemsetAsync(partial_dev, 0, (size_t)n * (size_t)tiles_total(e) * 4 * KG_PARTIAL_SLOTS, e->stream));
    kg_status st = launch_eval(e, now_ns, pod_begin, n, nullptr, nullptr, partial_dev, false, nullptr, true);
    if (st) return st;
    // reservation nodes: entries of every reservation node (the snapshot is replicated across
    // ranks in the multi-GPU placement, so each rank holds all of them), rows 0..n of E / O
    if (rsv_args(e).rsv) {
        if (n > KG_RSV_POD_CHUNK) return set_err(e, KG_ERR_RANGE, "chunk larger than the reservation entry buffer");
        return rsv_eval_chunk(e, now_ns, pod_begin, n, nullptr, nullptr, nullptr, 0, 0, true);
    }
    return KG_OK;
}

// defer_last: the chunk's last pod is only selected (out_node / out_score); its Reserve is host_reserve's
kg_status chunk_resolve(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n, const uint32_t *partial_dev,
                        int32_t *out_node_dev, int64_t *out_score_dev, bool defer_last,
                        const int32_t *prev_nodes_dev = nullptr, int32_t n_prev = 0,
                        unsigned long long *pvkeys = nullptr) {
    if (pod_begin < 0 || n < 0 || n > KG_MAX_CHUNK || pod_begin + (int64_t)n > e->n_pods)
        return set_err(e, KG_ERR_RANGE, "bad chunk");
    if (n == 0) return KG_OK;
    kg_status st = quota_ready(e);
    if (st) return st;
    e->ctr.resolved += (uint64_t)n;
    RsvArgs ra = rsv_args(e);
    if (ra.rsv) {  // this chunk's entries were written by kg_place_chunk_eval from row 0
        if (n > KG_RSV_POD_CHUNK) return set_err(e, KG_ERR_RANGE, "chunk larger than the reservation entry buffer");
    }
    st = slow_refresh(e);
    if (st) return st;
    const bool numa = (e->consts.plugins & KG_PLUGIN_NUMA) != 0;
    // NodeNUMAResource: the previous chunk's nodes keyed for every pod at once (pvkeys: n × n_prev, the caller's)
    const bool pv = numa && pvkeys && n_prev > 0 && !ra.rsv && n <= KG_NUMA_CHUNK_PODS && n_prev <= KG_NUMA_CHUNK_PODS;
    if (pv) {
        hipLaunchKernelGGL(k_prev_keys, dim3((unsigned)(n * n_prev)), dim3(64), 0, e->stream, e->consts, e->pl,
                           e->pods + pod_begin, n, prev_nodes_dev, n_prev, e->n_nodes, now_ns, pvkeys);
        HIP_TRY(e, hipGetLastError());
    }
    auto *kres = ra.rsv ? (numa ? k_resolve<true, true> : k_resolve<true, false>)
                        : (numa ? k_resolve<false, true> : k_resolve<false, false>);
    hipLaunchKernelGGL(kres, dim3(1), dim3(KG_RESOLVE_THREADS), 0, e->stream,
                       e->consts, e->pl, e->pods, pod_begin, n,
                       partial_dev, (int32_t)tiles_total(e), e->n_nodes, now_ns, out_node_dev, out_score_dev, ra,
                       numa && n > e->numa_chunk_pods ? 1 : KG_PARTIAL_SLOTS, e->slow_list, e->slow_count,
                       numa ? 0 : 1,   // the NUMA chunk kernels list slow nodes themselves (exact pair path)
                       defer_last ? 1 : 0, prev_nodes_dev, n_prev, pv ? pvkeys : nullptr);
    HIP_TRY(e, hipGetLastError());
    e->generation++;   // the resolve commits the chunk's winners to the snapshot
    return KG_OK;
}

// Reserve of `pod` on `node` with the cpuset part on the host (NodeNUMAResource.Reserve, plugin.go:375-419):
// when the pod binds a cpuset there, resourceManager.Allocate runs on the pre-Reserve row and the node's CPU
// table (kg_cpuset_allocate — the hint's zones through the kernels' own per-pair code, then the CPU
// accumulator); if it fails the Reserve fails and nothing changes (*failed = true; the scheduler's Unreserve
// + ForgetPod).  Otherwise the device commits every plugin's Reserve (k_commit_one: zone allocations of the
// same hint, AssumePod, LoadAware, ElasticQuota) and the host writes the taken CPUs into the table and the
// node's cpuset counts into its row.
// host_reserve's upload area at the head of the scratch buffer: the row, then (256-B aligned) its node index;
// kg_place keeps its partial keys after it
constexpr size_t kHostRowOff = 0, kHostNodeOff = (sizeof(kg_node_row) + 255) / 256 * 256;
constexpr size_t kHostReserveHead = kHostNodeOff + 256;
static_assert(kHostNodeOff >= kHostRowOff + sizeof(kg_node_row) && kHostNodeOff + 4 <= kHostReserveHead,
              "the row and its node index fit the head");
kg_status host_reserve(kg_engine *e, int32_t pod, int32_t node, bool *failed) {
    *failed = false;
    kg_node_row row;
    HIP_TRY(e, hipMemcpyAsync(&row, e->pl.rows + node, sizeof(row), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    kg_pod_dev pd;
    kg_pod_dev_from_row(e->cfg, e->pod_rows_h[(size_t)pod], pd);
    int required, take;
    const bool bind = (e->consts.plugins & KG_PLUGIN_NUMA) && kg_numa_binds(row, pd, required, take);
    std::vector<uint8_t> taken;
    kg_engine::CpuTable *tab = nullptr;
    if (bind) {
        auto it = e->cpu_tab.find(node);
        if (it == e->cpu_tab.end())
            return set_err(e, KG_ERR_STATE, "node %d: cpuset Reserve needs the node's CPUs (kg_cpus_set)", node);
        tab = &it->second;
        const int32_t nc = (int32_t)tab->cpus.size();
        taken.assign((size_t)nc, 0);
        if (kg_cpuset_allocate(e->consts, row, pd, required, take, tab->cpus.data(), nc, tab->max_ref, tab->strategy,
                               taken.data()) != 0) {
            *failed = true;
            return KG_OK;
        }
    }
    hipLaunchKernelGGL(k_commit_one, dim3(1), dim3(1), 0, e->stream, e->consts, e->pl, e->pods, pod, node, rsv_args(e));
    HIP_TRY(e, hipGetLastError());
    if (bind) {
        const int32_t nc = (int32_t)tab->cpus.size();
        kg_cpuset_apply(pd, tab->cpus.data(), nc, taken.data());
        HIP_TRY(e, hipMemcpyAsync(&row, e->pl.rows + node, sizeof(row), hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(e, hipStreamSynchronize(e->stream));
        kg_cpuset_row_fields(row, tab->cpus.data(), nc, tab->max_ref);
        // the row back, its planes re-derived (k_upsert)
        kg_status st = ensure_scratch(e, kHostReserveHead);
        if (st) return st;
        char *sc = (char *)e->scratch;
        HIP_TRY(e, h2d(e, sc + kHostRowOff, &row, sizeof(row), e->stream));
        HIP_TRY(e, h2d(e, sc + kHostNodeOff, &node, 4, e->stream));
        hipLaunchKernelGGL(k_upsert, dim3(1), dim3(256), 0, e->stream, e->consts, e->pl, (const kg_node_row *)(sc + kHostRowOff),
                           (const int32_t *)(sc + kHostNodeOff), 1);
        HIP_TRY(e, hipGetLastError());
    }
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->slow_valid = false;   // the commit may move the node off (or onto) the fast paths
    e->generation++;
    return KG_OK;
}

}  // namespace

extern "C" {

kg_status kg_place_chunk_eval(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n, uint32_t *partial_dev) {
    kg_status st = check_engine(e);
    if (st) return st;
    st = bind_ready(e, true);
    if (st) return st;
    hipStream_t main_s = e->stream;
    if (e->eval_stream) e->stream = e->eval_stream;   // chunk_eval launches on e->stream
    st = chunk_eval(e, now_ns, pod_begin, n, partial_dev);
    e->stream = main_s;
    if (st) return st;
    if (e->eval_stream) {   // the resolve that reads these partials waits for them (eval_join)
        int k = 0;
        while (k < kg_engine::kEvalEvents && e->ev_eval_buf[k] != partial_dev) k++;
        if (k == kg_engine::kEvalEvents) {   // a new buffer: the least recently assigned slot
            k = e->ev_eval_next;
            e->ev_eval_next = (k + 1) % kg_engine::kEvalEvents;
            e->ev_eval_buf[k] = partial_dev;
        }
        if (!e->ev_eval[k]) HIP_TRY(e, hipEventCreateWithFlags(&e->ev_eval[k], hipEventDisableTiming));
        HIP_TRY(e, hipEventRecord(e->ev_eval[k], e->eval_stream));
    }
    return KG_OK;
}

}  // extern "C"

namespace {
// a chunk resolve after kg_place_chunk_eval on the eval stream: the engine stream waits for the evaluation that wrote
// partial_dev (its latest record), not for whatever the caller enqueued on the eval stream after it — a caller that
// enqueues eval(i + 1) before resolve(i) keeps its overlap.  Partials no evaluation wrote (the caller's own) join
// nothing.
kg_status eval_join(kg_engine *e, const void *partial_dev) {
    if (!e->eval_stream) return KG_OK;
    for (int k = 0; k < kg_engine::kEvalEvents; k++)
        if (e->ev_eval_buf[k] == partial_dev && e->ev_eval[k]) HIP_TRY(e, hipStreamWaitEvent(e->stream, e->ev_eval[k], 0));
    return KG_OK;
}
}  // namespace

extern "C" {

#ifdef KG_RESOLVE_TIMING
int32_t kg_debug_resolve_times(unsigned long long *out, int32_t n_pods) {
    int pods = 0;
    if (hipMemcpyFromSymbol(&pods, HIP_SYMBOL(g_rtimes_pod), sizeof(int)) != hipSuccess) return -1;
    if (pods > n_pods) pods = n_pods;
    if (pods > 65536) pods = 65536;
    if (pods > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rtimes), sizeof(unsigned long long) * 16 * (size_t)pods) != hipSuccess) return -1;
    return pods;
}
#endif

kg_status kg_set_forms(kg_engine *e, uint32_t forms) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (forms & ~(KG_FORM_PLACE_PIPELINE | KG_FORM_PLACE_SEQUENTIAL | KG_FORM_NUMA_QUEUED | KG_FORM_NUMA_CHUNK_TILE |
                  KG_FORM_NUMA_NO_CACHE | KG_FORM_NUMA_FUSED))
        return set_err(e, KG_ERR_INVALID_ARG, "unknown kernel form bits 0x%x", forms);
    if ((forms & KG_FORM_PLACE_PIPELINE) && (forms & KG_FORM_PLACE_SEQUENTIAL))
        return set_err(e, KG_ERR_INVALID_ARG, "pipelined and sequential placement together");
    e->forms = forms;
    e->numa_chunk_pods = (forms & KG_FORM_NUMA_CHUNK_TILE) ? 0 : KG_NUMA_CHUNK_PODS;
    return KG_OK;
}

kg_status kg_set_eval_stream(kg_engine *e, void *s) {
    kg_status st = check_engine(e);
    if (st) return st;
    e->eval_stream = (hipStream_t)s;
    return KG_OK;
}

kg_status kg_place_chunk_resolve_prev(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n,
                                      const uint32_t *partial_dev, int32_t *out_node_dev, int64_t *out_score_dev,
                                      const int32_t *prev_nodes_dev, int32_t n_prev) {
    kg_status st = check_engine(e);
    if (st) return st;
    st = bind_ready(e, true);
    if (st) return st;
    if (n_prev < 0 || n_prev > KG_MAX_CHUNK || (n_prev > 0 && !prev_nodes_dev))
        return set_err(e, KG_ERR_RANGE, "bad previous-chunk node list");
    if (n_prev > 0 && rsv_args(e).rsv)
        return set_err(e, KG_ERR_UNSUPPORTED, "pipelined resolve with reservations (chunk_eval writes their entries)");
    st = eval_join(e, partial_dev);
    if (st) return st;
    return chunk_resolve(e, now_ns, pod_begin, n, partial_dev, out_node_dev, out_score_dev, false, prev_nodes_dev, n_prev);
}

kg_status kg_place_chunk_resolve(kg_engine *e, int64_t now_ns, int32_t pod_begin, int32_t n, const uint32_t *partial_dev,
                                 int32_t *out_node_dev, int64_t *out_score_dev) {
    kg_status st = check_engine(e);
    if (st) return st;
    st = bind_ready(e, true);
    if (st) return st;
    st = eval_join(e, partial_dev);
    if (st) return st;
    return chunk_resolve(e, now_ns, pod_begin, n, partial_dev, out_node_dev, out_score_dev, false);
}

}  // extern "C"

namespace {

// Pipelined placement: chunk i + 1's evaluation (second stream) runs while chunk i resolves.  It starts once
// chunk i − 1's resolve is done, so the snapshot it reads differs from chunk i + 1's true pre-state only by
// chunk i's commits — and those nodes go to chunk i + 1's resolve as touched (prev_nodes): their keys are
// skipped and they are re-scored exactly, while every other node's key is exact (its planes did not change).
// Partial buffers alternate; a buffer is rewritten only after the resolve that read it (eval i + 2 waits for
// resolve i).  Not used with reservations (one entry buffer) or cpuset pods (host Reserve between chunks).
kg_status merge_partials(kg_engine *e, uint32_t *part, int32_t n, hipStream_t s, bool failed = false);
kg_status merge_verdict(kg_engine *e, const uint32_t *part, int32_t n);
kg_status comm_agree(kg_engine *e, kg_status mine);

// the NodeNUMAResource cache of the batch's distinct rows over the shard (kg_engine::ncache), on the engine stream:
// matrix mode (k_eval_numa2) over eq_pods into the buffer's tail, then k_ncache_init
kg_status ncache_build(kg_engine *e, int64_t now_ns) {
    const int32_t U = e->eq_n;
    const int64_t width = e->shard_end - e->shard_begin;
    const int64_t words = (width + 63) / 64, stride = words * 64;
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t cache_b = up((size_t)U * (size_t)stride), mask_b = up((size_t)U * (size_t)words * 8),
                 score_b = up((size_t)U * (size_t)stride * 4), numa_b = up((size_t)U * (size_t)stride),
                 part_b = up((size_t)U * (size_t)tiles_total(e) * 4);
    const size_t need = cache_b + mask_b + score_b + numa_b + part_b;
    if (need > e->ncache_bytes) {
        HIP_TRY(e, hipStreamSynchronize(e->stream));
        if (e->ncache_mem) HIP_TRY(e, hipFree(e->ncache_mem));
        e->ncache_mem = nullptr;
        e->ncache_bytes = 0;
        HIP_TRY(e, hipMalloc(&e->ncache_mem, need));
        e->ncache_bytes = need;
    }
    char *m = (char *)e->ncache_mem;
    uint8_t *cache = (uint8_t *)m;
    unsigned long long *mask = (unsigned long long *)(m + cache_b);
    uint16_t *scores = (uint16_t *)(m + cache_b + mask_b);
    uint8_t *numa = (uint8_t *)(m + cache_b + mask_b + score_b);
    uint32_t *part = (uint32_t *)(m + cache_b + mask_b + score_b + numa_b);
    HIP_TRY(e, hipMemsetAsync(part, 0, part_b, e->stream));
    // the distinct batch in place of the batch (as eval_eq), restored on every path
    const kg_counters ctr0 = e->ctr;
    const int32_t P = e->n_pods;
    std::swap(e->pods, e->eq_pods);
    std::swap(e->hot, e->eq_hot);
    std::swap(e->numa_perm, e->eq_perm);
    std::swap(e->numa_perm_on, e->eq_perm_on);
    e->n_pods = U;
    e->reps_in = true;
    kg_status st = launch_eval(e, now_ns, 0, U, (uint64_t *)mask, scores, part, false, numa);
    e->reps_in = false;
    e->n_pods = P;
    std::swap(e->pods, e->eq_pods);
    std::swap(e->hot, e->eq_hot);
    std::swap(e->numa_perm, e->eq_perm);
    std::swap(e->numa_perm_on, e->eq_perm_on);
    e->ctr = ctr0;
    if (st) return st;
    const int64_t total = (int64_t)U * stride;
    if (total > 0) {   // (an empty shard has no cache columns)
        hipLaunchKernelGGL(k_ncache_init, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, e->stream, mask, numa, U,
                           (int32_t)words, stride, width, cache);
        HIP_TRY(e, hipGetLastError());
    }
    e->ncache = cache;
    e->ncache_stride = stride;
    return KG_OK;
}

// chunk i − 2's committed nodes re-evaluated in the cache, on stream s (after that chunk's resolve)
kg_status ncache_refresh(kg_engine *e, int64_t now_ns, const int32_t *nodes, int32_t n, hipStream_t s) {
    const int64_t total = (int64_t)e->eq_n * n;
    if (total <= 0) return KG_OK;
    if (n > KG_NUMA_CHUNK_PODS) return set_err(e, KG_ERR_RANGE, "cache refresh of more than %d nodes", KG_NUMA_CHUNK_PODS);
    hipLaunchKernelGGL(k_ncache_refresh, dim3((unsigned)total), dim3(64), 0, s, e->consts, e->pl,
                       e->eq_pods, e->eq_n, nodes, n, now_ns, e->ncache, e->ncache_stride, e->shard_begin, e->shard_end);
    HIP_TRY(e, hipGetLastError());
    return KG_OK;
}

kg_status place_pipelined(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score, int32_t chunk,
                          bool merge = false) {
    const int32_t P = e->n_pods;
    const size_t part_b = (size_t)chunk * (size_t)tiles_total(e) * 4 * KG_PARTIAL_SLOTS + 4;   // + the status word
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t pvk_b = up((size_t)chunk * (size_t)chunk * 8);
    hipStream_t main_s = e->stream;
    // NodeNUMAResource over a batch of repeated rows: the chunks read the distinct rows' cached outcomes (built on the
    // engine stream before the fork below; ncache_live off again on every return)
    struct NcacheScope {
        kg_engine *e;
        ~NcacheScope() { e->ncache_live = false; }
    } ncache_scope{e};
    // this rank's setup (scratch, streams, events, the outcome cache); sharded (merge): the ranks agree on it before
    // the first collective of the loop
    auto setup = [&]() -> kg_status {
        kg_status st = ensure_scratch(e, 2 * up(part_b) + up((size_t)P * 4) + up((size_t)P * 8) + pvk_b + 256);
        if (st) return st;
        if (!e->stream2) {
            HIP_TRY(e, hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking));
            HIP_TRY(e, hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
            HIP_TRY(e, hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
        }
        if (!e->ev_res[0])
            for (int k = 0; k < 3; k++) HIP_TRY(e, hipEventCreateWithFlags(&e->ev_res[k], hipEventDisableTiming));
        // (the refresh re-evaluates U pairs per committed node where a chunk evaluation takes one per node: worth it
        // while the distinct rows are a fraction of the shard's nodes; the build's matrix outputs stay within 8 GiB)
        const int64_t ncache_width = e->shard_end - e->shard_begin;
        if ((e->consts.plugins & KG_PLUGIN_NUMA) && e->eq_on && !e->consts.numa_bz && !(e->forms & KG_FORM_NUMA_NO_CACHE) &&
            P > 2 * chunk && chunk <= e->numa_chunk_pods && 4 * (int64_t)e->eq_n <= ncache_width &&
            (int64_t)e->eq_n * ((ncache_width + 63) / 64 * 64) * 7 <= (int64_t)8 << 30) {
            st = ncache_build(e, now_ns);
            if (st) return st;
            e->ncache_live = true;
        }
        return KG_OK;
    };
    kg_status st = setup();
    if (merge) st = comm_agree(e, st);
    if (st) return st;
    char *s = (char *)e->scratch;
    uint32_t *part[2] = {(uint32_t *)s, (uint32_t *)(s + up(part_b))};
    int32_t *dnode = (int32_t *)(s + 2 * up(part_b));
    int64_t *dscore = (int64_t *)(s + 2 * up(part_b) + up((size_t)P * 4));
    unsigned long long *pvkeys = (unsigned long long *)(s + 2 * up(part_b) + up((size_t)P * 4) + up((size_t)P * 8));
    hipStream_t eval_s = e->stream2;
    HIP_TRY(e, hipEventRecord(e->ev_fork, main_s));   // the eval stream starts after everything queued so far
    HIP_TRY(e, hipStreamWaitEvent(eval_s, e->ev_fork, 0));
    // an error return leaves no evaluation in flight behind the engine stream (it may write the scratch buffer)
    auto fail = [&](kg_status code) {
        (void)hipEventRecord(e->ev_join, eval_s);
        (void)hipStreamWaitEvent(main_s, e->ev_join, 0);
        if (merge) e->stale = true;   // the replicas stopped at different chunks
        return code;
    };
    // sharded: a step of this rank that fails (not the collective itself) turns the rest of the loop into merges of
    // zero keys flagged as failed, so that no peer waits in a collective this rank never issues; every rank then
    // returns an error (this one its own, the others KG_ERR_STATE from the last chunk's status word)
    kg_status local = KG_OK;
    int32_t prev_b = 0, prev_n = 0, last_n = 0;
    int32_t i = 0;
    for (int32_t b = 0; b < P; b += chunk, i++) {
        const int32_t n = P - b < chunk ? P - b : chunk;
        last_n = n;
        if (i >= 2) HIP_TRY(e, hipStreamWaitEvent(eval_s, e->ev_res[(i - 2) % 3], 0));
        if (!local && i >= 2 && e->ncache_live) {   // chunk i − 2 (full-size) resolved: its nodes' cache entries re-evaluated
            st = ncache_refresh(e, now_ns, dnode + (b - 2 * chunk), chunk, eval_s);
            if (st) local = st;
        }
        if (!local) {
            e->stream = eval_s;   // chunk_eval launches on e->stream
            st = chunk_eval(e, now_ns, b, n, part[i & 1]);
            e->stream = main_s;
            if (st) local = st;
        }
        if (local && !merge) return fail(local);
        if (merge) {   // the shards' partials merged beside the resolve (kg_place_sharded)
            st = merge_partials(e, part[i & 1], n, eval_s, local != KG_OK);
            if (st) return fail(st);
        }
        if (local) continue;
        HIP_TRY(e, hipEventRecord(e->ev_join, eval_s));
        HIP_TRY(e, hipStreamWaitEvent(main_s, e->ev_join, 0));
        st = chunk_resolve(e, now_ns, b, n, part[i & 1], dnode + b, dscore + b, false, i ? dnode + prev_b : nullptr,
                           i ? prev_n : 0, pvkeys);
        if (st) {
            if (!merge) return fail(st);
            local = st;
            continue;
        }
        HIP_TRY(e, hipEventRecord(e->ev_res[i % 3], main_s));
        prev_b = b;
        prev_n = n;
    }
    if (local) {
        (void)fail(local);
        (void)hipStreamSynchronize(eval_s);
        return local;
    }
    HIP_TRY(e, hipMemcpyAsync(out_node, dnode, (size_t)P * 4, hipMemcpyDeviceToHost, main_s));
    HIP_TRY(e, hipMemcpyAsync(out_score, dscore, (size_t)P * 8, hipMemcpyDeviceToHost, main_s));
    HIP_TRY(e, hipStreamSynchronize(main_s));
    HIP_TRY(e, hipStreamSynchronize(eval_s));
    if (merge && i > 0) return merge_verdict(e, part[(i - 1) & 1], last_n);
    return KG_OK;
}

}  // namespace

extern "C" {

kg_status place_impl(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score);
kg_status place_loop(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score, bool sharded);

}  // extern "C"

namespace {
// the engine's communicator (either kind) released
void comm_drop(kg_engine *e) {
    if (e->comm) (void)rccl().comm_destroy(e->comm);
    e->comm = nullptr;
    if (e->shm) kg_shm_comm_close(e->shm);
    e->shm = nullptr;
    if (e->shm_stage) (void)hipHostFree(e->shm_stage);
    e->shm_stage = nullptr;
    e->comm_world = 0;
}
}  // namespace

extern "C" {

kg_status kg_comm_init_loopback(kg_engine *e, int32_t rank, int32_t world, const char *name) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (!name || world < 1 || rank < 0 || rank >= world) return set_err(e, KG_ERR_INVALID_ARG, "bad rank / world / name");
    if (!e->plane_mem) return set_err(e, KG_ERR_STATE, "kg_comm_init_loopback sizes its slots from the snapshot: load it first");
    comm_drop(e);
    // one slot holds the largest merge: a chunk's partial keys + the status word (merge_partials)
    const size_t slot = ((size_t)KG_MAX_CHUNK * (size_t)tiles_total(e) * KG_PARTIAL_SLOTS + 1) * 4;
    std::string err;
    kg_shm_comm *c = kg_shm_comm_open(name, rank, world, slot, 120.0, err);
    if (!c) return set_err(e, KG_ERR_STATE, "%s", err.c_str());
    if (hipHostMalloc((void **)&e->shm_stage, slot, hipHostMallocDefault) != hipSuccess) {
        kg_shm_comm_abort(c);   // the peers' next wait fails instead of hanging
        kg_shm_comm_close(c);
        e->shm_stage = nullptr;
        return set_err(e, KG_ERR_STATE, "hipHostMalloc(%zu) for the loopback staging buffer failed", slot);
    }
    e->shm = c;
    e->comm_rank = rank;
    e->comm_world = world;
    return KG_OK;
}

int32_t kg_comm_kind(const kg_engine *e) {
    if (!e) return KG_COMM_NONE;
    return e->comm ? KG_COMM_RCCL : e->shm ? KG_COMM_LOOPBACK : KG_COMM_NONE;
}

kg_status kg_comm_unique_id(void *out) {
    if (!out) return KG_ERR_INVALID_ARG;
    Rccl &r = rccl();
    if (!r.h) return KG_ERR_UNSUPPORTED;
    ncclUniqueId id;
    if (r.get_unique_id(&id) != ncclSuccess) return KG_ERR_HIP;
    memcpy(out, &id, sizeof(id));
    return KG_OK;
}

kg_status kg_comm_init(kg_engine *e, int32_t rank, int32_t world, const void *unique_id) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (!unique_id || world < 1 || rank < 0 || rank >= world) return set_err(e, KG_ERR_INVALID_ARG, "bad rank / world");
    Rccl &r = rccl();
    if (!r.h) return set_err(e, KG_ERR_UNSUPPORTED, "librccl not found");
    comm_drop(e);
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    const ncclResult_t res = r.comm_init_rank(&e->comm, world, id, rank);
    if (res != ncclSuccess) {
        e->comm = nullptr;
        return set_err(e, KG_ERR_HIP, "ncclCommInitRank: %s", r.error_string(res));
    }
    e->comm_rank = rank;
    e->comm_world = world;
    return KG_OK;
}

kg_status kg_place_sharded(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score) {
    const uint64_t resolved0 = e ? e->ctr.resolved : 0;
    kg_status st = check_engine(e);
    if (st) return st;
    if (!out_node || !out_score) return set_err(e, KG_ERR_INVALID_ARG, "null outputs");
    if (!e->plane_mem) return set_err(e, KG_ERR_STATE, "snapshot not initialised");
    if (!e->comm && !e->shm) return set_err(e, KG_ERR_STATE, "kg_place_sharded needs kg_comm_init or kg_comm_init_loopback");
    st = place_loop(e, now_ns, out_node, out_score, true);
    if (st == KG_OK) st = bounds_verdict(e);
    if (st == KG_OK) {
        e->ctr.resolved = resolved0 + (uint64_t)e->n_pods;
        for (int32_t p = 0; p < e->n_pods; p++) e->ctr.placed += out_node[p] >= 0 ? 1u : 0u;
    }
    return st;
}

kg_status kg_place(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score) {
    const uint64_t resolved0 = e ? e->ctr.resolved : 0;
    kg_status st = place_impl(e, now_ns, out_node, out_score);
    if (st == KG_OK) st = bounds_verdict(e);
    if (st == KG_OK) {
        e->ctr.resolved = resolved0 + (uint64_t)e->n_pods;   // (the chunk resolves inside counted the same pods)
        for (int32_t p = 0; p < e->n_pods; p++) e->ctr.placed += out_node[p] >= 0 ? 1u : 0u;
    }
    return st;
}

kg_status place_loop(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score, bool sharded);

kg_status place_impl(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (!out_node || !out_score) return set_err(e, KG_ERR_INVALID_ARG, "null outputs");
    if (!e->plane_mem) return set_err(e, KG_ERR_STATE, "snapshot not initialised");
    if (e->shard_begin != 0 || e->shard_end != e->n_nodes)
        return set_err(e, KG_ERR_STATE, "kg_place runs on the whole snapshot; use kg_place_sharded for shards");
    return place_loop(e, now_ns, out_node, out_score, false);
}

}  // extern "C"

namespace {
// dev[0..count) := max over the ranks, in place, on stream s: ncclAllReduce on the RCCL communicator; through the host
// shared-memory segment on the loopback one (device → pinned staging, the exchange, back; synchronous on s)
kg_status comm_allreduce_max(kg_engine *e, uint32_t *dev, size_t count, hipStream_t s) {
    if (e->comm) {
        const ncclResult_t r = rccl().all_reduce(dev, dev, count, ncclUint32, ncclMax, e->comm, s);
        if (r != ncclSuccess) return set_err(e, KG_ERR_HIP, "ncclAllReduce: %s", rccl().error_string(r));
        return KG_OK;
    }
    if (!e->shm) return set_err(e, KG_ERR_STATE, "no communicator");
    if (count * 4 > kg_shm_comm_slot_bytes(e->shm)) return set_err(e, KG_ERR_RANGE, "merge larger than the loopback slot");
    HIP_TRY(e, hipMemcpyAsync(e->shm_stage, dev, count * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(e, hipStreamSynchronize(s));
    std::string err;
    if (!kg_shm_comm_allreduce_max_u32(e->shm, e->shm_stage, count, err)) return set_err(e, KG_ERR_STATE, "%s", err.c_str());
    HIP_TRY(e, hipMemcpyAsync(dev, e->shm_stage, count * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(e, hipStreamSynchronize(s));
    return KG_OK;
}

// the partial-key buffer of a chunk carries one status word after its n rows: 0 from a healthy rank, 1 from a rank
// whose own steps failed (it keeps joining the merges with zero keys so that no peer blocks in a collective), merged
// by the same max — a rank learns from the last chunk's word that a peer failed
size_t merge_count(const kg_engine *e, int32_t n) { return (size_t)n * (size_t)tiles_total(e) * KG_PARTIAL_SLOTS; }

// every rank's partial keys of a chunk merged in place (max over ranks: a tile's slots come from one rank, the
// others hold zeros), on stream s; failed: this rank's step failed (its keys zeroed, the status word set)
kg_status merge_partials(kg_engine *e, uint32_t *part, int32_t n, hipStream_t s, bool failed) {
    const size_t count = merge_count(e, n);
    if (failed) HIP_TRY(e, hipMemsetAsync(part, 0, count * 4, s));
    HIP_TRY(e, hipMemsetD32Async((hipDeviceptr_t)(part + count), failed ? 1 : 0, 1, s));
    return comm_allreduce_max(e, part, count + 1, s);
}

// the merged status word of the last chunk (after the loop's final synchronisation): a peer failed ⇒ this rank's
// placements came from incomplete keys — an error, and the replicas may differ (stale until reloaded)
kg_status merge_verdict(kg_engine *e, const uint32_t *part, int32_t n) {
    uint32_t w = 0;
    HIP_TRY(e, hipMemcpy(&w, part + merge_count(e, n), 4, hipMemcpyDeviceToHost));
    if (w) {
        e->stale = true;
        return set_err(e, KG_ERR_STATE, "a peer rank failed during kg_place_sharded: placements are not valid and the "
                                        "snapshot replicas may differ (reload with kg_snapshot_reset)");
    }
    return KG_OK;
}

// the ranks agree that every one of them is ready for the chunk loop (one all-reduce of a status flag after each
// rank's own allocations and checks): a rank that failed returns its error, the others KG_ERR_STATE, none enters
// the loop, so no rank waits in a collective its peer never issues
kg_status comm_agree(kg_engine *e, kg_status mine) {
    uint32_t v = mine != KG_OK ? 1u : 0u;
    kg_status st = KG_OK;
    if (!e->comm_word && hipMalloc((void **)&e->comm_word, 256) != hipSuccess) {
        e->comm_word = nullptr;
        return mine ? mine : set_err(e, KG_ERR_HIP, "hipMalloc of the status word");
    }
    if (hipMemcpyAsync(e->comm_word, &v, 4, hipMemcpyHostToDevice, e->stream) != hipSuccess)
        return mine ? mine : set_err(e, KG_ERR_HIP, "status word upload");
    st = comm_allreduce_max(e, e->comm_word, 1, e->stream);
    if (st) return mine ? mine : st;
    if (hipMemcpyAsync(&v, e->comm_word, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        return mine ? mine : set_err(e, KG_ERR_HIP, "status word download");
    if (mine) return mine;
    if (v) return set_err(e, KG_ERR_STATE, "a peer rank failed to set up kg_place_sharded (nothing was placed)");
    return KG_OK;
}
}  // namespace

extern "C" {

// kg_place's chunk loop; sharded: this rank evaluates its node shard and the chunk's partial keys are merged over
// the communicator before the (replicated, identical) resolve and host Reserve steps
kg_status place_loop(kg_engine *e, int64_t now_ns, int32_t *out_node, int64_t *out_score, bool sharded) {
    const int32_t P = e->n_pods;
    kg_status st = bind_ready(e, true, true);
    if (P == 0) return st;   // (the same batch on every rank: no rank enters a collective)
    int32_t chunk = e->cfg.place_chunk > 0 ? e->cfg.place_chunk : 16;
    if (chunk > KG_MAX_CHUNK) chunk = KG_MAX_CHUNK;
    // a pod that may bind a cpuset (its own PreFilter decision, or a cpu request where nodes have a CPU bind
    // policy) ends its chunk, and its Reserve runs on the host before the next chunk is evaluated
    const bool bind_mode = (e->consts.plugins & KG_PLUGIN_NUMA) && (e->batch_bind || e->n_node_bind_nodes > 0);
    const uint8_t may_mask = e->n_node_bind_nodes > 0 ? 3 : 1;
    // the pipeline pays two cross-stream event hops per chunk: it wins where the chunk evaluation is long
    // (NodeNUMAResource: config 3 5.0k → 6.1k pods/s) and loses where it is short (config 2: 82k → 61k)
    const bool pipelined = !bind_mode && !rsv_args(e).rsv && !(e->forms & KG_FORM_PLACE_SEQUENTIAL) &&
                           ((e->forms & KG_FORM_PLACE_PIPELINE) || (e->consts.plugins & KG_PLUGIN_NUMA));
    if (!st) st = quota_ready(e);   // (before the pipeline: chunk_resolve checks it too, with an evaluation in flight)
    if (st) {
        if (sharded) (void)comm_agree(e, st);   // the peers' one agreement of this call (here or in place_pipelined)
        return st;
    }
    if (pipelined) return place_pipelined(e, now_ns, out_node, out_score, chunk, sharded);
    const size_t part_b = (size_t)chunk * (size_t)tiles_total(e) * 4 * KG_PARTIAL_SLOTS + 4;   // + the status word
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    // the host Reserve's row upload uses the head of the scratch buffer: the partials live after it
    const size_t head = kHostReserveHead;
    st = ensure_scratch(e, head + up(part_b) + up((size_t)P * 4) + up((size_t)P * 8) + 256);
    if (sharded) st = comm_agree(e, st);
    if (st) return st;
    char *s = (char *)e->scratch + head;
    uint32_t *part = (uint32_t *)s;
    int32_t *dnode = (int32_t *)(s + up(part_b));
    int64_t *dscore = (int64_t *)(s + up(part_b) + up((size_t)P * 4));
    // the placement kernels answer cpusets on NUMA-policy nodes for this batch (kg_consts.numa_bz)
    struct BzScope {
        kg_consts &k;
        BzScope(kg_consts &c, bool on) : k(c) { k.numa_bz = on ? 1 : 0; }
        ~BzScope() { k.numa_bz = 0; }
    } bz_scope(e->consts, bind_mode && e->n_numa_policy_nodes > 0);
    // sharded: a failing step of this rank turns the rest of its loop into flagged merges of zero keys (see
    // place_pipelined); chunk boundaries depend only on the batch, so every rank issues the same merges
    kg_status local = KG_OK;
    int32_t last_n = 0;
    for (int32_t b = 0; b < P;) {
        int32_t n = P - b < chunk ? P - b : chunk;
        bool defer = false;
        if (bind_mode)
            for (int32_t k = 0; k < n; k++)
                if (e->pod_may_bind[(size_t)(b + k)] & may_mask) {
                    n = k + 1;
                    defer = true;
                    break;
                }
        last_n = n;
        if (!local) {
            st = chunk_eval(e, now_ns, b, n, part);
            if (st) {
                if (!sharded) return st;
                local = st;
            }
        }
        if (sharded) {
            st = merge_partials(e, part, n, e->stream, local != KG_OK);
            if (st) {
                e->stale = true;
                return st;
            }
        }
        if (!local) {
            st = chunk_resolve(e, now_ns, b, n, part, dnode + b, dscore + b, defer);
            if (st) {
                if (!sharded) return st;
                local = st;
            }
        }
        if (defer && !local) {
            const int32_t j = b + n - 1;
            int32_t node = -1;
            st = KG_OK;
            if (hipMemcpyAsync(&node, dnode + j, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
                hipStreamSynchronize(e->stream) != hipSuccess)
                st = set_err(e, KG_ERR_HIP, "download of a deferred placement");
            if (!st && node >= 0) {
                bool failed = false;
                st = host_reserve(e, j, node, &failed);
                if (!st && failed) {   // the Reserve failed: the pod is not placed
                    const int32_t no = -1;
                    const int64_t ns = -1;
                    if (h2d(e, dnode + j, &no, 4, e->stream) != hipSuccess || h2d(e, dscore + j, &ns, 8, e->stream) != hipSuccess ||
                        hipStreamSynchronize(e->stream) != hipSuccess)
                        st = set_err(e, KG_ERR_HIP, "upload of a failed Reserve's outcome");
                }
            }
            if (st) {
                if (!sharded) return st;
                local = st;
            }
        }
        b += n;
    }
    if (local) {
        e->stale = true;   // the replicas stopped at different chunks
        return local;
    }
    HIP_TRY(e, hipMemcpyAsync(out_node, dnode, (size_t)P * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipMemcpyAsync(out_score, dscore, (size_t)P * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    if (sharded) return merge_verdict(e, part, last_n);
    return KG_OK;
}

kg_status kg_cpus_set(kg_engine *e, const kg_cluster_view *view, const int32_t *view_index, const int32_t *snap_index,
                      int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (!view || n < 0) return set_err(e, KG_ERR_INVALID_ARG, "bad CPU table arguments");
    // validate everything first: a failed call changes no table
    std::vector<std::pair<int32_t, kg_engine::CpuTable>> tab;
    std::vector<int32_t> dropped;
    for (int32_t k = 0; k < n; k++) {
        const int32_t vi = view_index ? view_index[k] : k, si = snap_index ? snap_index[k] : k;
        if (vi < 0 || vi >= view->n_nodes) return set_err(e, KG_ERR_RANGE, "view node %d out of range", vi);
        if (si < 0 || si >= e->n_nodes) return set_err(e, KG_ERR_RANGE, "snapshot node %d out of range", si);
        const kg_node_spec &ns = view->nodes[vi];
        const kg_numa_spec *nmp = ns.numa >= 0 && ns.numa < view->n_numa && view->numa ? &view->numa[ns.numa] : nullptr;
        if (ns.numa >= 0 && !nmp) return set_err(e, KG_ERR_RANGE, "node %d: bad NUMA spec index", vi);
        if (!nmp || nmp->n_cpus <= 0) {
            dropped.push_back(si);
            continue;
        }
        const kg_numa_spec &nm = *nmp;
        if (nm.n_cpus > KG_MAX_NODE_CPUS || nm.first_cpu < 0 || nm.first_cpu + (int64_t)nm.n_cpus > view->n_cpus || !view->cpus)
            return set_err(e, KG_ERR_RANGE, "node %d: bad CPU range", vi);
        if (nm.numa_allocate_strategy < KG_NUMA_ALLOC_DEFAULT || nm.numa_allocate_strategy > KG_NUMA_ALLOC_DISTRIBUTE_EVENLY)
            return set_err(e, KG_ERR_INVALID_ARG, "node %d: bad NUMA allocate strategy", vi);
        kg_engine::CpuTable t;
        t.max_ref = nm.max_ref_count > 0 ? nm.max_ref_count : 1;
        t.strategy = kg_cpuset_strategy(e->cfg, nm.numa_allocate_strategy);
        t.cpus.assign(view->cpus + nm.first_cpu, view->cpus + nm.first_cpu + nm.n_cpus);
        tab.emplace_back(si, std::move(t));
    }
    for (int32_t si : dropped) e->cpu_tab.erase(si);
    for (auto &kv : tab) e->cpu_tab[kv.first] = std::move(kv.second);
    return KG_OK;
}

kg_status kg_cpus_download(kg_engine *e, int32_t node, kg_cpu_info *out, int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    auto it = e->cpu_tab.find(node);
    if (it == e->cpu_tab.end()) return set_err(e, KG_ERR_RANGE, "node %d has no CPU table", node);
    if (n != (int32_t)it->second.cpus.size() || (n > 0 && !out))
        return set_err(e, KG_ERR_RANGE, "node %d has %zu CPUs, asked for %d", node, it->second.cpus.size(), n);
    memcpy(out, it->second.cpus.data(), sizeof(kg_cpu_info) * (size_t)n);
    return KG_OK;
}

kg_status kg_set_profiling(kg_engine *e, int32_t on) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (on && !e->ev0[0]) {
        for (int k = 0; k < kg_engine::kRing; k++) {
            HIP_TRY(e, hipEventCreate(&e->ev0[k]));
            HIP_TRY(e, hipEventCreate(&e->ev1[k]));
        }
    }
    e->profiling = on != 0;
    e->ev_count = 0;
    e->ev_acc = 0;
    return KG_OK;
}

kg_status kg_counters_get(kg_engine *e, kg_counters *out) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (!out) return set_err(e, KG_ERR_INVALID_ARG, "null output");
    if (e->profiling) {   // the timed launches not summed yet (prof_begin sums a ring slot before reusing it)
        for (; e->ev_acc < e->ev_count; e->ev_acc++) HIP_TRY(e, prof_sum(e, e->ev_acc));
    }
    *out = e->ctr;
    return KG_OK;
}

kg_status kg_counters_reset(kg_engine *e) {
    kg_status st = check_engine(e);
    if (st) return st;
    e->ctr = kg_counters{};
    e->ev_acc = e->ev_count;
    return KG_OK;
}

int32_t kg_eval_kernel_times(kg_engine *e, float *ms, int32_t n) {
    if (check_engine(e) != KG_OK || !ms || n < 0) return KG_ERR_INVALID_ARG;
    if (!e->profiling) return set_err(e, KG_ERR_STATE, "profiling is off");
    const int64_t have = e->ev_count < kg_engine::kRing ? e->ev_count : kg_engine::kRing;
    const int32_t k = n < have ? n : (int32_t)have;
    for (int32_t j = 0; j < k; j++) {
        const int64_t slot = (e->ev_count - k + j) % kg_engine::kRing;
        HIP_TRY(e, hipEventSynchronize(e->ev1[slot]));
        HIP_TRY(e, hipEventElapsedTime(&ms[j], e->ev0[slot], e->ev1[slot]));
    }
    return k;
}

kg_status kg_rsv_set(kg_engine *e, const kg_reservation *rsv, int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (!(e->consts.plugins & KG_PLUGIN_RESERVATION)) return set_err(e, KG_ERR_STATE, "Reservation plugin not enabled");
    if (!e->plane_mem) return set_err(e, KG_ERR_STATE, "snapshot not initialised");
    if (n < 0 || (n > 0 && !rsv)) return set_err(e, KG_ERR_INVALID_ARG, "bad reservation list");
    std::vector<int32_t> order((size_t)n);
    std::vector<int32_t> per_node_count;
    std::map<int32_t, int32_t> count;
    for (int32_t i = 0; i < n; i++) {
        if (rsv[i].node < 0 || rsv[i].node >= e->n_nodes) return set_err(e, KG_ERR_RANGE, "reservation %d: bad node", i);
        if (++count[rsv[i].node] > KG_MAX_RSV_PER_NODE)
            return set_err(e, KG_ERR_UNSUPPORTED, "node %d: more than %d reservations", rsv[i].node, KG_MAX_RSV_PER_NODE);
        if (rsv[i].policy < KG_RSV_POLICY_DEFAULT || rsv[i].policy > KG_RSV_POLICY_RESTRICTED)
            return set_err(e, KG_ERR_INVALID_ARG, "reservation %d: bad allocate policy", i);
        order[(size_t)i] = i;
    }
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return rsv[a].node < rsv[b].node; });
    std::vector<kg_reservation> slots((size_t)n);
    std::vector<int32_t> rfirst, rnode;
    std::vector<int32_t> rsv_of((size_t)e->pl.cap, -1);
    for (int32_t k = 0; k < n; k++) {
        slots[(size_t)k] = rsv[order[(size_t)k]];
        const int32_t node = slots[(size_t)k].node;
        if (rnode.empty() || rnode.back() != node) {
            rsv_of[(size_t)node] = (int32_t)rnode.size();
            rnode.push_back(node);
            rfirst.push_back(k);
        }
    }
    rfirst.push_back(n);
    const int32_t n_rn = (int32_t)rnode.size();
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t sb = up(sizeof(kg_reservation) * (size_t)(n > 0 ? n : 1)), fb = up(4 * rfirst.size()),
                 nb = up(4 * (size_t)(n_rn > 0 ? n_rn : 1)),
                 eb = up(8 * (size_t)KG_RSV_POD_CHUNK * (size_t)(n_rn > 0 ? n_rn : 1));
    // the placement split: scored-entry lists [chunk][n_rn], their counts, per-group keys [chunk][groups]; only
    // when the resolve's touched-group flags cover the groups (rsv_args), else nothing reads it
    const bool split = (n_rn + KG_RSV_GROUP - 1) / KG_RSV_GROUP <= KG_RSV_MAX_GROUPS;
    const size_t mb = split ? up(sizeof(kg_rsv_ment) * (size_t)KG_RSV_POD_CHUNK * (size_t)(n_rn > 0 ? n_rn : 1)) : 0,
                 cb = split ? up(4 * (size_t)KG_RSV_POD_CHUNK) : 0,
                 gb = split ? up(8 * (size_t)KG_RSV_POD_CHUNK * (size_t)((n_rn + KG_RSV_GROUP - 1) / KG_RSV_GROUP + 1)) : 0;
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    if (e->rsv_mem) HIP_TRY(e, hipFree(e->rsv_mem));
    e->rsv_mem = nullptr;
    HIP_TRY(e, hipMalloc(&e->rsv_mem, sb + fb + nb + 2 * eb + mb + cb + gb));
    char *m = (char *)e->rsv_mem;
    e->rsv = (kg_reservation *)m;
    e->rfirst = (int32_t *)(m + sb);
    e->rnode = (int32_t *)(m + sb + fb);
    e->rsv_e = (unsigned long long *)(m + sb + fb + nb);
    e->rsv_o = (int64_t *)(m + sb + fb + nb + eb);
    e->rsv_m = split ? (kg_rsv_ment *)(m + sb + fb + nb + 2 * eb) : nullptr;
    e->rsv_mn = split ? (int32_t *)(m + sb + fb + nb + 2 * eb + mb) : nullptr;
    e->rsv_g = split ? (unsigned long long *)(m + sb + fb + nb + 2 * eb + mb + cb) : nullptr;
    if (n) HIP_TRY(e, h2d(e, e->rsv, slots.data(), sizeof(kg_reservation) * (size_t)n, e->stream));
    HIP_TRY(e, h2d(e, e->rfirst, rfirst.data(), 4 * rfirst.size(), e->stream));
    if (n_rn) HIP_TRY(e, h2d(e, e->rnode, rnode.data(), 4 * (size_t)n_rn, e->stream));
    HIP_TRY(e, h2d(e, e->pl.rsv_of, rsv_of.data(), 4 * rsv_of.size(), e->stream));
    e->n_rsv = n;
    e->n_rn = n_rn;
    e->rsv_perm = order;
    // re-derive every node's planes: reservation nodes leave the fast paths, the others rejoin
    hipLaunchKernelGGL(k_finalize_range, dim3((unsigned)((e->pl.cap + 255) / 256)), dim3(256), 0, e->stream, e->consts,
                       e->pl, (int64_t)0, e->pl.cap);
    HIP_TRY(e, hipGetLastError());
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->slow_valid = false;
    return KG_OK;
}

kg_status kg_rsv_download(kg_engine *e, kg_reservation *out, int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (n != e->n_rsv || (n > 0 && !out)) return set_err(e, KG_ERR_RANGE, "download %d reservations, have %d", n, e->n_rsv);
    if (n == 0) return KG_OK;
    std::vector<kg_reservation> slots((size_t)n);
    HIP_TRY(e, hipMemcpyAsync(slots.data(), e->rsv, sizeof(kg_reservation) * (size_t)n, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    for (int32_t k = 0; k < n; k++) out[e->rsv_perm[(size_t)k]] = slots[(size_t)k];
    return KG_OK;
}

kg_status kg_quota_set(kg_engine *e, const kg_quota *q, int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (!(e->consts.plugins & KG_PLUGIN_ELASTICQUOTA)) return set_err(e, KG_ERR_STATE, "ElasticQuota plugin not enabled");
    if (n < 0 || (n > 0 && !q)) return set_err(e, KG_ERR_INVALID_ARG, "bad quota list");
    for (int32_t g = 0; g < n; g++) {  // parent chains end at the root within KG_QUOTA_MAX_DEPTH steps (no cycles)
        if (q[g].parent == g)   // the usual cause: a zero-filled record (the root is parent = -1, not 0)
            return set_err(e, KG_ERR_INVALID_ARG,
                           "quota %d is its own parent: a group directly under the root has parent = -1", g);
        int32_t a = q[g].parent, d = 0;
        for (; a >= 0 && a < n && d < KG_QUOTA_MAX_DEPTH; a = q[a].parent) d++;
        if (a < -1 || a >= n) return set_err(e, KG_ERR_INVALID_ARG, "quota %d: parent index %d out of range", g, a);
        if (a >= 0) return set_err(e, KG_ERR_INVALID_ARG, "quota %d: parent chain cyclic or deeper than %d", g,
                                   KG_QUOTA_MAX_DEPTH);
    }
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    if (e->quota) HIP_TRY(e, hipFree(e->quota));
    e->quota = nullptr;
    HIP_TRY(e, hipMalloc(&e->quota, sizeof(kg_quota) * (size_t)(n > 0 ? n : 1)));
    if (n) HIP_TRY(e, h2d(e, e->quota, q, sizeof(kg_quota) * (size_t)n, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    e->n_quota = n;
    return KG_OK;
}

kg_status kg_quota_download(kg_engine *e, kg_quota *out, int32_t n) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (n != e->n_quota || (n > 0 && !out)) return set_err(e, KG_ERR_RANGE, "download %d quotas, have %d", n, e->n_quota);
    if (n == 0) return KG_OK;
    HIP_TRY(e, hipMemcpyAsync(out, e->quota, sizeof(kg_quota) * (size_t)n, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    return KG_OK;
}

kg_status kg_commit(kg_engine *e, int32_t pod, int32_t node) {
    kg_status st = check_engine(e);
    if (st) return st;
    if (pod < 0 || pod >= e->n_pods || node < 0 || node >= e->n_nodes) return set_err(e, KG_ERR_RANGE, "bad commit");
    st = bind_ready(e, true, true);
    if (st) return st;
    st = quota_ready(e);   // the pod's quota group must exist before its usage is committed
    if (st) return st;
    bool failed = false;
    st = host_reserve(e, pod, node, &failed);
    if (st) return st;
    if (failed) return set_err(e, KG_NOT_FOUND, "pod %d on node %d: not enough cpus available to satisfy request", pod, node);
    e->ctr.placed++;
    return KG_OK;
}

}  // extern "C"
