// kg_cpuset.cpp — NodeNUMAResource's cpuset take at Reserve (the CPU accumulator), on the host.
//
// A Reserve of a cpuset-bound pod picks WHICH logical CPUs the pod gets: branchy, sort-heavy work on one
// node's few hundred CPUs, once per placed pod — host work by nature (SURVEY §8f "later"), run by the
// engine's placement loop between device chunks.  Restates:
//   takePreferredCPUs / takeCPUs            nodenumaresource/cpu_accumulator.go:29-232
//   cpuAccumulator and its orderings         cpu_accumulator.go:234-822
//   NodeAllocation.getAvailableCPUs          node_allocation.go:134-155
//   filterCPUsByRequiredCPUBindPolicy        resource_manager.go:534-566
//   satisfiedRequiredCPUBindPolicy           resource_manager.go:568-589
// Every ordering the reference sorts with a total order is a std::sort with that comparator; the two
// sorts without a tie-break (cpu_accumulator.go:142, :161: socket groups by length, which Go's pdqsort
// insertion-sorts at these sizes, i.e. stably) are std::stable_sort.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "kg_host.h"

namespace {

constexpr int kBindFull = KG_CPU_BIND_FULL_PCPUS, kBindSpread = KG_CPU_BIND_SPREAD_BY_PCPUS;
constexpr int kExclPCPU = KG_CPU_EXCL_PCPU_LEVEL, kExclNUMA = KG_CPU_EXCL_NUMA_NODE_LEVEL;

// compact ids: the reference keys its maps by the reported core / node / socket ids
struct Topo {
    int n = 0;
    std::vector<int> core, node, sock;            // per cpu: compact index
    std::vector<int> core_id, node_id, sock_id;   // compact index → reported id
    int per_core = 0, per_node = 0, per_socket = 0;

    static int intern(std::vector<int> &ids, int id) {
        for (size_t i = 0; i < ids.size(); i++)
            if (ids[i] == id) return (int)i;
        ids.push_back(id);
        return (int)ids.size() - 1;
    }
    Topo(const kg_cpu_info *cpus, int n_cpus) : n(n_cpus), core(n_cpus), node(n_cpus), sock(n_cpus) {
        for (int c = 0; c < n; c++) {
            core[c] = intern(core_id, cpus[c].core);
            node[c] = intern(node_id, cpus[c].node);
            sock[c] = intern(sock_id, cpus[c].socket);
        }
        // CPUsPerCore / CPUsPerNode / CPUsPerSocket (cpu_topology.go): total CPUs over distinct ids
        per_core = core_id.empty() ? 0 : n / (int)core_id.size();
        per_node = node_id.empty() ? 0 : n / (int)node_id.size();
        per_socket = sock_id.empty() ? 0 : n / (int)sock_id.size();
    }
};

using List = std::vector<int>;
using Groups = std::vector<List>;

struct Accumulator {
    const Topo &t;
    int max_ref;
    std::vector<uint8_t> avail;        // allocatableCPUs
    std::vector<int32_t> ref;          // their RefCount (maxRefCount > 1)
    std::vector<uint8_t> excl_core;    // exclusiveInCores (compact core)
    std::vector<uint8_t> excl_node;    // exclusiveInNUMANodes (compact node)
    bool exclusive;
    int excl_policy, strategy, need;
    std::vector<uint8_t> result;

    Accumulator(const Topo &topo, const kg_cpu_info *cpus, int max_ref_, const uint8_t *available, int need_, int excl,
                int strategy_)
        : t(topo), max_ref(max_ref_), avail(topo.n), ref(topo.n, 0), excl_core(topo.core_id.size(), 0),
          excl_node(topo.node_id.size(), 0), exclusive(excl == kExclPCPU || excl == kExclNUMA), excl_policy(excl),
          strategy(strategy_), need(need_), result(topo.n, 0) {
        for (int c = 0; c < t.n; c++) {
            avail[c] = available[c] != 0;
            if (max_ref > 1) ref[c] = cpus[c].refcount;
            if (cpus[c].refcount > 0) {   // allocatedCPUs: the exclusive policy the holders asked for
                if (cpus[c].exclusive == kExclPCPU) excl_core[t.core[c]] = 1;
                else if (cpus[c].exclusive == kExclNUMA) excl_node[t.node[c]] = 1;
            }
        }
    }
    int n_avail() const { return (int)std::count(avail.begin(), avail.end(), (uint8_t)1); }
    bool needs(int k) const { return need >= k; }
    bool satisfied() const { return need < 1; }
    void take(const int *cpus, int k) {
        for (int i = 0; i < k; i++) {
            const int c = cpus[i];
            result[c] = 1;
            avail[c] = 0;
            if (exclusive) {
                if (excl_policy == kExclPCPU) excl_core[t.core[c]] = 1;
                else if (excl_policy == kExclNUMA) excl_node[t.node[c]] = 1;
            }
        }
        need -= k;
    }
    bool excl_pcpu(int c) const { return excl_policy == kExclPCPU && excl_core[t.core[c]]; }
    bool excl_numa(int c) const { return excl_policy == kExclNUMA && excl_node[t.node[c]]; }
    bool most() const { return strategy == KG_STRATEGY_MOST_ALLOCATED; }
    // a free-score order: NUMAMostAllocated ascending, LeastAllocated descending; 0 on a tie
    int by_free(int x, int y) const { return x == y ? 0 : (most() ? (x < y ? -1 : 1) : (x > y ? -1 : 1)); }
    int core_ref(int k) const {   // getCoreRefCount over the allocatable CPUs
        int r = 0;
        for (int c = 0; c < t.n; c++)
            if (avail[c] && t.core[c] == k) r += ref[c];
        return r;
    }
    void sort_cpus(List &cpus) const {   // sort.Ints, then sortCPUsByRefCount when maxRefCount > 1
        std::sort(cpus.begin(), cpus.end());
        if (max_ref > 1)
            std::sort(cpus.begin(), cpus.end(), [&](int i, int j) { return ref[i] != ref[j] ? ref[i] < ref[j] : i < j; });
    }
    List extract_cpu(const List &cpus) const {   // the first CPU of each core, in order
        std::vector<uint8_t> seen(t.core_id.size(), 0);
        List out;
        for (int c : cpus)
            if (!seen[t.core[c]]) {
                seen[t.core[c]] = 1;
                out.push_back(c);
            }
        return out;
    }
    List spread(const List &cpus) const {   // spreadCPUs: one CPU per core per pass
        if ((int)cpus.size() <= t.per_core) return cpus;
        List prep = cpus, out;
        while (!prep.empty()) {
            std::vector<uint8_t> seen(t.core_id.size(), 0);
            List rest;
            for (int c : prep) {
                if (seen[t.core[c]]) {
                    rest.push_back(c);
                    continue;
                }
                seen[t.core[c]] = 1;
                out.push_back(c);
            }
            prep.swap(rest);
        }
        return out;
    }

    // freeCoresInNode (by_node) / freeCoresInSocket: the CPUs of the (full-)free cores grouped by NUMA node /
    // socket; cores by sortCores, groups by the free scores
    Groups free_cores(bool by_node, bool full_only, bool skip_numa_excl) const {
        const int ncore = (int)t.core_id.size();
        std::vector<List> in_core(ncore);
        std::vector<int> sock_free(t.sock_id.size(), 0);
        for (int c = 0; c < t.n; c++) {
            if (!avail[c] || (skip_numa_excl && excl_numa(c))) continue;
            in_core[t.core[c]].push_back(c);
            sock_free[t.sock[c]]++;
        }
        const int ng = (int)(by_node ? t.node_id.size() : t.sock_id.size());
        std::vector<List> cores_of(ng);
        for (int k = 0; k < ncore; k++) {
            if (in_core[k].empty() || (full_only && (int)in_core[k].size() != t.per_core)) continue;
            const int c0 = in_core[k][0];
            cores_of[by_node ? t.node[c0] : t.sock[c0]].push_back(k);
        }
        std::vector<int> order;
        std::vector<List> cpus_of(ng);
        std::vector<int> grp_sock(ng, 0);
        for (int g = 0; g < ng; g++) {
            if (cores_of[g].empty()) continue;
            std::sort(cores_of[g].begin(), cores_of[g].end(), [&](int i, int j) {   // sortCores
                if (in_core[i].size() != in_core[j].size()) return in_core[i].size() > in_core[j].size();
                if (max_ref > 1) {
                    const int ri = core_ref(i), rj = core_ref(j);
                    if (ri != rj) return ri < rj;
                }
                return t.core_id[i] < t.core_id[j];
            });
            for (int k : cores_of[g]) {
                List cs = in_core[k];
                std::sort(cs.begin(), cs.end());
                cpus_of[g].insert(cpus_of[g].end(), cs.begin(), cs.end());
            }
            grp_sock[g] = t.sock[cpus_of[g][0]];
            order.push_back(g);
        }
        std::sort(order.begin(), order.end(), [&](int i, int j) {
            int r = by_free((int)cpus_of[i].size(), (int)cpus_of[j].size());
            if (r) return r < 0;
            if (by_node) {
                r = by_free(sock_free[grp_sock[i]], sock_free[grp_sock[j]]);
                if (r) return r < 0;
                return t.node_id[i] < t.node_id[j];
            }
            return t.sock_id[i] < t.sock_id[j];
        });
        Groups out;
        for (int g : order) out.push_back(cpus_of[g]);
        return out;
    }

    // freeCPUsInNode (by_node) / freeCPUsInSocket
    Groups free_cpus_in(bool by_node, bool filter_excl) const {
        const int ng = (int)(by_node ? t.node_id.size() : t.sock_id.size());
        std::vector<List> cpus_of(ng);
        std::vector<int> node_free(t.node_id.size(), 0), sock_free(t.sock_id.size(), 0), grp_sock(ng, 0);
        for (int c = 0; c < t.n; c++) {
            if (!avail[c]) continue;
            if (filter_excl && (excl_pcpu(c) || (by_node && excl_numa(c)))) continue;
            cpus_of[by_node ? t.node[c] : t.sock[c]].push_back(c);
            node_free[t.node[c]]++;
            sock_free[t.sock[c]]++;
            if (by_node) grp_sock[t.node[c]] = t.sock[c];
        }
        std::vector<int> order;
        for (int g = 0; g < ng; g++) {
            if (cpus_of[g].empty()) continue;
            sort_cpus(cpus_of[g]);
            if (filter_excl) cpus_of[g] = extract_cpu(cpus_of[g]);
            order.push_back(g);
        }
        std::sort(order.begin(), order.end(), [&](int i, int j) {
            if (by_node) {   // scores counted before extractCPU (cpu_accumulator.go:544, :575)
                int r = by_free(node_free[i], node_free[j]);
                if (r) return r < 0;
                r = by_free(sock_free[grp_sock[i]], sock_free[grp_sock[j]]);
                if (r) return r < 0;
                return t.node_id[i] < t.node_id[j];
            }
            const int r = by_free((int)cpus_of[i].size(), (int)cpus_of[j].size());   // after extractCPU (:637)
            if (r) return r < 0;
            return t.sock_id[i] < t.sock_id[j];
        });
        Groups out;
        for (int g : order) out.push_back(cpus_of[g]);
        return out;
    }

    // freeCPUs: cores by socket colocation with the result, socket / node free scores, free CPUs on the
    // core, socket id, refcount, core id; each core's CPUs ascending (then by refcount)
    List free_cpus(bool filter_excl) const {
        const int ncore = (int)t.core_id.size();
        std::vector<List> in_core(ncore);
        std::vector<int> sock_free(t.sock_id.size(), 0), node_free(t.node_id.size(), 0), colo(t.sock_id.size(), 0);
        std::vector<int> csock(ncore, 0), cnode(ncore, 0);
        for (int c = 0; c < t.n; c++) {
            if (!avail[c] || (filter_excl && (excl_pcpu(c) || excl_numa(c)))) continue;
            in_core[t.core[c]].push_back(c);
            csock[t.core[c]] = t.sock[c];
            cnode[t.core[c]] = t.node[c];
            node_free[t.node[c]]++;
            sock_free[t.sock[c]]++;
        }
        for (int c = 0; c < t.n; c++)
            if (result[c]) colo[t.sock[c]]++;
        std::vector<int> cores;
        for (int k = 0; k < ncore; k++)
            if (!in_core[k].empty()) cores.push_back(k);
        std::sort(cores.begin(), cores.end(), [&](int i, int j) {
            const int si = csock[i], sj = csock[j];
            if (colo[si] != colo[sj]) return colo[si] > colo[sj];
            int r = by_free(sock_free[si], sock_free[sj]);
            if (r) return r < 0;
            r = by_free(node_free[cnode[i]], node_free[cnode[j]]);
            if (r) return r < 0;
            if (in_core[i].size() != in_core[j].size()) return in_core[i].size() < in_core[j].size();
            if (t.sock_id[si] != t.sock_id[sj]) return t.sock_id[si] < t.sock_id[sj];
            if (max_ref > 1) {
                const int ri = core_ref(i), rj = core_ref(j);
                if (ri != rj) return ri < rj;
            }
            return t.core_id[i] < t.core_id[j];
        });
        List out;
        for (int k : cores) {
            List cs = in_core[k];
            sort_cpus(cs);
            out.insert(out.end(), cs.begin(), cs.end());
        }
        return out;
    }
};

// takeCPUs (cpu_accumulator.go:87-232); true ⇔ satisfied, result in acc.result
bool take_cpus(Accumulator &a, int bind) {
    const Topo &t = a.t;
    if (a.satisfied()) return true;
    if (a.need > a.n_avail()) return false;
    const bool full = bind == kBindFull;
    if (full || t.per_core == 1) {
        if (a.need <= t.per_node) {
            for (int fe = 1; fe >= 0; fe--)
                for (const List &g : a.free_cores(true, true, fe == 1))
                    if ((int)g.size() >= a.need) {
                        a.take(g.data(), a.need);
                        return true;
                    }
        }
        if (a.need <= t.per_socket)
            for (const List &g : a.free_cores(false, true, false))
                if ((int)g.size() >= a.need) {
                    a.take(g.data(), a.need);
                    return true;
                }
        Groups socks = a.free_cores(false, true, false);
        std::stable_sort(socks.begin(), socks.end(), [](const List &x, const List &y) { return x.size() > y.size(); });
        Groups unsat;
        for (const List &g : socks) {
            if (!a.needs((int)g.size())) {
                unsat.push_back(g);
            } else {
                a.take(g.data(), (int)g.size());
                if (a.satisfied()) return true;
            }
        }
        if (a.needs(t.per_core)) {
            std::stable_sort(unsat.begin(), unsat.end(), [](const List &x, const List &y) { return x.size() < y.size(); });
            for (const List &g : unsat)
                for (size_t i = 0; i < g.size(); i += (size_t)t.per_core) {
                    a.take(g.data() + i, t.per_core);
                    if (a.satisfied()) return true;
                    if (!a.needs(t.per_core)) break;
                }
        }
    }
    if (!full) {
        if (a.need <= t.per_node)
            for (int fe = 1; fe >= 0; fe--)
                for (const List &g : a.free_cpus_in(true, fe == 1))
                    if ((int)g.size() >= a.need) {
                        const List s = a.spread(g);
                        a.take(s.data(), a.need);
                        return true;
                    }
        if (a.need <= t.per_socket)
            for (int fe = 1; fe >= 0; fe--)
                for (const List &g : a.free_cpus_in(false, fe == 1))
                    if ((int)g.size() >= a.need) {
                        const List s = a.spread(g);
                        a.take(s.data(), a.need);
                        return true;
                    }
    }
    for (int fe = 1; fe >= 0; fe--) {
        const List s = a.spread(a.free_cpus(fe == 1));
        for (int c : s) {
            if (a.needs(1)) a.take(&c, 1);
            if (a.satisfied()) return true;
        }
    }
    return false;
}

}  // namespace

// takeCPUs over `available` (per cpu id); the node's allocated CPU details come from `cpus` (refcount,
// exclusive).  0 ⇔ `need` CPUs taken into `result`.
int kg_cpuset_take_cpus(const kg_cpu_info *cpus, int32_t n_cpus, int32_t max_ref, const uint8_t *available, int32_t need,
                        int32_t bind, int32_t exclusive, int32_t strategy, uint8_t *result) {
    const Topo t(cpus, n_cpus);
    Accumulator a(t, cpus, max_ref, available, need, exclusive, strategy);
    memset(result, 0, (size_t)n_cpus);
    if (!take_cpus(a, bind)) return -1;
    memcpy(result, a.result.data(), (size_t)n_cpus);
    return 0;
}

// NodeAllocation.getAvailableCPUs (node_allocation.go:134-155): allocated once RefCount ≥ maxRefCount;
// reserved CPUs are never available (no preferred CPUs on the engine path)
void kg_cpuset_available(const kg_cpu_info *cpus, int32_t n_cpus, int32_t max_ref, uint8_t *available) {
    for (int c = 0; c < n_cpus; c++)
        available[c] = !(cpus[c].refcount > 0 && cpus[c].refcount >= max_ref) && !cpus[c].reserved;
}

// filterCPUsByRequiredCPUBindPolicy (resource_manager.go:534-566): FullPCPUs keeps the CPUs of wholly
// available cores, SpreadByPCPUs the lowest available CPU of each core
void kg_cpuset_filter_required(const kg_cpu_info *cpus, int32_t n_cpus, int32_t bind, uint8_t *available) {
    const Topo t(cpus, n_cpus);
    std::vector<int> cnt(t.core_id.size(), 0), first(t.core_id.size(), -1);
    for (int c = 0; c < n_cpus; c++)
        if (available[c]) {
            cnt[t.core[c]]++;
            if (first[t.core[c]] < 0) first[t.core[c]] = c;
        }
    for (int c = 0; c < n_cpus; c++) {
        if (!available[c]) continue;
        if (bind == kBindFull) available[c] = cnt[t.core[c]] == t.per_core;
        else if (bind == kBindSpread) available[c] = first[t.core[c]] == c;
    }
}

// satisfiedRequiredCPUBindPolicy (resource_manager.go:568-589)
bool kg_cpuset_satisfies_required(const kg_cpu_info *cpus, int32_t n_cpus, int32_t bind, const uint8_t *taken) {
    const Topo t(cpus, n_cpus);
    std::vector<uint8_t> seen(t.core_id.size(), 0);
    int ncpu = 0, ncore = 0;
    for (int c = 0; c < n_cpus; c++)
        if (taken[c]) {
            ncpu++;
            if (!seen[t.core[c]]) {
                seen[t.core[c]] = 1;
                ncore++;
            }
        }
    if (bind == kBindFull) return ncore * t.per_core == ncpu;
    if (bind == kBindSpread) return ncore == ncpu;
    return true;
}

// The row's cpuset facts from the node's logical CPUs (what kg_build_node_rows derives from the view, and what
// a Reserve re-derives after it took CPUs): CPUsPerCore, the available CPUs (getAvailableCPUs: allocated once
// RefCount ≥ maxRefCount, reserved CPUs out) node-wide and per zone — all of them, those of wholly available
// cores, cores with one — and the cpuset pods' CPUs (allocatedCPUs, RefCount > 0) with their amplified
// terms.  Returns the allocated CPU count.
int32_t kg_cpuset_row_fields(kg_node_row &row, const kg_cpu_info *ci, int32_t n, int32_t max_ref) {
    if (max_ref < 1) max_ref = 1;
    std::vector<int32_t> core_id, core_total, core_avail, core_zone;
    int32_t nalloc = 0, zone_alloc[KG_MAX_ZONES] = {};
    for (int32_t c = 0; c < n; c++) {
        size_t k = 0;
        while (k < core_id.size() && core_id[k] != ci[c].core) k++;
        if (k == core_id.size()) {
            core_id.push_back(ci[c].core);
            core_total.push_back(0);
            core_avail.push_back(0);
            core_zone.push_back(-1);
        }
        core_total[k]++;
        if (!(ci[c].refcount > 0 && ci[c].refcount >= max_ref) && !ci[c].reserved) core_avail[k]++;
        for (int z = 0; z < row.n_zones && z < KG_MAX_ZONES; z++)
            if (row.zone_id[z] == ci[c].node) {
                core_zone[k] = z;   // the zone of each core (its CPUs' NUMA node); −1 ⇔ no zone
                if (ci[c].refcount > 0) zone_alloc[z]++;
            }
        if (ci[c].refcount > 0) nalloc++;
    }
    const int32_t ncores = (int32_t)core_id.size();
    row.cpus_per_core = ncores ? n / ncores : 0;
    row.cpuset_full_free_cpus = row.cpuset_free_cores = row.cpuset_avail_cpus = 0;
    for (int z = 0; z < KG_MAX_ZONES; z++) row.zone_cpus_avail[z] = row.zone_cpus_full[z] = row.zone_cores_free[z] = 0;
    for (int32_t k = 0; k < ncores; k++) {
        const bool full = core_avail[k] == row.cpus_per_core;
        if (full) row.cpuset_full_free_cpus += core_avail[k];
        if (core_avail[k] > 0) row.cpuset_free_cores++;
        row.cpuset_avail_cpus += core_avail[k];
        const int32_t z = core_zone[k];
        if (z < 0) continue;
        row.zone_cpus_avail[z] = (int16_t)(row.zone_cpus_avail[z] + core_avail[k]);
        if (full) row.zone_cpus_full[z] = (int16_t)(row.zone_cpus_full[z] + core_avail[k]);
        if (core_avail[k] > 0) row.zone_cores_free[z]++;
    }
    // the amplified-CPU terms of filterAmplifiedCPUs / scoreWithAmplifiedCPUs / getAvailableNUMANodeResources
    const double ratio = row.cpu_amplification_ratio;
    const auto amplify = [ratio](int64_t x) { return ratio > 1.0 ? (int64_t)ceil((double)x * ratio) : x; };
    row.cpuset_milli = (int64_t)nalloc * 1000;
    row.cpuset_amp_milli = amplify(row.cpuset_milli);
    for (int z = 0; z < KG_MAX_ZONES; z++)
        row.zone_cpuset_amp[z] = amplify((int64_t)zone_alloc[z] * 1000) - (int64_t)zone_alloc[z] * 1000;
    return nalloc;
}

// resourceManager.Allocate's cpuset part for a pod that binds on the node (resource_manager.go:171-195,
// 273-360): the zones of the Filter's hint (allocateResourcesByHint on the original requests, through the same
// per-pair code the kernels run) and allocateCPUSet — available CPUs, the required policy's filter, per
// allocated zone min(its available CPUs, its cpu / 1000) through the accumulator, the rest node-wide, and
// satisfiedRequiredCPUBindPolicy.  0 ⇔ a cpuset was taken into taken[n]; −1 ⇔ Allocate fails.
int kg_cpuset_allocate(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, int required, int take,
                       const kg_cpu_info *cpus, int32_t n, int32_t max_ref, int32_t strategy, uint8_t *taken) {
    if (max_ref < 1) max_ref = 1;
    memset(taken, 0, (size_t)n);
    if (!(row.flags & KG_NODE_NUMA_TOPO_VALID) || n <= 0) return -1;   // ErrInvalidCPUTopology
    const int64_t pcpu = p.numa_req[KG_RES_CPU];
    const int need_all = (int)(pcpu / 1000);   // numCPUsNeeded
    // PodAllocation.CPUExclusivePolicy = the pod's preferredCPUExclusivePolicy (set by its own PreFilter only)
    const int excl = (p.flags & KG_POD_NUMA_CPU_BIND) ? (int)((p.cpu_bind >> 8) & 15u) : KG_CPU_EXCL_UNSET;
    kg_numa_out o;
    o.feasible = true;
    o.score = 0;
    o.n_alloc = 0;
    const bool opts = (row.flags & KG_NODE_NUMA_OPTIONS) != 0;
    if (opts && row.numa_policy != KG_NUMA_NONE) {   // a hint exists only where the Filter admitted one
        const double ratio = row.cpu_amplification_ratio;
        const int64_t pcpu_eff = pcpu != 0 && ratio > 1.0 ? (int64_t)ceil((double)pcpu * ratio) : pcpu;
        kg_numa_bind_zoned(c, row, p, o, row.requested, row.numa_policy, pcpu_eff, required);
        if (!o.feasible) return -1;
    }
    std::vector<uint8_t> avail((size_t)n), zav((size_t)n), got((size_t)n);
    kg_cpuset_available(cpus, n, max_ref, avail.data());
    if (required != KG_CPU_BIND_UNSET) kg_cpuset_filter_required(cpus, n, required, avail.data());
    int navail = 0;
    for (int32_t k = 0; k < n; k++) navail += avail[k];
    if (navail < need_all) return -1;   // "not enough cpus available to satisfy request"
    int need = need_all;
    if (o.n_alloc > 0) {
        int taken_n = 0;
        for (int j = 0; j < o.n_alloc; j++) {   // allocatedNUMANodes in ascending affinity id
            const int32_t zid = row.zone_id[o.zone[j]];
            int cnt = 0;
            for (int32_t k = 0; k < n; k++) {
                zav[k] = (uint8_t)(avail[k] && cpus[k].node == zid);
                cnt += zav[k];
            }
            const int64_t want = o.alloc[j][KG_RES_CPU] / 1000;
            if (want < cnt) cnt = (int)want;
            if (kg_cpuset_take_cpus(cpus, n, max_ref, zav.data(), cnt, take, excl, strategy, got.data()) != 0) return -1;
            for (int32_t k = 0; k < n; k++)
                if (got[k] && !taken[k]) {
                    taken[k] = 1;
                    taken_n++;
                }
        }
        need -= taken_n;
        if (need != 0) return -1;
    }
    if (need > 0) {
        for (int32_t k = 0; k < n; k++) zav[k] = (uint8_t)(avail[k] && !taken[k]);
        if (kg_cpuset_take_cpus(cpus, n, max_ref, zav.data(), need, take, excl, strategy, got.data()) != 0) return -1;
        for (int32_t k = 0; k < n; k++) taken[k] |= got[k];
    }
    if (required != KG_CPU_BIND_UNSET && !kg_cpuset_satisfies_required(cpus, n, required, taken)) return -1;
    return 0;
}

// NodeAllocation.addPodAllocation (node_allocation.go:72-100) for the cpuset: RefCount + 1 and the pod's
// exclusive policy on every taken CPU
void kg_cpuset_apply(const kg_pod_dev &p, kg_cpu_info *cpus, int32_t n, const uint8_t *taken) {
    const int excl = (p.flags & KG_POD_NUMA_CPU_BIND) ? (int)((p.cpu_bind >> 8) & 15u) : KG_CPU_EXCL_UNSET;
    for (int32_t k = 0; k < n; k++)
        if (taken[k]) {
            cpus[k].refcount++;
            cpus[k].exclusive = excl;
        }
}

// the accumulator's strategy for a node: its label, else the plugin default (util.go:27-41); only
// NUMAMostAllocated changes the orderings (cpu_accumulator.go:434-733)
int32_t kg_cpuset_strategy(const kg_config &cfg, int32_t label) {
    if (label == KG_NUMA_ALLOC_MOST) return KG_STRATEGY_MOST_ALLOCATED;
    if (label == KG_NUMA_ALLOC_LEAST || label == KG_NUMA_ALLOC_DISTRIBUTE_EVENLY) return KG_STRATEGY_LEAST_ALLOCATED;
    return cfg.numa_hint_strategy == KG_STRATEGY_MOST_ALLOCATED ? KG_STRATEGY_MOST_ALLOCATED : KG_STRATEGY_LEAST_ALLOCATED;
}

extern "C" kg_status kg_cpuset_take(const kg_cpu_info *cpus, int32_t n_cpus, int32_t max_ref_count,
                                    const uint8_t *available, int32_t need, int32_t bind_policy,
                                    int32_t exclusive_policy, int32_t numa_strategy, uint8_t *result) {
    if (!cpus || !available || !result || n_cpus <= 0 || n_cpus > KG_MAX_NODE_CPUS || need < 0)
        return KG_ERR_INVALID_ARG;
    return kg_cpuset_take_cpus(cpus, n_cpus, max_ref_count > 0 ? max_ref_count : 1, available, need, bind_policy,
                               exclusive_policy, numa_strategy, result) == 0
               ? KG_OK
               : KG_NOT_FOUND;
}
