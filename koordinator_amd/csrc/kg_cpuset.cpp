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
