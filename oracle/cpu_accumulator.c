/*
 * cpu_accumulator.c — CPU restatement of NodeNUMAResource's cpuset take (the "later" row of SURVEY §8:
 * cpuset binding of LSE / LSR prod pods).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker of the engine's cpuset path; only tests/ load it.
 *
 * Follows the reference object by object:
 *   takePreferredCPUs / takeCPUs        nodenumaresource/cpu_accumulator.go:29-232
 *   cpuAccumulator (take, needs, the free-core / free-CPU orderings, spreadCPUs)
 *                                        cpu_accumulator.go:234-822
 *   NodeAllocation.getAvailableCPUs     node_allocation.go:134-155 (allocated = refcount ≥ maxRefCount)
 *   filterCPUsByRequiredCPUBindPolicy   resource_manager.go:534-566
 *   satisfiedRequiredCPUBindPolicy      resource_manager.go:568-589
 * Go maps become arrays indexed by dense CPU ids and by compact core / node / socket indices; every
 * sort the reference does with a total order is a qsort here, and the one sort without a tie-break
 * (cpu_accumulator.go:142 / :161, ≤ a handful of sockets, which Go's pdqsort insertion-sorts, i.e.
 * stably) is a stable insertion sort.  Parity is pinned by cpu_accumulator_test.go's cases
 * (tests/golden/cpu_accumulator_kat.json).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KGO_MAX_CPUS 1024

enum { BIND_NONE = 0, BIND_FULL_PCPUS = 1, BIND_SPREAD_BY_PCPUS = 2 };
enum { EXCL_NONE = 0, EXCL_PCPU = 1, EXCL_NUMA = 2 };
enum { STRATEGY_LEAST = 0, STRATEGY_MOST = 1 };

/* CPUTopology (cpu_topology.go): cpu id → socket, NUMA node, core (ids as reported) */
typedef struct kgo_cpu_topo {
    int32_t n_cpus;            /* cpu ids 0..n_cpus-1 present */
    const int32_t *socket, *node, *core;
} kgo_cpu_topo;

typedef struct {
    const kgo_cpu_topo *t;
    int ncores, nnodes, nsockets;       /* distinct ids */
    int cpus_per_core, cpus_per_node, cpus_per_socket;
    int core_ix[KGO_MAX_CPUS], node_ix[KGO_MAX_CPUS], sock_ix[KGO_MAX_CPUS];   /* compact indices per cpu */
    int core_id[KGO_MAX_CPUS], node_id[KGO_MAX_CPUS], sock_id[KGO_MAX_CPUS];   /* compact index → id */
} topo_t;

static int find_or_add(int *ids, int *n, int id) {
    for (int i = 0; i < *n; i++)
        if (ids[i] == id) return i;
    ids[*n] = id;
    return (*n)++;
}

static void topo_init(topo_t *T, const kgo_cpu_topo *t) {
    memset(T, 0, sizeof(*T));
    T->t = t;
    for (int c = 0; c < t->n_cpus; c++) {
        T->core_ix[c] = find_or_add(T->core_id, &T->ncores, t->core[c]);
        T->node_ix[c] = find_or_add(T->node_id, &T->nnodes, t->node[c]);
        T->sock_ix[c] = find_or_add(T->sock_id, &T->nsockets, t->socket[c]);
    }
    T->cpus_per_core = T->ncores ? t->n_cpus / T->ncores : 0;       /* CPUsPerCore */
    T->cpus_per_node = T->nnodes ? t->n_cpus / T->nnodes : 0;       /* CPUsPerNode */
    T->cpus_per_socket = T->nsockets ? t->n_cpus / T->nsockets : 0; /* CPUsPerSocket */
}

/* ordered groups of cpu lists ([][]int) */
typedef struct {
    int n;
    int start[KGO_MAX_CPUS + 1];
    int cpus[KGO_MAX_CPUS];
} groups_t;

typedef struct {
    const topo_t *T;
    int max_ref;
    uint8_t avail[KGO_MAX_CPUS];         /* allocatableCPUs */
    int32_t ref[KGO_MAX_CPUS];           /* RefCount of allocatable cpus (maxRefCount > 1) */
    uint8_t excl_core[KGO_MAX_CPUS];     /* exclusiveInCores (compact core index) */
    uint8_t excl_node[KGO_MAX_CPUS];     /* exclusiveInNUMANodes (compact node index) */
    int exclusive, excl_policy, strategy;
    int need;
    uint8_t result[KGO_MAX_CPUS];
} acc_t;

static int n_avail(const acc_t *a) {
    int n = 0;
    for (int c = 0; c < a->T->t->n_cpus; c++) n += a->avail[c];
    return n;
}
static int needs(const acc_t *a, int n) { return a->need >= n; }
static int satisfied(const acc_t *a) { return a->need < 1; }

static void take(acc_t *a, const int *cpus, int n) {
    for (int i = 0; i < n; i++) {
        const int c = cpus[i];
        a->result[c] = 1;
        a->avail[c] = 0;
        if (a->exclusive) {
            if (a->excl_policy == EXCL_PCPU) a->excl_core[a->T->core_ix[c]] = 1;
            else if (a->excl_policy == EXCL_NUMA) a->excl_node[a->T->node_ix[c]] = 1;
        }
    }
    a->need -= n;
}

static int excl_pcpu(const acc_t *a, int c) { return a->excl_policy == EXCL_PCPU && a->excl_core[a->T->core_ix[c]]; }
static int excl_numa(const acc_t *a, int c) { return a->excl_policy == EXCL_NUMA && a->excl_node[a->T->node_ix[c]]; }

/* ---- sort helpers (comparators read a file-scope context: the oracle is single-threaded per call) ---- */
static __thread const acc_t *g_acc;
static __thread const int *g_key1, *g_key2;   /* per compact index */
static __thread int g_most;

static int core_refcount(const acc_t *a, int core_ix) {   /* getCoreRefCount over allocatableCPUs */
    int r = 0;
    for (int c = 0; c < a->T->t->n_cpus; c++)
        if (a->avail[c] && a->T->core_ix[c] == core_ix) r += a->ref[c];
    return r;
}

static int cmp_int(const void *x, const void *y) { return *(const int *)x - *(const int *)y; }

static int cmp_cpu_ref(const void *x, const void *y) {   /* sortCPUsByRefCount */
    const int i = *(const int *)x, j = *(const int *)y;
    if (g_acc->ref[i] != g_acc->ref[j]) return g_acc->ref[i] < g_acc->ref[j] ? -1 : 1;
    return i - j;
}

static void sort_cpus(const acc_t *a, int *cpus, int n) {
    qsort(cpus, n, sizeof(int), cmp_int);
    if (a->max_ref > 1) {
        g_acc = a;
        qsort(cpus, n, sizeof(int), cmp_cpu_ref);
    }
}

/* sortCores: count desc, refcount asc (maxRefCount > 1), core id asc.  g_key1 = cpus per core index */
static int cmp_core(const void *x, const void *y) {
    const int i = *(const int *)x, j = *(const int *)y;
    if (g_key1[i] != g_key1[j]) return g_key1[i] > g_key1[j] ? -1 : 1;
    if (g_acc->max_ref > 1) {
        const int ri = core_refcount(g_acc, i), rj = core_refcount(g_acc, j);
        if (ri != rj) return ri < rj ? -1 : 1;
    }
    return g_acc->T->core_id[i] < g_acc->T->core_id[j] ? -1 : g_acc->T->core_id[i] > g_acc->T->core_id[j];
}

/* a free-score comparison: NUMAMostAllocated ascending, otherwise descending */
static int by_free(int x, int y) {
    if (x == y) return 0;
    return g_most ? (x < y ? -1 : 1) : (x > y ? -1 : 1);
}

/* node groups: key1 = node free score, key2 = socket free score of the node (by compact node index) */
static int cmp_node(const void *x, const void *y) {
    const int i = *(const int *)x, j = *(const int *)y;
    int r = by_free(g_key1[i], g_key1[j]);
    if (r) return r;
    r = by_free(g_key2[i], g_key2[j]);
    if (r) return r;
    return g_acc->T->node_id[i] < g_acc->T->node_id[j] ? -1 : g_acc->T->node_id[i] > g_acc->T->node_id[j];
}

static int cmp_socket(const void *x, const void *y) {
    const int i = *(const int *)x, j = *(const int *)y;
    const int r = by_free(g_key1[i], g_key1[j]);
    if (r) return r;
    return g_acc->T->sock_id[i] < g_acc->T->sock_id[j] ? -1 : g_acc->T->sock_id[i] > g_acc->T->sock_id[j];
}

/* cpus of each core (compact index) among the allocatable cpus passing `skip` */
typedef int (*skip_fn)(const acc_t *, int);
static int skip_none(const acc_t *a, int c) { (void)a; (void)c; return 0; }
static int skip_numa(const acc_t *a, int c) { return excl_numa(a, c); }
static int skip_pcpu(const acc_t *a, int c) { return excl_pcpu(a, c); }
static int skip_both(const acc_t *a, int c) { return excl_pcpu(a, c) || excl_numa(a, c); }

/* freeCoresInNode (level 0) / freeCoresInSocket (level 1): logical cpus of the (full-)free cores,
 * grouped by NUMA node / socket, cores sorted by sortCores, groups by free scores */
static void free_cores_in(const acc_t *a, int level, int full_only, skip_fn skip, groups_t *out) {
    const topo_t *T = a->T;
    const int n = T->t->n_cpus;
    static __thread int core_cnt[KGO_MAX_CPUS], sock_free[KGO_MAX_CPUS], grp_len[KGO_MAX_CPUS], sock_of_grp[KGO_MAX_CPUS];
    static __thread int cores_of[KGO_MAX_CPUS], ncores_of[KGO_MAX_CPUS], order[KGO_MAX_CPUS];
    memset(core_cnt, 0, sizeof(int) * T->ncores);
    memset(sock_free, 0, sizeof(int) * T->nsockets);
    for (int c = 0; c < n; c++) {
        if (!a->avail[c] || skip(a, c)) continue;
        core_cnt[T->core_ix[c]]++;
        sock_free[T->sock_ix[c]]++;
    }
    const int ng = level == 0 ? T->nnodes : T->nsockets;
    memset(grp_len, 0, sizeof(int) * ng);
    memset(ncores_of, 0, sizeof(int) * ng);
    /* the group of a core = group of its cpus (a core's cpus share node and socket) */
    int core_grp[KGO_MAX_CPUS];
    for (int k = 0; k < T->ncores; k++) core_grp[k] = -1;
    for (int c = 0; c < n; c++)
        if (a->avail[c] && !skip(a, c)) {
            core_grp[T->core_ix[c]] = level == 0 ? T->node_ix[c] : T->sock_ix[c];
            if (level == 0) sock_of_grp[T->node_ix[c]] = T->sock_ix[c];
        }
    /* per group: its cores (compact), in any order; sorted below */
    static __thread int members[KGO_MAX_CPUS * 2];
    int pos = 0;
    for (int g = 0; g < ng; g++) {
        cores_of[g] = pos;
        for (int k = 0; k < T->ncores; k++) {
            if (core_grp[k] != g || core_cnt[k] == 0) continue;
            if (full_only && core_cnt[k] != T->cpus_per_core) continue;
            members[pos++] = k;
            ncores_of[g]++;
            grp_len[g] += core_cnt[k];
        }
    }
    g_acc = a;
    g_key1 = core_cnt;
    for (int g = 0; g < ng; g++) qsort(members + cores_of[g], ncores_of[g], sizeof(int), cmp_core);
    int m = 0;
    for (int g = 0; g < ng; g++)
        if (ncores_of[g] > 0) order[m++] = g;
    g_most = a->strategy == STRATEGY_MOST;
    if (level == 0) {
        static __thread int sock_free_of_node[KGO_MAX_CPUS];
        for (int g = 0; g < ng; g++) sock_free_of_node[g] = sock_free[sock_of_grp[g]];
        g_key1 = grp_len;
        g_key2 = sock_free_of_node;
        qsort(order, m, sizeof(int), cmp_node);
    } else {
        g_key1 = grp_len;
        qsort(order, m, sizeof(int), cmp_socket);
    }
    out->n = 0;
    int w = 0;
    for (int oi = 0; oi < m; oi++) {
        const int g = order[oi];
        out->start[out->n++] = w;
        for (int q = 0; q < ncores_of[g]; q++) {
            const int k = members[cores_of[g] + q];
            const int first = w;
            for (int c = 0; c < n; c++)
                if (a->avail[c] && !skip(a, c) && T->core_ix[c] == k) out->cpus[w++] = c;
            qsort(out->cpus + first, w - first, sizeof(int), cmp_int);   /* sort.Ints(cpus) */
        }
    }
    out->start[out->n] = w;
}

/* extractCPU: the first cpu of each core, in list order */
static int extract_cpu(const acc_t *a, int *cpus, int n) {
    static __thread uint8_t seen[KGO_MAX_CPUS];
    memset(seen, 0, (size_t)a->T->ncores);
    int w = 0;
    for (int i = 0; i < n; i++) {
        const int k = a->T->core_ix[cpus[i]];
        if (seen[k]) continue;
        seen[k] = 1;
        cpus[w++] = cpus[i];
    }
    return w;
}

/* freeCPUsInNode (level 0) / freeCPUsInSocket (level 1) */
static void free_cpus_in(const acc_t *a, int level, int filter_excl, groups_t *out) {
    const topo_t *T = a->T;
    const int n = T->t->n_cpus;
    const skip_fn skip = !filter_excl ? skip_none : level == 0 ? skip_both : skip_pcpu;
    static __thread int node_free[KGO_MAX_CPUS], sock_free[KGO_MAX_CPUS], sock_of[KGO_MAX_CPUS], len[KGO_MAX_CPUS];
    static __thread int order[KGO_MAX_CPUS], buf[KGO_MAX_CPUS], bstart[KGO_MAX_CPUS + 1];
    const int ng = level == 0 ? T->nnodes : T->nsockets;
    memset(node_free, 0, sizeof(int) * T->nnodes);
    memset(sock_free, 0, sizeof(int) * T->nsockets);
    for (int c = 0; c < n; c++) {
        if (!a->avail[c] || skip(a, c)) continue;
        node_free[T->node_ix[c]]++;
        sock_free[T->sock_ix[c]]++;
        if (level == 0) sock_of[T->node_ix[c]] = T->sock_ix[c];
    }
    int w = 0, m = 0;
    for (int g = 0; g < ng; g++) {
        bstart[g] = w;
        for (int c = 0; c < n; c++)
            if (a->avail[c] && !skip(a, c) && (level == 0 ? T->node_ix[c] : T->sock_ix[c]) == g) buf[w++] = c;
        sort_cpus(a, buf + bstart[g], w - bstart[g]);
        int l = w - bstart[g];
        if (filter_excl) l = extract_cpu(a, buf + bstart[g], l);
        w = bstart[g] + l;
        len[g] = l;
        if (l > 0) order[m++] = g;
    }
    bstart[ng] = w;
    g_acc = a;
    g_most = a->strategy == STRATEGY_MOST;
    if (level == 0) {
        static __thread int sf[KGO_MAX_CPUS];
        for (int g = 0; g < ng; g++) sf[g] = sock_free[sock_of[g]];
        g_key1 = node_free;     /* counted before extractCPU (cpu_accumulator.go:544, :575) */
        g_key2 = sf;
        qsort(order, m, sizeof(int), cmp_node);
    } else {
        g_key1 = len;           /* len(cpusInSockets) after extractCPU (:637) */
        qsort(order, m, sizeof(int), cmp_socket);
    }
    out->n = 0;
    int o = 0;
    for (int oi = 0; oi < m; oi++) {
        const int g = order[oi];
        out->start[out->n++] = o;
        memcpy(out->cpus + o, buf + bstart[g], sizeof(int) * len[g]);
        o += len[g];
    }
    out->start[out->n] = o;
}

/* freeCPUs: cores sorted by result colocation of their socket, socket / node free scores, core free
 * count, socket, refcount, core id; each core's cpus ascending (then by refcount) */
static __thread int *g_colo, *g_sfree, *g_nfree, *g_ccnt, *g_csock, *g_cnode;
static int cmp_free_core(const void *x, const void *y) {
    const int i = *(const int *)x, j = *(const int *)y;
    const int si = g_csock[i], sj = g_csock[j];
    if (g_colo[si] != g_colo[sj]) return g_colo[si] > g_colo[sj] ? -1 : 1;
    int r = by_free(g_sfree[si], g_sfree[sj]);
    if (r) return r;
    r = by_free(g_nfree[g_cnode[i]], g_nfree[g_cnode[j]]);
    if (r) return r;
    if (g_ccnt[i] != g_ccnt[j]) return g_ccnt[i] < g_ccnt[j] ? -1 : 1;
    const int sid_i = g_acc->T->sock_id[si], sid_j = g_acc->T->sock_id[sj];
    if (sid_i != sid_j) return sid_i < sid_j ? -1 : 1;
    if (g_acc->max_ref > 1) {
        const int ri = core_refcount(g_acc, i), rj = core_refcount(g_acc, j);
        if (ri != rj) return ri < rj ? -1 : 1;
    }
    return g_acc->T->core_id[i] < g_acc->T->core_id[j] ? -1 : g_acc->T->core_id[i] > g_acc->T->core_id[j];
}

static int free_cpus(const acc_t *a, int filter_excl, int *out) {
    const topo_t *T = a->T;
    const int n = T->t->n_cpus;
    const skip_fn skip = filter_excl ? skip_both : skip_none;
    static __thread int colo[KGO_MAX_CPUS], sfree[KGO_MAX_CPUS], nfree[KGO_MAX_CPUS], ccnt[KGO_MAX_CPUS];
    static __thread int csock[KGO_MAX_CPUS], cnode[KGO_MAX_CPUS], cores[KGO_MAX_CPUS];
    memset(sfree, 0, sizeof(int) * T->nsockets);
    memset(nfree, 0, sizeof(int) * T->nnodes);
    memset(ccnt, 0, sizeof(int) * T->ncores);
    memset(colo, 0, sizeof(int) * T->nsockets);
    for (int c = 0; c < n; c++) {
        if (!a->avail[c] || skip(a, c)) continue;
        ccnt[T->core_ix[c]]++;
        csock[T->core_ix[c]] = T->sock_ix[c];
        cnode[T->core_ix[c]] = T->node_ix[c];
        nfree[T->node_ix[c]]++;
        sfree[T->sock_ix[c]]++;
    }
    for (int c = 0; c < n; c++)   /* CPUsInSockets(socket) ∩ result */
        if (a->result[c]) colo[T->sock_ix[c]]++;
    int m = 0;
    for (int k = 0; k < T->ncores; k++)
        if (ccnt[k] > 0) cores[m++] = k;
    g_acc = a;
    g_most = a->strategy == STRATEGY_MOST;
    g_colo = colo, g_sfree = sfree, g_nfree = nfree, g_ccnt = ccnt, g_csock = csock, g_cnode = cnode;
    qsort(cores, m, sizeof(int), cmp_free_core);
    int w = 0;
    for (int q = 0; q < m; q++) {
        const int first = w;
        for (int c = 0; c < n; c++)
            if (a->avail[c] && !skip(a, c) && T->core_ix[c] == cores[q]) out[w++] = c;
        sort_cpus(a, out + first, w - first);
    }
    return w;
}

/* spreadCPUs: round-robin over cores, one cpu per core per pass, in list order */
static int spread_cpus(const acc_t *a, int *cpus, int n) {
    if (n <= a->T->cpus_per_core) return n;
    static __thread int prep[KGO_MAX_CPUS], res[KGO_MAX_CPUS], rest[KGO_MAX_CPUS];
    static __thread uint8_t seen[KGO_MAX_CPUS];
    memcpy(prep, cpus, sizeof(int) * n);
    int np = n, w = 0;
    while (np > 0) {
        memset(seen, 0, (size_t)a->T->ncores);
        int nr = 0;
        for (int i = 0; i < np; i++) {
            const int k = a->T->core_ix[prep[i]];
            if (seen[k]) {
                rest[nr++] = prep[i];
                continue;
            }
            res[w++] = prep[i];
            seen[k] = 1;
        }
        memcpy(prep, rest, sizeof(int) * nr);
        np = nr;
    }
    memcpy(cpus, res, sizeof(int) * n);
    return n;
}

/* stable insertion sort of group indices by group length (desc / asc) */
static void sort_groups_by_len(const groups_t *g, int *idx, int m, int desc) {
    for (int i = 1; i < m; i++) {
        const int v = idx[i];
        const int lv = g->start[v + 1] - g->start[v];
        int j = i - 1;
        while (j >= 0) {
            const int lj = g->start[idx[j] + 1] - g->start[idx[j]];
            if (desc ? lj < lv : lj > lv) {
                idx[j + 1] = idx[j];
                j--;
            } else
                break;
        }
        idx[j + 1] = v;
    }
}

/* takeCPUs (cpu_accumulator.go:87-232).  available / result: per cpu id; alloc_ref / alloc_excl: the
 * node's allocated CPU details (RefCount, ExclusivePolicy; alloc_excl is set only for allocated cpus).
 * Returns 0 on success, −1 on failure. */
int kgo_take_cpus(const kgo_cpu_topo *topo, int max_ref, const uint8_t *available, const int32_t *alloc_ref,
                  const int8_t *alloc_excl, int need, int bind, int excl_policy, int strategy, uint8_t *result) {
    static __thread topo_t T;
    static __thread acc_t A;
    static __thread groups_t G;
    static __thread int list[KGO_MAX_CPUS];
    if (topo->n_cpus > KGO_MAX_CPUS) return -2;
    topo_init(&T, topo);
    acc_t *a = &A;
    memset(a, 0, sizeof(*a));
    a->T = &T;
    a->max_ref = max_ref;
    a->need = need;
    a->excl_policy = excl_policy;
    a->strategy = strategy;
    a->exclusive = excl_policy == EXCL_PCPU || excl_policy == EXCL_NUMA;
    for (int c = 0; c < topo->n_cpus; c++) {
        a->avail[c] = available[c] != 0;
        if (max_ref > 1) a->ref[c] = alloc_ref ? alloc_ref[c] : 0;
        if (alloc_excl) {   /* allocatedCPUs entries (CPUDetails of the node allocation) */
            if (alloc_excl[c] == EXCL_PCPU) a->excl_core[T.core_ix[c]] = 1;
            else if (alloc_excl[c] == EXCL_NUMA) a->excl_node[T.node_ix[c]] = 1;
        }
    }
    memset(result, 0, (size_t)topo->n_cpus);
#define DONE()                                                 \
    do {                                                       \
        memcpy(result, a->result, (size_t)topo->n_cpus);       \
        return 0;                                              \
    } while (0)
    if (satisfied(a)) DONE();
    if (a->need > n_avail(a)) return -1;
    const int full = bind == BIND_FULL_PCPUS;
    if (full || T.cpus_per_core == 1) {
        if (a->need <= T.cpus_per_node) {
            for (int fe = 1; fe >= 0; fe--) {
                free_cores_in(a, 0, 1, fe ? skip_numa : skip_none, &G);
                for (int g = 0; g < G.n; g++)
                    if (G.start[g + 1] - G.start[g] >= a->need) {
                        take(a, G.cpus + G.start[g], a->need);
                        DONE();
                    }
            }
        }
        if (a->need <= T.cpus_per_socket) {
            free_cores_in(a, 1, 1, skip_none, &G);
            for (int g = 0; g < G.n; g++)
                if (G.start[g + 1] - G.start[g] >= a->need) {
                    take(a, G.cpus + G.start[g], a->need);
                    DONE();
                }
        }
        free_cores_in(a, 1, 1, skip_none, &G);
        int idx[KGO_MAX_CPUS], unsat[KGO_MAX_CPUS], nu = 0;
        for (int g = 0; g < G.n; g++) idx[g] = g;
        sort_groups_by_len(&G, idx, G.n, 1);
        for (int q = 0; q < G.n; q++) {
            const int g = idx[q], len = G.start[g + 1] - G.start[g];
            if (!needs(a, len)) {
                unsat[nu++] = g;
            } else {
                take(a, G.cpus + G.start[g], len);
                if (satisfied(a)) DONE();
            }
        }
        if (needs(a, T.cpus_per_core)) {
            sort_groups_by_len(&G, unsat, nu, 0);
            const int cpc = T.cpus_per_core;
            for (int q = 0; q < nu; q++) {
                const int g = unsat[q], len = G.start[g + 1] - G.start[g];
                for (int i = 0; i < len; i += cpc) {
                    take(a, G.cpus + G.start[g] + i, cpc);
                    if (satisfied(a)) DONE();
                    if (!needs(a, cpc)) break;
                }
            }
        }
    }
    if (!full) {
        if (a->need <= T.cpus_per_node) {
            for (int fe = 1; fe >= 0; fe--) {
                free_cpus_in(a, 0, fe, &G);
                for (int g = 0; g < G.n; g++) {
                    const int len = G.start[g + 1] - G.start[g];
                    if (len >= a->need) {
                        memcpy(list, G.cpus + G.start[g], sizeof(int) * len);
                        spread_cpus(a, list, len);
                        take(a, list, a->need);
                        DONE();
                    }
                }
            }
        }
        if (a->need <= T.cpus_per_socket) {
            for (int fe = 1; fe >= 0; fe--) {
                free_cpus_in(a, 1, fe, &G);
                for (int g = 0; g < G.n; g++) {
                    const int len = G.start[g + 1] - G.start[g];
                    if (len >= a->need) {
                        memcpy(list, G.cpus + G.start[g], sizeof(int) * len);
                        spread_cpus(a, list, len);
                        take(a, list, a->need);
                        DONE();
                    }
                }
            }
        }
    }
    for (int fe = 1; fe >= 0; fe--) {
        const int len = free_cpus(a, fe, list);
        spread_cpus(a, list, len);
        for (int i = 0; i < len; i++) {
            if (needs(a, 1)) take(a, list + i, 1);
            if (satisfied(a)) DONE();
        }
    }
#undef DONE
    return -1;
}

/* takePreferredCPUs (cpu_accumulator.go:29-85) */
int kgo_take_preferred_cpus(const kgo_cpu_topo *topo, int max_ref, const uint8_t *available, const uint8_t *preferred,
                            const int32_t *alloc_ref, const int8_t *alloc_excl, int need, int bind, int excl_policy,
                            int strategy, uint8_t *result) {
    const int n = topo->n_cpus;
    if (n > KGO_MAX_CPUS) return -2;
    uint8_t pref[KGO_MAX_CPUS], avail[KGO_MAX_CPUS], part[KGO_MAX_CPUS];
    int npref = 0;
    for (int c = 0; c < n; c++) {
        pref[c] = available[c] && preferred && preferred[c];
        npref += pref[c];
        avail[c] = available[c] != 0;
    }
    memset(result, 0, (size_t)n);
    if (npref > 0) {
        const int needed = need > npref ? npref : need;
        if (kgo_take_cpus(topo, max_ref, pref, alloc_ref, alloc_excl, needed, bind, excl_policy, strategy, part) != 0)
            return -1;
        for (int c = 0; c < n; c++) {
            result[c] |= part[c];
            need -= part[c];
            if (pref[c]) avail[c] = 0;
        }
    }
    if (need > 0) {
        if (kgo_take_cpus(topo, max_ref, avail, alloc_ref, alloc_excl, need, bind, excl_policy, strategy, part) != 0) {
            memset(result, 0, (size_t)n);
            return -1;
        }
        for (int c = 0; c < n; c++) result[c] |= part[c];
    }
    return 0;
}

/* NodeAllocation.getAvailableCPUs (node_allocation.go:134-155): a cpu is allocated once its refcount
 * (less one per preferred cpu it holds) reaches maxRefCount; reserved cpus are never available */
void kgo_available_cpus(const kgo_cpu_topo *topo, int max_ref, const int32_t *alloc_ref, const uint8_t *reserved,
                        const uint8_t *preferred, uint8_t *available, int32_t *ref_out) {
    for (int c = 0; c < topo->n_cpus; c++) {
        int32_t r = alloc_ref ? alloc_ref[c] : 0;
        if (preferred && preferred[c] && r > 0) r--;
        if (ref_out) ref_out[c] = r;
        available[c] = !(r > 0 && r >= max_ref) && !(reserved && reserved[c]);
    }
}

/* filterCPUsByRequiredCPUBindPolicy (resource_manager.go:534-566): FullPCPUs keeps the cpus of cores
 * whose every cpu is available; SpreadByPCPUs keeps the first (lowest) available cpu of each core */
void kgo_filter_required_bind(const kgo_cpu_topo *topo, int bind, uint8_t *available) {
    static __thread topo_t T;
    topo_init(&T, topo);
    const int n = topo->n_cpus;
    int cnt[KGO_MAX_CPUS] = {0}, first[KGO_MAX_CPUS];
    for (int k = 0; k < T.ncores; k++) first[k] = -1;
    for (int c = 0; c < n; c++)
        if (available[c]) {
            cnt[T.core_ix[c]]++;
            if (first[T.core_ix[c]] < 0) first[T.core_ix[c]] = c;
        }
    for (int c = 0; c < n; c++) {
        if (!available[c]) continue;
        if (bind == BIND_FULL_PCPUS) available[c] = cnt[T.core_ix[c]] == T.cpus_per_core;
        else if (bind == BIND_SPREAD_BY_PCPUS) available[c] = first[T.core_ix[c]] == c;
    }
}

/* satisfiedRequiredCPUBindPolicy (resource_manager.go:568-589) */
int kgo_satisfied_required_bind(const kgo_cpu_topo *topo, int bind, const uint8_t *cpus) {
    static __thread topo_t T;
    topo_init(&T, topo);
    uint8_t seen[KGO_MAX_CPUS] = {0};
    int ncpu = 0, ncore = 0;
    for (int c = 0; c < topo->n_cpus; c++)
        if (cpus[c]) {
            ncpu++;
            if (!seen[T.core_ix[c]]) {
                seen[T.core_ix[c]] = 1;
                ncore++;
            }
        }
    if (bind == BIND_FULL_PCPUS) return ncore * T.cpus_per_core == ncpu;
    if (bind == BIND_SPREAD_BY_PCPUS) return ncore == ncpu;
    return 1;
}
