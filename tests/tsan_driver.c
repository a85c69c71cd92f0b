/* ThreadSanitizer driver for the oracle's threaded CPU baselines (tests/test_tsan_cpu.py): reads a cluster view
 * dumped by the test (config, the view's ten arrays, the pod queue, now), runs the Parallelizer restatements
 * (kgo_eval_parallel, kgo_schedule_parallel) and the threaded Reservation + ElasticQuota cycle
 * (kgo_schedule2_parallel) on 8 threads and checks them against the sequential cycle (kgo_eval_matrix5's top-1,
 * kgo_schedule, kgo_schedule2).  Built with -fsanitize=thread together with the oracle sources;
 * test infrastructure only. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "koord_gpu.h"

int kgo_eval_parallel(const kg_config *c, const kg_cluster_view *v, const int32_t *pod_index, int32_t P, int64_t now_ns,
                      int32_t workers, uint64_t *top1);
int kgo_eval_matrix5(const kg_config *c, const kg_cluster_view *v, const int32_t *pod_index, int32_t P, int64_t now_ns,
                     uint8_t *mask, uint8_t *fit, uint8_t *la, uint8_t *numa, uint8_t *rsv, uint64_t *top1);
int kgo_schedule(const kg_config *c, const kg_cluster_view *v, const int32_t *pod_index, int32_t P, int64_t now_ns,
                 int32_t *out_node, int64_t *out_score);
int kgo_schedule_parallel(const kg_config *c, const kg_cluster_view *v, const int32_t *pod_index, int32_t P,
                          int64_t now_ns, int32_t workers, int32_t *out_node, int64_t *out_score);
int kgo_schedule2(const kg_config *c, const kg_cluster_view *v, const int32_t *pod_index, int32_t P, int64_t now_ns,
                  int32_t *out_node, int64_t *out_score, kg_reservation *out_rsv, kg_quota *out_quota);
int kgo_schedule2_parallel(const kg_config *c, const kg_cluster_view *v, const int32_t *pod_index, int32_t P,
                           int64_t now_ns, int32_t workers, int32_t *out_node, int64_t *out_score,
                           kg_reservation *out_rsv, kg_quota *out_quota);

static void *chunk(FILE *f, int64_t elem, int64_t *count) {
    int64_t hdr[2];
    if (fread(hdr, sizeof(hdr), 1, f) != 1) exit(3);
    if (hdr[0] != elem) {
        fprintf(stderr, "element size %lld, expected %lld\n", (long long)hdr[0], (long long)elem);
        exit(4);
    }
    *count = hdr[1];
    void *p = calloc((size_t)(hdr[1] > 0 ? hdr[1] : 1), (size_t)elem);
    if (hdr[1] > 0 && fread(p, (size_t)elem, (size_t)hdr[1], f) != (size_t)hdr[1]) exit(5);
    return p;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    int64_t n;
    kg_config *cfg = (kg_config *)chunk(f, sizeof(kg_config), &n);
    kg_cluster_view v;
    memset(&v, 0, sizeof(v));
    v.pods = (const kg_pod_spec *)chunk(f, sizeof(kg_pod_spec), &n), v.n_pods = (int32_t)n;
    v.containers = (const kg_container *)chunk(f, sizeof(kg_container), &n), v.n_containers = (int32_t)n;
    v.nodes = (const kg_node_spec *)chunk(f, sizeof(kg_node_spec), &n), v.n_nodes = (int32_t)n;
    v.aggregated = (const kg_aggregated_usage *)chunk(f, sizeof(kg_aggregated_usage), &n), v.n_aggregated = (int32_t)n;
    v.pod_metrics = (const kg_pod_metric *)chunk(f, sizeof(kg_pod_metric), &n), v.n_pod_metrics = (int32_t)n;
    v.assigned = (const kg_assigned_pod *)chunk(f, sizeof(kg_assigned_pod), &n), v.n_assigned = (int32_t)n;
    v.numa = (const kg_numa_spec *)chunk(f, sizeof(kg_numa_spec), &n), v.n_numa = (int32_t)n;
    v.reservations = (const kg_reservation *)chunk(f, sizeof(kg_reservation), &n), v.n_reservations = (int32_t)n;
    v.quotas = (const kg_quota *)chunk(f, sizeof(kg_quota), &n), v.n_quotas = (int32_t)n;
    v.cpus = (const kg_cpu_info *)chunk(f, sizeof(kg_cpu_info), &n), v.n_cpus = (int32_t)n;
    int64_t P;
    const int32_t *idx = (const int32_t *)chunk(f, sizeof(int32_t), &P);
    int64_t one;
    const int64_t *now = (const int64_t *)chunk(f, sizeof(int64_t), &one);
    fclose(f);
    const int64_t N = v.n_nodes;
    // the Parallelizer baselines restate the Fit / LoadAware / NodeNUMAResource profiles (bench configs 2 and 3);
    // a view with reservations or quota groups is checked through the Reservation + ElasticQuota cycle only
    const int rsv_quota = v.n_reservations > 0 || v.n_quotas > 0;
    uint64_t *top_par = calloc((size_t)P, 8), *top_seq = calloc((size_t)P, 8);
    uint8_t *planes = calloc((size_t)(P * N * 5), 1);
    if (!rsv_quota && kgo_eval_parallel(cfg, &v, idx, (int32_t)P, *now, 8, top_par) != 0) return 6;
    if (kgo_eval_matrix5(cfg, &v, idx, (int32_t)P, *now, planes, planes + P * N, planes + 2 * P * N, planes + 3 * P * N,
                         planes + 4 * P * N, top_seq) != 0)
        return 7;
    if (!rsv_quota && memcmp(top_par, top_seq, (size_t)P * 8) != 0) {
        fprintf(stderr, "kgo_eval_parallel differs from the sequential top-1\n");
        return 8;
    }
    int32_t *node_par = calloc((size_t)P, 4), *node_seq = calloc((size_t)P, 4);
    int64_t *score_par = calloc((size_t)P, 8), *score_seq = calloc((size_t)P, 8);
    if (!rsv_quota && kgo_schedule_parallel(cfg, &v, idx, (int32_t)P, *now, 8, node_par, score_par) != 0) return 9;
    if (!rsv_quota && kgo_schedule(cfg, &v, idx, (int32_t)P, *now, node_seq, score_seq) != 0) return 10;
    if (!rsv_quota && (memcmp(node_par, node_seq, (size_t)P * 4) != 0 || memcmp(score_par, score_seq, (size_t)P * 8) != 0)) {
        fprintf(stderr, "kgo_schedule_parallel differs from the sequential cycle\n");
        return 11;
    }
    const size_t nr = (size_t)(v.n_reservations > 0 ? v.n_reservations : 1), nq = (size_t)(v.n_quotas > 0 ? v.n_quotas : 1);
    kg_reservation *rsv_par = calloc(nr, sizeof(kg_reservation)), *rsv_seq = calloc(nr, sizeof(kg_reservation));
    kg_quota *q_par = calloc(nq, sizeof(kg_quota)), *q_seq = calloc(nq, sizeof(kg_quota));
    if (kgo_schedule2_parallel(cfg, &v, idx, (int32_t)P, *now, 8, node_par, score_par, v.n_reservations ? rsv_par : NULL,
                               v.n_quotas ? q_par : NULL) != 0)
        return 12;
    if (kgo_schedule2(cfg, &v, idx, (int32_t)P, *now, node_seq, score_seq, v.n_reservations ? rsv_seq : NULL,
                      v.n_quotas ? q_seq : NULL) != 0)
        return 13;
    if (memcmp(node_par, node_seq, (size_t)P * 4) != 0 || memcmp(score_par, score_seq, (size_t)P * 8) != 0 ||
        memcmp(rsv_par, rsv_seq, nr * sizeof(kg_reservation)) != 0 || memcmp(q_par, q_seq, nq * sizeof(kg_quota)) != 0) {
        fprintf(stderr, "kgo_schedule2_parallel differs from the sequential cycle\n");
        return 14;
    }
    int placed = 0;
    for (int64_t i = 0; i < P; i++) placed += node_seq[i] >= 0;
    printf("tsan workload ok: %lld pods x %lld nodes, %d placed\n", (long long)P, (long long)N, placed);
    return 0;
}
