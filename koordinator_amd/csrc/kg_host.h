// kg_host.h — host-side helpers shared between kg_host.cpp and kg_engine.hip (not part of the C-ABI).
#pragma once
#include "kg_common.h"

void kg_consts_from_config(const kg_config &c, kg_consts &k);
const char *kg_res_name(const kg_config &c, int r);   // the resource-name key of slot r ("" ⇔ an unused named slot)
void kg_res_sorted_order(const kg_config &c, int8_t out[KG_NUM_RES]);
void kg_pod_dev_from_row(const kg_config &c, const kg_pod_row &row, kg_pod_dev &d);
bool kg_pod_row_in_bounds(const kg_pod_row &row);
int kg_numa_list_count(const kg_pod_row &row);   // NodeNUMAResource hint lists the pod can produce
// Fills the S-slot hot row (slot s ↔ resource slot_res[s]) and returns the pod's resources that
// need a slot (compared or scored), so the caller can check the profile covers them.
template <int S>
uint32_t kg_pod_hot_from_row(const kg_config &c, const kg_pod_row &row, const int32_t *slot_res, kg_pod_hot_t<S> &h);

// kg_cpuset.cpp — the CPU accumulator (cpuset take at Reserve) and NodeAllocation's available CPUs
int kg_cpuset_take_cpus(const kg_cpu_info *cpus, int32_t n_cpus, int32_t max_ref, const uint8_t *available, int32_t need,
                        int32_t bind, int32_t exclusive, int32_t strategy, uint8_t *result);
void kg_cpuset_available(const kg_cpu_info *cpus, int32_t n_cpus, int32_t max_ref, uint8_t *available);
void kg_cpuset_filter_required(const kg_cpu_info *cpus, int32_t n_cpus, int32_t bind, uint8_t *available);
bool kg_cpuset_satisfies_required(const kg_cpu_info *cpus, int32_t n_cpus, int32_t bind, const uint8_t *taken);
int32_t kg_cpuset_row_fields(kg_node_row &row, const kg_cpu_info *cpus, int32_t n, int32_t max_ref);
int kg_cpuset_allocate(const kg_consts &c, const kg_node_row &row, const kg_pod_dev &p, int required, int take,
                       const kg_cpu_info *cpus, int32_t n, int32_t max_ref, int32_t strategy, uint8_t *taken);
void kg_cpuset_apply(const kg_pod_dev &p, kg_cpu_info *cpus, int32_t n, const uint8_t *taken);
int32_t kg_cpuset_strategy(const kg_config &cfg, int32_t label);
