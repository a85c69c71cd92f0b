// kg_host.h — host-side helpers shared between kg_host.cpp and kg_engine.hip (not part of the C-ABI).
#pragma once
#include "kg_common.h"

void kg_consts_from_config(const kg_config &c, kg_consts &k);
void kg_pod_dev_from_row(const kg_config &c, const kg_pod_row &row, kg_pod_dev &d);
bool kg_pod_row_in_bounds(const kg_pod_row &row);
