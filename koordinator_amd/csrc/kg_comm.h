// kg_comm.h — the host shared-memory communicator (kg_comm.cpp) behind kg_comm_init_loopback; not part of the C-ABI.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

struct kg_shm_comm;
// every rank opens the same name ("/…") with the same world and slot size; returns when all have joined (or nullptr
// and err after timeout_s)
kg_shm_comm *kg_shm_comm_open(const char *name, int rank, int world, size_t slot_bytes, double timeout_s, std::string &err);
void kg_shm_comm_close(kg_shm_comm *c);
// every later wait of every rank fails (a rank that cannot continue releases its peers)
void kg_shm_comm_abort(kg_shm_comm *c);
// buf[0..count) := max over the ranks' buf, element-wise (every rank calls it in the same order)
bool kg_shm_comm_allreduce_max_u32(kg_shm_comm *c, uint32_t *buf, size_t count, std::string &err);
int kg_shm_comm_rank(const kg_shm_comm *c);
int kg_shm_comm_world(const kg_shm_comm *c);
size_t kg_shm_comm_slot_bytes(const kg_shm_comm *c);
