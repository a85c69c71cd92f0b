// C shim over the loopback communicator (koordinator_amd/csrc/kg_comm.cpp) for tests/test_shm_comm_cpu.py: the
// barrier, the double-buffered slot sets, the timeout and the abort are host code and are tested on the CPU, in
// several processes, without a GPU.
#include <cstdint>
#include <cstring>
#include <string>

#include "kg_comm.h"

static std::string g_err;

extern "C" {
void *shim_open(const char *name, int rank, int world, size_t slot_bytes, double timeout_s) {
    return kg_shm_comm_open(name, rank, world, slot_bytes, timeout_s, g_err);
}
int shim_allreduce(void *c, uint32_t *buf, size_t count) {
    return kg_shm_comm_allreduce_max_u32((kg_shm_comm *)c, buf, count, g_err) ? 0 : 1;
}
void shim_abort(void *c) { kg_shm_comm_abort((kg_shm_comm *)c); }
void shim_close(void *c) { kg_shm_comm_close((kg_shm_comm *)c); }
const char *shim_error() { return g_err.c_str(); }
}
