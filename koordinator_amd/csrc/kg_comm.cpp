// kg_comm.cpp — the loopback communicator of the native sharded placement (kg_comm_init_loopback).
//
// kg_place_sharded merges each chunk's per-(pod, tile) partial keys over the ranks with one max-reduction
// (the shards' local top-k merged before the replicated resolve).  On hardware that is an
// ncclAllReduce over RCCL.  This communicator runs the same C++ chunk loop with ranks that cannot form an RCCL
// communicator — several processes sharing one GPU (RCCL refuses two ranks on one device), or hosts without
// peer access — by exchanging the keys through a POSIX shared-memory segment on the host:
//
//   header (one page) | slot set 0: world × slot_bytes | slot set 1: world × slot_bytes
//
// An all-reduce of round k writes the rank's buffer into slot set k mod 2, meets every rank at a barrier and
// reduces every rank's slot of that set into the caller's buffer.  The next round writes the other set, and
// the round after that (the same set again) starts only after every rank has passed round k + 1's barrier,
// i.e. after every rank finished reading round k: one barrier per all-reduce.
//
// The barrier is a generation counter in the segment (process-shared atomics), with a deadline: a rank that
// never arrives ends the wait with an error instead of hanging the others, and kg_shm_comm_abort wakes every
// waiter with an error.  The segment is unlinked as soon as every rank has mapped it, so nothing is left in
// /dev/shm when a process dies.
#include "kg_comm.h"

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

constexpr uint32_t kMagic = 0x4b47434du;   // "KGCM"
constexpr size_t kHeaderBytes = 4096;

struct ShmHeader {
    std::atomic<uint32_t> world;     // set once by the first rank (CAS 0 → world); the others check it
    std::atomic<uint32_t> magic;
    std::atomic<uint32_t> joined;    // ranks that mapped the segment
    std::atomic<uint32_t> arrive;    // ranks at the current barrier
    std::atomic<uint64_t> gen;       // barrier generation
    std::atomic<uint32_t> aborted;   // kg_shm_comm_abort: every wait fails
    std::atomic<uint64_t> slot_bytes;
};
static_assert(sizeof(ShmHeader) <= kHeaderBytes, "header fits its page");
static_assert(std::atomic<uint64_t>::is_always_lock_free && std::atomic<uint32_t>::is_always_lock_free,
              "process-shared atomics must be lock-free");

}  // namespace

struct kg_shm_comm {
    int rank = 0, world = 0;
    size_t slot_bytes = 0, map_bytes = 0;
    void *map = nullptr;
    ShmHeader *hdr = nullptr;
    uint64_t round = 0;
    double timeout_s = 120.0;
};

namespace {

char *slot(kg_shm_comm *c, int set, int rank) {
    return (char *)c->map + kHeaderBytes + ((size_t)set * (size_t)c->world + (size_t)rank) * c->slot_bytes;
}

bool wait_until(kg_shm_comm *c, const char *what, std::string &err, bool (*done)(kg_shm_comm *, uint64_t), uint64_t arg) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; spin++) {
        if (done(c, arg)) return true;
        if (c->hdr->aborted.load(std::memory_order_acquire)) {
            err = std::string(what) + ": the communicator was aborted by a rank";
            return false;
        }
        if ((spin & 1023) == 1023) {
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (s > c->timeout_s) {
                char b[160];
                snprintf(b, sizeof(b), "%s: rank %d waited %.0f s for the other ranks", what, c->rank, s);
                err = b;
                return false;
            }
            sched_yield();
        }
    }
}

bool barrier(kg_shm_comm *c, std::string &err) {
    ShmHeader *h = c->hdr;
    const uint64_t g = h->gen.load(std::memory_order_acquire);
    if (h->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->world) {
        h->arrive.store(0, std::memory_order_relaxed);
        h->gen.store(g + 1, std::memory_order_release);
        return true;
    }
    return wait_until(c, "loopback barrier", err, [](kg_shm_comm *cc, uint64_t gg) {
        return cc->hdr->gen.load(std::memory_order_acquire) != gg;
    }, g);
}

}  // namespace

kg_shm_comm *kg_shm_comm_open(const char *name, int rank, int world, size_t slot_bytes, double timeout_s,
                              std::string &err) {
    if (!name || name[0] != '/' || strchr(name + 1, '/') || world < 1 || rank < 0 || rank >= world || slot_bytes == 0) {
        err = "loopback communicator: bad name (\"/…\"), rank, world or slot size";
        return nullptr;
    }
    slot_bytes = (slot_bytes + 255) / 256 * 256;
    const size_t total = kHeaderBytes + 2 * (size_t)world * slot_bytes;
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        err = std::string("shm_open(") + name + "): " + strerror(errno);
        return nullptr;
    }
    struct stat sb;
    if (fstat(fd, &sb) != 0 || (sb.st_size != 0 && (size_t)sb.st_size != total)) {
        close(fd);
        err = std::string("loopback communicator ") + name + ": the segment exists with another size (ranks disagree on "
              "the world or the snapshot's tile count)";
        return nullptr;
    }
    if ((size_t)sb.st_size != total && ftruncate(fd, (off_t)total) != 0) {
        err = std::string("ftruncate: ") + strerror(errno);
        close(fd);
        return nullptr;
    }
    void *m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        err = std::string("mmap: ") + strerror(errno);
        return nullptr;
    }
    auto *c = new kg_shm_comm;
    c->rank = rank;
    c->world = world;
    c->slot_bytes = slot_bytes;
    c->map_bytes = total;
    c->map = m;
    c->hdr = reinterpret_cast<ShmHeader *>(m);   // zero-filled by ftruncate: every atomic starts at 0
    c->timeout_s = timeout_s > 0 ? timeout_s : 120.0;
    uint32_t w0 = 0;
    if (!c->hdr->world.compare_exchange_strong(w0, (uint32_t)world) && w0 != (uint32_t)world) {
        err = "loopback communicator: ranks disagree on the world size";
        kg_shm_comm_close(c);
        return nullptr;
    }
    uint32_t m0 = 0;
    c->hdr->magic.compare_exchange_strong(m0, kMagic);
    if (c->hdr->magic.load() != kMagic) {
        err = "loopback communicator: the segment is not a kg_comm segment";
        kg_shm_comm_close(c);
        return nullptr;
    }
    c->hdr->joined.fetch_add(1, std::memory_order_acq_rel);
    if (!wait_until(c, "loopback join", err, [](kg_shm_comm *cc, uint64_t) {
            return cc->hdr->joined.load(std::memory_order_acquire) >= (uint32_t)cc->world;
        }, 0)) {
        shm_unlink(name);   // the job failed: leave nothing in /dev/shm (a late rank then fails on its own)
        kg_shm_comm_close(c);
        return nullptr;
    }
    // every rank has the mapping: the name can go (nothing stays in /dev/shm after the processes end)
    if (rank == 0) shm_unlink(name);
    return c;
}

void kg_shm_comm_close(kg_shm_comm *c) {
    if (!c) return;
    if (c->map) munmap(c->map, c->map_bytes);
    delete c;
}

void kg_shm_comm_abort(kg_shm_comm *c) {
    if (c && c->hdr) c->hdr->aborted.store(1, std::memory_order_release);
}

int kg_shm_comm_rank(const kg_shm_comm *c) { return c ? c->rank : -1; }
int kg_shm_comm_world(const kg_shm_comm *c) { return c ? c->world : 0; }
size_t kg_shm_comm_slot_bytes(const kg_shm_comm *c) { return c ? c->slot_bytes : 0; }

bool kg_shm_comm_allreduce_max_u32(kg_shm_comm *c, uint32_t *buf, size_t count, std::string &err) {
    if (count * 4 > c->slot_bytes) {
        err = "loopback all-reduce larger than the communicator's slot";
        return false;
    }
    const int set = (int)(c->round++ & 1);
    memcpy(slot(c, set, c->rank), buf, count * 4);
    if (!barrier(c, err)) return false;
    for (int r = 0; r < c->world; r++) {
        if (r == c->rank) continue;
        const uint32_t *o = reinterpret_cast<const uint32_t *>(slot(c, set, r));
        for (size_t i = 0; i < count; i++) buf[i] = buf[i] > o[i] ? buf[i] : o[i];
    }
    return true;
}
