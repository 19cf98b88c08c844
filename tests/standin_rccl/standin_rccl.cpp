// standin_rccl.cpp -- TEST INFRASTRUCTURE ONLY, never part of the package.
//
// A stand-in for the four RCCL entry points the native observation exchange binds at run time
// (cf2_xchg_bind, csrc/cf2sim_exchange.hip: ncclGetUniqueId, ncclCommInitRank, ncclAllGather,
// ncclCommDestroy), so that the exchange's multi-rank code -- the [world][nb][words] receive
// layout, the per-rank look-ahead counts, the setup agreement -- runs with world_size > 1 on a
// one-GPU test box, where RCCL itself refuses two ranks on the same device.
//
// The all-gather is host-staged through a POSIX shared-memory segment named by the unique id: a
// rank waits for its stream's prior work, copies its send buffer into its slot of the segment,
// meets the other ranks at a barrier, copies all slots into its receive buffer and meets them
// again before returning.  The call therefore completes before it returns (a stricter ordering
// than RCCL's stream-ordered collective, so everything the exchange orders after it on the stream
// sees the gathered data).  Slower than RCCL by far; it is a correctness vehicle, not a transport.
//
// Environment (tests only): CF2_STANDIN_FAIL_RANK=r makes rank r's ncclCommInitRank fail (the
// exchange's all-ranks fallback); CF2_STANDIN_SLOT_MB sizes each rank's slot (default 48 MB);
// CF2_STANDIN_TIMEOUT_S bounds every barrier wait (default 60 s: a peer that never arrives makes
// the call fail instead of hanging).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <fcntl.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

namespace {

struct Ctl {                               // first page of the segment
    std::atomic<uint32_t> arrived;
    std::atomic<uint32_t> generation;
};
constexpr size_t CTL_BYTES = 4096;

double env_num(const char* name, double dflt) {
    const char* v = getenv(name);
    return v && *v ? atof(v) : dflt;
}

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

}  // namespace

struct ncclComm {
    int rank, world;
    size_t slot;                          // bytes per rank
    size_t map_bytes;
    Ctl* ctl;
    uint8_t* data;                        // [world][slot]
    char name[64];
    double timeout_s;
};

// every rank of the communicator meets here (sense by generation); false after the timeout
static bool barrier(ncclComm* c) {
    const uint32_t gen = c->ctl->generation.load(std::memory_order_acquire);
    if (c->ctl->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->world) {
        c->ctl->arrived.store(0, std::memory_order_relaxed);
        c->ctl->generation.fetch_add(1, std::memory_order_acq_rel);
        return true;
    }
    const auto t0 = std::chrono::steady_clock::now();
    while (c->ctl->generation.load(std::memory_order_acquire) == gen) {
        sched_yield();
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) return false;
    }
    return true;
}

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof(*id));
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    snprintf(id->internal, sizeof(id->internal), "/cf2standin_%d_%lx_%lx", (int)getpid(), (unsigned long)ts.tv_sec,
             (unsigned long)ts.tv_nsec);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks || id.internal[0] != '/') return ncclInvalidArgument;
    *comm = nullptr;
    if ((int)env_num("CF2_STANDIN_FAIL_RANK", -1) == rank) return ncclSystemError;
    ncclComm* c = new ncclComm();
    c->rank = rank;
    c->world = nranks;
    c->slot = (size_t)(env_num("CF2_STANDIN_SLOT_MB", 48) * (1 << 20));
    c->timeout_s = env_num("CF2_STANDIN_TIMEOUT_S", 60);
    snprintf(c->name, sizeof(c->name), "%s", id.internal);
    c->map_bytes = CTL_BYTES + (size_t)nranks * c->slot;
    const int fd = shm_open(c->name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) { delete c; return ncclSystemError; }
    if (ftruncate(fd, (off_t)c->map_bytes) != 0) { close(fd); delete c; return ncclSystemError; }
    void* m = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) { delete c; return ncclSystemError; }
    c->ctl = static_cast<Ctl*>(m);          // a fresh segment is zero-filled: counters start at 0
    c->data = static_cast<uint8_t*>(m) + CTL_BYTES;
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
    if (!comm || !sendbuff || !recvbuff) return ncclInvalidArgument;
    const size_t tb = type_bytes(datatype);
    const size_t bytes = sendcount * tb;
    if (tb == 0 || bytes > comm->slot) return ncclInvalidArgument;
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    if (bytes && hipMemcpy(comm->data + (size_t)comm->rank * comm->slot, sendbuff, bytes, hipMemcpyDeviceToHost) !=
                     hipSuccess)
        return ncclUnhandledCudaError;
    if (!barrier(comm)) return ncclSystemError;
    for (int r = 0; r < comm->world && bytes; ++r)
        if (hipMemcpy(static_cast<uint8_t*>(recvbuff) + (size_t)r * bytes, comm->data + (size_t)r * comm->slot, bytes,
                      hipMemcpyHostToDevice) != hipSuccess)
            return ncclUnhandledCudaError;
    if (!barrier(comm)) return ncclSystemError;          // nobody refills a slot another rank still reads
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclSuccess;
    munmap(comm->ctl, comm->map_bytes);
    shm_unlink(comm->name);                 // every rank: the name goes with the first, ENOENT after
    delete comm;
    return ncclSuccess;
}

}  // extern "C"
