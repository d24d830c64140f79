// RCCL transport (HIP build): one communicator per process / GPU, every
// collective enqueued on the backend's HIP stream so that it is ordered after
// the kernels that produced its input and before those that consume it.
//
// Pairwise exchanges (the only bulk traffic: distributed qubit swaps, see
// src/core/router.cpp) are ncclSend + ncclRecv inside one group, i.e. both
// directions of the single direct xGMI link between the two GPUs at once.
// Scalars (probabilities, norms, inner products) use ncclAllReduce on a small
// device buffer.  Replaces the reference's blocking MPI_Sendrecv /
// MPI_Allreduce / MPI_Bcast calls (QuEST_cpu_distributed.c:41-512, 1236-1305).
//
// librccl is loaded with dlopen: inside a Python process that already loaded
// PyTorch we bind to torch's RCCL (same HIP runtime); standalone C programs
// get /opt/rocm's.
//
// QUEST_COMM=socket selects the test transport instead: the TCP socket mesh
// of comm_socket.cpp with every device buffer staged through pinned host
// memory, so that several ranks can share one GPU (RCCL refuses that).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../hip/qa_hip.h"
#include "comm.hpp"

namespace qa {
namespace comm {

namespace {

struct Rccl {
    void* lib = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char* (*errorString)(ncclResult_t) = nullptr;
    ncclResult_t (*getVersion)(int*) = nullptr;
    ncclResult_t (*getAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;  // optional
    ncclResult_t (*commAbort)(ncclComm_t) = nullptr;                      // optional
} R;

int g_rank = 0, g_size = 1;
bool g_socket = false;          // QUEST_COMM=socket test transport
char* g_stage = nullptr;        // pinned staging for the socket transport
size_t g_stageBytes = 0;
ncclComm_t g_comm = nullptr;
// communication stream of the pipelined exchange and its events
hipStream_t g_cstream = nullptr;
hipEvent_t g_ready = nullptr, g_done[2] = {nullptr, nullptr};
double* g_dScalars = nullptr;   // device scratch for scalar collectives
double* g_hScalars = nullptr;   // pinned host mirror
std::string g_libName;

void die(const char* what, ncclResult_t r) {
    fprintf(stderr, "QuEST RCCL error (rank %d): %s: %s\n", g_rank, what, R.errorString ? R.errorString(r) : "?");
    exit(EXIT_FAILURE);
}

#define QA_NCCL(call, what)                  \
    do {                                     \
        ncclResult_t _r = (call);            \
        if (_r != ncclSuccess) die(what, _r); \
    } while (0)

template <typename F>
void sym(F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(R.lib, name));
    if (!f) {
        fprintf(stderr, "QuEST: symbol %s missing from %s\n", name, g_libName.c_str());
        exit(EXIT_FAILURE);
    }
}

bool loadRccl() {
    if (R.lib) return true;
    const char* env = getenv("QUEST_RCCL_LIB");
    const char* candidates[] = {env, "librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
    for (int i = 0; i < 4 && !R.lib; i++) {
        if (!candidates[i]) continue;
        // prefer a copy already mapped into the process (e.g. PyTorch's)
        R.lib = dlopen(candidates[i], RTLD_NOW | RTLD_NOLOAD);
        if (!R.lib) R.lib = dlopen(candidates[i], RTLD_NOW | RTLD_GLOBAL);
        if (R.lib) g_libName = candidates[i];
    }
    if (!R.lib) {
        fprintf(stderr, "QuEST: could not load librccl (%s)\n", dlerror());
        return false;
    }
    sym(R.getUniqueId, "ncclGetUniqueId");
    sym(R.commInitRank, "ncclCommInitRank");
    sym(R.commDestroy, "ncclCommDestroy");
    sym(R.send, "ncclSend");
    sym(R.recv, "ncclRecv");
    sym(R.allReduce, "ncclAllReduce");
    sym(R.broadcast, "ncclBroadcast");
    sym(R.allGather, "ncclAllGather");
    sym(R.groupStart, "ncclGroupStart");
    sym(R.groupEnd, "ncclGroupEnd");
    sym(R.errorString, "ncclGetErrorString");
    sym(R.getVersion, "ncclGetVersion");
    R.getAsyncError = reinterpret_cast<decltype(R.getAsyncError)>(dlsym(R.lib, "ncclCommGetAsyncError"));
    R.commAbort = reinterpret_cast<decltype(R.commAbort)>(dlsym(R.lib, "ncclCommAbort"));
    return true;
}

hipStream_t S() { return hipk::stream(); }

// Failure detection while the host waits on the stream (hipk::syncStream):
// an asynchronous RCCL error (e.g. a peer's connection dropped) or no
// progress for QUEST_COMM_TIMEOUT seconds (default 900; 0 = never) aborts the
// communicator and ends this rank with a report, rather than leaving every
// rank of the job blocked in a collective whose peer is gone.
double commTimeout() {
    static const double t = [] {
        const char* e = getenv("QUEST_COMM_TIMEOUT");
        return e ? atof(e) : 900.0;
    }();
    return t;
}

[[noreturn]] void abortComm(const char* why) {
    fprintf(stderr, "QuEST: rank %d: %s; aborting the RCCL communicator\n", g_rank, why);
    fflush(stderr);
    if (R.commAbort && g_comm) R.commAbort(g_comm);
    g_comm = nullptr;
    exit(EXIT_FAILURE);
}

void watchdog(double elapsed) {
    if (!g_comm) return;
    if (R.getAsyncError) {
        ncclResult_t r = ncclSuccess;
        if (R.getAsyncError(g_comm, &r) == ncclSuccess && r != ncclSuccess && r != ncclInProgress) {
            char msg[256];
            snprintf(msg, sizeof msg, "RCCL reported an asynchronous error: %s", R.errorString(r));
            abortComm(msg);
        }
    }
    if (commTimeout() > 0 && elapsed > commTimeout()) {
        char msg[256];
        snprintf(msg, sizeof msg, "no progress for %.0f s (QUEST_COMM_TIMEOUT) -- a peer rank may have failed",
                 elapsed);
        abortComm(msg);
    }
}

// pinned host staging of at least `bytes` (socket transport)
char* stage(size_t bytes) {
    if (bytes > g_stageBytes) {
        if (g_stage) QA_HIP_CHECK(hipHostFree(g_stage));
        g_stageBytes = bytes < ((size_t)1 << 20) ? ((size_t)1 << 20) : bytes;
        QA_HIP_CHECK(hipHostMalloc(&g_stage, g_stageBytes, hipHostMallocDefault));
    }
    return g_stage;
}

}  // namespace

void init(int rank, int size) {
    g_rank = rank;
    g_size = size;
    if (size == 1) return;
    const char* mode = getenv("QUEST_COMM");
    g_socket = mode && !strcmp(mode, "socket");
    if (g_socket) {
        sock::init(rank, size);
        return;
    }
    // RCCL unique id from rank 0; then every rank reports whether its
    // communicator came up, and if any did not, all fall back together to
    // the socket transport (staged through host memory) rather than hang
    int ok = loadRccl() ? 1 : 0;
    ncclUniqueId id;
    memset(&id, 0, sizeof id);
    if (rank == 0 && ok && R.getUniqueId(&id) != ncclSuccess) ok = 0;
    std::string all((size_t)size * sizeof id, '\0');
    boot::allgather(rank, size, &id, &all[0], sizeof id);
    memcpy(&id, all.data(), sizeof id);  // rank 0's id
    std::vector<int> oks(size, 0);
    boot::allgather(rank, size, &ok, oks.data(), sizeof(int));
    for (int r = 0; r < size; r++) ok = ok && oks[r];  // rank 0 failing to make an id fails everyone
    if (ok) {
        const ncclResult_t rc = R.commInitRank(&g_comm, size, id, rank);
        int mine = rc == ncclSuccess ? 1 : 0;
        if (!mine) fprintf(stderr, "QuEST: ncclCommInitRank failed on rank %d: %s\n", rank, R.errorString(rc));
        boot::allgather(rank, size, &mine, oks.data(), sizeof(int));
        for (int r = 0; r < size; r++) ok = ok && oks[r];
        if (!ok && mine) {
            R.commDestroy(g_comm);
            g_comm = nullptr;
        }
    }
    if (!ok) {
        if (rank == 0) fprintf(stderr, "QuEST: RCCL unavailable, using the socket transport (slow)\n");
        g_socket = true;
        sock::init(rank, size);
        return;
    }
    QA_HIP_CHECK(hipMalloc(&g_dScalars, sizeof(double) * 64));
    QA_HIP_CHECK(hipHostMalloc(&g_hScalars, sizeof(double) * 64, hipHostMallocDefault));
    QA_HIP_CHECK(hipStreamCreateWithFlags(&g_cstream, hipStreamNonBlocking));
    QA_HIP_CHECK(hipEventCreateWithFlags(&g_ready, hipEventDisableTiming));
    for (hipEvent_t& e : g_done) QA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipk::setSyncWatchdog(watchdog);
}

void finalize() {
    if (g_socket) {
        sock::finalize();
        if (g_stage) (void)hipHostFree(g_stage);
        g_stage = nullptr;
        g_stageBytes = 0;
        g_socket = false;
    }
    if (g_comm) {
        hipk::syncStream();
        hipk::setSyncWatchdog(nullptr);
        R.commDestroy(g_comm);
        g_comm = nullptr;
        if (g_cstream) {
            (void)hipStreamSynchronize(g_cstream);
            (void)hipEventDestroy(g_ready);
            for (hipEvent_t e : g_done) (void)hipEventDestroy(e);
            (void)hipStreamDestroy(g_cstream);
            g_cstream = nullptr;
        }
        (void)hipFree(g_dScalars);
        (void)hipHostFree(g_hScalars);
        g_dScalars = g_hScalars = nullptr;
    }
    g_size = 1;
}

bool active() { return g_size > 1; }

void sendrecv(int peer, const void* send, void* recv, size_t bytes) {
    if (peer == g_rank) {
        QA_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, S()));
        return;
    }
    if (g_socket) {
        char* h = stage(2 * bytes);
        QA_HIP_CHECK(hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, S()));
        hipk::syncStream();
        sock::sendrecv(peer, h, h + bytes, bytes);
        QA_HIP_CHECK(hipMemcpyAsync(recv, h + bytes, bytes, hipMemcpyHostToDevice, S()));
        hipk::syncStream();
        return;
    }
    QA_NCCL(R.groupStart(), "ncclGroupStart");
    QA_NCCL(R.send(send, bytes, ncclUint8, peer, g_comm, S()), "ncclSend");
    QA_NCCL(R.recv(recv, bytes, ncclUint8, peer, g_comm, S()), "ncclRecv");
    QA_NCCL(R.groupEnd(), "ncclGroupEnd");
}

void exchange(const Xfer* x, int n) {
    if (g_socket || g_size == 1) {
        for (int i = 0; i < n; i++) sendrecv(x[i].peer, x[i].send, x[i].recv, x[i].bytes);
        return;
    }
    // one group: RCCL drives every peer's xGMI link at once
    QA_NCCL(R.groupStart(), "ncclGroupStart");
    for (int i = 0; i < n; i++) {
        QA_NCCL(R.send(x[i].send, x[i].bytes, ncclUint8, x[i].peer, g_comm, S()), "ncclSend");
        QA_NCCL(R.recv(x[i].recv, x[i].bytes, ncclUint8, x[i].peer, g_comm, S()), "ncclRecv");
    }
    QA_NCCL(R.groupEnd(), "ncclGroupEnd");
}

bool pipelined() {
    static const bool off = getenv("QUEST_EXCHANGE_PIPELINE") && atoi(getenv("QUEST_EXCHANGE_PIPELINE")) == 0;
    return !off && !g_socket && g_size > 1 && g_cstream;
}

void exchangeAsync(const Xfer* x, int n, int slot) {
    if (!pipelined()) {
        exchange(x, n);
        return;
    }
    QA_HIP_CHECK(hipEventRecord(g_ready, S()));
    QA_HIP_CHECK(hipStreamWaitEvent(g_cstream, g_ready, 0));
    QA_NCCL(R.groupStart(), "ncclGroupStart");
    for (int i = 0; i < n; i++) {
        QA_NCCL(R.send(x[i].send, x[i].bytes, ncclUint8, x[i].peer, g_comm, g_cstream), "ncclSend");
        QA_NCCL(R.recv(x[i].recv, x[i].bytes, ncclUint8, x[i].peer, g_comm, g_cstream), "ncclRecv");
    }
    QA_NCCL(R.groupEnd(), "ncclGroupEnd");
    QA_HIP_CHECK(hipEventRecord(g_done[slot & 1], g_cstream));
}

void exchangeWait(int slot) {
    if (!pipelined()) return;
    QA_HIP_CHECK(hipStreamWaitEvent(S(), g_done[slot & 1], 0));
}

void allreduceSum(double* vals, int n) {
    if (g_size == 1) return;
    if (g_socket) {
        sock::allreduceSum(vals, n);
        return;
    }
    for (int off = 0; off < n; off += 64) {
        int k = n - off < 64 ? n - off : 64;
        memcpy(g_hScalars, vals + off, sizeof(double) * k);
        QA_HIP_CHECK(hipMemcpyAsync(g_dScalars, g_hScalars, sizeof(double) * k, hipMemcpyHostToDevice, S()));
        QA_NCCL(R.allReduce(g_dScalars, g_dScalars, (size_t)k, ncclFloat64, ncclSum, g_comm, S()), "ncclAllReduce");
        QA_HIP_CHECK(hipMemcpyAsync(g_hScalars, g_dScalars, sizeof(double) * k, hipMemcpyDeviceToHost, S()));
        hipk::syncStream();
        memcpy(vals + off, g_hScalars, sizeof(double) * k);
    }
}

int allreduceAnd(int v) {
    double d = v ? 0.0 : 1.0;
    allreduceSum(&d, 1);
    return d == 0.0 ? 1 : 0;
}

void bcastHost(void* buf, size_t bytes, int root) {
    if (g_size == 1) return;
    if (g_socket) {
        sock::bcastHost(buf, bytes, root);
        return;
    }
    char* p = (char*)buf;
    const size_t cap = sizeof(double) * 64;
    for (size_t off = 0; off < bytes; off += cap) {
        size_t k = bytes - off < cap ? bytes - off : cap;
        if (g_rank == root) memcpy(g_hScalars, p + off, k);
        QA_HIP_CHECK(hipMemcpyAsync(g_dScalars, g_hScalars, k, hipMemcpyHostToDevice, S()));
        QA_NCCL(R.broadcast(g_dScalars, g_dScalars, k, ncclUint8, root, g_comm, S()), "ncclBroadcast");
        QA_HIP_CHECK(hipMemcpyAsync(g_hScalars, g_dScalars, k, hipMemcpyDeviceToHost, S()));
        hipk::syncStream();
        memcpy(p + off, g_hScalars, k);
    }
}

void allgather(const void* send, void* recv, size_t bytesPerRank) {
    if (g_size == 1) {
        QA_HIP_CHECK(hipMemcpyAsync(recv, send, bytesPerRank, hipMemcpyDeviceToDevice, S()));
        return;
    }
    if (g_socket) {
        const size_t all = bytesPerRank * (size_t)g_size;
        char* h = stage(bytesPerRank + all);
        QA_HIP_CHECK(hipMemcpyAsync(h, send, bytesPerRank, hipMemcpyDeviceToHost, S()));
        hipk::syncStream();
        sock::allgatherHost(h, h + bytesPerRank, bytesPerRank);
        QA_HIP_CHECK(hipMemcpyAsync(recv, h + bytesPerRank, all, hipMemcpyHostToDevice, S()));
        hipk::syncStream();
        return;
    }
    QA_NCCL(R.allGather(send, recv, bytesPerRank, ncclUint8, g_comm, S()), "ncclAllGather");
}

void barrier() {
    double d = 1;
    allreduceSum(&d, 1);
}

std::string describe() {
    if (g_size == 1) return "single process";
    if (g_socket) return "TCP socket mesh, device buffers staged through host (QUEST_COMM=socket)";
    int v = 0;
    if (R.getVersion) R.getVersion(&v);
    char buf[256];
    snprintf(buf, sizeof buf, "RCCL %d over xGMI (%d ranks, %s)", v, g_size, g_libName.c_str());
    return buf;
}

}  // namespace comm
}  // namespace qa
