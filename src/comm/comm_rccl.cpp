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
// Other transports, only on explicit request (a communicator that fails to
// come up is a fatal error, never a silent downgrade):
//   QUEST_COMM=ipc     ranks sharing one GPU: device buffers exchanged through
//                      HIP IPC handles with the SAME communication stream and
//                      event protocol (comm_ipc.hpp), scalars over sockets;
//   QUEST_COMM=socket  the TCP socket mesh of comm_socket.cpp with every
//                      device buffer staged through pinned host memory.
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
#include "comm_ipc.hpp"

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
enum class Mode { Single, Rccl, Ipc, Socket };
Mode g_mode = Mode::Single;
bool g_socket = false;          // QUEST_COMM=socket test transport
bool g_sharedGpu = false;       // QUEST_RCCL_SHARED_GPU=1: RCCL ranks sharing one GPU
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
    if (g_mode == Mode::Ipc) {
        if (commTimeout() > 0 && elapsed > commTimeout()) {
            fprintf(stderr, "QuEST: rank %d: no progress for %.0f s (QUEST_COMM_TIMEOUT) -- a peer rank may have "
                            "failed\n", g_rank, elapsed);
            fflush(stderr);
            exit(EXIT_FAILURE);
        }
        return;
    }
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

void createStreams() {
    QA_HIP_CHECK(hipMalloc(&g_dScalars, sizeof(double) * 64));
    QA_HIP_CHECK(hipHostMalloc(&g_hScalars, sizeof(double) * 64, hipHostMallocDefault));
    QA_HIP_CHECK(hipStreamCreateWithFlags(&g_cstream, hipStreamNonBlocking));
    QA_HIP_CHECK(hipEventCreateWithFlags(&g_ready, hipEventDisableTiming));
    for (hipEvent_t& e : g_done) QA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipk::setSyncWatchdog(watchdog);
}

void init(int rank, int size) {
    g_rank = rank;
    g_size = size;
    g_mode = Mode::Single;
    if (size == 1) return;
    const char* mode = getenv("QUEST_COMM");
    const std::string m = mode ? mode : "rccl";
    if (m == "socket") {
        g_mode = Mode::Socket;
        g_socket = true;
        sock::init(rank, size);
        return;
    }
    if (m == "ipc") {
        g_mode = Mode::Ipc;
        sock::init(rank, size);
        ipc::init(rank, size);
        createStreams();
        return;
    }
    if (m != "rccl") {
        fprintf(stderr, "QuEST: unknown QUEST_COMM=%s (rccl, ipc or socket)\n", mode);
        exit(EXIT_FAILURE);
    }
    // QUEST_RCCL_SHARED_GPU=1: several ranks on ONE GPU still run RCCL.  RCCL
    // refuses two ranks on one device of one host ("Duplicate GPU"), so each
    // rank presents its own host id (NCCL_HOSTID, read when the communicator
    // is made) and RCCL connects them through its network transport over
    // loopback.  Every RCCL call of the data path (grouped send / recv of the
    // pipelined exchange, allreduce, broadcast, allgather) then runs with N
    // ranks on a one-GPU machine; only the link differs from xGMI.
    g_sharedGpu = getenv("QUEST_RCCL_SHARED_GPU") && atoi(getenv("QUEST_RCCL_SHARED_GPU")) != 0;
    if (g_sharedGpu) {
        char host[64];
        snprintf(host, sizeof host, "quest-shared-gpu-rank-%d", rank);
        setenv("NCCL_HOSTID", host, 1);
        setenv("NCCL_SOCKET_IFNAME", "lo", 0);
        setenv("NCCL_IB_DISABLE", "1", 0);
    }
    // RCCL unique id from rank 0; then every rank reports whether its
    // communicator came up.  If any did not, every rank stops with the
    // reason: a job launched for RCCL over xGMI must not quietly continue on
    // a host-staged transport (QUEST_COMM=ipc / socket select those).
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
    std::string why = ok ? "" : "librccl could not be loaded or ncclGetUniqueId failed";
    if (ok) {
        const ncclResult_t rc = R.commInitRank(&g_comm, size, id, rank);
        int mine = rc == ncclSuccess ? 1 : 0;
        if (!mine) fprintf(stderr, "QuEST: ncclCommInitRank failed on rank %d: %s\n", rank, R.errorString(rc));
        boot::allgather(rank, size, &mine, oks.data(), sizeof(int));
        for (int r = 0; r < size; r++) ok = ok && oks[r];
        if (!ok) {
            why = "ncclCommInitRank failed on a rank (several ranks on one GPU? set QUEST_RCCL_SHARED_GPU=1 or use "
                  "QUEST_COMM=ipc)";
            if (mine) R.commDestroy(g_comm);
            g_comm = nullptr;
        }
    }
    if (!ok) {
        fprintf(stderr, "QuEST: rank %d: the RCCL transport could not start: %s; set QUEST_COMM=ipc or "
                        "QUEST_COMM=socket to use another transport explicitly\n", rank, why.c_str());
        fflush(stderr);
        exit(EXIT_FAILURE);
    }
    g_mode = Mode::Rccl;
    createStreams();
}

void finalize() {
    if (g_mode == Mode::Single) {
        g_size = 1;
        return;
    }
    if (g_cstream) {
        hipk::syncStream();
        (void)hipStreamSynchronize(g_cstream);
        hipk::setSyncWatchdog(nullptr);
    }
    if (g_mode == Mode::Ipc) ipc::finalize();
    if (g_mode == Mode::Socket || g_mode == Mode::Ipc) sock::finalize();
    if (g_stage) (void)hipHostFree(g_stage);
    g_stage = nullptr;
    g_stageBytes = 0;
    g_socket = false;
    if (g_comm) R.commDestroy(g_comm);
    g_comm = nullptr;
    if (g_cstream) {
        (void)hipEventDestroy(g_ready);
        for (hipEvent_t e : g_done) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(g_cstream);
        g_cstream = nullptr;
        (void)hipFree(g_dScalars);
        (void)hipHostFree(g_hScalars);
        g_dScalars = g_hScalars = nullptr;
    }
    g_mode = Mode::Single;
    g_size = 1;
}

bool active() { return g_size > 1; }

void bufferFreed(const void* p) {
    if (g_mode == Mode::Ipc) ipc::forget(p);
}

namespace {

// The device-side exchange of one slice set on `stream` (RCCL: one group,
// every peer's xGMI link at once; IPC: pulls from the peers' buffers).
// `producer` is the stream whose queued work filled the send buffers.
void deviceExchange(const Xfer* x, int n, int slot, hipStream_t producer, hipStream_t stream) {
    if (g_mode == Mode::Ipc) {
        ipc::transfer(x, n, slot, producer, stream);
        if (stream == producer) ipc::complete(slot);  // not pipelined: done on return
        return;
    }
    QA_NCCL(R.groupStart(), "ncclGroupStart");
    for (int i = 0; i < n; i++) {
        QA_NCCL(R.send(x[i].send, x[i].bytes, ncclUint8, x[i].peer, g_comm, stream), "ncclSend");
        QA_NCCL(R.recv(x[i].recv, x[i].bytes, ncclUint8, x[i].peer, g_comm, stream), "ncclRecv");
    }
    QA_NCCL(R.groupEnd(), "ncclGroupEnd");
}

// host staging of a device exchange for the socket transport
void socketExchange(const Xfer& x) {
    char* h = stage(2 * x.bytes);
    QA_HIP_CHECK(hipMemcpyAsync(h, x.send, x.bytes, hipMemcpyDeviceToHost, S()));
    hipk::syncStream();
    sock::sendrecv(x.peer, h, h + x.bytes, x.bytes);
    QA_HIP_CHECK(hipMemcpyAsync(x.recv, h + x.bytes, x.bytes, hipMemcpyHostToDevice, S()));
    hipk::syncStream();
}

}  // namespace

void sendrecv(int peer, const void* send, void* recv, size_t bytes) {
    hipk::settleSwaps();   // an overlapped swap's transfers come first on every rank
    if (peer == g_rank) {
        QA_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, S()));
        return;
    }
    const Xfer x{peer, send, recv, bytes};
    if (g_mode == Mode::Socket)
        socketExchange(x);
    else
        deviceExchange(&x, 1, 0, S(), S());
}

void exchange(const Xfer* x, int n) {
    hipk::settleSwaps();   // an overlapped swap's transfers come first on every rank
    if (g_mode == Mode::Socket || g_mode == Mode::Single) {
        for (int i = 0; i < n; i++) sendrecv(x[i].peer, x[i].send, x[i].recv, x[i].bytes);
        return;
    }
    deviceExchange(x, n, 0, S(), S());
}

bool sendsFromState() { return g_mode == Mode::Rccl; }

bool swapsInPlace() {
    // mapped address ranges (QUEST_ALLOC_MODE=3) have no IPC handle
    static const bool on = (!getenv("QUEST_IPC_SWAP") || atoi(getenv("QUEST_IPC_SWAP")) != 0) &&
                           !(getenv("QUEST_ALLOC_MODE") && atoi(getenv("QUEST_ALLOC_MODE")) == 3);
    return on && g_mode == Mode::Ipc;
}

void mapPeerArrays(const int* peers, int n, void* const* arrays, int nArr, void** peerPtr) {
    ipc::mapArrays(peers, n, arrays, nArr, peerPtr, S());
}

void peersDone(const int* peers, int n) { ipc::done(peers, n, S()); }

bool pipelined() {
    static const bool off = getenv("QUEST_EXCHANGE_PIPELINE") && atoi(getenv("QUEST_EXCHANGE_PIPELINE")) == 0;
    return !off && (g_mode == Mode::Rccl || g_mode == Mode::Ipc) && g_cstream;
}

bool exchangeStreamOrdered() { return g_mode == Mode::Rccl && pipelined(); }

void exchangeAsync(const Xfer* x, int n, int slot) {
    if (!pipelined()) {
        exchange(x, n);
        return;
    }
    // the communication stream starts after everything queued so far on the
    // compute stream (the packs of this slice, the unpacks that freed its
    // receive buffers)
    QA_HIP_CHECK(hipEventRecord(g_ready, S()));
    QA_HIP_CHECK(hipStreamWaitEvent(g_cstream, g_ready, 0));
    deviceExchange(x, n, slot, S(), g_cstream);
    QA_HIP_CHECK(hipEventRecord(g_done[slot & 1], g_cstream));
}

void exchangeWait(int slot) {
    if (!pipelined()) return;
    if (g_mode == Mode::Ipc) ipc::complete(slot);
    QA_HIP_CHECK(hipStreamWaitEvent(S(), g_done[slot & 1], 0));
}

namespace {
// RCCL collectives on host values staged through the device scratch
void rcclAllreduceSum(double* vals, int n) {
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

void rcclBcast(void* buf, size_t bytes, int root) {
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
}  // namespace

void allreduceSum(double* vals, int n) {
    hipk::settleSwaps();   // an overlapped swap's transfers come first on every rank
    if (g_size == 1) return;
    if (g_mode == Mode::Socket || g_mode == Mode::Ipc) {
        sock::allreduceSum(vals, n);
        return;
    }
    rcclAllreduceSum(vals, n);
}

int allreduceAnd(int v) {
    hipk::settleSwaps();   // an overlapped swap's transfers come first on every rank
    double d = v ? 0.0 : 1.0;
    allreduceSum(&d, 1);
    return d == 0.0 ? 1 : 0;
}

void bcastHost(void* buf, size_t bytes, int root) {
    hipk::settleSwaps();   // an overlapped swap's transfers come first on every rank
    if (g_size == 1) return;
    if (g_mode == Mode::Socket || g_mode == Mode::Ipc) {
        sock::bcastHost(buf, bytes, root);
        return;
    }
    rcclBcast(buf, bytes, root);
}

void allgather(const void* send, void* recv, size_t bytesPerRank) {
    hipk::settleSwaps();   // an overlapped swap's transfers come first on every rank
    if (g_size == 1) {
        QA_HIP_CHECK(hipMemcpyAsync(recv, send, bytesPerRank, hipMemcpyDeviceToDevice, S()));
        return;
    }
    if (g_mode == Mode::Socket || g_mode == Mode::Ipc) {
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
    hipk::settleSwaps();   // an overlapped swap's transfers come first on every rank
    double d = 1;
    allreduceSum(&d, 1);
}

// One-rank RCCL communicator driven through the production code paths: the
// pipelined exchange (communication stream, ready / done events, double
// buffering, grouped send + recv -- to itself), the staged scalar allreduce
// and broadcast, allgather and the async-error watchdog, in one process
// (several ranks on one GPU: QUEST_RCCL_SHARED_GPU=1 in comm::init).
bool selfTest(std::string& report, void* const* userSend, void* const* userRecv, int nBuf, size_t bufBytes) {
    char msg[768];
    if (g_size != 1 || g_mode != Mode::Single) {
        report = "self-test needs a single-process job";
        return false;
    }
    if (!loadRccl()) {
        report = "librccl could not be loaded";
        return false;
    }
    ncclUniqueId id;
    QA_NCCL(R.getUniqueId(&id), "ncclGetUniqueId");
    QA_NCCL(R.commInitRank(&g_comm, 1, id, 0), "ncclCommInitRank");
    g_mode = Mode::Rccl;
    g_rank = 0;
    createStreams();
    bool ok = pipelined();
    size_t freeComm = 0, totalMem = 0;
    (void)hipMemGetInfo(&freeComm, &totalMem);   // with the communicator up
    // caller's buffers (a swap's exchange buffers): two sets of nBuf / 2
    // peers -- every peer is this rank -- through the pipelined exchange,
    // 4 slices alternating the sets; a byte pattern per buffer and slice,
    // checked at both ends and in the middle of every receive buffer
    bool userOk = true;
    if (userSend && nBuf >= 2) {
        const int np = nBuf / 2;
        std::vector<Xfer> xs[2] = {std::vector<Xfer>((size_t)np), std::vector<Xfer>((size_t)np)};
        const size_t words = bufBytes / 4, probe = std::min<size_t>(words, 1 << 16);
        std::vector<unsigned> back(probe);
        auto check = [&](int set, int slice) {
            for (int p = 0; p < np; p++) {
                const unsigned want = 0x5a000000u + (unsigned)(slice * 256 + set * np + p);
                const unsigned* dev = static_cast<const unsigned*>(userRecv[set * np + p]);
                for (size_t at : {(size_t)0, (words - probe) / 2, words - probe}) {
                    QA_HIP_CHECK(hipMemcpyAsync(back.data(), dev + at, probe * 4, hipMemcpyDeviceToHost, S()));
                    hipk::syncStream();
                    for (size_t i = 0; i < probe; i++) userOk = userOk && back[i] == want;
                }
            }
        };
        for (int s = 0; s < 4; s++) {
            const int b = s & 1;
            for (int p = 0; p < np; p++) {
                const unsigned pat = 0x5a000000u + (unsigned)(s * 256 + b * np + p);
                QA_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)userSend[b * np + p], (int)pat, words, S()));
                xs[b][(size_t)p] = {0, userSend[b * np + p], userRecv[b * np + p], bufBytes};
            }
            exchangeAsync(xs[b].data(), np, b);
            if (s > 0) {
                exchangeWait(1 - b);
                check(1 - b, s - 1);
            }
        }
        exchangeWait(1);
        check(1, 3);
        ok = ok && userOk;
    }
    // exchange: 5 slices through 2 buffer sets, as router::multiSwap does
    const size_t N = (size_t)1 << 20;
    std::vector<double> host(N), back(N);
    double *send[2], *recv[2];
    for (int b = 0; b < 2; b++) {
        QA_HIP_CHECK(hipMalloc(&send[b], N * sizeof(double)));
        QA_HIP_CHECK(hipMalloc(&recv[b], N * sizeof(double)));
    }
    for (int s = 0; s < 5; s++) {
        const int b = s & 1;
        for (size_t i = 0; i < N; i++) host[i] = (double)s * 1e7 + (double)i;
        QA_HIP_CHECK(hipMemcpyAsync(send[b], host.data(), N * sizeof(double), hipMemcpyHostToDevice, S()));
        hipk::syncStream();  // host buffer reused next iteration
        const Xfer x{0, send[b], recv[b], N * sizeof(double)};
        exchangeAsync(&x, 1, b);
        if (s > 0) exchangeWait(1 - b);
        if (s > 0) {
            QA_HIP_CHECK(hipMemcpyAsync(back.data(), recv[1 - b], N * sizeof(double), hipMemcpyDeviceToHost, S()));
            hipk::syncStream();
            for (size_t i = 0; i < N; i++) ok = ok && back[i] == (double)(s - 1) * 1e7 + (double)i;
        }
    }
    exchangeWait(0);
    QA_HIP_CHECK(hipMemcpyAsync(back.data(), recv[0], N * sizeof(double), hipMemcpyDeviceToHost, S()));
    hipk::syncStream();
    for (size_t i = 0; i < N; i++) ok = ok && back[i] == 4e7 + (double)i;
    const bool exchangeOk = ok;
    // scalars
    double vals[70];
    for (int i = 0; i < 70; i++) vals[i] = 0.5 * i;
    rcclAllreduceSum(vals, 70);
    for (int i = 0; i < 70; i++) ok = ok && vals[i] == 0.5 * i;
    unsigned long seeds[2] = {12345ul, 678ul};
    rcclBcast(seeds, sizeof seeds, 0);
    ok = ok && seeds[0] == 12345ul && seeds[1] == 678ul;
    QA_NCCL(R.allGather(send[0], recv[1], N * sizeof(double), ncclUint8, g_comm, S()), "ncclAllGather");
    QA_HIP_CHECK(hipMemcpyAsync(back.data(), recv[1], N * sizeof(double), hipMemcpyDeviceToHost, S()));
    hipk::syncStream();  // polls the watchdog (async errors) while waiting
    for (size_t i = 0; i < N; i++) ok = ok && back[i] == 4e7 + (double)i;
    watchdog(0.0);
    int v = 0;
    R.getVersion(&v);
    int at = snprintf(msg, sizeof msg, "RCCL %d (%s): pipelined exchange %s (5 slices, 2 buffer sets), allreduce, "
                      "broadcast, allgather %s; %.2f GiB free with the communicator up", v, g_libName.c_str(),
                      exchangeOk ? "ok" : "WRONG", ok ? "ok" : "WRONG", freeComm / 1073741824.0);
    if (userSend && nBuf >= 2 && at > 0 && at < (int)sizeof msg)
        snprintf(msg + at, sizeof msg - (size_t)at, "; exchange through the caller's %d x 2 buffers of %.0f MiB %s",
                 nBuf, bufBytes / 1048576.0, userOk ? "ok" : "WRONG");
    report = msg;
    for (int b = 0; b < 2; b++) {
        QA_HIP_CHECK(hipFree(send[b]));
        QA_HIP_CHECK(hipFree(recv[b]));
    }
    finalize();
    return ok;
}

std::string describe() {
    if (g_size == 1) return "single process";
    if (g_mode == Mode::Socket) return "TCP socket mesh, device buffers staged through host (QUEST_COMM=socket)";
    if (g_mode == Mode::Ipc) return ipc::describe() + " (QUEST_COMM=ipc)";
    int v = 0;
    if (R.getVersion) R.getVersion(&v);
    char buf[256];
    if (g_sharedGpu)
        snprintf(buf, sizeof buf, "RCCL %d, ranks sharing one GPU over its network transport (%d ranks, %s, "
                 "QUEST_RCCL_SHARED_GPU=1)", v, g_size, g_libName.c_str());
    else
        snprintf(buf, sizeof buf, "RCCL %d over xGMI (%d ranks, %s)", v, g_size, g_libName.c_str());
    return buf;
}

}  // namespace comm
}  // namespace qa
