// Device IPC transport for ranks sharing one GPU (QUEST_COMM=ipc); protocol
// in comm_ipc.hpp.  Control tokens travel over the socket mesh
// (comm_socket.cpp), amplitudes only through HBM (hipMemcpyAsync from the
// peer's IPC-mapped send buffer into our receive buffer).
#include "comm_ipc.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../hip/qa_hip.h"

namespace qa {
namespace ipc {

namespace {

int g_rank = 0, g_size = 1;
bool g_events = true;  // GPU-side waits on interprocess events (QUEST_IPC_EVENTS=0: host sync)
hipEvent_t g_ready[2] = {nullptr, nullptr};    // ours, interprocess
hipEvent_t g_drained[2] = {nullptr, nullptr};
std::vector<hipEvent_t> g_peerReady, g_peerDrained;  // [peer * 2 + slot], opened from peers' handles

// send buffers we have exported (base allocation -> IPC handle, id)
struct Exported {
    char* base;
    size_t size;
    unsigned long long id;
    hipIpcMemHandle_t handle;
};
std::vector<Exported> g_exported;
unsigned long long g_nextId = 1;

// peers' send buffers we have opened
struct Imported {
    int peer;
    unsigned long long id;
    char* ptr;
    unsigned long long lastUse;
};
std::vector<Imported> g_imported;
unsigned long long g_clock = 0;
constexpr size_t kMaxImportedPerPeer = 16;

struct Token {
    unsigned long long id;
    hipIpcMemHandle_t handle;
    unsigned long long offset, bytes;
};

struct EventHandles {
    hipIpcEventHandle_t ready[2], drained[2];
};

const Exported& exportBuffer(const void* p) {
    const char* c = static_cast<const char*>(p);
    for (const Exported& e : g_exported)
        if (c >= e.base && c < e.base + e.size) return e;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    QA_HIP_CHECK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p));
    Exported e;
    e.base = static_cast<char*>(base);
    e.size = size;
    e.id = g_nextId++;
    QA_HIP_CHECK(hipIpcGetMemHandle(&e.handle, base));
    g_exported.push_back(e);
    return g_exported.back();
}

char* importBuffer(int peer, const Token& t) {
    g_clock++;
    size_t mine = 0, lru = (size_t)-1;
    for (size_t i = 0; i < g_imported.size(); i++) {
        Imported& m = g_imported[i];
        if (m.peer != peer) continue;
        if (m.id == t.id) {
            m.lastUse = g_clock;
            return m.ptr;
        }
        mine++;
        if (lru == (size_t)-1 || m.lastUse < g_imported[lru].lastUse) lru = i;
    }
    if (mine >= kMaxImportedPerPeer) {
        // the peer re-allocated its buffers; unmap the least recently used
        // one once nothing on this device still reads it
        QA_HIP_CHECK(hipDeviceSynchronize());
        QA_HIP_CHECK(hipIpcCloseMemHandle(g_imported[lru].ptr));
        g_imported.erase(g_imported.begin() + (long)lru);
    }
    void* ptr = nullptr;
    QA_HIP_CHECK(hipIpcOpenMemHandle(&ptr, t.handle, hipIpcMemLazyEnablePeerAccess));
    g_imported.push_back({peer, t.id, static_cast<char*>(ptr), g_clock});
    return static_cast<char*>(ptr);
}

}  // namespace

void init(int rank, int size) {
    g_rank = rank;
    g_size = size;
    const char* e = getenv("QUEST_IPC_EVENTS");
    g_events = !(e && atoi(e) == 0);
    if (!g_events) return;
    EventHandles mine;
    for (int s = 0; s < 2; s++) {
        QA_HIP_CHECK(hipEventCreateWithFlags(&g_ready[s], hipEventInterprocess | hipEventDisableTiming));
        QA_HIP_CHECK(hipEventCreateWithFlags(&g_drained[s], hipEventInterprocess | hipEventDisableTiming));
        QA_HIP_CHECK(hipIpcGetEventHandle(&mine.ready[s], g_ready[s]));
        QA_HIP_CHECK(hipIpcGetEventHandle(&mine.drained[s], g_drained[s]));
    }
    std::vector<EventHandles> all((size_t)size);
    sock::allgatherHost(&mine, all.data(), sizeof(EventHandles));
    g_peerReady.assign((size_t)size * 2, nullptr);
    g_peerDrained.assign((size_t)size * 2, nullptr);
    for (int p = 0; p < size; p++) {
        if (p == rank) continue;
        for (int s = 0; s < 2; s++) {
            QA_HIP_CHECK(hipIpcOpenEventHandle(&g_peerReady[(size_t)p * 2 + s], all[(size_t)p].ready[s]));
            QA_HIP_CHECK(hipIpcOpenEventHandle(&g_peerDrained[(size_t)p * 2 + s], all[(size_t)p].drained[s]));
        }
    }
}

void finalize() {
    (void)hipDeviceSynchronize();
    for (Imported& m : g_imported) (void)hipIpcCloseMemHandle(m.ptr);
    g_imported.clear();
    g_exported.clear();
    for (hipEvent_t& ev : g_peerReady)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t& ev : g_peerDrained)
        if (ev) (void)hipEventDestroy(ev);
    g_peerReady.clear();
    g_peerDrained.clear();
    for (int s = 0; s < 2; s++) {
        if (g_ready[s]) (void)hipEventDestroy(g_ready[s]);
        if (g_drained[s]) (void)hipEventDestroy(g_drained[s]);
        g_ready[s] = g_drained[s] = nullptr;
    }
    g_size = 1;
}

void transfer(const comm::Xfer* x, int n, int slot, hipStream_t producer, hipStream_t stream) {
    slot &= 1;
    // 1. our send buffers are complete once the producer reaches this point
    if (g_events)
        QA_HIP_CHECK(hipEventRecord(g_ready[slot], producer));
    else
        QA_HIP_CHECK(hipStreamSynchronize(producer));
    // 2. tell each peer where its data is, learn where ours is
    std::vector<Token> mine((size_t)n), theirs((size_t)n);
    for (int i = 0; i < n; i++) {
        const Exported& e = exportBuffer(x[i].send);
        memset(&mine[(size_t)i], 0, sizeof(Token));
        mine[(size_t)i].id = e.id;
        mine[(size_t)i].handle = e.handle;
        mine[(size_t)i].offset = (unsigned long long)(static_cast<const char*>(x[i].send) - e.base);
        mine[(size_t)i].bytes = x[i].bytes;
    }
    for (int i = 0; i < n; i++) sock::sendrecv(x[i].peer, &mine[(size_t)i], &theirs[(size_t)i], sizeof(Token));
    // 3. pull
    for (int i = 0; i < n; i++) {
        const Token& t = theirs[(size_t)i];
        if (t.bytes != x[i].bytes) {
            fprintf(stderr, "QuEST ipc: rank %d expected %zu bytes from rank %d, peer offers %llu\n", g_rank,
                    x[i].bytes, x[i].peer, t.bytes);
            exit(EXIT_FAILURE);
        }
        char* src = importBuffer(x[i].peer, t) + t.offset;
        if (g_events) QA_HIP_CHECK(hipStreamWaitEvent(stream, g_peerReady[(size_t)x[i].peer * 2 + slot], 0));
        QA_HIP_CHECK(hipMemcpyAsync(x[i].recv, src, x[i].bytes, hipMemcpyDeviceToDevice, stream));
    }
    // 4./5. we are done reading the peers' buffers
    if (g_events)
        QA_HIP_CHECK(hipEventRecord(g_drained[slot], stream));
    else
        QA_HIP_CHECK(hipStreamSynchronize(stream));
    for (int i = 0; i < n; i++) {
        int a = 1, b = 0;
        sock::sendrecv(x[i].peer, &a, &b, sizeof a);
    }
    // 6. and so are they with ours
    if (g_events)
        for (int i = 0; i < n; i++)
            QA_HIP_CHECK(hipStreamWaitEvent(stream, g_peerDrained[(size_t)x[i].peer * 2 + slot], 0));
}

void forget(const void* p) {
    const char* c = static_cast<const char*>(p);
    for (size_t i = 0; i < g_exported.size(); i++)
        if (c >= g_exported[i].base && c < g_exported[i].base + g_exported[i].size) {
            g_exported.erase(g_exported.begin() + (long)i);
            return;
        }
}

std::string describe() {
    return g_events ? "HIP IPC on one device (interprocess events, GPU-side waits)"
                    : "HIP IPC on one device (host-synchronised, QUEST_IPC_EVENTS=0)";
}

}  // namespace ipc
}  // namespace qa
