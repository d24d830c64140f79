// HIP backend for MI355X (gfx950): device/stream management, the gate queue
// and its fused tile passes, and the thin wrappers around the kernels.
//
// One process per GPU.  All work of this process is issued on ONE
// non-blocking HIP stream; RCCL exchanges are enqueued on the same stream
// (src/comm/comm_rccl.cpp), so pack -> send/recv -> unpack needs no host
// synchronisation.  The host blocks only when a value must come back
// (reductions, amplitude reads) or at syncQuESTEnv.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "../core/backend.hpp"
#include "../core/router.hpp"
#include "qa_hip.h"
#include "../core/trace.hpp"

namespace qa {
namespace hipk {

namespace {
hipStream_t g_stream = nullptr;
int g_device = 0;
int g_numCUs = 256;
hipDeviceProp_t g_prop;

// Ring of pinned upload slots for tile programs; a slot is reused only after
// the event recorded behind its last use has completed.
// A slot holds the program of one flush: at most kMaxQueued ops, as many
// phases and as many dense 2^R x 2^R blocks (every phase and block holds at
// least one op).
constexpr int kSlots = 32;
constexpr size_t kSlotBytes = 1 << 20;
char* g_progHost = nullptr;
char* g_progDev = nullptr;
hipEvent_t g_slotEvent[kSlots];
bool g_slotUsed[kSlots];
int g_nextSlot = 0;

void (*g_watchdog)(double) = nullptr;
double syncTimeout() {
    static const double t = [] {
        const char* e = getenv("QUEST_SYNC_TIMEOUT");
        return e ? atof(e) : 0.0;
    }();
    return t;
}
}  // namespace

void setSyncWatchdog(void (*poll)(double)) { g_watchdog = poll; }

void syncStream(hipEvent_t ev) {
    if (!g_watchdog && syncTimeout() <= 0) {
        if (ev)
            QA_HIP_CHECK(hipEventSynchronize(ev));
        else
            QA_HIP_CHECK(hipStreamSynchronize(g_stream));
        return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    double nextPoll = 0.01;
    for (long spin = 0;; spin++) {
        const hipError_t e = ev ? hipEventQuery(ev) : hipStreamQuery(g_stream);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) fatal(ev ? "hipEventQuery" : "hipStreamQuery", hipGetErrorString(e), __FILE__, __LINE__);
        (void)hipGetLastError();  // "not ready" is not an error; keep it out of the next launch check
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (syncTimeout() > 0 && el > syncTimeout()) {
            fprintf(stderr,
                    "QuEST: rank %d: device work has not finished after %.1f s (QUEST_SYNC_TIMEOUT); exiting\n",
                    rt().rank, el);
            fflush(stderr);
            exit(EXIT_FAILURE);
        }
        if (g_watchdog && el >= nextPoll) {
            g_watchdog(el);
            nextPoll = el + 0.01;
        }
        if (spin > 2000) usleep(20);
    }
}

Tuning& tuning() {
    static Tuning t = [] {
        Tuning x;
        auto env = [](const char* n, int d) {
            const char* e = getenv(n);
            return e ? atoi(e) : d;
        };
        x.directKernels = env("QUEST_DIRECT_KERNELS", 1);
        x.tileMode = env("QUEST_TILE_MODE", 0);
        x.tileWgPerCU = env("QUEST_TILE_WG_PER_CU", 2);
        x.tileQubits = env("QUEST_TILE_QUBITS", 0);
        x.directLayout = env("QUEST_DIRECT_LAYOUT", 1);
        x.directLowToTile = env("QUEST_DIRECT_LOW_TO_TILE", 1);
        return x;
    }();
    return t;
}

void fatal(const char* expr, const char* err, const char* file, int line) {
    fprintf(stderr, "QuEST HIP error: %s failed: %s (%s:%d)\n", expr, err, file, line);
    fflush(stderr);
    exit(EXIT_FAILURE);
}

hipStream_t stream() { return g_stream; }
int numCUs() { return g_numCUs; }

}  // namespace hipk

namespace be {

using namespace hipk;

namespace {

constexpr size_t kMaxQueued = 256;
static_assert(kMaxQueued * (sizeof(TileOp) + sizeof(TilePhase) + sizeof(real) * 2 * (1 << (2 * kRegSlots))) <=
                  kSlotBytes,
              "upload slot too small for a full flush");

int tileQubits(int L) {
    const int cmin = sizeof(real) == 8 ? 4 : 5;
    int kmax = rt().fuseMaxQubits > 0 ? rt().fuseMaxQubits
                                      : (tuning().tileQubits > 0 ? tuning().tileQubits : kTileQubits);
    kmax = std::min(kmax, 13);
    // keep at least ~128 tiles in flight for small chunks
    int k = std::min(kmax, std::max(cmin + 4, L - 7));
    return std::min(k, L);
}

int contiguousLow(const TilePass& ps) {
    int c = 0;
    while (c < ps.k && ps.pos[c] == c) c++;
    return c;
}

bool directEnabled() { return tuning().directKernels != 0; }

void runProgram(real* re, real* im, int L, const std::vector<Op>& src, TileProgram& prog, int tileMode) {
    // phase op ranges relative to their pass (the kernel sees the pass's ops)
    std::vector<TilePhase> rel = prog.phases;
    for (const TilePass& ps : prog.passes)
        for (int h = ps.phaseBegin; h < ps.phaseEnd; h++) {
            rel[h].opBegin -= ps.opBegin;
            rel[h].opEnd -= ps.opBegin;
        }
    const size_t opBytes = sizeof(TileOp) * prog.ops.size();
    const size_t phBytes = sizeof(TilePhase) * rel.size();
    const size_t matBytes = sizeof(real) * prog.mats.size();
    const size_t total = opBytes + phBytes + matBytes;
    if (total > kSlotBytes) fatal("tile program", "too many ops in one flush", __FILE__, __LINE__);
    const int s = g_nextSlot;
    g_nextSlot = (g_nextSlot + 1) % kSlots;
    if (g_slotUsed[s]) syncStream(g_slotEvent[s]);
    char* h = g_progHost + s * kSlotBytes;
    char* d = g_progDev + s * kSlotBytes;
    memcpy(h, prog.ops.data(), opBytes);
    if (phBytes) memcpy(h + opBytes, rel.data(), phBytes);
    if (matBytes) memcpy(h + opBytes + phBytes, prog.mats.data(), matBytes);
    QA_HIP_CHECK(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, g_stream));
    const TileOp* dOps = reinterpret_cast<const TileOp*>(d);
    const TilePhase* dPh = reinterpret_cast<const TilePhase*>(d + opBytes);
    const real* dMats = reinterpret_cast<const real*>(d + opBytes + phBytes);
    for (const TilePass& ps : prog.passes) {
        const int nOps = ps.opEnd - ps.opBegin;
        stats().passes++;
        if (nOps > 1) stats().fusedOps += nOps;
        if (nOps == 1 && directEnabled() && launchDirectOp(re, im, L, src[ps.opBegin])) continue;
        TileArgs a;
        a.L = L;
        a.k = ps.k;
        a.c = contiguousLow(ps);
        a.nOps = nOps;
        a.nPhases = ps.phaseEnd - ps.phaseBegin;
        a.pad = 0;
        a.numTiles = 1ll << (L - ps.k);
        for (int i = 0; i < 32; i++) a.pos[i] = i < ps.k ? ps.pos[i] : 0;
        launchTilePass(re, im, a, dOps + ps.opBegin, dPh + ps.phaseBegin, dMats, tileMode);
    }
    QA_HIP_CHECK(hipEventRecord(g_slotEvent[s], g_stream));
    g_slotUsed[s] = true;
}

}  // namespace

void envInit(int rank, int numRanks, int localRank) {
    (void)rank;
    (void)numRanks;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        printf("Trying to run GPU code with no GPU available\n");
        exit(EXIT_FAILURE);
    }
    g_device = localRank % count;
    QA_HIP_CHECK(hipSetDevice(g_device));
    QA_HIP_CHECK(hipGetDeviceProperties(&g_prop, g_device));
    g_numCUs = g_prop.multiProcessorCount > 0 ? g_prop.multiProcessorCount : 256;
    QA_HIP_CHECK(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
    QA_HIP_CHECK(hipHostMalloc(&g_progHost, kSlots * kSlotBytes, hipHostMallocDefault));
    QA_HIP_CHECK(hipMalloc(&g_progDev, kSlots * kSlotBytes));
    for (int i = 0; i < kSlots; i++) {
        QA_HIP_CHECK(hipEventCreateWithFlags(&g_slotEvent[i], hipEventDisableTiming));
        g_slotUsed[i] = false;
    }
}

void envFinalize() {
    if (!g_stream) return;
    syncStream();
    for (int i = 0; i < kSlots; i++) (void)hipEventDestroy(g_slotEvent[i]);
    (void)hipHostFree(g_progHost);
    (void)hipFree(g_progDev);
    (void)hipStreamDestroy(g_stream);
    g_stream = nullptr;
    g_progHost = g_progDev = nullptr;
}

void deviceSync() {
    if (g_stream) syncStream();
}

std::string describe() {
    char buf[512];
    snprintf(buf, sizeof buf, "%s (%s), %d CUs, %.1f GiB HBM, device %d", g_prop.name, g_prop.gcnArchName, g_numCUs,
             (double)g_prop.totalGlobalMem / (1024.0 * 1024 * 1024), g_device);
    return buf;
}

const char* shortName() { return "HIP"; }
bool stateOnHost() { return false; }

// The re and im arrays of a register.  QUEST_ALLOC_MODE=1 places both in
// one allocation, im starting QUEST_IM_OFFSET bytes after the end of re
// (HBM channel / TLB placement experiments); the default is two allocations.
void allocState(QuregImpl& q) {
    const size_t bytes = sizeof(real) * (size_t)q.numAmpsPerChunk;
    const char* mode = getenv("QUEST_ALLOC_MODE");
    if (mode && atoi(mode) == 1) {
        const char* o = getenv("QUEST_IM_OFFSET");
        size_t off = o ? (size_t)atoll(o) : 0;
        off = (off + 255) & ~(size_t)255;
        char* base = nullptr;
        if (hipMalloc(&base, 2 * bytes + off) != hipSuccess) {
            fprintf(stderr, "QuEST: out of device memory allocating 2 x %.2f GiB for a %d-qubit register\n",
                    (double)bytes / (1 << 30), q.nSV);
            exit(EXIT_FAILURE);
        }
        q.re = reinterpret_cast<real*>(base);
        q.im = reinterpret_cast<real*>(base + bytes + off);
        q.jointAlloc = true;
        return;
    }
    if (hipMalloc(&q.re, bytes) != hipSuccess || hipMalloc(&q.im, bytes) != hipSuccess) {
        fprintf(stderr, "QuEST: out of device memory allocating 2 x %.2f GiB for a %d-qubit register\n",
                (double)bytes / (1 << 30), q.nSV);
        exit(EXIT_FAILURE);
    }
    q.jointAlloc = false;
}

void freeState(QuregImpl& q) {
    deviceSync();
    (void)hipFree(q.re);
    if (!q.jointAlloc) (void)hipFree(q.im);
    q.re = q.im = nullptr;
}

void* allocComm(size_t bytes) {
    void* p = nullptr;
    QA_HIP_CHECK(hipMalloc(&p, bytes ? bytes : 16));
    return p;
}

void freeComm(void* p) {
    deviceSync();
    (void)hipFree(p);
}

void enqueue(QuregImpl& q, const Op& op) {
    q.pending.push_back(op);
    if (q.pending.size() >= kMaxQueued) flush(q);
}

void flush(QuregImpl& q) {
    if (q.pending.empty()) return;
    trace::Range range("quest.flush");
    const size_t opsIn = q.pending.size();
    TileProgram prog;
    const int cmin = sizeof(real) == 8 ? 4 : 5;
    std::vector<Op> raw;
    if (rt().verify) raw = q.pending;
    planTiles(q.pending, q.L, tileQubits(q.L), cmin, rt().fusion, prog);
    if (tuning().tileMode == 1)
        planPhases(prog, kTileQubits, kRegSlots);
    else if (tuning().tileMode == 2)
        planDenseBlocks(prog, kTileQubits, kRegSlots);
    if (trace::on())
        trace::event("flush", "\"qubits\": %d, \"ops\": %zu, \"ops_fused\": %zu, \"passes\": %zu", q.L, opsIn,
                     q.pending.size(), prog.passes.size());
    std::vector<Op> src;
    src.swap(q.pending);
    if (!rt().verify) {
        runProgram(q.re, q.im, q.L, src, prog, tuning().tileMode);
        return;
    }
    // debug mode: the same ops one pass each (no fusion, no reordering, the
    // direct kernels where they apply) on a shadow copy, then compare
    const size_t bytes = sizeof(real) * (size_t)q.numAmpsPerChunk;
    real *sr = nullptr, *si = nullptr;
    QA_HIP_CHECK(hipMalloc(&sr, bytes));
    QA_HIP_CHECK(hipMalloc(&si, bytes));
    QA_HIP_CHECK(hipMemcpyAsync(sr, q.re, bytes, hipMemcpyDeviceToDevice, g_stream));
    QA_HIP_CHECK(hipMemcpyAsync(si, q.im, bytes, hipMemcpyDeviceToDevice, g_stream));
    runProgram(q.re, q.im, q.L, src, prog, tuning().tileMode);
    const Stats keep = stats();
    TileProgram ref;
    planTiles(raw, q.L, tileQubits(q.L), cmin, false, ref);
    runProgram(sr, si, q.L, raw, ref, 0);
    stats() = keep;
    if (rt().verifyInject) {
        rt().verifyInject = false;
        launchFill(q.re, q.im, 1, (real)0.5, (real)0);
    }
    const double diff = reduceMaxDiff(q.re, q.im, sr, si, q.numAmpsPerChunk);
    QA_HIP_CHECK(hipFree(sr));
    QA_HIP_CHECK(hipFree(si));
    verifyFlush(q.L, raw.size(), prog.passes.size(), diff);
}

void fill(QuregImpl& q, real re, real im) {
    flush(q);
    launchFill(q.re, q.im, q.numAmpsPerChunk, re, im);
}

void setAmp(QuregImpl& q, i64 local, real re, real im) {
    flush(q);
    launchFill(q.re + local, q.im + local, 1, re, im);
}

void initDebug(QuregImpl& q, i64 globalOffset) {
    flush(q);
    launchInitDebug(q.re, q.im, q.numAmpsPerChunk, globalOffset);
}

void fillWhereBit(QuregImpl& q, int bit, int outcome, real val) {
    flush(q);
    launchFillWhereBit(q.re, q.im, q.numAmpsPerChunk, bit, outcome, val);
}

void writeAmps(QuregImpl& q, i64 local, const real* re, const real* im, i64 n) {
    flush(q);
    QA_HIP_CHECK(hipMemcpyAsync(q.re + local, re, sizeof(real) * n, hipMemcpyHostToDevice, g_stream));
    QA_HIP_CHECK(hipMemcpyAsync(q.im + local, im, sizeof(real) * n, hipMemcpyHostToDevice, g_stream));
    syncStream();
}

void readAmps(QuregImpl& q, i64 local, real* re, real* im, i64 n) {
    flush(q);
    QA_HIP_CHECK(hipMemcpyAsync(re, q.re + local, sizeof(real) * n, hipMemcpyDeviceToHost, g_stream));
    QA_HIP_CHECK(hipMemcpyAsync(im, q.im + local, sizeof(real) * n, hipMemcpyDeviceToHost, g_stream));
    syncStream();
}

void copyState(QuregImpl& dst, QuregImpl& src) {
    flush(src);
    flush(dst);
    const size_t bytes = sizeof(real) * (size_t)dst.numAmpsPerChunk;
    QA_HIP_CHECK(hipMemcpyAsync(dst.re, src.re, bytes, hipMemcpyDeviceToDevice, g_stream));
    QA_HIP_CHECK(hipMemcpyAsync(dst.im, src.im, bytes, hipMemcpyDeviceToDevice, g_stream));
}

double sumSq(QuregImpl& q, int bit, int bitVal) {
    flush(q);
    return reduceSumSq(q.re, q.im, q.numAmpsPerChunk, bit, bitVal);
}

void innerProduct(QuregImpl& bra, QuregImpl& ket, double out[2]) {
    flush(bra);
    flush(ket);
    reduceInner(bra.re, bra.im, ket.re, ket.im, bra.numAmpsPerChunk, out);
}

double densDiagSum(QuregImpl& q, const u64* offs, int n, int skipBit, i64 chunkStart) {
    flush(q);
    return reduceDensDiag(q.re, q.numAmpsPerChunk, offs, n, skipBit, chunkStart);
}

void axpby(QuregImpl& a, real alpha, QuregImpl& b, real beta) {
    flush(a);
    flush(b);
    launchAxpby(a.re, a.im, alpha, b.re, b.im, beta, a.numAmpsPerChunk);
}

void densInitPure(QuregImpl& rho, const real* pr, const real* pi, int n, i64 chunkStart) {
    flush(rho);
    launchDensInitPure(rho.re, rho.im, rho.numAmpsPerChunk, pr, pi, n, chunkStart);
}

double densFidelity(QuregImpl& rho, const real* pr, const real* pi, int n, i64 chunkStart) {
    flush(rho);
    return reduceDensFidelity(rho.re, rho.im, rho.numAmpsPerChunk, pr, pi, n, chunkStart);
}

void packBits(QuregImpl& q, const int* pos, int k, u64 setMask, i64 start, i64 count, real* br, real* bi) {
    flush(q);
    launchPackBits(q.re, q.im, pos, k, setMask, start, count, br, bi, false);
}

void unpackBits(QuregImpl& q, const int* pos, int k, u64 setMask, i64 start, i64 count, const real* br,
                const real* bi) {
    flush(q);
    launchPackBits(q.re, q.im, pos, k, setMask, start, count, const_cast<real*>(br), const_cast<real*>(bi), true);
}

void toBuffer(QuregImpl& q, i64 local, i64 n, real* br, real* bi) {
    flush(q);
    QA_HIP_CHECK(hipMemcpyAsync(br, q.re + local, sizeof(real) * n, hipMemcpyDeviceToDevice, g_stream));
    QA_HIP_CHECK(hipMemcpyAsync(bi, q.im + local, sizeof(real) * n, hipMemcpyDeviceToDevice, g_stream));
}

void fromBuffer(QuregImpl& q, i64 local, i64 n, const real* br, const real* bi) {
    flush(q);
    QA_HIP_CHECK(hipMemcpyAsync(q.re + local, br, sizeof(real) * n, hipMemcpyDeviceToDevice, g_stream));
    QA_HIP_CHECK(hipMemcpyAsync(q.im + local, bi, sizeof(real) * n, hipMemcpyDeviceToDevice, g_stream));
}

void bufferToHost(const real* buf, real* host, i64 n) {
    QA_HIP_CHECK(hipMemcpyAsync(host, buf, sizeof(real) * n, hipMemcpyDeviceToHost, g_stream));
    syncStream();
}

void hostToBuffer(const real* host, real* buf, i64 n) {
    QA_HIP_CHECK(hipMemcpyAsync(buf, host, sizeof(real) * n, hipMemcpyHostToDevice, g_stream));
    syncStream();
}

}  // namespace be
}  // namespace qa

namespace qa {
namespace be {
bool setTuning(const char* key, int value) {
    std::string k(key);
    if (k == "direct_kernels") hipk::tuning().directKernels = value;
    else if (k == "tile_mode") hipk::tuning().tileMode = value;
    else if (k == "tile_qubits") hipk::tuning().tileQubits = value;
    else if (k == "direct_layout") hipk::tuning().directLayout = value;
    else if (k == "direct_low_to_tile") hipk::tuning().directLowToTile = value;
    else if (k == "tile_wg_per_cu") hipk::tuning().tileWgPerCU = value;
    else return false;
    return true;
}
}  // namespace be
}  // namespace qa
