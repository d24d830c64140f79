// Binary checkpoint / restart of a register (quest_amd.h).
//
// The reference's only persistence is the CSV pair reportState ->
// initStateFromSingleFile (QuEST_common.c:166-182, QuEST_cpu.c:1507-1547),
// which prints 12 decimals and parses text: fine for 3 qubits, not for a
// 16-256 GiB state.  Here every rank streams its canonical chunk, in slices,
// to "<path>.<rank>" as raw qreals behind a 64-byte header; a checkpoint
// written by R ranks can be restored on any number of ranks (each rank reads
// its global range from whichever files hold it).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "QuEST.h"
#include "quest_amd.h"

#include "../comm/comm.hpp"
#include "../core/backend.hpp"
#include "../core/router.hpp"
#include "validation.hpp"

namespace qa {
namespace {

struct CkptHeader {
    char magic[8];  // "QAMDCKP1"
    int32_t version;
    int32_t realBytes;
    int32_t numQubits;  // represented
    int32_t isDensity;
    int32_t numChunks;
    int32_t chunkId;
    int64_t ampsPerChunk;
    int64_t ampsTotal;
    char pad[16];
};
static_assert(sizeof(CkptHeader) == 64, "checkpoint header must be 64 bytes");

constexpr i64 kSlice = (i64)1 << 22;  // amplitudes per host staging slice

std::string fileOf(const char* path, int rank) { return std::string(path) + "." + std::to_string(rank); }

bool readHeader(FILE* f, CkptHeader& h) {
    return fread(&h, sizeof h, 1, f) == 1 && !memcmp(h.magic, "QAMDCKP1", 8) && h.version == 1;
}

}  // namespace
}  // namespace qa

using namespace qa;

extern "C" int saveQuregCheckpoint(Qureg qureg, const char* path) {
    QuregImpl& q = *impl(qureg);
    router::canonicalise(q);
    FILE* f = fopen(fileOf(path, q.chunkId).c_str(), "wb");
    int ok = f != nullptr;
    if (ok) {
        CkptHeader h;
        memset(&h, 0, sizeof h);
        memcpy(h.magic, "QAMDCKP1", 8);
        h.version = 1;
        h.realBytes = (int32_t)sizeof(real);
        h.numQubits = q.nRep;
        h.isDensity = q.isDensity ? 1 : 0;
        h.numChunks = q.numChunks;
        h.chunkId = q.chunkId;
        h.ampsPerChunk = q.numAmpsPerChunk;
        h.ampsTotal = q.numAmpsTotal;
        ok = fwrite(&h, sizeof h, 1, f) == 1;
        std::vector<real> re((size_t)std::min(kSlice, q.numAmpsPerChunk)), im(re.size());
        // all re, then all im (each array contiguous in the file)
        for (int part = 0; part < 2 && ok; part++)
            for (i64 off = 0; off < q.numAmpsPerChunk && ok; off += kSlice) {
                const i64 n = std::min(kSlice, q.numAmpsPerChunk - off);
                be::readAmps(q, off, re.data(), im.data(), n);
                ok = fwrite(part == 0 ? re.data() : im.data(), sizeof(real), (size_t)n, f) == (size_t)n;
            }
        ok = (fclose(f) == 0) && ok;
    }
    if (comm::active()) ok = comm::allreduceAnd(ok);
    if (!ok) v::fileOpened(0, __func__);
    return ok;
}

// Every source file this rank will read is opened and validated (header
// fields agree with the rank-0 header and the register, file long enough for
// its chunk) BEFORE the register is touched, so a missing, truncated or
// foreign file leaves the state as it was.
extern "C" int loadQuregCheckpoint(Qureg qureg, const char* path) {
    QuregImpl& q = *impl(qureg);
    // the writer's rank count comes from the rank-0 file
    CkptHeader h0;
    FILE* f0 = fopen(fileOf(path, 0).c_str(), "rb");
    int ok = f0 != nullptr && readHeader(f0, h0);
    if (f0) fclose(f0);
    if (comm::active()) ok = comm::allreduceAnd(ok);
    if (!ok) {
        v::fileOpened(0, __func__);
        return 0;
    }
    int match = h0.numQubits == q.nRep && h0.isDensity == (q.isDensity ? 1 : 0) &&
                h0.realBytes == (int)sizeof(real) && h0.ampsTotal == q.numAmpsTotal && h0.numChunks > 0 &&
                h0.ampsPerChunk > 0 && (i64)h0.numChunks * h0.ampsPerChunk == h0.ampsTotal;
    if (comm::active()) match = comm::allreduceAnd(match);
    if (!match) {
        raiseError(E_CHECKPOINT_MISMATCH, __func__);
        return 0;
    }
    const i64 srcChunk = h0.ampsPerChunk;
    const i64 c0 = (i64)q.chunkId * q.numAmpsPerChunk, c1 = c0 + q.numAmpsPerChunk;
    struct Src {
        int chunk;
        FILE* f;
    };
    std::vector<Src> srcs;
    for (int s = (int)(c0 / srcChunk); s < h0.numChunks && (i64)s * srcChunk < c1; s++) {
        FILE* f = fopen(fileOf(path, s).c_str(), "rb");
        CkptHeader h;
        bool good = f != nullptr && readHeader(f, h) && h.chunkId == s && h.ampsPerChunk == srcChunk &&
                    h.numChunks == h0.numChunks && h.numQubits == h0.numQubits && h.isDensity == h0.isDensity &&
                    h.realBytes == h0.realBytes && h.ampsTotal == h0.ampsTotal;
        if (good) {
            const long long need = (long long)sizeof h + 2ll * (long long)sizeof(real) * srcChunk;
            good = fseeko(f, 0, SEEK_END) == 0 && (long long)ftello(f) >= need;
        }
        if (f) srcs.push_back({s, f});
        ok = ok && good;
    }
    if (comm::active()) ok = comm::allreduceAnd(ok);
    if (!ok) {
        for (Src& x : srcs) fclose(x.f);
        v::fileOpened(0, __func__);
        return 0;
    }
    router::prepareOverwrite(q);
    std::vector<real> re((size_t)std::min(kSlice, q.numAmpsPerChunk)), im(re.size());
    for (Src& x : srcs) {
        const i64 s0 = (i64)x.chunk * srcChunk;
        const i64 lo = std::max(c0, s0), hi = std::min(c1, s0 + srcChunk);
        for (i64 g = lo; ok && g < hi; g += kSlice) {
            const i64 n = std::min(kSlice, hi - g);
            const off_t reOff = (off_t)(sizeof(CkptHeader) + sizeof(real) * (size_t)(g - s0));
            const off_t imOff = (off_t)(sizeof(CkptHeader) + sizeof(real) * (size_t)(srcChunk + g - s0));
            ok = fseeko(x.f, reOff, SEEK_SET) == 0 && fread(re.data(), sizeof(real), (size_t)n, x.f) == (size_t)n &&
                 fseeko(x.f, imOff, SEEK_SET) == 0 && fread(im.data(), sizeof(real), (size_t)n, x.f) == (size_t)n;
            if (ok) be::writeAmps(q, g - c0, re.data(), im.data(), n);
        }
        fclose(x.f);
    }
    if (comm::active()) ok = comm::allreduceAnd(ok);
    if (!ok) v::fileOpened(0, __func__);
    return ok;
}
