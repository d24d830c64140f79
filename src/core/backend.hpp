// Hardware backend interface.  Exactly one implementation is linked into a
// library build (compile-time choice, like the reference's
// QuEST/src/CMakeLists.txt:1-15): src/hip/ (MI355X, gfx950) or src/cpu/
// (host plumbing build used on machines without a GPU and as the oracle).
//
// Every function acts on THIS rank's chunk only; all index arguments are
// physical and chunk-local unless stated otherwise.  Reductions return this
// chunk's partial sums (fp64 accumulation); the router combines ranks.
#pragma once

#include "core.hpp"

namespace qa {
namespace be {

// ---- environment -------------------------------------------------------
void envInit(int rank, int numRanks, int localRank);
void envFinalize();
void deviceSync();                 // wait for all queued device work
std::string describe();            // device/backend description for reports
const char* shortName();           // "HIP" or "CPU"
bool stateOnHost();                // CPU build: amplitudes are host memory
bool setTuning(const char* key, int value);  // backend knobs; false if unknown
bool getTuning(const char* key, int* value);  // current value; false if unknown

// ---- memory --------------------------------------------------------------
// Free / total bytes of the memory the state lives in (HIP: device HBM from
// hipMemGetInfo).  False if unknown (host build).  QUEST_DEVICE_MEM_MB
// overrides the free amount on any build (tests of the budget check).
bool memoryInfo(size_t* freeBytes, size_t* totalBytes);
void allocState(QuregImpl& q);     // sets q.re / q.im (numAmpsPerChunk each)
void freeState(QuregImpl& q);
void* allocComm(size_t bytes);     // buffer usable by the comm transport
void freeComm(void* p);

// ---- gate queue ----------------------------------------------------------
// Ops are queued per register and applied, possibly fused, at the latest
// when flush() is called.  Every other backend function flushes first.
void enqueue(QuregImpl& q, const Op& op);
void flush(QuregImpl& q);

// ---- state initialisation -------------------------------------------------
void fill(QuregImpl& q, real re, real im);                     // every amp
void setAmp(QuregImpl& q, i64 local, real re, real im);        // one amp
void initDebug(QuregImpl& q, i64 globalOffset);                // amp[g] = (2g + i(2g+1))/10
// amplitudes whose physical bit `bit` equals `outcome` := val, others 0
void fillWhereBit(QuregImpl& q, int bit, int outcome, real val);
void writeAmps(QuregImpl& q, i64 local, const real* re, const real* im, i64 n);   // host -> chunk
void readAmps(QuregImpl& q, i64 local, real* re, real* im, i64 n);                // chunk -> host
void copyState(QuregImpl& dst, QuregImpl& src);

// Move the qubit on every local position p to dest[p] (a permutation of the
// local positions) by the backend's own means (wave relabelling passes); false
// if it has none for this register (the caller then uses SWAP ops).
bool permuteLocal(QuregImpl& q, const int* dest);

// ---- reductions (partials of this chunk) -----------------------------------
// sum |amp|^2 over amplitudes whose physical bit `bit` == bitVal (bit < 0: all)
double sumSq(QuregImpl& q, int bit, int bitVal);
// every local bit at once (one pass): zeroSums[b] = sumSq(q, b, 0) for b < q.L,
// *total = sumSq(q, -1, 0)
void marginals(QuregImpl& q, double* zeroSums, double* total);
// sum conj(bra) * ket
void innerProduct(QuregImpl& bra, QuregImpl& ket, double out[2]);
// The same for two registers whose local qubits sit on different positions
// (no relayout): sig[p] (p < L) = ket's position of the qubit bra holds at
// local position p; bra's amplitude i pairs with ket's sigma(i).
void innerProductPerm(QuregImpl& bra, QuregImpl& ket, const int* sig, double out[2]);
// Density-matrix diagonal: sum over logical row r in [0, 2^n) of Re rho(r,r),
// restricted to r with logical bit `skipBit` == 0 when skipBit >= 0.  The
// physical flat index of rho(r,r) is sum_{j : bit j of r} offs[j]; only
// indices inside [chunkStart, chunkStart + numAmpsPerChunk) contribute.
double densDiagSum(QuregImpl& q, const u64* offs, int n, int skipBit, i64 chunkStart);

// ---- non-unitary local ops --------------------------------------------------
// a := alpha a + beta b
void axpby(QuregImpl& a, real alpha, QuregImpl& b, real beta);
// the same with b's local qubits on other positions (sig as innerProductPerm)
void axpbyPerm(QuregImpl& a, real alpha, QuregImpl& b, real beta, const int* sig);
// density matrix from a full pure state held in a comm buffer (2^n amps):
// element at chunk-local k (global g = chunkStart + k, r = g mod 2^n,
// c = g div 2^n) := psi_r conj(psi_c)
void densInitPure(QuregImpl& rho, const real* psiRe, const real* psiIm, int n, i64 chunkStart);
// sum_{r,c in chunk} Re[conj(psi_r) rho(r,c) psi_c]
double densFidelity(QuregImpl& rho, const real* psiRe, const real* psiIm, int n, i64 chunkStart);

// ---- distributed support -----------------------------------------------------
// Gather / scatter the amplitudes whose local bits pos[0..k) equal the
// matching bits of setMask (k <= 8), in increasing index order: items
// [start, start+count) of that sub-sequence.
// Swap this chunk's amplitudes whose bits pos[0..k) = myMask with the
// peer's (arrays peerRe / peerIm, mapped into this process) whose bits =
// peerMask, at equal packed index in [start, start + count)
// (comm::swapsInPlace)
void swapPartsWithPeer(QuregImpl& q, real* peerRe, real* peerIm, const int* pos, int k, u64 myMask, u64 peerMask,
                       i64 start, i64 count);
void packBits(QuregImpl& q, const int* pos, int k, u64 setMask, i64 start, i64 count, real* bufRe, real* bufIm);
void unpackBits(QuregImpl& q, const int* pos, int k, u64 setMask, i64 start, i64 count, const real* bufRe,
                const real* bufIm);
// chunk amplitudes [local, local+n) -> comm buffer / comm buffer -> chunk
void toBuffer(QuregImpl& q, i64 local, i64 n, real* bufRe, real* bufIm);
void fromBuffer(QuregImpl& q, i64 local, i64 n, const real* bufRe, const real* bufIm);
// host <-> comm buffer
void bufferToHost(const real* buf, real* host, i64 n);
void hostToBuffer(const real* host, real* buf, i64 n);

// ---- overlapped swaps ----------------------------------------------------------
// swapOverlapBegin(q, lpos, k, myG), right after the pre-swap flush: the
// swap's packs / unpacks (and the transport's stream-ordered exchanges) go to
// a stream of their own, started after everything queued so far; returns
// false (nothing changed) if this backend or configuration cannot overlap.
// swapOverlapEnd(q): the swap is issued.  Until it is settled, passes of q
// whose tiles avoid the swapped local positions lpos run at once on the part
// of the chunk the swap leaves in place (local bits lpos = myG) and their
// other parts are deferred; the first operation that needs the whole chunk
// (any other backend call on q, a pass that includes an lpos, a device sync)
// waits for the swap and runs the deferred parts first, in order.
bool swapOverlapBegin(QuregImpl& q, const int* lpos, int k, int myG);
void swapOverlapEnd(QuregImpl& q);
// Before the pre-swap flush (router planSwap, victims chosen ahead of it and
// kept out of tiles through q.tileAvoid): passes of q launched from now until
// swapOverlapBegin whose tiles avoid lpos run at once on the parts the swap
// sends (local bits lpos != myG) -- so the sends can start -- and on the part
// it keeps only once the swap has been issued, next to the transfer.  False
// if this backend does not split (nothing changed).
bool preSwap(QuregImpl& q, const int* lpos, int k, int myG);
// Receive-side overlap (round 6; the swapped positions may be tile bits): the
// exchange's slices arrive in the order of the chunk's top local positions
// other than lpos -- rangePos[0..b), b <= 3 -- and swapRangeLanded(q, v) is
// called once every slice of range v (rangePos bits = v) has been unpacked.
// Passes of q launched while the swap is in flight whose tiles avoid rangePos
// then run range by range, each range once it has landed, next to the
// transfer of the later ranges; flushes meanwhile keep rangePos out of tile
// padding.  Call after swapOverlapBegin returned true, before any slice.
void swapRanges(QuregImpl& q, const int* rangePos, int b);
void swapRangeLanded(QuregImpl& q, int v);
// Local positions the ops queued for q target, plus the low positions every
// planned tile holds: swap victims outside them are never a tile bit of the
// passes that flush plans.
u64 queuedTargets(const QuregImpl& q);

// ---- swap timing (QuESTStats.swapMicros) --------------------------------------
// swapMark(true) / swapMark(false) bracket one qubit swap on the device
// timeline (HIP: events on the compute stream, so the interval starts when the
// passes queued before the swap have run; host build: wall clock).
// swapMicros(drain) returns the total of the completed intervals, waiting for
// pending ones when drain is set; swapMicrosReset() clears it.
void swapMark(bool begin);
long long swapMicros(bool drain);
void swapMicrosReset();

}  // namespace be
}  // namespace qa
