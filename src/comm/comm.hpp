// Inter-rank communication used by the distributed router (src/core/router.cpp).
//
// Replaces the reference's MPI layer (QuEST/src/CPU/QuEST_cpu_distributed.c,
// call sites listed in SURVEY.md §2.5).  One process per GPU; the transport is
// chosen at compile time with the backend:
//   HIP build  -> RCCL (comm_rccl.cpp): pairwise ncclSend/ncclRecv over the
//                 direct xGMI link, ncclAllReduce / ncclBroadcast, all ordered
//                 on the backend's HIP stream (no host round trip per slice);
//   CPU build  -> TCP sockets (comm_socket.cpp), used for multi-process tests;
//   HIP build with QUEST_COMM=socket -> the same sockets with device buffers
//                 staged through pinned host memory (several ranks on one GPU,
//                 for tests; RCCL needs one GPU per rank).
// Both are bootstrapped by bootstrap.cpp from torchrun-style environment
// variables (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT) or
// QUEST_BOOTSTRAP_ADDR / QUEST_BOOTSTRAP_PORT.
#pragma once

#include <cstddef>
#include <string>

namespace qa {
namespace comm {

// Rank / world discovered from the environment (1 rank when unset).
void discover(int* rank, int* size, int* localRank);

void init(int rank, int size);
void finalize();
bool active();  // true when size > 1
// A buffer from be::allocComm is about to be freed (transports that cache
// per-buffer state, e.g. IPC handles, drop it).
void bufferFreed(const void* p);

// Exchange `bytes` with `peer`: send from `send`, receive into `recv`
// (both backend comm buffers; must not overlap).
void sendrecv(int peer, const void* send, void* recv, size_t bytes);
// Simultaneous exchanges with several peers (each peer at most once; send
// and recv buffers distinct).  Every rank lists its peers in increasing
// order of (peer XOR rank), so that transports that pair ranks one at a time
// proceed through perfect matchings and cannot deadlock.
struct Xfer {
    int peer;
    const void* send;
    void* recv;
    size_t bytes;
};
void exchange(const Xfer* x, int n);
// Pipelined form: the exchange is ordered after everything already queued on
// the compute stream but runs on a communication stream of its own, so the
// compute stream can pack / unpack other slices meanwhile; exchangeWait(slot)
// orders later compute-stream work after the exchange issued with that slot
// (0 or 1).  Stream-less transports finish inside exchangeAsync.
void exchangeAsync(const Xfer* x, int n, int slot);
void exchangeWait(int slot);
// Whether exchangeAsync / exchangeWait are stream-ordered device operations
// without host waits (RCCL): a swap built from them can run on a stream of
// its own, next to gate passes (overlapped swaps, router multiSwap).
bool exchangeStreamOrdered();
// Whether the transport can send from any device memory (RCCL: the state
// itself), not only from comm buffers (IPC exports them, sockets stage them).
bool sendsFromState();
// In-place part swaps through the peers' mapped device memory (the IPC
// transport: ranks of one node whose memory is mutually mappable).  Instead of
// pack -> send -> receive -> unpack, one rank of each pair runs a kernel that
// reads both parts and writes them swapped (router multiSwap / restore).
// QUEST_IPC_SWAP=0 turns it off (the buffered pipeline then runs).
bool swapsInPlace();
// Collective with the listed peers (each must list this rank, in the same
// pairwise (peer ^ rank) order): once the device work every one of them has
// queued so far is complete, peerPtr[i * nArr + a] is a device pointer to
// peer i's arrays[a] (the same role on every rank).
void mapPeerArrays(const int* peers, int n, void* const* arrays, int nArr, void** peerPtr);
// The device work this rank queued on the peers' memory is complete; returns
// once every listed peer has said the same.
void peersDone(const int* peers, int n);
// In-place sum of host doubles across ranks.
void allreduceSum(double* vals, int n);
// In-place logical AND of a host int across ranks.
int allreduceAnd(int v);
// Broadcast host bytes from root.
void bcastHost(void* buf, size_t bytes, int root);
// Gather `bytesPerRank` from every rank into recv (rank order); comm buffers.
void allgather(const void* send, void* recv, size_t bytesPerRank);
void barrier();
std::string describe();
// Run the device transport's own code paths with a one-rank communicator
// (HIP build: RCCL); false with a reason if unavailable or wrong.  With
// buffers (nBuf send + nBuf recv comm buffers of bufBytes each, nBuf even):
// the pipelined exchange runs through them, two sets of nBuf / 2 peers, as
// a swap with nBuf / 2 peers would use them.
bool selfTest(std::string& report, void* const* send = nullptr, void* const* recv = nullptr, int nBuf = 0,
              size_t bufBytes = 0);

}  // namespace comm

// ---- TCP socket mesh on host buffers (comm_socket.cpp) ------------------------
namespace sock {
void init(int rank, int size);
void finalize();
void sendrecv(int peer, const void* send, void* recv, size_t bytes);
void allreduceSum(double* vals, int n);
void bcastHost(void* buf, size_t bytes, int root);
void allgatherHost(const void* send, void* recv, size_t bytesPerRank);
}  // namespace sock

// ---- bootstrap (bootstrap.cpp) ----------------------------------------------
namespace boot {
// Star rendezvous through rank 0 over TCP.  Every rank contributes `bytes`;
// every rank receives all contributions in rank order.
void allgather(int rank, int size, const void* mine, void* all, size_t bytes);
// Local IPv4 address string of this host, as seen by rank 0's listener.
std::string hostAddress();
}  // namespace boot

}  // namespace qa
