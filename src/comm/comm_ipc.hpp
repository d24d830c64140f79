// Device IPC transport (HIP build, QUEST_COMM=ipc): ranks that share ONE GPU
// exchange device buffers directly through HIP IPC memory handles, with the
// same stream/event protocol the RCCL transport uses (comm_rccl.cpp).
//
// RCCL refuses two ranks on one device ("Duplicate GPU detected"), so on a
// single-GPU machine this is the transport that runs the distributed data
// path -- pack on the compute stream, exchange on the communication stream,
// unpack after an event wait, double-buffered -- on real hardware.  The data
// never leaves HBM; only 16-byte control tokens go over the socket mesh of
// comm_socket.cpp.
//
// Protocol of one exchange with peers x[0..n) (buffers from allocComm):
//   1. a local event recorded on the producer stream behind the packs; the
//      host waits for it (the send buffers of this slot are complete);
//   2. token round 1 (socket, pairwise in the router's (peer ^ rank) order):
//      every rank tells each peer where the send buffer meant for it lives
//      (allocation id + IPC memory handle + offset + bytes);
//   3. the transfer stream copies each peer's send buffer into this rank's
//      receive buffer (a pull through the IPC mapping) and records a local
//      "copied" event -- transfer() returns here, the copies run while the
//      compute stream goes on unpacking / packing other slices;
//   4. complete(slot), called when the compute stream is about to depend on
//      the slot (comm::exchangeWait) or before the slot is reused: the host
//      waits for the "copied" event, then token round 2 tells the peers that
//      their send buffers are free again.
// No rank ever copies from a buffer its owner has not finished (step 1
// precedes the token), and no rank repacks a send buffer before every reader
// has confirmed its copy (step 4 precedes the next use of the slot).  All
// waits are on local events; interprocess events (whose stream waits failed
// intermittently on ROCm 7.2 with hipErrorInvalidValue on the following copy)
// are not needed.
#pragma once

#include <hip/hip_runtime.h>

#include "comm.hpp"

namespace qa {
namespace ipc {

// After the socket control mesh is up (comm_socket.cpp).
void init(int rank, int size);
void finalize();
// Steps 1-3 of one exchange; `producer` is the stream that packs the send
// buffers, `stream` the one the copies run on (may be the same).
void transfer(const comm::Xfer* x, int n, int slot, hipStream_t producer, hipStream_t stream);
// Step 4 for the exchange last issued with `slot` (no-op if none pending).
void complete(int slot);
// In-place swaps (comm::mapPeerArrays / peersDone): the host waits for
// `producer`, then one token round per peer trades IPC handles of the listed
// arrays (any device allocation, the state included); done() waits for
// `producer` again and trades a completion token with each peer.
void mapArrays(const int* peers, int n, void* const* arrays, int nArr, void** out, hipStream_t producer);
void done(const int* peers, int n, hipStream_t producer);
// A comm buffer is about to be freed: forget its handle (a later allocation
// at the same address gets a new id, so peers re-open it).
void forget(const void* p);
// Close every mapping of a peer's state array (mapArrays): before a register
// is freed (forget) -- destroying one is collective, so all ranks release
// their mappings of each other's states there.
void releaseStateMappings();
std::string describe();

}  // namespace ipc
}  // namespace qa
