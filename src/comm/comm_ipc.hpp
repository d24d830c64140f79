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
//   1. the producer stream records this rank's interprocess event READY[slot]
//      (its send buffers are packed once that event fires);
//   2. token round 1 (socket, pairwise in the router's (peer ^ rank) order):
//      every rank tells each peer where the send buffer meant for it lives
//      (allocation id + IPC memory handle + offset + bytes);
//   3. the transfer stream waits on the peer's READY[slot] and copies the
//      peer's send buffer into this rank's receive buffer (a pull);
//   4. the transfer stream records DRAINED[slot] (this rank has finished
//      reading every peer's send buffer);
//   5. token round 2: "DRAINED recorded";
//   6. the transfer stream waits on every peer's DRAINED[slot], so whoever
//      waits on the transfer stream afterwards knows both that the data has
//      arrived and that its own send buffers are free again.
// Every wait is a GPU-side wait on an event the peer recorded BEFORE it sent
// the token that let us issue the wait, so no rank ever waits on a record
// that has not been issued.  QUEST_IPC_EVENTS=0 replaces the GPU-side waits
// by host synchronisation before each token (slower, no interprocess
// events needed).
#pragma once

#include <hip/hip_runtime.h>

#include "comm.hpp"

namespace qa {
namespace ipc {

// Collective: socket control mesh (already up), interprocess events.
void init(int rank, int size);
void finalize();
// One exchange as above; `producer` is the stream that packs the send
// buffers, `stream` the one the copies run on (may be the same).
void transfer(const comm::Xfer* x, int n, int slot, hipStream_t producer, hipStream_t stream);
// A comm buffer is about to be freed: forget its handle (a later allocation
// at the same address gets a new id, so peers re-open it).
void forget(const void* p);
std::string describe();

}  // namespace ipc
}  // namespace qa
