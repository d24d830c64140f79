// comm:: for the host (CPU) build: the socket mesh of comm_socket.cpp on
// host buffers (the state lives in host memory).
#include <cstdio>
#include <cstdlib>
#include "comm.hpp"

namespace qa {
namespace comm {

namespace {
int g_size = 1;
}

void init(int rank, int size) {
    g_size = size;
    sock::init(rank, size);
}
void finalize() {
    sock::finalize();
    g_size = 1;
}
bool active() { return g_size > 1; }
void bufferFreed(const void*) {}
void sendrecv(int peer, const void* send, void* recv, size_t bytes) { sock::sendrecv(peer, send, recv, bytes); }
void exchange(const Xfer* x, int n) {
    for (int i = 0; i < n; i++) sock::sendrecv(x[i].peer, x[i].send, x[i].recv, x[i].bytes);
}
void exchangeAsync(const Xfer* x, int n, int) { exchange(x, n); }
bool sendsFromState() { return false; }
bool exchangeStreamOrdered() { return false; }
bool swapsInPlace() { return false; }
void mapPeerArrays(const int*, int, void* const*, int, void**) {
    fprintf(stderr, "QuEST: in-place peer swaps need the device IPC transport\n");
    exit(EXIT_FAILURE);
}
void peersDone(const int*, int) {}
void exchangeWait(int) {}
void allreduceSum(double* vals, int n) { sock::allreduceSum(vals, n); }
int allreduceAnd(int v) {
    double d = v ? 0.0 : 1.0;  // count failures
    sock::allreduceSum(&d, 1);
    return d == 0.0 ? 1 : 0;
}
void bcastHost(void* buf, size_t bytes, int root) { sock::bcastHost(buf, bytes, root); }
void allgather(const void* send, void* recv, size_t bytesPerRank) { sock::allgatherHost(send, recv, bytesPerRank); }
void barrier() {
    double d = 1;
    sock::allreduceSum(&d, 1);
}
bool selfTest(std::string& report, void* const*, void* const*, int, size_t) {
    report = "host build: no device transport";
    return false;
}
std::string describe() { return g_size > 1 ? "TCP socket mesh (host build)" : "single process"; }

}  // namespace comm
}  // namespace qa
