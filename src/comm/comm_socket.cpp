// TCP-socket transport: a full mesh of sockets between ranks on host
// buffers.  The CPU build's only transport (comm_host.cpp), and in the HIP
// build the test transport selected by QUEST_COMM=socket (comm_rccl.cpp stages
// device buffers through pinned host memory), which lets several ranks share
// ONE GPU without RCCL (which needs QUEST_RCCL_SHARED_GPU=1 for that) -- so the distributed router
// and its GPU kernels are tested on a single-GPU box (the analogue of the
// reference's oversubscribed `mpiexec -n 4` runs).
#include "comm.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace qa {
namespace sock {

namespace {
int g_rank = 0, g_size = 1;
std::vector<int> g_fd;  // socket to each peer (-1 for self)

void die(const char* m) {
    fprintf(stderr, "QuEST socket comm error (rank %d): %s (%s)\n", g_rank, m, strerror(errno));
    exit(EXIT_FAILURE);
}

struct Endpoint {
    char ip[64];
    int port;
};

void setNoDelay(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

// Failure detection: a peer that makes no progress for QUEST_COMM_TIMEOUT
// seconds (default 900; 0 = wait forever) is reported and this rank exits,
// instead of the whole job hanging on a dead or stuck rank.
int timeoutMs() {
    static const int ms = [] {
        const char* e = getenv("QUEST_COMM_TIMEOUT");
        const double sec = e ? atof(e) : 900.0;
        return sec <= 0 ? -1 : (int)(sec * 1000.0);
    }();
    return ms;
}

int peerOf(int fd) {
    for (int r = 0; r < (int)g_fd.size(); r++)
        if (g_fd[r] == fd) return r;
    return -1;
}

// wait until fd is ready for `events`; exits on timeout
short waitFd(int fd, short events) {
    for (;;) {
        pollfd p{fd, events, 0};
        const int rc = poll(&p, 1, timeoutMs());
        if (rc < 0) {
            if (errno == EINTR) continue;
            die("poll");
        }
        if (rc == 0) {
            fprintf(stderr,
                    "QuEST socket comm error (rank %d): no progress from peer rank %d for %.0f s "
                    "(QUEST_COMM_TIMEOUT); giving up\n",
                    g_rank, peerOf(fd), timeoutMs() / 1000.0);
            exit(EXIT_FAILURE);
        }
        return p.revents;
    }
}

void blockingWrite(int fd, const void* b, size_t n) {
    const char* p = (const char*)b;
    while (n) {
        waitFd(fd, POLLOUT);
        ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
        if (k < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) continue;
        if (k <= 0) die("send");
        p += k;
        n -= (size_t)k;
    }
}

void blockingRead(int fd, void* b, size_t n) {
    char* p = (char*)b;
    while (n) {
        waitFd(fd, POLLIN);
        ssize_t k = ::recv(fd, p, n, MSG_DONTWAIT);
        if (k < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) continue;
        if (k == 0) die("peer closed the connection");
        if (k < 0) die("recv");
        p += k;
        n -= (size_t)k;
    }
}

// simultaneous send and receive on one socket (avoids the deadlock of two
// blocking sends of large messages)
void duplex(int fd, const void* sbuf, void* rbuf, size_t n) {
    const char* s = (const char*)sbuf;
    char* r = (char*)rbuf;
    size_t sent = 0, got = 0;
    while (sent < n || got < n) {
        short ev = 0;
        if (sent < n) ev |= POLLOUT;
        if (got < n) ev |= POLLIN;
        const short rev = waitFd(fd, ev);
        if ((rev & POLLOUT) && sent < n) {
            ssize_t k = ::send(fd, s + sent, n - sent, MSG_NOSIGNAL | MSG_DONTWAIT);
            if (k > 0) sent += (size_t)k;
            else if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) die("send");
        }
        if ((rev & (POLLIN | POLLHUP | POLLERR)) && got < n) {
            ssize_t k = ::recv(fd, r + got, n - got, MSG_DONTWAIT);
            if (k > 0) got += (size_t)k;
            else if (k == 0) die("peer closed the connection");
            else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) die("recv");
        }
    }
}
}  // namespace

void init(int rank, int size) {
    g_rank = rank;
    g_size = size;
    g_fd.assign(size, -1);
    if (size == 1) return;

    int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) die("socket");
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = 0;
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (bind(ls, (sockaddr*)&sa, sizeof sa) != 0) die("bind");
    // room for every peer's connect plus retries (as the bootstrap listener)
    if (listen(ls, size * 8 > SOMAXCONN ? size * 8 : SOMAXCONN) != 0) die("listen");
    socklen_t len = sizeof sa;
    getsockname(ls, (sockaddr*)&sa, &len);

    Endpoint me{};
    std::string host = boot::hostAddress();
    snprintf(me.ip, sizeof me.ip, "%s", host.c_str());
    me.port = ntohs(sa.sin_port);
    std::vector<Endpoint> all(size);
    boot::allgather(rank, size, &me, all.data(), sizeof(Endpoint));

    // connect to lower ranks, accept from higher ranks
    for (int j = 0; j < rank; j++) {
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in to{};
        to.sin_family = AF_INET;
        to.sin_port = htons((uint16_t)all[j].port);
        inet_pton(AF_INET, all[j].ip, &to.sin_addr);
        int tries = 0;
        while (connect(fd, (sockaddr*)&to, sizeof to) != 0) {
            if (++tries > 5000) die("connect");
            close(fd);
            fd = socket(AF_INET, SOCK_STREAM, 0);
            usleep(2000);
        }
        setNoDelay(fd);
        blockingWrite(fd, &rank, sizeof rank);
        g_fd[j] = fd;
    }
    for (int k = rank + 1; k < size; k++) {
        waitFd(ls, POLLIN);  // a rank that never connects times out here
        int fd = accept(ls, nullptr, nullptr);
        if (fd < 0) die("accept");
        setNoDelay(fd);
        int r = -1;
        blockingRead(fd, &r, sizeof r);
        if (r <= rank || r >= size) die("bad peer rank");
        g_fd[r] = fd;
    }
    close(ls);
}

void finalize() {
    for (int& fd : g_fd)
        if (fd >= 0) {
            close(fd);
            fd = -1;
        }
    g_size = 1;
}

void sendrecv(int peer, const void* send, void* recv, size_t bytes) {
    if (peer == g_rank) {
        memcpy(recv, send, bytes);
        return;
    }
    duplex(g_fd[peer], send, recv, bytes);
}

void allreduceSum(double* vals, int n) {
    if (g_size == 1) return;
    std::vector<double> tmp(n);
    if (g_rank == 0) {
        for (int r = 1; r < g_size; r++) {
            blockingRead(g_fd[r], tmp.data(), sizeof(double) * n);
            for (int i = 0; i < n; i++) vals[i] += tmp[i];
        }
        for (int r = 1; r < g_size; r++) blockingWrite(g_fd[r], vals, sizeof(double) * n);
    } else {
        blockingWrite(g_fd[0], vals, sizeof(double) * n);
        blockingRead(g_fd[0], vals, sizeof(double) * n);
    }
}

void bcastHost(void* buf, size_t bytes, int root) {
    if (g_size == 1) return;
    if (g_rank == root) {
        for (int r = 0; r < g_size; r++)
            if (r != root) blockingWrite(g_fd[r], buf, bytes);
    } else {
        blockingRead(g_fd[root], buf, bytes);
    }
}

void allgatherHost(const void* send, void* recv, size_t bytesPerRank) {
    char* out = (char*)recv;
    memcpy(out + (size_t)g_rank * bytesPerRank, send, bytesPerRank);
    for (int r = 0; r < g_size; r++) bcastHost(out + (size_t)r * bytesPerRank, bytesPerRank, r);
}

}  // namespace sock
}  // namespace qa
