// TCP star rendezvous used once at createQuESTEnv() time to exchange the RCCL
// unique id (HIP build) or the socket-mesh endpoints (CPU build).
// The reference bootstraps with MPI_Init (QuEST_cpu_distributed.c:135-164);
// MPI is not part of this stack, so the rendezvous is a few hundred bytes
// over one TCP listener on rank 0.
#include "comm.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace qa {
namespace boot {

static std::string envOr(const char* a, const char* b, const char* dflt) {
    if (const char* v = getenv(a)) return v;
    if (b)
        if (const char* v = getenv(b)) return v;
    return dflt;
}

static int bootstrapPort() {
    if (const char* p = getenv("QUEST_BOOTSTRAP_PORT")) return atoi(p);
    if (const char* p = getenv("MASTER_PORT")) return atoi(p) + 1;
    return 29517;
}

static void fatal(const char* what) {
    fprintf(stderr, "QuEST bootstrap error: %s\n", what);
    exit(EXIT_FAILURE);
}

// Non-fatal forms for rank 0's accept loop: a peer that gave up on an earlier
// connection (greeting timeout) leaves a dead socket in the backlog.
static bool tryWriteAll(int fd, const void* buf, size_t n) {
    const char* p = (const char*)buf;
    while (n) {
        ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k <= 0) return false;
        p += k;
        n -= (size_t)k;
    }
    return true;
}

static bool tryReadAll(int fd, void* buf, size_t n) {
    char* p = (char*)buf;
    while (n) {
        ssize_t k = ::recv(fd, p, n, 0);
        if (k <= 0) return false;
        p += k;
        n -= (size_t)k;
    }
    return true;
}

static void writeAll(int fd, const void* buf, size_t n) {
    const char* p = (const char*)buf;
    while (n) {
        ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k <= 0) fatal("send failed");
        p += k;
        n -= (size_t)k;
    }
}

static void readAll(int fd, void* buf, size_t n) {
    char* p = (char*)buf;
    while (n) {
        ssize_t k = ::recv(fd, p, n, 0);
        if (k <= 0) fatal("recv failed");
        p += k;
        n -= (size_t)k;
    }
}

static bool selfConnected(int fd) {
    sockaddr_in a{}, b{};
    socklen_t la = sizeof a, lb = sizeof b;
    if (getsockname(fd, (sockaddr*)&a, &la) != 0 || getpeername(fd, (sockaddr*)&b, &lb) != 0) return false;
    return a.sin_port == b.sin_port && a.sin_addr.s_addr == b.sin_addr.s_addr;
}

static double timeoutSeconds() {
    if (const char* t = getenv("QUEST_BOOTSTRAP_TIMEOUT")) return atof(t);
    return 300.0;
}

std::string hostAddress() {
    return envOr("QUEST_BOOTSTRAP_ADDR", "MASTER_ADDR", "127.0.0.1");
}

// Rank 0's listener, opened at the first rendezvous and kept for the life of
// the process.  Every rendezvous uses it: a rank connects for rendezvous g + 1
// only after rank 0 has answered it for g, i.e. after rank 0 accepted every
// connection of g, so rendezvous never mix.  (Opening a new port per
// rendezvous collided with RCCL, which listens on ephemeral ports of its own
// once its communicator exists: a later rendezvous could not bind, and its
// peers connected to RCCL's listener instead.)
static int g_listener = -1;
// rank 0 greets every connection with this word: a rank that reached some
// other listener on the port (or its own socket) notices and retries
static const unsigned long long kGreeting = 0x5175455354414d44ull;   // "QuESTAMD"

static bool readGreeting(int fd, double seconds) {
    timeval tv{};
    tv.tv_sec = (long)seconds;
    tv.tv_usec = (long)((seconds - (double)tv.tv_sec) * 1e6);
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    unsigned long long g = 0;
    size_t got = 0;
    while (got < sizeof g) {
        const ssize_t k = ::recv(fd, (char*)&g + got, sizeof g - got, 0);
        if (k <= 0) return false;
        got += (size_t)k;
    }
    tv = timeval{};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);   // blocking again
    return g == kGreeting;
}

void allgather(int rank, int size, const void* mine, void* all, size_t bytes) {
    char* out = (char*)all;
    memcpy(out + (size_t)rank * bytes, mine, bytes);
    if (size == 1) return;

    const std::string addr = hostAddress();
    const int port = bootstrapPort();

    if (rank == 0) {
        if (g_listener < 0) {
            int ls = socket(AF_INET, SOCK_STREAM, 0);
            if (ls < 0) fatal("socket");
            int one = 1;
            setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
            sockaddr_in sa{};
            sa.sin_family = AF_INET;
            sa.sin_port = htons((uint16_t)port);
            sa.sin_addr.s_addr = htonl(INADDR_ANY);
            // a peer's connect loop can hold the port for a moment (see the
            // self-connect note below): retry the bind for a few seconds
            for (int tries = 0; bind(ls, (sockaddr*)&sa, sizeof sa) != 0; tries++) {
                if (errno != EADDRINUSE || tries >= 250) fatal("bind (is QUEST_BOOTSTRAP_PORT free?)");
                std::this_thread::sleep_for(std::chrono::milliseconds(20));
            }
            // room for connections that ranks abandoned (greeting timeouts)
            // and retried, so new connects never stall on a full accept queue
            if (listen(ls, std::max(size * 8, SOMAXCONN)) != 0) fatal("listen");
            g_listener = ls;
        }
        std::vector<int> fds(size, -1);
        for (int k = 1; k < size;) {
            int fd = accept(g_listener, nullptr, nullptr);
            if (fd < 0) fatal("accept");
            int r = -1;
            if (!tryWriteAll(fd, &kGreeting, sizeof kGreeting) || !tryReadAll(fd, &r, sizeof r)) {
                close(fd);   // a connection its rank abandoned; the rank retries
                continue;
            }
            if (r <= 0 || r >= size) {   // not one of ours (another job on a reused port)
                close(fd);
                continue;
            }
            if (!tryReadAll(fd, out + (size_t)r * bytes, bytes)) {
                close(fd);
                continue;
            }
            if (fds[r] >= 0) {
                // the rank gave up on an earlier connection (greeting timeout)
                // after rank 0 had accepted it: keep the newest
                close(fds[r]);
                fds[r] = fd;
                continue;
            }
            fds[r] = fd;
            k++;
        }
        for (int r = 1; r < size; r++) {
            writeAll(fds[r], out, bytes * (size_t)size);
            close(fds[r]);
        }
        return;
    }

    // non-root: connect with retries until rank 0 listens and greets
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(addr.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
        fatal("cannot resolve bootstrap address");
    auto t0 = std::chrono::steady_clock::now();
    int fd = -1;
    while (true) {
        fd = socket(AF_INET, SOCK_STREAM, 0);
        // A TCP connect to a local port nobody listens on yet can pick that
        // same port as its ephemeral source and "succeed" against itself
        // (simultaneous open): rank 0 then cannot bind the port and this rank
        // waits forever on its own socket.  Drop such a connection, and one
        // that does not greet like rank 0, and retry.
        // (rank 0 greets when it reaches this rendezvous: wait long enough for
        // a rank 0 still busy with device or RCCL initialisation)
        // (each attempt waits at most 60 s, and never past the budget, so a
        // connection that lands on a listener that never greets is retried)
        const double left =
            timeoutSeconds() - std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (connect(fd, res->ai_addr, res->ai_addrlen) == 0 && !selfConnected(fd) &&
            readGreeting(fd, std::max(1.0, std::min(60.0, left))))
            break;
        close(fd);
        double waited =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (waited > timeoutSeconds()) fatal("timed out connecting to rank 0");
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    freeaddrinfo(res);
    writeAll(fd, &rank, sizeof rank);
    writeAll(fd, mine, bytes);
    readAll(fd, out, bytes * (size_t)size);
    close(fd);
}

}  // namespace boot

namespace comm {

void discover(int* rank, int* size, int* localRank) {
    auto geti = [](const char* a, const char* b, int d) {
        if (const char* v = getenv(a)) return atoi(v);
        if (b)
            if (const char* v = getenv(b)) return atoi(v);
        return d;
    };
    *size = geti("WORLD_SIZE", "QUEST_WORLD_SIZE", 1);
    *rank = geti("RANK", "QUEST_RANK", 0);
    *localRank = geti("LOCAL_RANK", "QUEST_LOCAL_RANK", *rank);
    if (*size < 1) *size = 1;
    if (*rank < 0 || *rank >= *size) {
        fprintf(stderr, "QuEST: RANK=%d outside WORLD_SIZE=%d\n", *rank, *size);
        exit(EXIT_FAILURE);
    }
    if (*size & (*size - 1)) {
        fprintf(stderr, "QuEST: WORLD_SIZE=%d must be a power of 2\n", *size);
        exit(EXIT_FAILURE);
    }
}

}  // namespace comm
}  // namespace qa
