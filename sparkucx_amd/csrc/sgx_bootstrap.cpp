// Multi-process bootstrap of the RCCL communicator (§8(f) row 4): the host control plane
// that hands every executor the 128-byte ncclUniqueId.  It replaces the reference's
// ExecutorAdded / IntroduceAllExecutors exchange (shuffle/ucx/rpc/UcxDriverRpcEndpoint
// .scala:21-42, UcxExecutorRpcEndpoint.scala:19-39; CommonUcxShuffleManager.scala:67-100),
// where the driver collects every executor's UCX worker address and introduces all of them
// to each other.  Here one process (the driver role, usually rank 0) serves the id over TCP;
// every other rank joins with its rank number and receives {nranks, id}.  Within a Spark
// deployment the same 128 bytes can ride Spark RPC instead; this is the path for hosts
// without one (JNI tests, the bench, multi-node runs over RoCE/IB with RCCL's own bootstrap
// interface selection).
//
// Wire format (all little-endian): join -> server: magic u32 'SGXB', rank i32.
//                                  server -> join: magic u32, nranks i32, id[128].
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/sgx.h"
#include "sgx_host.h"

#include <algorithm>

namespace {

constexpr uint32_t MAGIC = 0x42584753u;  // "SGXB"

using clk = std::chrono::steady_clock;

int64_t ms_left(clk::time_point deadline) {
    return std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clk::now()).count();
}

// full-length send / recv with a deadline
bool io_all(int fd, void *buf, size_t len, bool send_dir, clk::time_point deadline) {
    char *p = (char *)buf;
    while (len > 0) {
        pollfd pf{fd, (short)(send_dir ? POLLOUT : POLLIN), 0};
        const int64_t left = ms_left(deadline);
        if (left <= 0) return false;
        const int pr = poll(&pf, 1, (int)std::min<int64_t>(left, 1000));
        if (pr < 0 && errno != EINTR) return false;
        if (pr <= 0) continue;
        const ssize_t r = send_dir ? send(fd, p, len, MSG_NOSIGNAL) : recv(fd, p, len, 0);
        if (r <= 0) {
            if (r < 0 && (errno == EINTR || errno == EAGAIN)) continue;
            return false;
        }
        p += r;
        len -= (size_t)r;
    }
    return true;
}

}  // namespace

extern "C" int sgx_bootstrap_serve(int32_t port, int32_t nranks, const uint8_t id[128], int32_t timeout_ms) {
    if (!id || nranks < 1 || port <= 0 || port > 65535 || timeout_ms <= 0)
        return sgx::fail_msg(SGX_ERR_INVALID, "sgx_bootstrap_serve: bad arguments");
    if (nranks == 1) return SGX_OK;
    const clk::time_point deadline = clk::now() + std::chrono::milliseconds(timeout_ms);
    const int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return sgx::fail_msg(SGX_ERR_COMM, "bootstrap: socket: %s", strerror(errno));
    const int one = 1;
    (void)setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (bind(ls, (sockaddr *)&a, sizeof(a)) != 0 || listen(ls, nranks) != 0) {
        const int err = errno;
        close(ls);
        return sgx::fail_msg(SGX_ERR_COMM, "bootstrap: bind/listen on port %d: %s", port, strerror(err));
    }
    std::vector<char> joined((size_t)nranks, 0);
    joined[0] = 1;  // the server is rank 0's side of the handshake
    int have = 1, rc = SGX_OK;
    while (have < nranks) {
        pollfd pf{ls, POLLIN, 0};
        const int64_t left = ms_left(deadline);
        if (left <= 0) {
            rc = sgx::fail_msg(SGX_ERR_TIMEOUT, "bootstrap: %d of %d ranks joined before the timeout", have, nranks);
            break;
        }
        if (poll(&pf, 1, (int)std::min<int64_t>(left, 1000)) <= 0) continue;
        const int c = accept(ls, nullptr, nullptr);
        if (c < 0) continue;
        uint32_t hdr[2] = {0, 0};
        bool ok = io_all(c, hdr, sizeof(hdr), false, deadline) && hdr[0] == MAGIC;
        const int32_t r = (int32_t)hdr[1];
        ok = ok && r > 0 && r < nranks && !joined[(size_t)r];
        if (ok) {
            uint8_t reply[8 + 128];
            const uint32_t m = MAGIC;
            std::memcpy(reply, &m, 4);
            std::memcpy(reply + 4, &nranks, 4);
            std::memcpy(reply + 8, id, 128);
            if (io_all(c, reply, sizeof(reply), true, deadline)) {
                joined[(size_t)r] = 1;
                ++have;
            }
        }
        close(c);  // a malformed or duplicate join is dropped; the rank may retry
    }
    close(ls);
    return rc;
}

extern "C" int sgx_bootstrap_join(const char *host, int32_t port, int32_t rank, int32_t timeout_ms,
                                  uint8_t out_id[128], int32_t *out_nranks) {
    if (!host || !out_id || !out_nranks || rank < 1 || port <= 0 || port > 65535 || timeout_ms <= 0)
        return sgx::fail_msg(SGX_ERR_INVALID, "sgx_bootstrap_join: bad arguments");
    const clk::time_point deadline = clk::now() + std::chrono::milliseconds(timeout_ms);
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    char ps[16];
    snprintf(ps, sizeof(ps), "%d", port);
    if (getaddrinfo(host, ps, &hints, &res) != 0 || !res)
        return sgx::fail_msg(SGX_ERR_COMM, "bootstrap: cannot resolve %s", host);
    int rc = SGX_ERR_TIMEOUT;
    while (ms_left(deadline) > 0) {
        const int s = socket(AF_INET, SOCK_STREAM, 0);
        if (s < 0) break;
        if (connect(s, res->ai_addr, res->ai_addrlen) == 0) {
            const uint32_t hdr[2] = {MAGIC, (uint32_t)rank};
            uint8_t reply[8 + 128];
            if (io_all(s, (void *)hdr, sizeof(hdr), true, deadline) && io_all(s, reply, sizeof(reply), false, deadline)) {
                uint32_t m;
                std::memcpy(&m, reply, 4);
                if (m == MAGIC) {
                    std::memcpy(out_nranks, reply + 4, 4);
                    std::memcpy(out_id, reply + 8, 128);
                    rc = SGX_OK;
                }
            }
            close(s);
            if (rc == SGX_OK) break;
        } else {
            close(s);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(50));  // the server is not up yet
    }
    freeaddrinfo(res);
    if (rc != SGX_OK) return sgx::fail_msg(SGX_ERR_TIMEOUT, "bootstrap: rank %d could not join %s:%d", rank, host, port);
    return SGX_OK;
}
