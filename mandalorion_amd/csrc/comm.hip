// comm.cpp — the one exchange step of the sharded D module: every rank clusters,
// orients and builds consensi for its own loci, then rank 0 collects all ranks' results for the
// ordered writer (the reference's single-process Pool writer, defineIsoforms.py:130-166).
//
// Transport:
//   * rendezvous: a TCP star — rank 0 listens on addr:port, the other ranks connect and announce
//     their rank.  This is how the ncclUniqueId travels (rank 0 draws it, the star ships it).
//   * data: RCCL over xGMI when the communicator is bound to a device context (one process per GPU);
//     RCCL has no allgatherv, so the byte all-gather is one ncclAllGather of every rank's bytes padded
//     to the largest rank's count (the byte counts travel first), compacted on the way to the host.
//   * host mode (ctx == NULL): the star itself carries the bytes (CPU-only runs and tests).
// Byte counts, barriers and the max-over-ranks timing reduction always use the star (tiny messages).
#include <arpa/inet.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mando.h"
#include "internal.h"

struct mando_comm {
    int nranks = 1, rank = 0;
    std::vector<int> fd;  // rank 0: fd[r] = socket to rank r (fd[0] = listening socket); others: fd[0]
    mando_ctx *ctx = nullptr;
    ncclComm_t nccl = nullptr;
    hipStream_t stream = nullptr;
    int device = -1;
    void *dsend = nullptr, *drecv = nullptr;
    size_t dsend_cap = 0, drecv_cap = 0;
};

namespace {

double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int send_all(int fd, const void *p, size_t n) {
    const char *c = static_cast<const char *>(p);
    while (n > 0) {
        const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            return mando::set_error(MANDO_E_INTERNAL, std::string("comm send: ") + strerror(errno));
        }
        c += k;
        n -= (size_t)k;
    }
    return MANDO_OK;
}

int recv_all(int fd, void *p, size_t n) {
    char *c = static_cast<char *>(p);
    while (n > 0) {
        const ssize_t k = ::recv(fd, c, n, 0);
        if (k == 0) return mando::set_error(MANDO_E_INTERNAL, "comm recv: peer closed the connection");
        if (k < 0) {
            if (errno == EINTR) continue;
            return mando::set_error(MANDO_E_INTERNAL, std::string("comm recv: ") + strerror(errno));
        }
        c += k;
        n -= (size_t)k;
    }
    return MANDO_OK;
}

int resolve(const char *addr, int port, sockaddr_in *out) {
    memset(out, 0, sizeof(*out));
    out->sin_family = AF_INET;
    out->sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, addr, &out->sin_addr) == 1) return MANDO_OK;
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(addr, nullptr, &hints, &res) != 0 || !res)
        return mando::set_error(MANDO_E_ARG, std::string("comm: cannot resolve ") + addr);
    out->sin_addr = reinterpret_cast<sockaddr_in *>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
    return MANDO_OK;
}

void nodelay(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

// rank 0: listen and accept nranks-1 peers, each announcing its rank
int star_listen(mando_comm *c, const sockaddr_in &sa, double timeout_s) {
    const int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return mando::set_error(MANDO_E_INTERNAL, std::string("comm socket: ") + strerror(errno));
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    c->fd.assign((size_t)c->nranks, -1);
    c->fd[0] = ls;
    if (bind(ls, reinterpret_cast<const sockaddr *>(&sa), sizeof(sa)) != 0)
        return mando::set_error(MANDO_E_INTERNAL, std::string("comm bind: ") + strerror(errno));
    if (listen(ls, c->nranks + 8) != 0)
        return mando::set_error(MANDO_E_INTERNAL, std::string("comm listen: ") + strerror(errno));
    const double t_end = now_s() + timeout_s;
    for (int got = 1; got < c->nranks;) {
        pollfd p{ls, POLLIN, 0};
        const int ms = (int)std::max(1.0, (t_end - now_s()) * 1e3);
        if (now_s() > t_end || poll(&p, 1, ms) <= 0)
            return mando::set_error(MANDO_E_INTERNAL, "comm: timed out waiting for " +
                                                          std::to_string(c->nranks - got) + " rank(s) to connect");
        const int s = accept(ls, nullptr, nullptr);
        if (s < 0) continue;
        nodelay(s);
        int32_t r = -1;
        if (recv_all(s, &r, 4) != MANDO_OK || r <= 0 || r >= c->nranks || c->fd[(size_t)r] >= 0) {
            close(s);
            return mando::set_error(MANDO_E_INTERNAL, "comm: bad rank announcement " + std::to_string(r));
        }
        c->fd[(size_t)r] = s;
        ++got;
    }
    return MANDO_OK;
}

// rank > 0: connect to rank 0 (retried until the deadline: rank 0 may not be listening yet)
int star_connect(mando_comm *c, const sockaddr_in &sa, double timeout_s) {
    const double t_end = now_s() + timeout_s;
    for (;;) {
        const int s = socket(AF_INET, SOCK_STREAM, 0);
        if (s < 0) return mando::set_error(MANDO_E_INTERNAL, std::string("comm socket: ") + strerror(errno));
        if (connect(s, reinterpret_cast<const sockaddr *>(&sa), sizeof(sa)) == 0) {
            nodelay(s);
            c->fd.assign(1, s);
            const int32_t r = c->rank;
            return send_all(s, &r, 4);
        }
        close(s);
        if (now_s() > t_end)
            return mando::set_error(MANDO_E_INTERNAL, "comm: rank " + std::to_string(c->rank) +
                                                          " could not reach rank 0 before the timeout");
        usleep(20000);
    }
}

// every rank's bytes, concatenated in rank order, on every rank (counts[r] = rank r's byte count)
int star_allgather(mando_comm *c, const void *send, int64_t n, std::vector<uint8_t> *all, std::vector<int64_t> *counts) {
    const int R = c->nranks;
    counts->assign((size_t)R, 0);
    if (c->rank == 0) {
        std::vector<std::vector<uint8_t>> parts((size_t)R);
        parts[0].assign(static_cast<const uint8_t *>(send), static_cast<const uint8_t *>(send) + n);
        (*counts)[0] = n;
        for (int r = 1; r < R; ++r) {
            int64_t k = 0;
            int rc = recv_all(c->fd[(size_t)r], &k, 8);
            if (rc) return rc;
            parts[(size_t)r].resize((size_t)k);
            if (k > 0 && (rc = recv_all(c->fd[(size_t)r], parts[(size_t)r].data(), (size_t)k))) return rc;
            (*counts)[(size_t)r] = k;
        }
        all->clear();
        for (auto &p : parts) all->insert(all->end(), p.begin(), p.end());
        for (int r = 1; r < R; ++r) {
            int rc = send_all(c->fd[(size_t)r], counts->data(), 8 * (size_t)R);
            if (!rc && !all->empty()) rc = send_all(c->fd[(size_t)r], all->data(), all->size());
            if (rc) return rc;
        }
        return MANDO_OK;
    }
    int rc = send_all(c->fd[0], &n, 8);
    if (!rc && n > 0) rc = send_all(c->fd[0], send, (size_t)n);
    if (!rc) rc = recv_all(c->fd[0], counts->data(), 8 * (size_t)R);
    if (rc) return rc;
    int64_t tot = 0;
    for (int64_t k : *counts) tot += k;
    all->resize((size_t)tot);
    return tot > 0 ? recv_all(c->fd[0], all->data(), (size_t)tot) : MANDO_OK;
}

// every rank's bytes on rank 0 only (rank order; the other ranks receive nothing)
int star_gather(mando_comm *c, const void *send, int64_t n, std::vector<uint8_t> *all, std::vector<int64_t> *counts) {
    const int R = c->nranks;
    counts->assign((size_t)R, 0);
    if (c->rank != 0) {
        int rc = send_all(c->fd[0], &n, 8);
        if (!rc && n > 0) rc = send_all(c->fd[0], send, (size_t)n);
        return rc;
    }
    all->assign(static_cast<const uint8_t *>(send), static_cast<const uint8_t *>(send) + n);
    (*counts)[0] = n;
    for (int r = 1; r < R; ++r) {
        int64_t k = 0;
        int rc = recv_all(c->fd[(size_t)r], &k, 8);
        if (rc) return rc;
        const size_t at = all->size();
        all->resize(at + (size_t)k);
        if (k > 0 && (rc = recv_all(c->fd[(size_t)r], all->data() + at, (size_t)k))) return rc;
        (*counts)[(size_t)r] = k;
    }
    return MANDO_OK;
}

int nccl_fail(ncclResult_t r, const char *what) {
    return mando::set_error(MANDO_E_INTERNAL, std::string(what) + ": " + ncclGetErrorString(r));
}

int ensure_dev(void **p, size_t *cap, size_t need) {
    if (need <= *cap && *p) return MANDO_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t nb = std::max<size_t>(need, 4096);
    if (hipMalloc(p, nb) != hipSuccess) {
        *p = nullptr;
        (void)hipGetLastError();
        return mando::set_error(MANDO_E_NOMEM, "comm: hipMalloc(" + std::to_string(nb) + ") failed");
    }
    *cap = nb;
    return MANDO_OK;
}

}  // namespace

extern "C" {

int mando_comm_init(mando_ctx *ctx, int nranks, int rank, const char *addr, int port, double timeout_s,
                    mando_comm **out) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && (!addr || port <= 0 || port > 65535)))
        return mando::set_error(MANDO_E_ARG, "mando_comm_init: bad argument");
    *out = nullptr;
    mando_comm *c = new mando_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->ctx = ctx;
    int rc = MANDO_OK;
    if (nranks > 1) {
        sockaddr_in sa;
        rc = resolve(addr, port, &sa);
        if (!rc) rc = rank == 0 ? star_listen(c, sa, timeout_s > 0 ? timeout_s : 300.0)
                                : star_connect(c, sa, timeout_s > 0 ? timeout_s : 300.0);
    }
    if (!rc && ctx) {
        // RCCL on the context's device; rank 0 draws the unique id and ships it over the star
        c->device = mando::ctx_device(ctx);
        c->stream = mando::ctx_stream(ctx);
        ncclUniqueId id;
        static_assert(sizeof(id) == NCCL_UNIQUE_ID_BYTES, "ncclUniqueId size");
        if (rank == 0) {
            const ncclResult_t r = ncclGetUniqueId(&id);
            if (r != ncclSuccess) rc = nccl_fail(r, "ncclGetUniqueId");
            for (int p = 1; p < nranks && !rc; ++p) rc = send_all(c->fd[(size_t)p], &id, sizeof(id));
        } else {
            rc = recv_all(c->fd[0], &id, sizeof(id));
        }
        if (!rc && hipSetDevice(c->device) != hipSuccess) rc = mando::set_error(MANDO_E_HIP, "comm: hipSetDevice failed");
        if (!rc) {
            const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, id, rank);
            if (r != ncclSuccess) {
                c->nccl = nullptr;
                rc = nccl_fail(r, "ncclCommInitRank");
            }
        }
    }
    if (rc) {
        mando_comm_destroy(c);
        return rc;
    }
    *out = c;
    return MANDO_OK;
}

int mando_comm_backend(const mando_comm *c) { return c && c->nccl ? 1 : 0; }

int mando_allgather_counts(mando_comm *c, int64_t n, int64_t *counts) {
    if (!c || !counts || n < 0) return mando::set_error(MANDO_E_ARG, "mando_allgather_counts: bad argument");
    if (c->nranks == 1) {
        counts[0] = n;
        return MANDO_OK;
    }
    std::vector<uint8_t> all;
    std::vector<int64_t> cnt;
    int rc = star_allgather(c, &n, 8, &all, &cnt);
    if (rc) return rc;
    memcpy(counts, all.data(), 8 * (size_t)c->nranks);
    return MANDO_OK;
}

// The RCCL paths' marshalling, kept apart from the transfers so that the CPU suite can replay it
// against the host transport (tests/test_comm.py) without a device.
int mando_rccl_allgather_plan(int nranks, const int64_t *recv_counts, int64_t *maxc, int64_t *dev_off,
                              int64_t *host_off) {
    if (nranks < 1 || !recv_counts || !maxc || !dev_off || !host_off)
        return mando::set_error(MANDO_E_ARG, "mando_rccl_allgather_plan: bad argument");
    int64_t m = 1, o = 0;
    for (int r = 0; r < nranks; ++r) {
        if (recv_counts[r] < 0) return mando::set_error(MANDO_E_ARG, "mando_rccl_allgather_plan: negative count");
        m = std::max(m, recv_counts[r]);
    }
    for (int r = 0; r < nranks; ++r) {
        dev_off[r] = (int64_t)r * m;  // ncclAllGather places rank r's padded slice at r * maxc
        host_off[r] = o;
        o += recv_counts[r];
    }
    *maxc = m;
    return MANDO_OK;
}

int mando_rccl_gather_plan(int nranks, int rank, const int64_t *recv_counts, int64_t *peer_off, int64_t *peer_len,
                           int64_t *d2h_off, int64_t *d2h_len) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !recv_counts || !peer_off || !peer_len || !d2h_off || !d2h_len)
        return mando::set_error(MANDO_E_ARG, "mando_rccl_gather_plan: bad argument");
    int64_t o = 0;
    for (int r = 0; r < nranks; ++r) {
        if (recv_counts[r] < 0) return mando::set_error(MANDO_E_ARG, "mando_rccl_gather_plan: negative count");
        // rank 0 receives peer p's bytes at their offset in the concatenation; a peer sends its own to 0
        peer_off[r] = rank == 0 && r > 0 ? o : 0;
        peer_len[r] = rank == 0 ? (r > 0 ? recv_counts[r] : 0) : (r == 0 ? recv_counts[rank] : 0);
        o += recv_counts[r];
    }
    *d2h_off = rank == 0 ? recv_counts[0] : 0;
    *d2h_len = rank == 0 ? o - recv_counts[0] : 0;
    return MANDO_OK;
}

int mando_allgather_bytes(mando_comm *c, const uint8_t *send, int64_t n, uint8_t *recv, const int64_t *recv_counts) {
    if (!c || !recv_counts || n < 0 || (n > 0 && !send)) return mando::set_error(MANDO_E_ARG, "mando_allgather_bytes: bad argument");
    const int R = c->nranks;
    if (recv_counts[c->rank] != n) return mando::set_error(MANDO_E_ARG, "mando_allgather_bytes: recv_counts[rank] != n");
    int64_t tot = 0;
    std::vector<int64_t> off((size_t)R + 1, 0);
    for (int r = 0; r < R; ++r) {
        if (recv_counts[r] < 0) return mando::set_error(MANDO_E_ARG, "mando_allgather_bytes: negative count");
        off[(size_t)r + 1] = off[(size_t)r] + recv_counts[r];
    }
    tot = off[(size_t)R];
    if (tot > 0 && !recv) return mando::set_error(MANDO_E_ARG, "mando_allgather_bytes: null recv");
    if (R == 1 && !c->nccl) {
        if (n > 0) memcpy(recv, send, (size_t)n);
        return MANDO_OK;
    }
    if (!c->nccl) {
        std::vector<uint8_t> all;
        std::vector<int64_t> cnt;
        int rc = star_allgather(c, send, n, &all, &cnt);
        if (rc) return rc;
        for (int r = 0; r < R; ++r)
            if (cnt[(size_t)r] != recv_counts[r]) return mando::set_error(MANDO_E_ARG, "mando_allgather_bytes: counts disagree");
        if (tot > 0) memcpy(recv, all.data(), (size_t)tot);
        return MANDO_OK;
    }
    // RCCL has no allgatherv: one ncclAllGather of every rank's bytes padded to the largest count
    // (SURVEY.md §8(e)), then each rank's slice is compacted on the way back to the host
    if (hipSetDevice(c->device) != hipSuccess) return mando::set_error(MANDO_E_HIP, "comm: hipSetDevice failed");
    int64_t maxc = 0;
    std::vector<int64_t> dev_off((size_t)R), host_off((size_t)R);
    int rc = mando_rccl_allgather_plan(R, recv_counts, &maxc, dev_off.data(), host_off.data());
    if (!rc) rc = ensure_dev(&c->dsend, &c->dsend_cap, (size_t)maxc);
    if (!rc) rc = ensure_dev(&c->drecv, &c->drecv_cap, (size_t)maxc * (size_t)R);
    if (rc) return rc;
    if (n > 0 && hipMemcpyAsync(c->dsend, send, (size_t)n, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return mando::set_error(MANDO_E_HIP, "comm: H2D copy failed");
    const ncclResult_t r = ncclAllGather(c->dsend, c->drecv, (size_t)maxc, ncclUint8, c->nccl, c->stream);
    if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
    for (int root = 0; root < R; ++root) {
        if (recv_counts[root] == 0) continue;
        if (hipMemcpyAsync(recv + host_off[(size_t)root], static_cast<uint8_t *>(c->drecv) + dev_off[(size_t)root],
                           (size_t)recv_counts[root], hipMemcpyDeviceToHost, c->stream) != hipSuccess)
            return mando::set_error(MANDO_E_HIP, "comm: D2H copy failed");
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return mando::set_error(MANDO_E_HIP, "comm: stream sync failed");
    return MANDO_OK;
}

int mando_gather_bytes(mando_comm *c, const uint8_t *send, int64_t n, uint8_t *recv, const int64_t *recv_counts) {
    if (!c || !recv_counts || n < 0 || (n > 0 && !send)) return mando::set_error(MANDO_E_ARG, "mando_gather_bytes: bad argument");
    const int R = c->nranks;
    if (recv_counts[c->rank] != n) return mando::set_error(MANDO_E_ARG, "mando_gather_bytes: recv_counts[rank] != n");
    std::vector<int64_t> off((size_t)R + 1, 0);
    for (int r = 0; r < R; ++r) {
        if (recv_counts[r] < 0) return mando::set_error(MANDO_E_ARG, "mando_gather_bytes: negative count");
        off[(size_t)r + 1] = off[(size_t)r] + recv_counts[r];
    }
    const int64_t tot = off[(size_t)R];
    const bool root = c->rank == 0;
    if (root && tot > 0 && !recv) return mando::set_error(MANDO_E_ARG, "mando_gather_bytes: null recv on rank 0");
    if (R == 1) {
        if (n > 0) memcpy(recv, send, (size_t)n);
        return MANDO_OK;
    }
    if (!c->nccl) {
        std::vector<uint8_t> all;
        std::vector<int64_t> cnt;
        int rc = star_gather(c, send, n, &all, &cnt);
        if (rc || !root) return rc;
        for (int r = 0; r < R; ++r)
            if (cnt[(size_t)r] != recv_counts[r]) return mando::set_error(MANDO_E_ARG, "mando_gather_bytes: counts disagree");
        if (tot > 0) memcpy(recv, all.data(), (size_t)tot);
        return MANDO_OK;
    }
    // RCCL: point-to-point sends to rank 0 in one group (rank 0 receives each rank's bytes at its
    // offset); no rank but 0 holds more than its own bytes, unlike the padded all-gather
    if (hipSetDevice(c->device) != hipSuccess) return mando::set_error(MANDO_E_HIP, "comm: hipSetDevice failed");
    std::vector<int64_t> peer_off((size_t)R), peer_len((size_t)R);
    int64_t d2h_off = 0, d2h_len = 0;
    int rc = mando_rccl_gather_plan(R, c->rank, recv_counts, peer_off.data(), peer_len.data(), &d2h_off, &d2h_len);
    if (!rc) rc = ensure_dev(&c->dsend, &c->dsend_cap, (size_t)std::max<int64_t>(n, 1));
    if (!rc && root) rc = ensure_dev(&c->drecv, &c->drecv_cap, (size_t)std::max<int64_t>(tot, 1));
    if (rc) return rc;
    if (n > 0 && hipMemcpyAsync(c->dsend, send, (size_t)n, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return mando::set_error(MANDO_E_HIP, "comm: H2D copy failed");
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess) {
        for (int p = 0; p < R && r == ncclSuccess; ++p) {
            if (peer_len[(size_t)p] == 0) continue;
            r = root ? ncclRecv(static_cast<uint8_t *>(c->drecv) + peer_off[(size_t)p], (size_t)peer_len[(size_t)p],
                                ncclUint8, p, c->nccl, c->stream)
                     : ncclSend(c->dsend, (size_t)peer_len[(size_t)p], ncclUint8, p, c->nccl, c->stream);
        }
        const ncclResult_t e = ncclGroupEnd();
        if (r == ncclSuccess) r = e;
    }
    if (r != ncclSuccess) return nccl_fail(r, "ncclSend/ncclRecv gather");
    if (root) {
        if (n > 0) memcpy(recv, send, (size_t)n);  // rank 0's own bytes never leave the host
        if (d2h_len > 0 && hipMemcpyAsync(recv + d2h_off, static_cast<uint8_t *>(c->drecv) + d2h_off, (size_t)d2h_len,
                                          hipMemcpyDeviceToHost, c->stream) != hipSuccess)
            return mando::set_error(MANDO_E_HIP, "comm: D2H copy failed");
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return mando::set_error(MANDO_E_HIP, "comm: stream sync failed");
    return MANDO_OK;
}

int mando_rccl_alltoallv_plan(int nranks, const int64_t *send_counts, const int64_t *recv_counts, int64_t *send_off,
                              int64_t *recv_off) {
    if (nranks < 1 || !send_counts || !recv_counts || !send_off || !recv_off)
        return mando::set_error(MANDO_E_ARG, "mando_rccl_alltoallv_plan: bad argument");
    int64_t so = 0, ro = 0;
    for (int r = 0; r < nranks; ++r) {
        if (send_counts[r] < 0 || recv_counts[r] < 0)
            return mando::set_error(MANDO_E_ARG, "mando_rccl_alltoallv_plan: negative count");
        send_off[r] = so;  // the send buffer holds the parts for ranks 0..R-1 in order, so does recv
        recv_off[r] = ro;
        so += send_counts[r];
        ro += recv_counts[r];
    }
    return MANDO_OK;
}

int mando_alltoallv_bytes(mando_comm *c, const uint8_t *send, const int64_t *send_counts, uint8_t *recv,
                          const int64_t *recv_counts) {
    if (!c || !send_counts || !recv_counts) return mando::set_error(MANDO_E_ARG, "mando_alltoallv_bytes: bad argument");
    const int R = c->nranks, me = c->rank;
    std::vector<int64_t> soff((size_t)R), roff((size_t)R);
    int rc = mando_rccl_alltoallv_plan(R, send_counts, recv_counts, soff.data(), roff.data());
    if (rc) return rc;
    const int64_t stot = soff[(size_t)R - 1] + send_counts[R - 1], rtot = roff[(size_t)R - 1] + recv_counts[R - 1];
    if ((stot > 0 && !send) || (rtot > 0 && !recv)) return mando::set_error(MANDO_E_ARG, "mando_alltoallv_bytes: null buffer");
    if (send_counts[me] != recv_counts[me]) return mando::set_error(MANDO_E_ARG, "mando_alltoallv_bytes: own part sizes differ");
    if (send_counts[me] > 0) memcpy(recv + roff[(size_t)me], send + soff[(size_t)me], (size_t)send_counts[me]);
    if (R == 1) return MANDO_OK;
    if (!c->nccl)  // the host transport has no point-to-point exchange: the caller all-gathers instead
        return mando::set_error(MANDO_E_UNSUPPORTED, "mando_alltoallv_bytes: RCCL communicators only");
    // RCCL: one group of point-to-point sends and receives with every other rank (the own part never
    // leaves the host)
    if (hipSetDevice(c->device) != hipSuccess) return mando::set_error(MANDO_E_HIP, "comm: hipSetDevice failed");
    rc = ensure_dev(&c->dsend, &c->dsend_cap, (size_t)std::max<int64_t>(stot, 1));
    if (!rc) rc = ensure_dev(&c->drecv, &c->drecv_cap, (size_t)std::max<int64_t>(rtot, 1));
    if (rc) return rc;
    if (stot > 0 && hipMemcpyAsync(c->dsend, send, (size_t)stot, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return mando::set_error(MANDO_E_HIP, "comm: H2D copy failed");
    ncclResult_t r = ncclGroupStart();
    for (int p = 0; p < R && r == ncclSuccess; ++p) {
        if (p == me) continue;
        if (send_counts[p] > 0)
            r = ncclSend(static_cast<uint8_t *>(c->dsend) + soff[(size_t)p], (size_t)send_counts[p], ncclUint8, p, c->nccl,
                         c->stream);
        if (r == ncclSuccess && recv_counts[p] > 0)
            r = ncclRecv(static_cast<uint8_t *>(c->drecv) + roff[(size_t)p], (size_t)recv_counts[p], ncclUint8, p, c->nccl,
                         c->stream);
    }
    const ncclResult_t e = ncclGroupEnd();
    if (r == ncclSuccess) r = e;
    if (r != ncclSuccess) return nccl_fail(r, "ncclSend/ncclRecv alltoallv");
    for (int p = 0; p < R; ++p) {
        if (p == me || recv_counts[p] == 0) continue;
        if (hipMemcpyAsync(recv + roff[(size_t)p], static_cast<uint8_t *>(c->drecv) + roff[(size_t)p],
                           (size_t)recv_counts[p], hipMemcpyDeviceToHost, c->stream) != hipSuccess)
            return mando::set_error(MANDO_E_HIP, "comm: D2H copy failed");
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return mando::set_error(MANDO_E_HIP, "comm: stream sync failed");
    return MANDO_OK;
}

int mando_allreduce_max_f64(mando_comm *c, double *v) {
    if (!c || !v) return mando::set_error(MANDO_E_ARG, "mando_allreduce_max_f64: bad argument");
    if (c->nranks == 1) return MANDO_OK;
    std::vector<uint8_t> all;
    std::vector<int64_t> cnt;
    int rc = star_allgather(c, v, 8, &all, &cnt);
    if (rc) return rc;
    double m = *v;
    for (int r = 0; r < c->nranks; ++r) {
        double x;
        memcpy(&x, all.data() + 8 * (size_t)r, 8);
        m = x > m ? x : m;
    }
    *v = m;
    return MANDO_OK;
}

int mando_comm_barrier(mando_comm *c) {
    if (!c) return mando::set_error(MANDO_E_ARG, "mando_comm_barrier: null comm");
    if (c->nranks == 1) return MANDO_OK;
    std::vector<uint8_t> all;
    std::vector<int64_t> cnt;
    return star_allgather(c, nullptr, 0, &all, &cnt);
}

void mando_comm_destroy(mando_comm *c) {
    if (!c) return;
    if (c->nccl) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        ncclCommDestroy(c->nccl);
    }
    if (c->dsend) (void)hipFree(c->dsend);
    if (c->drecv) (void)hipFree(c->drecv);
    for (int f : c->fd)
        if (f >= 0) close(f);
    delete c;
}

}  // extern "C"
