/*
 * rfec_net.c -- batched UDP I/O for the datagram slots of the wire codec
 * (host C, no HIP).
 *
 * The reference moves one datagram per system call: the session thread's
 * loop (sim_session.c:321-364) waits up to 5 ms in select and reads one
 * datagram with recvfrom (su_udp_recv, common/platform/posix/posix.c:245-275),
 * and every send is one sendto (sim_session_network_send, sim_session.c:286-296
 * -> su_udp_send, posix.c:240-243).  Here a batch of [N][dstride] slots --
 * what rfec_wire_frame_* writes and rfec_wire_parse reads -- moves with
 * sendmmsg / recvmmsg, up to 1024 datagrams per call, straight from / into the
 * (pinned) slot block, so the datagrams need no further host copy before the
 * H2D.  Behaviour kept from the reference: its socket options (su_udp_create,
 * posix.c:133-170), the 1500-byte receive buffer (sim_session.c:333), datagrams
 * shorter than SIM_HEADER_SIZE ignored (:339), zero-length sends refused
 * (:287-288), and the byte / datagram counters (:291-292, :343-344).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "razor_fec.h"
#include "rfec_internal.h"

#define NET_BATCH 1024 /* UIO_MAXIOV: the kernel's cap on messages per sendmmsg / recvmmsg */

static void to_sockaddr(const rfec_udp_addr* a, struct sockaddr_in* s)
{
    memset(s, 0, sizeof(*s));
    s->sin_family = AF_INET;
    s->sin_port = htons(a->port);
    s->sin_addr.s_addr = htonl(a->ip);
}

static void from_sockaddr(const struct sockaddr_in* s, rfec_udp_addr* a)
{
    a->ip = ntohl(s->sin_addr.s_addr);
    a->port = ntohs(s->sin_port);
    a->reserved = 0;
}

int rfec_udp_addr_of(const char* ip, uint16_t port, rfec_udp_addr* addr)
{
    struct in_addr in;
    if (!addr || !ip || inet_pton(AF_INET, ip, &in) != 1)
        return rfec_set_error_sys(RFEC_EINVAL, "udp: bad IPv4 address", 0);
    addr->ip = ntohl(in.s_addr);
    addr->port = port;
    addr->reserved = 0;
    return RFEC_OK;
}

int rfec_udp_open(const char* ip, uint16_t port, unsigned flags, uint32_t buf_bytes, int* fd, rfec_udp_addr* bound)
{
    if (!fd)
        return rfec_set_error_sys(RFEC_EINVAL, "udp: fd is NULL", 0);
    *fd = -1;
    struct sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_port = htons(port);
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (ip && ip[0] && inet_pton(AF_INET, ip, &a.sin_addr) != 1)
        return rfec_set_error_sys(RFEC_EINVAL, "udp: bad IPv4 address", 0);
    const int s = socket(AF_INET, SOCK_DGRAM, 0);
    if (s < 0)
        return rfec_set_error_sys(RFEC_EIO, "udp: socket", errno);
    /* posix.c:135-145: 1 MiB buffers for the server build, 128 KiB otherwise */
    const int bs = buf_bytes ? (int)buf_bytes : ((flags & RFEC_UDP_SERVER) ? 1024 * 1024 : 128 * 1024);
    (void)setsockopt(s, SOL_SOCKET, SO_SNDBUF, &bs, sizeof(bs));
    (void)setsockopt(s, SOL_SOCKET, SO_RCVBUF, &bs, sizeof(bs));
    if (flags & RFEC_UDP_SERVER) { /* su_socket_noblocking (posix.c:232-238) */
        const int fl = fcntl(s, F_GETFL, 0);
        if (fl < 0 || fcntl(s, F_SETFL, fl | O_NONBLOCK) < 0) {
            const int e = errno;
            close(s);
            return rfec_set_error_sys(RFEC_EIO, "udp: O_NONBLOCK", e);
        }
    }
    if (bind(s, (struct sockaddr*)&a, sizeof(a)) < 0) {
        const int e = errno;
        close(s);
        return rfec_set_error_sys(RFEC_EIO, "udp: bind", e);
    }
    if (bound) {
        struct sockaddr_in b;
        socklen_t bl = sizeof(b);
        if (getsockname(s, (struct sockaddr*)&b, &bl) < 0) {
            const int e = errno;
            close(s);
            return rfec_set_error_sys(RFEC_EIO, "udp: getsockname", e);
        }
        from_sockaddr(&b, bound);
    }
    *fd = s;
    return RFEC_OK;
}

void rfec_udp_close(int fd)
{
    if (fd >= 0)
        close(fd);
}

/* 1 when the socket became ready for `ev` within wait_ms, 0 on timeout, <0 on error */
static int wait_ready(int fd, short ev, uint32_t wait_ms)
{
    struct pollfd p = {fd, ev, 0};
    for (;;) {
        const int r = poll(&p, 1, (int)wait_ms);
        if (r >= 0)
            return r > 0;
        if (errno != EINTR)
            return -1;
    }
}

static int check_slots(uint32_t n, uint32_t dstride, const void* dgram, const void* dlen)
{
    if (n && (!dgram || !dlen))
        return rfec_set_error_sys(RFEC_EINVAL, "udp: slot buffers are NULL", 0);
    if (dstride == 0 || dstride > 65535u)
        return rfec_set_error_sys(RFEC_EINVAL, "udp: dstride must be in [1, 65535]", 0);
    return RFEC_OK;
}

int rfec_udp_send_batch(int fd, const rfec_udp_addr* peer, uint32_t n, uint32_t dstride, const uint8_t* dgram,
                        const uint16_t* dlen, uint32_t wait_ms, uint32_t* n_done, rfec_udp_stats* st)
{
    if (n_done)
        *n_done = 0;
    int rc = check_slots(n, dstride, dgram, dlen);
    if (rc)
        return rc;
    if (!peer)
        return rfec_set_error_sys(RFEC_EINVAL, "udp: peer is NULL", 0);
    for (uint32_t i = 0; i < n; ++i)
        if (dlen[i] > dstride)
            return rfec_set_error_sys(RFEC_EINVAL, "udp: datagram longer than its slot", 0);
    struct sockaddr_in to;
    to_sockaddr(peer, &to);
    struct mmsghdr msg[NET_BATCH];
    struct iovec iov[NET_BATCH];
    uint32_t slot_of[NET_BATCH];
    uint32_t i = 0; /* next slot not yet handed to the kernel */
    while (i < n) {
        uint32_t m = 0, j = i;
        for (; j < n && m < NET_BATCH; ++j) {
            if (dlen[j] == 0) { /* sim_session_network_send: nothing to send (sim_session.c:287-288) */
                if (st)
                    st->skipped++;
                continue;
            }
            iov[m].iov_base = (void*)(dgram + (size_t)j * dstride);
            iov[m].iov_len = dlen[j];
            memset(&msg[m].msg_hdr, 0, sizeof(msg[m].msg_hdr));
            msg[m].msg_hdr.msg_name = &to;
            msg[m].msg_hdr.msg_namelen = sizeof(to);
            msg[m].msg_hdr.msg_iov = &iov[m];
            msg[m].msg_hdr.msg_iovlen = 1;
            msg[m].msg_len = 0;
            slot_of[m] = j;
            ++m;
        }
        if (m == 0) { /* only empty slots left in this window */
            i = j;
            continue;
        }
        const int r = sendmmsg(fd, msg, m, MSG_DONTWAIT);
        if (st)
            st->syscalls++;
        if (r < 0) {
            const int e = errno;
            if (e == EINTR)
                continue;
            if (e == EAGAIN || e == EWOULDBLOCK || e == ENOBUFS) {
                if (st)
                    st->stalls++;
                const int w = wait_ms ? wait_ready(fd, POLLOUT, wait_ms) : 0;
                if (w > 0)
                    continue;
                if (n_done)
                    *n_done = i;
                return w < 0 ? rfec_set_error_sys(RFEC_EIO, "udp: poll", errno)
                             : rfec_set_error_sys(RFEC_EAGAIN, "udp: send buffer stayed full", 0);
            }
            if (n_done)
                *n_done = i;
            return rfec_set_error_sys(RFEC_EIO, "udp: sendmmsg", e);
        }
        if (st) {
            st->datagrams += (uint64_t)r;
            for (int q = 0; q < r; ++q)
                st->bytes += iov[q].iov_len;
        }
        /* the first r messages went out: resume after the last of them (a
           partial send leaves the rest, and the empty slots between, for the
           next round) */
        i = r == (int)m ? j : slot_of[r];
        if (n_done)
            *n_done = i;
    }
    return RFEC_OK;
}

int rfec_udp_recv_batch(int fd, uint32_t max, uint32_t dstride, uint8_t* dgram, uint16_t* dlen, rfec_udp_addr* from,
                        uint32_t wait_ms, uint32_t* n, rfec_udp_stats* st)
{
    if (!n)
        return rfec_set_error_sys(RFEC_EINVAL, "udp: n is NULL", 0);
    *n = 0;
    int rc = check_slots(max, dstride, dgram, dlen);
    if (rc)
        return rc;
    if (max == 0)
        return RFEC_OK;
    /* su_udp_recv: wait for the first datagram (select with `ms`) */
    if (wait_ms) {
        const int w = wait_ready(fd, POLLIN, wait_ms);
        if (w < 0)
            return rfec_set_error_sys(RFEC_EIO, "udp: poll", errno);
        if (st)
            st->stalls++;
        if (w == 0)
            return RFEC_OK;
    }
    const uint32_t cap = dstride < RFEC_UDP_RECV_BYTES ? dstride : RFEC_UDP_RECV_BYTES;
    struct mmsghdr msg[NET_BATCH];
    struct iovec iov[NET_BATCH];
    struct sockaddr_in src[NET_BATCH];
    uint32_t got = 0;
    while (got < max) {
        const uint32_t m = (max - got) < NET_BATCH ? (max - got) : NET_BATCH;
        for (uint32_t q = 0; q < m; ++q) {
            iov[q].iov_base = dgram + (size_t)(got + q) * dstride;
            iov[q].iov_len = cap;
            memset(&msg[q].msg_hdr, 0, sizeof(msg[q].msg_hdr));
            msg[q].msg_hdr.msg_name = &src[q];
            msg[q].msg_hdr.msg_namelen = sizeof(src[q]);
            msg[q].msg_hdr.msg_iov = &iov[q];
            msg[q].msg_hdr.msg_iovlen = 1;
            msg[q].msg_len = 0;
        }
        const int r = recvmmsg(fd, msg, m, MSG_DONTWAIT, NULL);
        if (st)
            st->syscalls++;
        if (r < 0) {
            const int e = errno;
            if (e == EINTR)
                continue;
            if (e == EAGAIN || e == EWOULDBLOCK)
                break; /* drained */
            *n = got;
            return rfec_set_error_sys(RFEC_EIO, "udp: recvmmsg", e);
        }
        if (r == 0)
            break;
        /* keep the datagrams the session loop would process (rc >= SIM_HEADER_SIZE,
           sim_session.c:339), packed to the front */
        uint32_t kept = 0;
        for (int q = 0; q < r; ++q) {
            const uint32_t len = msg[q].msg_len;
            if (msg[q].msg_hdr.msg_flags & MSG_TRUNC) {
                if (st)
                    st->truncated++;
            }
            if (len < RFEC_UDP_MIN_DGRAM) {
                if (st)
                    st->dropped++;
                continue;
            }
            const uint32_t dst = got + kept;
            if (dst != got + (uint32_t)q)
                memmove(dgram + (size_t)dst * dstride, dgram + (size_t)(got + q) * dstride, len);
            dlen[dst] = (uint16_t)len;
            if (from)
                from_sockaddr(&src[q], &from[dst]);
            if (st) {
                st->datagrams++;
                st->bytes += len;
            }
            ++kept;
        }
        got += kept;
        if ((uint32_t)r < m)
            break; /* the queue is empty (recvmmsg without MSG_WAITFORONE returns what is there) */
    }
    *n = got;
    return RFEC_OK;
}
