// ina_send.cpp -- host send path of libina.so.
//
// send_gradients keeps the reference's C signature (communicator.h:27) so the
// reference's ctypes loader (communicator.py:15-24) binds it unchanged.  Where
// communicator.cc:23-41 builds each 524-byte packet_t on the CPU (memcpy + 131
// htonl) and issues one sendto() per packet, this path copies the gradient slice
// to HBM once, builds all packets with the gfx950 pack kernel (ina_pack_c128),
// copies them back into a pinned buffer and hands them to the kernel in batches
// of up to 1024 datagrams per sendmmsg() call.
#include <hip/hip_runtime.h>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <vector>

#include "ina.h"
#include "ina_internal.h"

namespace {

struct Staging {   // per host thread (the reference fans send_gradients out over threads)
    uint32_t* d_grad = nullptr;
    uint8_t* d_pkts = nullptr;
    uint8_t* h_pkts = nullptr;
    size_t cap_pkts = 0;
    hipStream_t stream = nullptr;
    ~Staging() {
        if (d_grad) (void)hipFree(d_grad);
        if (d_pkts) (void)hipFree(d_pkts);
        if (h_pkts) (void)hipHostFree(h_pkts);
        if (stream) (void)hipStreamDestroy(stream);
    }
    int reserve(size_t npk) {
        if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess)
            return INA_EHIP;
        if (npk <= cap_pkts) return INA_OK;
        if (d_grad) (void)hipFree(d_grad);
        if (d_pkts) (void)hipFree(d_pkts);
        if (h_pkts) (void)hipHostFree(h_pkts);
        d_grad = nullptr; d_pkts = nullptr; h_pkts = nullptr; cap_pkts = 0;
        if (hipMalloc(&d_grad, npk * INA_C128_VALUES * 4) != hipSuccess) return INA_ENOMEM;
        if (hipMalloc(&d_pkts, npk * INA_C128_BYTES) != hipSuccess) return INA_ENOMEM;
        if (hipHostMalloc(&h_pkts, npk * INA_C128_BYTES, hipHostMallocDefault) != hipSuccess)
            return INA_ENOMEM;
        cap_pkts = npk;
        return INA_OK;
    }
};

thread_local Staging g_stage;

}  // namespace

extern "C" {

int ina_send_gradients_fd(int fd, const uint32_t* gradient_array, int packet_num, uint32_t dst_ip,
                          int worker_id, uint32_t aggregator_index, int tensor_index) {
    if (packet_num < 0) return ina::set_error(INA_EINVAL, "packet_num < 0%s", "");
    if (packet_num == 0) return 0;
    if (!gradient_array) return ina::set_error(INA_EINVAL, "null gradient array%s", "");
    size_t npk = (size_t)packet_num;
    if (int rc = g_stage.reserve(npk)) return ina::set_error(rc, "staging allocation failed%s", "");
    hipStream_t s = g_stage.stream;
    if (hipMemcpyAsync(g_stage.d_grad, gradient_array, npk * INA_C128_VALUES * 4,
                       hipMemcpyHostToDevice, s) != hipSuccess)
        return ina::set_error(INA_EHIP, "H2D gradient copy%s", "");
    if (int rc = ina_pack_c128(g_stage.d_grad, packet_num, worker_id, aggregator_index,
                               tensor_index, g_stage.d_pkts, s)) {
        (void)hipStreamSynchronize(s);   // the H2D copy still reads the caller's array
        return rc;
    }
    if (hipMemcpyAsync(g_stage.h_pkts, g_stage.d_pkts, npk * INA_C128_BYTES, hipMemcpyDeviceToHost,
                       s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return ina::set_error(INA_EHIP, "D2H packet copy%s", "");

    return ina_send_packets_fd(fd, g_stage.h_pkts, npk, INA_C128_BYTES, INA_C128_BYTES, dst_ip);
}

int ina_send_packets_fd(int fd, const uint8_t* host_pkts, size_t npk, size_t stride,
                        size_t pkt_len, uint32_t dst_ip) {
    if (npk == 0) return 0;
    if (!host_pkts || pkt_len == 0 || stride < pkt_len)
        return ina::set_error(INA_EINVAL, "bad packet buffer%s", "");
    sockaddr_in dst;
    memset(&dst, 0, sizeof dst);
    dst.sin_family = AF_INET;
    dst.sin_addr.s_addr = htonl(dst_ip);   // communicator.cc:8 (host-order argument)
    // an IPv4 destination only means something on an AF_INET socket (a connected or
    // AF_UNIX datagram socket, e.g. a capture socketpair, takes no address)
    int domain = AF_INET;
    socklen_t dl = sizeof domain;
    if (getsockopt(fd, SOL_SOCKET, SO_DOMAIN, &domain, &dl) == 0 && domain != AF_INET) dst_ip = 0;
    constexpr size_t kBatch = 1024;
    std::vector<mmsghdr> msgs(kBatch);
    std::vector<iovec> iov(kBatch);
    size_t sent = 0;
    while (sent < npk) {
        size_t nb = npk - sent < kBatch ? npk - sent : kBatch;
        for (size_t i = 0; i < nb; ++i) {
            iov[i].iov_base = const_cast<uint8_t*>(host_pkts) + (sent + i) * stride;
            iov[i].iov_len = pkt_len;
            memset(&msgs[i], 0, sizeof(mmsghdr));
            msgs[i].msg_hdr.msg_iov = &iov[i];
            msgs[i].msg_hdr.msg_iovlen = 1;
            if (dst_ip) {
                msgs[i].msg_hdr.msg_name = &dst;
                msgs[i].msg_hdr.msg_namelen = sizeof dst;
            }
        }
        int r = sendmmsg(fd, msgs.data(), (unsigned)nb, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            return ina::set_error(INA_ESOCK, "sendmmsg: %s", strerror(errno));
        }
        sent += (size_t)r;
    }
    if (sent > 0x7FFFFFFFu) sent = 0x7FFFFFFFu;
    return (int)sent;
}

int ina_recv_packets_fd(int fd, uint8_t* host_pkts, size_t max_pkts, size_t stride, size_t skip,
                        int timeout_ms, uint32_t* lens) {
    if (max_pkts == 0) return 0;
    if (!host_pkts || stride == 0) return ina::set_error(INA_EINVAL, "bad packet buffer%s", "");
    constexpr size_t kBatch = 1024;
    std::vector<mmsghdr> msgs(kBatch);
    std::vector<iovec> iov(2 * kBatch);
    std::vector<uint8_t> skipbuf(skip ? skip : 1);
    size_t got = 0;
    timespec t0{};
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const int64_t end_ns = (int64_t)t0.tv_sec * 1000000000LL + t0.tv_nsec +
                           (int64_t)(timeout_ms < 0 ? 0 : timeout_ms) * 1000000LL;
    // wait for data (poll) then drain what is queued (recvmmsg, non-blocking), until
    // max_pkts have arrived or the deadline passes
    while (got < max_pkts) {
        size_t nb = max_pkts - got < kBatch ? max_pkts - got : kBatch;
        for (size_t i = 0; i < nb; ++i) {
            int k = 0;
            if (skip) {                        // e.g. the 20-byte IPv4 header of a raw socket
                iov[2 * i].iov_base = skipbuf.data();
                iov[2 * i].iov_len = skip;
                k = 1;
            }
            iov[2 * i + k].iov_base = host_pkts + (got + i) * stride;
            iov[2 * i + k].iov_len = stride;
            memset(&msgs[i], 0, sizeof(mmsghdr));
            msgs[i].msg_hdr.msg_iov = &iov[2 * i];
            msgs[i].msg_hdr.msg_iovlen = (size_t)(k + 1);
        }
        int r = recvmmsg(fd, msgs.data(), (unsigned)nb, MSG_DONTWAIT, nullptr);
        if (r < 0) {
            if (errno == EINTR) continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK)
                return ina::set_error(INA_ESOCK, "recvmmsg: %s", strerror(errno));
            timespec now{};
            clock_gettime(CLOCK_MONOTONIC, &now);
            int64_t left = end_ns - ((int64_t)now.tv_sec * 1000000000LL + now.tv_nsec);
            if (left <= 0) break;
            pollfd pfd{fd, POLLIN, 0};
            int pr = poll(&pfd, 1, (int)((left + 999999) / 1000000));
            if (pr < 0 && errno != EINTR) return ina::set_error(INA_ESOCK, "poll: %s", strerror(errno));
            if (pr == 0) break;
            continue;
        }
        for (int i = 0; i < r; ++i) {
            size_t len = msgs[i].msg_len;
            len = len > skip ? len - skip : 0;
            if (lens) lens[got + i] = (uint32_t)len;
        }
        got += (size_t)r;
    }
    return (int)(got > 0x7FFFFFFFu ? 0x7FFFFFFFu : got);
}

// split rows on the socket (include/ina.h): datagram p = header row p's 15 bytes || payload
// row p's 4V bytes, two iovecs -- the bytes ina_send_packets_fd sends from packed rows
int ina_send_packets_split_fd(int fd, const uint8_t* host_hdr, const uint8_t* host_pay, size_t npk, int V,
                              uint32_t dst_ip) {
    if (npk == 0) return 0;
    if (!host_hdr || !host_pay || V <= 0) return ina::set_error(INA_EINVAL, "bad packet buffers%s", "");
    const size_t plen = 4u * (size_t)V;
    sockaddr_in dst;
    memset(&dst, 0, sizeof dst);
    dst.sin_family = AF_INET;
    dst.sin_addr.s_addr = htonl(dst_ip);
    int domain = AF_INET;
    socklen_t dl = sizeof domain;
    if (getsockopt(fd, SOL_SOCKET, SO_DOMAIN, &domain, &dl) == 0 && domain != AF_INET) dst_ip = 0;
    constexpr size_t kBatch = 1024;
    std::vector<mmsghdr> msgs(kBatch);
    std::vector<iovec> iov(2 * kBatch);
    size_t sent = 0;
    while (sent < npk) {
        size_t nb = npk - sent < kBatch ? npk - sent : kBatch;
        for (size_t i = 0; i < nb; ++i) {
            iov[2 * i].iov_base = const_cast<uint8_t*>(host_hdr) + (sent + i) * 16;
            iov[2 * i].iov_len = INA_NGA_HDR_BYTES;
            iov[2 * i + 1].iov_base = const_cast<uint8_t*>(host_pay) + (sent + i) * plen;
            iov[2 * i + 1].iov_len = plen;
            memset(&msgs[i], 0, sizeof(mmsghdr));
            msgs[i].msg_hdr.msg_iov = &iov[2 * i];
            msgs[i].msg_hdr.msg_iovlen = 2;
            if (dst_ip) {
                msgs[i].msg_hdr.msg_name = &dst;
                msgs[i].msg_hdr.msg_namelen = sizeof dst;
            }
        }
        int r = sendmmsg(fd, msgs.data(), (unsigned)nb, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            return ina::set_error(INA_ESOCK, "sendmmsg: %s", strerror(errno));
        }
        sent += (size_t)r;
    }
    if (sent > 0x7FFFFFFFu) sent = 0x7FFFFFFFu;
    return (int)sent;
}

int ina_recv_packets_split_fd(int fd, uint8_t* host_hdr, uint8_t* host_pay, size_t max_pkts, int V,
                              size_t skip, int timeout_ms, uint32_t* lens) {
    if (max_pkts == 0) return 0;
    if (!host_hdr || !host_pay || V <= 0) return ina::set_error(INA_EINVAL, "bad packet buffers%s", "");
    const size_t plen = 4u * (size_t)V;
    constexpr size_t kBatch = 1024;
    std::vector<mmsghdr> msgs(kBatch);
    std::vector<iovec> iov(3 * kBatch);
    std::vector<uint8_t> skipbuf(skip ? skip : 1);
    size_t got = 0;
    timespec t0{};
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const int64_t end_ns = (int64_t)t0.tv_sec * 1000000000LL + t0.tv_nsec +
                           (int64_t)(timeout_ms < 0 ? 0 : timeout_ms) * 1000000LL;
    while (got < max_pkts) {
        size_t nb = max_pkts - got < kBatch ? max_pkts - got : kBatch;
        for (size_t i = 0; i < nb; ++i) {
            int k = 0;
            if (skip) {
                iov[3 * i].iov_base = skipbuf.data();
                iov[3 * i].iov_len = skip;
                k = 1;
            }
            iov[3 * i + k].iov_base = host_hdr + (got + i) * 16;
            iov[3 * i + k].iov_len = INA_NGA_HDR_BYTES;
            iov[3 * i + k + 1].iov_base = host_pay + (got + i) * plen;
            iov[3 * i + k + 1].iov_len = plen;
            memset(&msgs[i], 0, sizeof(mmsghdr));
            msgs[i].msg_hdr.msg_iov = &iov[3 * i];
            msgs[i].msg_hdr.msg_iovlen = (size_t)(k + 2);
        }
        int r = recvmmsg(fd, msgs.data(), (unsigned)nb, MSG_DONTWAIT, nullptr);
        if (r < 0) {
            if (errno == EINTR) continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK)
                return ina::set_error(INA_ESOCK, "recvmmsg: %s", strerror(errno));
            timespec now{};
            clock_gettime(CLOCK_MONOTONIC, &now);
            int64_t left = end_ns - ((int64_t)now.tv_sec * 1000000000LL + now.tv_nsec);
            if (left <= 0) break;
            pollfd pfd{fd, POLLIN, 0};
            int pr = poll(&pfd, 1, (int)((left + 999999) / 1000000));
            if (pr < 0 && errno != EINTR) return ina::set_error(INA_ESOCK, "poll: %s", strerror(errno));
            if (pr == 0) break;
            continue;
        }
        for (int i = 0; i < r; ++i) {
            size_t len = msgs[i].msg_len;
            len = len > skip ? len - skip : 0;
            if (lens) lens[got + i] = (uint32_t)len;
        }
        got += (size_t)r;
    }
    return (int)(got > 0x7FFFFFFFu ? 0x7FFFFFFFu : got);
}

void send_gradients(uint32_t* gradient_array, int packet_num, uint32_t dst_ip, int worker_id,
                    uint32_t aggregator_index, int tensor_index) {
    int fd = socket(AF_INET, SOCK_RAW, IPPROTO_UDP);   // communicator.cc:10
    if (fd < 0) {
        perror("ERROR: Failed to create raw socket.\n");
        exit(-1);
    }
    int send_buff_size = 4096 * 4096;                  // communicator.cc:15-16
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &send_buff_size, sizeof(send_buff_size));
    clock_t start = clock();
    int rc = ina_send_gradients_fd(fd, gradient_array, packet_num, dst_ip, worker_id,
                                   aggregator_index, tensor_index);
    if (rc < 0) {
        if (rc == INA_ESOCK) perror("ERROR: Failed to call sendto()");
        else fprintf(stderr, "ERROR: %s\n", ina_last_error_string());
        close(fd);
        exit(-1);
    }
    clock_t end = clock();
    printf("Time consumed: %lf s\n", (double)(end - start) / CLOCKS_PER_SEC);   // communicator.cc:43-44
    close(fd);
}

}  // extern "C"
