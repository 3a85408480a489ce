/*
 * capture_shim.c -- TEST INFRASTRUCTURE ONLY, container-only (never on the GPU box).
 *
 * LD_PRELOAD interposer used by tests/golden/gen_golden.py while it drives the
 * reference's own send_gradients (communicator.cc, compiled into
 * oracle/_ref/send.so by oracle/Makefile).  Raw sockets are not available here,
 * so socket()/setsockopt()/sendto() are replaced by a capture sink: every
 * datagram handed to sendto() is appended to $INA_CAPTURE_FILE as
 * [u32 little-endian length][bytes].  Nothing is transmitted.
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

static int cap_fd = -1;

static int cap_open(void) {
    if (cap_fd >= 0) return cap_fd;
    const char* path = getenv("INA_CAPTURE_FILE");
    if (!path) return -1;
    cap_fd = open(path, O_WRONLY | O_CREAT | O_APPEND, 0644);
    return cap_fd;
}

int socket(int domain, int type, int protocol) {
    (void)domain; (void)type; (void)protocol;
    int fd = cap_open();
    return fd < 0 ? -1 : dup(fd);
}

int setsockopt(int fd, int level, int name, const void* val, socklen_t len) {
    (void)fd; (void)level; (void)name; (void)val; (void)len;
    return 0;
}

ssize_t sendto(int fd, const void* buf, size_t len, int flags, const struct sockaddr* addr,
               socklen_t alen) {
    (void)flags; (void)addr; (void)alen;
    uint32_t l = (uint32_t)len;
    if (write(fd, &l, 4) != 4) return -1;
    if (write(fd, buf, len) != (ssize_t)len) return -1;
    return (ssize_t)len;
}
