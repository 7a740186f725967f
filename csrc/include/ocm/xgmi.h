/*
 * Raw one-sided backend over xGMI peer mappings — the MI355X counterpart of
 * the reference's fabric backends, reference inc/io/rdma.h:36-45 (ib_init, ib_new,
 * ib_free, ib_connect, ib_disconnect, ib_read, ib_write, ib_poll) and
 * inc/io/extoll.h:50-59 (extoll_*). Used without any daemon: two processes
 * rendezvous on a named endpoint, exchange their buffer registrations (the
 * RDMA-CM private data {va, rkey, len} of reference src/rdma.h:37-41 becomes
 * {IPC handle | host-slab path, length, GPU}) and then read/write each other's
 * memory one-sidedly with the gfx950 transfer kernel.
 *
 * Connections are symmetric (like a connected RC QP): after xgmi_connect both
 * sides can read and write the other's buffer.
 */
#ifndef OCM_XGMI_H
#define OCM_XGMI_H

#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct xgmi_params {
    const char *endpoint; /* rendezvous name (abstract unix socket), like ib addr:port */
    int gpu;              /* device of the local buffer, -1 = pinned host memory */
    void *buf;            /* caller's buffer, NULL = allocate buf_len bytes */
    size_t buf_len;
};

typedef struct xgmi_alloc *xgmi_t;

int xgmi_init(void);
xgmi_t xgmi_new(const struct xgmi_params *p);
int xgmi_free(xgmi_t x);
/* Server: publish the endpoint and block until one client connected (like
 * rdma_listen + rdma_accept). Client: connect (retrying up to 10 s). */
int xgmi_connect(xgmi_t x, bool is_server);
int xgmi_disconnect(xgmi_t x, bool is_server);
/* local[src_offset .. +len] <- remote[dest_offset .. +len] */
int xgmi_read(xgmi_t x, size_t src_offset, size_t dest_offset, size_t len);
/* local[src_offset .. +len] -> remote[dest_offset .. +len] */
int xgmi_write(xgmi_t x, size_t src_offset, size_t dest_offset, size_t len);
/* wait for every posted read/write (reference ib_poll, src/rdma.c:266-302) */
int xgmi_poll(xgmi_t x);
void *xgmi_localbuf(xgmi_t x, size_t *len);
size_t xgmi_remote_len(xgmi_t x);
/* out-of-band control channel of the connection (test orchestration) */
int xgmi_send_ctrl(xgmi_t x, const char *text);
int xgmi_recv_ctrl(xgmi_t x, char *text, size_t cap, int timeout_ms);

#ifdef __cplusplus
}
#endif
#endif
