/*
 * oncillamem.h — public C ABI of libocm (MI355X-native OncillaMem).
 *
 * Parity: same entry points, enum values and struct layouts as the reference
 * app interface (reference inc/oncillamem.h:24-89):
 *   - enum ocm_kind values OCM_LOCAL_HOST=1 .. OCM_REMOTE_GPU=7
 *   - struct ocm_params       (48 B)  src/dest offsets, *_2 offsets, bytes, op_flag
 *   - struct ocm_alloc_params (24 B)  local_alloc_bytes, rem_alloc_bytes, kind
 *
 * What the kinds mean on MI355X (one backend, not a dispatch layer):
 *   OCM_LOCAL_HOST   page-aligned host memory of the calling process
 *   OCM_LOCAL_GPU    HBM of the calling process' GPU
 *   OCM_REMOTE_GPU   pair: local half in the app GPU's HBM, remote half in the
 *                    HBM of a peer MI355X (placed by rank0) reached over xGMI,
 *                    or in a daemon's pinned host tier when HBM is exhausted
 *   OCM_REMOTE_RDMA  pair whose local half is pinned host memory (CPU-visible,
 *   OCM_REMOTE_RMA   like the reference's malloc'd IB/EXTOLL bounce buffer);
 *                    remote half placed exactly like OCM_REMOTE_GPU
 *   OCM_LOCAL_RDMA / OCM_LOCAL_RMA  accepted as OCM_LOCAL_HOST (the reference
 *                    never implemented them).
 *
 * Functions added for MI355X (async put/get, striping, explicit placement,
 * daemon statistics) are declared after the reference block.
 */
#ifndef ONCILLAMEM_H
#define ONCILLAMEM_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lib_alloc *ocm_alloc_t;

enum ocm_kind {
    OCM_LOCAL_HOST = 1,
    OCM_LOCAL_RMA,
    OCM_REMOTE_RMA,
    OCM_LOCAL_RDMA,
    OCM_REMOTE_RDMA,
    OCM_LOCAL_GPU,
    OCM_REMOTE_GPU,
};

/* General parameters for one-sided / two-sided copies.
 * op_flag: read = 0, write = 1. */
struct ocm_params {
    uint64_t src_offset;
    uint64_t dest_offset;
    uint64_t src_offset_2;
    uint64_t dest_offset_2;
    uint64_t bytes;
    int op_flag;
};
typedef struct ocm_params *ocm_param_t;

struct ocm_alloc_params {
    uint64_t local_alloc_bytes;
    uint64_t rem_alloc_bytes;
    enum ocm_kind kind;
};
typedef struct ocm_alloc_params *ocm_alloc_param_t;

/* ---------------- reference API (inc/oncillamem.h:69-89) ---------------- */
int ocm_init(void);
int ocm_tini(void);
ocm_alloc_t ocm_alloc(ocm_alloc_param_t alloc_param);
int ocm_free(ocm_alloc_t a);
int ocm_localbuf(ocm_alloc_t a, void **buf, size_t *len);
bool ocm_is_remote(ocm_alloc_t a);
enum ocm_kind ocm_alloc_kind(ocm_alloc_t a);
int ocm_remote_sz(ocm_alloc_t a, size_t *len);
/* Implemented (stubs in the reference, src/lib.c:491-499):
 * copy_in  writes min(local,remote) bytes from `src` into the allocation
 *          (remote half for pairs, the buffer itself for local kinds);
 * copy_out reads them back into `dst`. Host or device pointers accepted. */
int ocm_copy_out(void *dst, ocm_alloc_t src);
int ocm_copy_in(ocm_alloc_t dst, void *src);
int ocm_copy(ocm_alloc_t dst, ocm_alloc_t src, ocm_param_t options);
int ocm_copy_onesided(ocm_alloc_t src, ocm_param_t options);

/* ---------------- MI355X extensions ---------------- */

enum ocm_alloc_flags {
    OCM_ALLOC_STRIPE      = 1u << 0, /* stripe the remote half over several peers (xGMI links) */
    OCM_ALLOC_HOST_TIER   = 1u << 1, /* place the remote half in a daemon's pinned host tier */
    OCM_ALLOC_NO_SPILL    = 1u << 2, /* fail instead of spilling to the host tier */
    OCM_ALLOC_ZERO        = 1u << 3, /* zero the remote half before returning */
    OCM_ALLOC_LOOPBACK    = 1u << 4, /* remote half in the origin daemon's own HBM */
};

struct ocm_alloc_ex_params {
    int32_t  remote_rank;   /* -1: rank0 places; >=0: honour this owner (reference field was unused) */
    uint32_t flags;         /* enum ocm_alloc_flags */
    uint32_t stripe_width;  /* 0: all peers; else max number of owners */
    uint32_t reserved;
    uint64_t stripe_unit;   /* bytes per stripe unit, 0: default (OCM_STRIPE_UNIT or 1 MiB) */
};

enum ocm_tier { OCM_TIER_NONE = 0, OCM_TIER_HOST = 1, OCM_TIER_GPU = 2 };

#define OCM_MAX_EXTENTS 8

struct ocm_remote_info {
    uint32_t n_extents;
    uint32_t tier[OCM_MAX_EXTENTS];       /* enum ocm_tier per extent */
    int32_t  owner_rank[OCM_MAX_EXTENTS];
    int32_t  owner_gpu[OCM_MAX_EXTENTS];  /* device ordinal on the node, -1 for host */
    uint64_t extent_bytes[OCM_MAX_EXTENTS];
    uint64_t stripe_unit;
    uint64_t alloc_id;
    uint64_t remote_bytes;
    uint32_t net_mask;   /* bit i: extent i is on another node (network tier) */
    uint32_t reserved;
};

struct ocm_daemon_stats {
    int32_t  rank;
    int32_t  gpu;
    int32_t  num_nodes;
    int32_t  num_apps;
    uint64_t gpu_capacity, gpu_used;
    uint64_t host_capacity, host_used;
    uint64_t n_alloc, n_free, n_reclaimed, n_spilled;
    uint64_t n_slabs;
    uint64_t ctrl_ticks;   /* allgather ticks of the RCCL/socket control transport (0 on TCP) */
    uint64_t n_leases;     /* capacity leases held on peers */
    uint64_t lease_allocs; /* allocations carved from them without a mesh round trip */
    uint32_t xgmi_peers;   /* GPUs on the node this daemon's GPU reaches over xGMI */
    uint16_t min_hops;     /* xGMI hop count over those links (0 when none) */
    uint16_t max_hops;
    uint32_t ctrl_transport; /* daemon<->daemon records: 0 TCP, 1 socket ticks, 2 RCCL ticks,
                                3 TCP after leaving a tick transport, 4 tick transport starting */
    uint32_t reserved;
};

ocm_alloc_t ocm_alloc_ex(ocm_alloc_param_t alloc_param, const struct ocm_alloc_ex_params *ex);
/* Non-blocking variants: enqueue on the allocation's stream; ocm_wait() completes them. */
int ocm_copy_onesided_async(ocm_alloc_t a, ocm_param_t options);
int ocm_wait(ocm_alloc_t a);
/* Batched one-sided copies on one remote pair: n_ops records with the
 * ocm_copy_onesided meaning (op_flag 1 = put local[src_offset] -> remote[dest_offset],
 * 0 = get), puts and gets mixed, run as ONE gfx950 kernel launch (scatter/gather
 * lists). Ops of one batch run concurrently: overlapping destinations have no
 * defined order. flags: OCM_BATCH_ASYNC completes later (ocm_wait). */
#define OCM_BATCH_ASYNC 1
int ocm_copy_onesided_batch(ocm_alloc_t a, const struct ocm_params *ops, int n_ops, int flags);
/* Stream interop (hipStream_t passed as void*, NULL = legacy default stream):
 * ocm_stream_wait:   a's next one-sided op starts after the work already queued on `stream`
 *                    (e.g. torch kernels that wrote the local half).
 * ocm_stream_signal: work queued on `stream` afterwards starts after a's queued async ops. */
int ocm_stream_wait(ocm_alloc_t a, void *stream);
int ocm_stream_signal(ocm_alloc_t a, void *stream);

/* Transfer plans: a fixed sequence of batch stages (each stage = one
 * ocm_copy_onesided_batch list on one allocation, run after the previous
 * stage), validated, planned and uploaded once, then captured into a HIP
 * graph. Every ocm_plan_launch replays the whole schedule as one graph launch
 * (data is read at replay time; the op lists are fixed). stream NULL: the
 * library stream, blocking; otherwise queued on `stream` (hipStream_t).
 * Allocations used by a plan cannot be freed before ocm_plan_destroy. */
typedef struct ocm_plan *ocm_plan_t;
ocm_plan_t ocm_plan_create(void);
int ocm_plan_add(ocm_plan_t p, ocm_alloc_t a, const struct ocm_params *ops, int n_ops);
int ocm_plan_launch(ocm_plan_t p, void *stream);
int ocm_plan_destroy(ocm_plan_t p);
int ocm_remote_info(ocm_alloc_t a, struct ocm_remote_info *info);
/* Device pointer of the remote half when it is a single extent (NULL if striped). */
void *ocm_remotebuf(ocm_alloc_t a);
int ocm_stats(int rank, struct ocm_daemon_stats *out); /* rank -1: local daemon */
int ocm_rank(void);        /* rank of the daemon this process is attached to */
int ocm_num_nodes(void);   /* daemons in the mesh */
int ocm_device(void);      /* HIP device the library copies on, -1 when CPU-only */
const char *ocm_last_error(void);

/* PyTorch pluggable-allocator hooks (torch.cuda.memory.CUDAPluggableAllocator;
 * Python wrapper: oncilla_amd.torch_pool.RemoteMemPool). A block is the remote
 * half of a single-extent pair with no local half, placed per
 * ocm_x_torch_pool_config (remote_rank -1: rank0 places; flags: enum
 * ocm_alloc_flags) and addressed in place by the caller's GPU. The process must
 * have called ocm_init; `device` must be the library's device. */
void *ocm_torch_alloc(ssize_t size, int device, void *stream);
void ocm_torch_free(void *ptr, ssize_t size, int device, void *stream);
void ocm_x_torch_pool_config(int remote_rank, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* ONCILLAMEM_H */
