/* Minimal OncillaMem program, unchanged from how the reference API is used:
 * attach to the local daemon, allocate a remote pair, write and read it back
 * one-sidedly, free, detach.
 *
 *   build/bin/ocmd nodefile --rank 0 &   (and the other ranks)
 *   OCM_DAEMON_RANK=0 build/bin/ocm_example_hello [MiB]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oncillamem.h"

int main(int argc, char **argv) {
    const size_t bytes = (argc > 1 ? (size_t)atoi(argv[1]) : 4) << 20;
    if (ocm_init() != 0) {
        fprintf(stderr, "ocm_init: %s\n", ocm_last_error());
        return 1;
    }
    /* OCM_REMOTE_RDMA: a pinned host local half + a remote half wherever rank0 places it
     * (peer HBM, the host tier, or another node). OCM_REMOTE_GPU keeps the local half in HBM. */
    struct ocm_alloc_params ap = {bytes, bytes, OCM_REMOTE_RDMA};
    ocm_alloc_t a = ocm_alloc(&ap);
    if (!a) {
        fprintf(stderr, "ocm_alloc: %s\n", ocm_last_error());
        return 1;
    }
    void *local = NULL;
    size_t len = 0;
    ocm_localbuf(a, &local, &len);
    for (size_t i = 0; i < len / 4; i++) ((unsigned *)local)[i] = (unsigned)i * 2654435761u;

    struct ocm_params put = {0, 0, 0, 0, bytes, 1}; /* local[0..) -> remote[0..) */
    struct ocm_params get = {0, 0, 0, 0, bytes, 0}; /* remote[0..) -> local[0..) */
    if (ocm_copy_onesided(a, &put) != 0) return fprintf(stderr, "put: %s\n", ocm_last_error()), 1;
    memset(local, 0, len);
    if (ocm_copy_onesided(a, &get) != 0) return fprintf(stderr, "get: %s\n", ocm_last_error()), 1;
    size_t bad = 0;
    for (size_t i = 0; i < len / 4; i++) bad += ((unsigned *)local)[i] != (unsigned)i * 2654435761u;

    struct ocm_remote_info info;
    ocm_remote_info(a, &info);
    printf("%zu MiB round trip through rank %d (%s), %zu bad words\n", bytes >> 20, info.owner_rank[0],
           info.tier[0] == OCM_TIER_GPU ? "HBM" : "host tier", bad);
    ocm_free(a);
    ocm_tini();
    return bad ? 1 : 0;
}
