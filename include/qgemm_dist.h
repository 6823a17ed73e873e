/*
 * qgemm_dist.h -- multi-GPU C-ABI of the quantized GEMM: M-sharding + RCCL all-gather over xGMI.
 *
 * The reference has no multi-GPU code; SURVEY.md s8(b) names the caller to serve ("the multi-GPU
 * driver: per-rank pointer offsets A+m0*K, C+m0*N") and s8(e) the partitioning and collective
 * (ncclAllGather of C, rccl.h:678).  The north star: "shard M across the 8 GPUs of one node with
 * RCCL all-gather of C over xGMI only for the whole-node number".
 *
 * Why this shards with no exchange: Cx is per row of A and Cw depends only on B, so rank r computes
 * the rows [m0, m0 + rows) of C from its rows of A and the replicated B -- bit-identical to the
 * one-GPU call (op_mm.cuh:67-101 has no cross-row state).  The all-gather exists only to assemble
 * the whole C on every GPU.
 *
 * Built as its own library (libqgemm_dist.so, links librccl) so libqgemm.so does not depend on
 * RCCL.  Same conventions as qgemm.h: device pointers, 0 or a hipError_t / ncclResult_t code
 * (ncclResult_t codes are returned as 1000 + code), work enqueued on `stream` (a hipStream_t).
 */
#ifndef QGEMM_DIST_H_
#define QGEMM_DIST_H_

#include <stddef.h>
#include <stdint.h>

#include "qgemm.h"

#ifdef __cplusplus
extern "C" {
#endif

#define QGEMM_COMM_ID_BYTES 128 /* = NCCL_UNIQUE_ID_BYTES (rccl.h:40) */

/* Balanced contiguous row shards: rank r owns rows [*m0, *m0 + *rows) of an m-row matrix split over
 * `world` ranks (the first m % world ranks get one row more).  Pure host arithmetic. */
QGEMM_API int qgemm_shard_rows(int m, int world, int rank, int *m0, int *rows);

/* This rank's share of op_mm_quantize(A, B, C, m, n, k): A and C are the FULL m-row matrices (row-major,
 * leading dimensions k and n) as every rank sees them; only rows [m0, m0+rows) of A are read and of C
 * written (pointer offsets A + m0*k, C + m0*n).  B (k x n) is replicated.  Bit-identical to those rows
 * of the one-GPU call. */
QGEMM_API int op_mm_quantize_shard(const float *A, const float *B, float *C, int m, int n, int k, int world,
                                   int rank, void *stream);

/* Communicators.  One process per GPU: rank 0 calls qgemm_comm_unique_id, shares the 128 bytes with the
 * other ranks (any host channel), every rank calls qgemm_comm_init_rank on its own device.  One process
 * driving ndev GPUs (the harness's -g): qgemm_comm_init_all fills comms[0..ndev). */
QGEMM_API int qgemm_comm_unique_id(void *id_out /* QGEMM_COMM_ID_BYTES */);
QGEMM_API int qgemm_comm_init_rank(void **comm, int world, const void *id, int rank);
QGEMM_API int qgemm_comm_init_all(void **comms, int ndev, const int *devices);
QGEMM_API int qgemm_comm_destroy(void *comm);
/* The communicator's size and this rank (ncclCommCount / ncclCommUserRank, rccl.h:378,400): what RCCL
 * itself saw, so a harness can prove its world size (bench.py's rccl_world). */
QGEMM_API int qgemm_comm_count(void *comm, int *count);
QGEMM_API int qgemm_comm_user_rank(void *comm, int *rank);

/* In-place all-gather of C's row shards over RCCL: on entry rank r holds rows
 * qgemm_shard_rows(m, world, r) of C (m x n row-major fp32, leading dimension n); on completion every
 * rank holds all m rows.  m % world == 0: one ncclAllGather (send buffer = C + m0*n inside the receive
 * buffer); otherwise one ncclBroadcast per owner inside a group.  Enqueued on `stream`. */
QGEMM_API int qgemm_allgather_rows(float *C, int m, int n, int world, int rank, void *comm, void *stream);
/* The collectives qgemm_allgather_rows enqueues, as data (no GPU, no RCCL): returns the number of operations
 * (0 when there is nothing to move; at most world) or -hipErrorInvalidValue.  Operation i moves count[i]
 * floats starting at element first[i] of C: root[i] == -1 is ONE in-place all-gather (rank r sends
 * C + first[i] + r*count[i], everyone receives C + first[i] .. + world*count[i]); root[i] >= 0 is an
 * in-place broadcast of [first[i], first[i] + count[i]) from rank root[i]. */
QGEMM_API int qgemm_allgather_plan(int m, int n, int world, int64_t *first, int64_t *count, int *root, int max_ops);

/* Pipelined whole-node step ("optionally pipeline the gather per row-chunk").  Rank r's rows
 * qgemm_shard_rows(m, world, r) are split into `chunks` balanced pieces (qgemm_shard_rows(rows, chunks, c));
 * chunk c of every rank is gathered by one in-place ncclBroadcast per owner (inside one group per chunk)
 * while chunk c + 1 computes.  The plan as data (no GPU, no RCCL), chunk-major, owners ascending, owners with
 * no rows in a chunk skipped: op i broadcasts count[i] floats at element first[i] of C from rank root[i].
 * Unlike qgemm_allgather_plan it also lists the broadcasts at world == 1 (each then an in-place no-op), so
 * the RCCL calls run on a one-GPU box.  Returns the number of operations (max_ops == 0 / NULL arrays: size
 * query) or -hipErrorInvalidValue. */
QGEMM_API int qgemm_allgather_chunk_plan(int m, int n, int world, int chunks, int64_t *first, int64_t *count,
                                         int *root, int max_ops);
/* Bytes of device workspace op_mm_quantize_shard_pipelined needs (B packed once + one chunk's A pack). */
QGEMM_API size_t op_mm_quantize_shard_pipelined_workspace_size(int m, int n, int k, int world, int chunks);
/* This rank's shard of op_mm_quantize(A, B, C, m, n, k) with the all-gather of C pipelined under it: B is
 * packed once (qgemm_pack_b), chunk c's rows run op_mm_quantize_prepacked_ws on `stream` (bit-identical to
 * op_mm_quantize_shard), then an event hands chunk c to `gather_stream`, where the chunk's broadcasts
 * (qgemm_allgather_chunk_plan) run under chunk c + 1's compute.  On return `stream` waits for the last
 * broadcast, so work enqueued after it sees the whole C.  comm may be NULL only when world == 1 (no gather).
 * After a local error past the argument checks (pack, compute, event) the remaining chunks are not computed but
 * their broadcast groups are still issued, so the peer ranks complete instead of blocking in RCCL; the first error
 * is returned and C's rows are unspecified. */
QGEMM_API int op_mm_quantize_shard_pipelined(const float *A, const float *B, float *C, int m, int n, int k, int world,
                                             int rank, int chunks, void *comm, void *workspace, size_t ws_bytes,
                                             void *stream, void *gather_stream);

/* One planned collective of the one-process node path: on device index `rank`, root < 0 is an in-place
 * ncclAllGather (send C + send_off, receive C + recv_off .. + ndev * count), root >= 0 an in-place
 * ncclBroadcast of count floats at C + recv_off (= send_off) from rank `root`. */
typedef struct qgemm_coll_op {
    int rank;
    int root;
    int64_t send_off;
    int64_t recv_off;
    int64_t count;
} qgemm_coll_op;

/* The collectives qgemm_node_mm_quantize (mode 1 / 2) enqueues, as data (no GPU, no RCCL), in the order it
 * issues them inside ONE ncclGroupStart/End: every rank's qgemm_allgather_plan operations, rank by rank.
 * ops == NULL: returns the count; else fills up to max_ops and returns the count, or -hipErrorInvalidValue. */
QGEMM_API int qgemm_node_allgather_plan(int m, int n, int ndev, qgemm_coll_op *ops, int max_ops);

/* One process, ndev GPUs (the harness's -g): the whole-node C4 step.  mode 0: every device's shard
 * (op_mm_quantize_shard on devices[r] with A[r], B[r], C[r], streams[r]); mode 1: the shards, then the
 * all-gather of C over comms[r]; mode 2: the all-gather alone (timed separately by the harness). */
QGEMM_API int qgemm_node_mm_quantize(const float *const *A, const float *const *B, float *const *C, int m, int n,
                                     int k, int ndev, const int *devices, void *const *comms,
                                     void *const *streams, int mode);

#ifdef __cplusplus
}
#endif

#endif /* QGEMM_DIST_H_ */
