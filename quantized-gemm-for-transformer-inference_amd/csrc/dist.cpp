// dist.cpp -- libqgemm_dist.so: M-sharded op_mm_quantize + RCCL all-gather of C over xGMI
// (include/qgemm_dist.h; SURVEY.md s8(b) multi-GPU driver, s8(e) partitioning and collective).
//
// No data-path collective in the compute: every rank packs its own rows of A and the replicated B and
// runs the int8 GEMM on them (Cx is per row, Cw depends on B only), so a shard is bit-identical to the
// same rows of the one-GPU call.  The all-gather only assembles the whole-node C.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <vector>

#include "../../include/qgemm_dist.h"

namespace {

int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? 0 : 1000 + (int)r; }

}  // namespace

extern "C" {

int qgemm_shard_rows(int m, int world, int rank, int *m0, int *rows) {
    if (m < 0 || world < 1 || rank < 0 || rank >= world || !m0 || !rows) return (int)hipErrorInvalidValue;
    const int q = m / world, r = m % world;
    *m0 = rank * q + (rank < r ? rank : r);
    *rows = q + (rank < r ? 1 : 0);
    return 0;
}

int op_mm_quantize_shard(const float *A, const float *B, float *C, int m, int n, int k, int world, int rank,
                         void *stream) {
    int m0 = 0, rows = 0;
    const int e = qgemm_shard_rows(m, world, rank, &m0, &rows);
    if (e) return e;
    if (!A || !B || !C || n < 0 || k < 1) return (int)hipErrorInvalidValue;
    if (rows == 0) return 0;
    // per-rank pointer offsets: A + m0*k, C + m0*n
    return op_mm_quantize_ex(A + (int64_t)m0 * k, k, 1, B, n, 1, C + (int64_t)m0 * n, n, 1, rows, n, k, 127.0f,
                             stream);
}

int qgemm_comm_unique_id(void *id_out) {
    if (!id_out) return (int)hipErrorInvalidValue;
    return nccl_rc(ncclGetUniqueId(static_cast<ncclUniqueId *>(id_out)));
}

int qgemm_comm_init_rank(void **comm, int world, const void *id, int rank) {
    if (!comm || !id || world < 1 || rank < 0 || rank >= world) return (int)hipErrorInvalidValue;
    ncclUniqueId uid;
    __builtin_memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    const int rc = nccl_rc(ncclCommInitRank(&c, world, uid, rank));
    *comm = c;
    return rc;
}

int qgemm_comm_init_all(void **comms, int ndev, const int *devices) {
    if (!comms || ndev < 1) return (int)hipErrorInvalidValue;
    return nccl_rc(ncclCommInitAll(reinterpret_cast<ncclComm_t *>(comms), ndev, devices));
}

int qgemm_comm_destroy(void *comm) {
    if (!comm) return 0;
    return nccl_rc(ncclCommDestroy(static_cast<ncclComm_t>(comm)));
}

int qgemm_comm_count(void *comm, int *count) {
    if (!comm || !count) return (int)hipErrorInvalidValue;
    return nccl_rc(ncclCommCount(static_cast<ncclComm_t>(comm), count));
}

int qgemm_comm_user_rank(void *comm, int *rank) {
    if (!comm || !rank) return (int)hipErrorInvalidValue;
    return nccl_rc(ncclCommUserRank(static_cast<ncclComm_t>(comm), rank));
}

int qgemm_allgather_plan(int m, int n, int world, int64_t *first, int64_t *count, int *root, int max_ops) {
    if (m < 0 || n < 0 || world < 1 || max_ops < 0 || (max_ops > 0 && (!first || !count || !root)))
        return -(int)hipErrorInvalidValue;
    if (world == 1 || m == 0 || n == 0) return 0;
    if (m % world == 0) {
        // ONE in-place all-gather: rank r's send buffer is its own rows inside the receive buffer,
        // recv + r * count, count = (m / world) * n floats per rank
        if (max_ops < 1) return -(int)hipErrorInvalidValue;
        first[0] = 0;
        count[0] = (int64_t)(m / world) * n;
        root[0] = -1;
        return 1;
    }
    // unequal shards: each owner broadcasts its rows in place (owners with no rows are skipped)
    int ops = 0;
    for (int r = 0; r < world; ++r) {
        int m0 = 0, rows = 0;
        qgemm_shard_rows(m, world, r, &m0, &rows);
        if (rows == 0) continue;
        if (ops >= max_ops) return -(int)hipErrorInvalidValue;
        first[ops] = (int64_t)m0 * n;
        count[ops] = (int64_t)rows * n;
        root[ops] = r;
        ++ops;
    }
    return ops;
}

namespace {

// the chunked plan, chunk-major, owners ascending; chunk_of (optional) records each op's chunk
int chunk_plan(int m, int n, int world, int chunks, int64_t *first, int64_t *count, int *root, int *chunk_of,
               int max_ops) {
    const bool query = first == nullptr;
    int ops = 0;
    for (int c = 0; c < chunks; ++c)
        for (int r = 0; r < world; ++r) {
            int m0 = 0, rows = 0, c0 = 0, crows = 0;
            qgemm_shard_rows(m, world, r, &m0, &rows);
            qgemm_shard_rows(rows, chunks, c, &c0, &crows);
            if (crows == 0 || n == 0) continue;
            if (!query) {
                if (ops >= max_ops) return -(int)hipErrorInvalidValue;
                first[ops] = (int64_t)(m0 + c0) * n;
                count[ops] = (int64_t)crows * n;
                root[ops] = r;
                if (chunk_of) chunk_of[ops] = c;
            }
            ++ops;
        }
    return ops;
}

}  // namespace

int qgemm_allgather_chunk_plan(int m, int n, int world, int chunks, int64_t *first, int64_t *count, int *root,
                               int max_ops) {
    if (m < 0 || n < 0 || world < 1 || chunks < 1 || max_ops < 0) return -(int)hipErrorInvalidValue;
    if (max_ops == 0 || !first || !count || !root) return chunk_plan(m, n, world, chunks, nullptr, nullptr, nullptr,
                                                                     nullptr, 0);
    return chunk_plan(m, n, world, chunks, first, count, root, nullptr, max_ops);
}

size_t op_mm_quantize_shard_pipelined_workspace_size(int m, int n, int k, int world, int chunks) {
    if (m < 0 || n < 1 || k < 1 || world < 1 || chunks < 1) return 0;
    // the largest chunk any rank computes: ceil(ceil(m / world) / chunks) rows
    const int rows = (m + world - 1) / world, crows = (rows + chunks - 1) / chunks;
    const size_t pb = (qgemm_packed_size(n, k) + 255) / 256 * 256;
    return pb + op_mm_quantize_prepacked_workspace_size(crows > 0 ? crows : 1, n, k);
}

int op_mm_quantize_shard_pipelined(const float *A, const float *B, float *C, int m, int n, int k, int world, int rank,
                                   int chunks, void *comm, void *workspace, size_t ws_bytes, void *stream,
                                   void *gather_stream) {
    int m0 = 0, rows = 0;
    const int e = qgemm_shard_rows(m, world, rank, &m0, &rows);
    if (e) return e;
    if (!A || !B || !C || n < 1 || k < 1 || chunks < 1 || !workspace || (world > 1 && !comm))
        return (int)hipErrorInvalidValue;
    if (ws_bytes < op_mm_quantize_shard_pipelined_workspace_size(m, n, k, world, chunks))
        return (int)hipErrorInvalidValue;
    const int nops = chunk_plan(m, n, world, chunks, nullptr, nullptr, nullptr, nullptr, 0);
    std::vector<int64_t> first((size_t)nops + 1), count((size_t)nops + 1);
    std::vector<int> root((size_t)nops + 1), chunk_of((size_t)nops + 1);
    if (nops > 0 &&
        chunk_plan(m, n, world, chunks, first.data(), count.data(), root.data(), chunk_of.data(), nops) != nops)
        return (int)hipErrorInvalidValue;
    hipStream_t s = static_cast<hipStream_t>(stream), g = static_cast<hipStream_t>(gather_stream);
    ncclComm_t cm = static_cast<ncclComm_t>(comm);
    const size_t pb_bytes = (qgemm_packed_size(n, k) + 255) / 256 * 256;
    char *ws = static_cast<char *>(workspace);
    // W packed ONCE for every chunk (the prepacked drop-in is bit-identical to op_mm_quantize)
    int rc = qgemm_pack_b(B, n, 1, k, n, 127.0f, ws, s);
    hipEvent_t ev = nullptr;
    hipError_t he = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (he != hipSuccess && rc == 0) rc = (int)he;
    // After a local error (pack, compute, event) the remaining chunks are not computed, but their broadcast groups
    // are still issued, in plan order: the peer ranks issue theirs and would otherwise block in RCCL for ever.  The
    // first error is returned and the rows of C are then unspecified.
    int op = 0;
    for (int c = 0; c < chunks; ++c) {
        int c0 = 0, crows = 0;
        qgemm_shard_rows(rows, chunks, c, &c0, &crows);
        if (crows > 0 && rc == 0)
            rc = op_mm_quantize_prepacked_ws(A + (int64_t)(m0 + c0) * k, k, ws, C + (int64_t)(m0 + c0) * n, n, crows,
                                             n, k, ws + pb_bytes, ws_bytes - pb_bytes, s);
        // this chunk's broadcasts (every owner's chunk c) on the gather stream, behind this rank's compute of it;
        // the event is re-recorded per chunk: hipStreamWaitEvent captures the record it follows
        const int o0 = op;
        while (op < nops && chunk_of[(size_t)op] == c) ++op;
        if (!cm || op == o0) continue;
        if (rc == 0 &&
            ((he = hipEventRecord(ev, s)) != hipSuccess || (he = hipStreamWaitEvent(g, ev, 0)) != hipSuccess))
            rc = (int)he;
        ncclResult_t r = ncclGroupStart();
        for (int i = o0; i < op && r == ncclSuccess; ++i)
            r = ncclBroadcast(C + first[(size_t)i], C + first[(size_t)i], (size_t)count[(size_t)i], ncclFloat32,
                              root[(size_t)i], cm, g);
        const ncclResult_t r2 = ncclGroupEnd();
        if (rc == 0) rc = nccl_rc(r != ncclSuccess ? r : r2);
    }
    // the caller's stream sees the whole C: it waits for the last broadcast
    if (rc == 0 && cm && op > 0) {
        if ((he = hipEventRecord(ev, g)) != hipSuccess || (he = hipStreamWaitEvent(s, ev, 0)) != hipSuccess)
            rc = (int)he;
    }
    if (ev) (void)hipEventDestroy(ev);  // released once its last record completes
    return rc;
}

int qgemm_node_allgather_plan(int m, int n, int ndev, qgemm_coll_op *ops, int max_ops) {
    if (m < 0 || n < 0 || ndev < 1 || max_ops < 0 || (max_ops > 0 && !ops)) return -(int)hipErrorInvalidValue;
    // the per-rank plan is the same for every rank (it depends on m, n, world only); RCCL matches a
    // communicator's collectives by their order inside the group, so every rank enqueues the list in plan order
    std::vector<int64_t> first((size_t)ndev), count((size_t)ndev);
    std::vector<int> root((size_t)ndev);
    const int nplan = qgemm_allgather_plan(m, n, ndev, first.data(), count.data(), root.data(), ndev);
    if (nplan < 0) return nplan;
    const int64_t total = (int64_t)nplan * ndev;
    if (ops == nullptr) return (int)total;  // size query
    if (total > max_ops) return -(int)hipErrorInvalidValue;
    int o = 0;
    for (int r = 0; r < ndev; ++r)
        for (int i = 0; i < nplan; ++i, ++o) {
            qgemm_coll_op &op = ops[o];
            op.rank = r;
            op.root = root[i];
            op.count = count[i];
            op.recv_off = first[i];
            // all-gather: rank r sends its own rows, in place inside the receive buffer; broadcast: the
            // owner's rows, in place on every rank
            op.send_off = root[i] < 0 ? first[i] + (int64_t)r * count[i] : first[i];
        }
    return o;
}

namespace {

// enqueue one planned collective on its rank's communicator (inside the caller's group, if any)
ncclResult_t issue(const qgemm_coll_op &op, float *C, ncclComm_t c, hipStream_t s) {
    if (op.root < 0) return ncclAllGather(C + op.send_off, C + op.recv_off, (size_t)op.count, ncclFloat32, c, s);
    return ncclBroadcast(C + op.send_off, C + op.recv_off, (size_t)op.count, ncclFloat32, op.root, c, s);
}

}  // namespace

int qgemm_allgather_rows(float *C, int m, int n, int world, int rank, void *comm, void *stream) {
    if (!C || !comm || m < 0 || n < 0 || world < 1 || rank < 0 || rank >= world) return (int)hipErrorInvalidValue;
    ncclComm_t c = static_cast<ncclComm_t>(comm);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the plan (qgemm_allgather_plan, tested on the CPU) executed on RCCL: at most world operations, sized
    // from world (no fixed cap on the communicator size)
    std::vector<int64_t> first((size_t)world), count((size_t)world);
    std::vector<int> root((size_t)world);
    const int ops = qgemm_allgather_plan(m, n, world, first.data(), count.data(), root.data(), world);
    if (ops < 0) return -ops;
    if (ops == 0) return 0;
    qgemm_coll_op op{};
    op.rank = rank;
    if (ops == 1 && root[0] < 0) {
        op.root = -1, op.count = count[0], op.recv_off = first[0], op.send_off = first[0] + (int64_t)rank * count[0];
        return nccl_rc(issue(op, C, c, s));
    }
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < ops && r == ncclSuccess; ++i) {
        op.root = root[i], op.count = count[i], op.recv_off = first[i], op.send_off = first[i];
        r = issue(op, C, c, s);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    return nccl_rc(r != ncclSuccess ? r : r2);
}

int qgemm_node_mm_quantize(const float *const *A, const float *const *B, float *const *C, int m, int n, int k,
                           int ndev, const int *devices, void *const *comms, void *const *streams, int mode) {
    if (!A || !B || !C || !devices || !streams || ndev < 1 || mode < 0 || mode > 2 || (mode && !comms))
        return (int)hipErrorInvalidValue;
    int prev = 0;
    hipError_t he = hipGetDevice(&prev);
    if (he != hipSuccess) return (int)he;
    int rc = 0;
    for (int r = 0; r < ndev && rc == 0 && mode != 2; ++r) {
        if ((he = hipSetDevice(devices[r])) != hipSuccess) rc = (int)he;
        else rc = op_mm_quantize_shard(A[r], B[r], C[r], m, n, k, ndev, r, streams[r]);
    }
    if (rc == 0 && mode != 0 && ndev > 1) {
        // one process drives every rank: ONE flat group holding every rank's planned collectives
        // (qgemm_node_allgather_plan, checked on the CPU for every ndev and m % ndev), no nested groups
        const int nops = qgemm_node_allgather_plan(m, n, ndev, nullptr, 0);
        if (nops < 0) rc = -nops;
        std::vector<qgemm_coll_op> ops(nops > 0 ? (size_t)nops : 0);
        if (rc == 0 && nops > 0) {
            const int got = qgemm_node_allgather_plan(m, n, ndev, ops.data(), nops);
            if (got < 0) rc = -got;
        }
        // every device is selected once BEFORE the group opens, so the only fallible steps inside it are the
        // enqueues themselves (a failure there leaves the communicators unusable, as any RCCL group error does)
        for (int r = 0; r < ndev && rc == 0 && nops > 0; ++r)
            if ((he = hipSetDevice(devices[r])) != hipSuccess) rc = (int)he;
        if (rc == 0 && nops > 0) {
            ncclResult_t g = ncclGroupStart();
            for (int i = 0; i < nops && rc == 0 && g == ncclSuccess; ++i) {
                const qgemm_coll_op &op = ops[(size_t)i];
                if ((he = hipSetDevice(devices[op.rank])) != hipSuccess) rc = (int)he;
                else g = issue(op, C[op.rank], static_cast<ncclComm_t>(comms[op.rank]),
                               static_cast<hipStream_t>(streams[op.rank]));
            }
            const ncclResult_t g2 = ncclGroupEnd();
            if (rc == 0) rc = nccl_rc(g != ncclSuccess ? g : g2);
        }
    }
    (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
