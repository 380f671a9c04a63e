/*
 * aijhip_mpi.h — the row-partitioned path on MI355X: one process per GPU,
 * the communicator RCCL (over xGMI) or the caller's own host transport,
 * MatMult_MPIAIJ over it, and KSPSolve_CG over that.
 *
 * Reference mapping. The reference runs PETSc's MPIAIJ on 1-16 MPI ranks
 * (/root/reference/runs/single-node-scaling.pbs:56-67); its patched
 * MatMult_SeqAIJ (src/openacc-step{1..4}/MatMult_SeqAIJ.patch) is the
 * diagonal-block product inside PETSc's MatMult_MPIAIJ [ext]:
 *     VecScatterBegin(x -> lvec); (*A->ops->mult)(A_d, x, y);
 *     VecScatterEnd;              (*B->ops->multadd)(A_o, lvec, y, y)
 * and its KSPSolve_CG [ext] reduces every dot with MPI_Allreduce
 * (/root/reference/src/main_ksp.cpp:103). Here:
 *     VecScatter        -> grouped RCCL send/recv (or all-gather) of the
 *                          ghost rows on a second HIP stream, overlapped with
 *                          the A_d product on the caller's stream
 *     MPI_Allreduce     -> RCCL all-reduce of 1-3 device doubles, enqueued on
 *                          the caller's stream (no host round trip)
 *     CG scalar logic   -> device kernels on the reduced values (every rank
 *                          holds the same sums, so every rank branches alike);
 *                          the host polls a stop flag every few iterations.
 *
 * The local blocks are ordinary aijhip_mat_t handles (include/aijhip.h): A_d
 * with local columns, A_o with columns numbered into the ghost vector
 * (PETSc's garray order). The handles here borrow them.
 *
 * Error convention as aijhip.h; AIJHIP_ERR_COMM for a failed or timed-out
 * collective (the communicator is aborted and every later call on it fails).
 */
#ifndef AIJHIP_MPI_H
#define AIJHIP_MPI_H

#include <stdint.h>

#include "aijhip.h"
#include "aijhip_gamg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define AIJHIP_ERR_COMM 6

typedef struct aijhip_comm *aijhip_comm_t;
typedef struct aijhip_mpiaij *aijhip_mpiaij_t;
typedef struct aijhip_kspmpi *aijhip_kspmpi_t;

enum { AIJHIP_COMM_RCCL = 1, AIJHIP_COMM_HOST = 2 };
enum { AIJHIP_HALO_P2P = 0, AIJHIP_HALO_ALLGATHER = 1 };

/* ---------------------------------------------------------------- comm */

/* RCCL's 128-byte ncclUniqueId, made on one rank and handed to all others by
 * the caller (e.g. over torch.distributed or MPI_Bcast). */
int aijhip_comm_rccl_unique_id(unsigned char id[128]);
/* ncclCommInitRank on `device` (collective over all nranks). RCCL is
 * resolved at run time from the process (the librccl.so.1 already loaded,
 * e.g. by PyTorch) or from /opt/rocm/lib. */
int aijhip_comm_create_rccl(const unsigned char id[128], int32_t nranks, int32_t rank, int32_t device,
                            aijhip_comm_t *out);

/* A host transport supplied by the caller (MPI, gloo, ...). Buffers are HOST
 * memory; the library stages device data through pinned buffers around each
 * call. allreduce: in-place sum of n doubles over all ranks (every rank must
 * end with identical values). exchange: the halo of operator `op` — `send` holds this rank's
 * packed send rows (peers in the order given to aijhip_mpiaij_create,
 * send_off delimiting them), `recv` receives the ghost vector (p2p: peer
 * segments at recv_off; all-gather: nranks x gather_len). Return 0 on
 * success. */
typedef int (*aijhip_host_allreduce_fn)(void *ctx, double *buf, int32_t n);
typedef int (*aijhip_host_exchange_fn)(void *ctx, aijhip_mpiaij_t op, const double *send, int64_t nsend,
                                       double *recv, int64_t nrecv);
int aijhip_comm_create_host(int32_t nranks, int32_t rank, int32_t device, aijhip_host_allreduce_fn allreduce,
                            aijhip_host_exchange_fn exchange, void *ctx, aijhip_comm_t *out);

/* The host transport's point-to-point exchange of variable-size messages,
 * used by the distributed GAMG set-up (aggregate ids, ghost rows of P,
 * Galerkin contributions to other ranks' coarse rows): send segment q —
 * send[send_off[q] .. send_off[q+1]), 8-byte words — to send_peer[q];
 * receive segment p into recv[recv_off[p] .. recv_off[p+1]) from
 * recv_peer[p]. Sizes are known on both sides (the library exchanges them
 * first); this rank never appears as a peer. Return 0 on success. */
typedef int (*aijhip_host_sendrecv_fn)(void *ctx, int32_t n_send, const int32_t *send_peer,
                                       const int64_t *send_off, const double *send, int32_t n_recv,
                                       const int32_t *recv_peer, const int64_t *recv_off, double *recv);
int aijhip_comm_set_host_sendrecv(aijhip_comm_t comm, aijhip_host_sendrecv_fn fn);

/* kind: AIJHIP_COMM_*; version: RCCL's ncclGetVersion code (0 for host). */
int aijhip_comm_info(aijhip_comm_t comm, int32_t *nranks, int32_t *rank, int32_t *kind, int32_t *version);
/* In-place sum of n device doubles over all ranks, enqueued on `stream`
 * (MPI_Allreduce(MPI_SUM) of VecDot / VecNorm). */
int aijhip_comm_allreduce_sum(aijhip_comm_t comm, double *d_buf, int32_t n, void *stream);
/* Seconds a blocking wait inside a solve may take before the communicator
 * is aborted and AIJHIP_ERR_COMM returned (default 300; <= 0 = forever). */
int aijhip_comm_set_timeout(aijhip_comm_t comm, double seconds);
int aijhip_comm_destroy(aijhip_comm_t comm);

/* ---------------------------------------------------- MatMult_MPIAIJ */

/* This rank's row block: A_d (mloc x mloc, local columns), A_o (mloc x
 * n_ghost_buf, may be NULL when no row has off-block entries).
 * Send side: peers send_peer[0..n_send) in that order; the local rows sent
 * to peer q are send_rows[send_off[q] .. send_off[q+1]).
 * Receive side, halo AIJHIP_HALO_P2P: ghost[recv_off[p] .. recv_off[p+1])
 * comes from recv_peer[p] (ghost length recv_off[n_recv]). A peer may be
 * this rank itself (a send/receive pair with itself is a local copy; PETSc's
 * VecScatter does the same for self entries).
 * AIJHIP_HALO_ALLGATHER: n_send must be 1 with send_peer[0] = -1 (the rows
 * every other rank needs from this one, padded by the library to
 * gather_len); the ghost vector is the all-gather, nranks x gather_len
 * (recv_* ignored). */
int aijhip_mpiaij_create(aijhip_comm_t comm, aijhip_mat_t A_d, aijhip_mat_t A_o, int32_t halo,
                         int32_t n_send, const int32_t *send_peer, const int64_t *send_off,
                         const int32_t *send_rows, int32_t n_recv, const int32_t *recv_peer,
                         const int64_t *recv_off, int32_t gather_len, aijhip_mpiaij_t *out);
/* y = A_d x + A_o x_ghost (MatMult_MPIAIJ): the ghost exchange runs on the
 * handle's exchange stream while A_d multiplies on `stream`. x, y: device
 * fp64[mloc], distinct. */
int aijhip_mpiaij_mult(aijhip_mpiaij_t M, const double *x, double *y, void *stream);
/* RCCL exchange placement: 1 on the operator's exchange stream beside A_d x
 * (forked from and joined to the caller's stream by events); 0 on the
 * caller's stream in order — pack, A_d x, the collective, A_o g — with no
 * cross-stream events (each fork / join costs ~6-13 us of device time on the
 * MI355X, profiles/r05/; the serial form exposes the exchange instead); -1
 * (the default at create): 1 when the process has at least 8 hardware queues
 * (GPU_MAX_HW_QUEUES, aijhip_info_t.hw_queues), else 0 — with HIP's default
 * 4 the exchange stream would share the compute stream's queue and run
 * behind it (the fork / join then costs 29.5 us, profiles/r05/e/). The host
 * transport is unaffected. */
int aijhip_mpiaij_set_overlap(aijhip_mpiaij_t M, int overlap);
/* The placement in effect (0 / 1) and the hardware-queue count it followed. */
int aijhip_mpiaij_get_overlap(aijhip_mpiaij_t M, int32_t *overlap, int32_t *hw_queues);
/* The ghost vector of the last mult (device fp64, *n entries), for tests. */
int aijhip_mpiaij_get_ghost(aijhip_mpiaij_t M, const double **ghost, int64_t *n);
int aijhip_mpiaij_destroy(aijhip_mpiaij_t M);

/* ------------------------------------------------- KSPSolve_CG over it */

/* KSPCG on the distributed operator. PC (aijhip_ksp.h values): NONE; JACOBI
 * = PETSc's bjacobi + jacobi sub-PC (the inverse diagonal of A_d); GAMG =
 * PETSc's agg GAMG over the whole operator (-pc_type gamg on an MPIAIJ
 * matrix): aggregates local to each rank, the prolongator smoothed and the
 * Galerkin products formed across ranks (ghost rows of P exchanged, coarse
 * contributions sent to their owners), every level a distributed operator
 * with its own p2p halo, one multiplicative V-cycle per application with
 * the halo exchanges inside (the operator must use AIJHIP_HALO_P2P:
 * set_pc_type refuses an all-gather operator at more than one rank); at one
 * rank the single-GPU PCGAMG set-up (bit-identical to aijhip_ksp's). The
 * V-cycle's smoothing SpMVs are fused with their vector passes on A_d and add
 * A_o's share afterwards, r = (b - A_d x) - A_o g, where PETSc's MatResidual
 * forms A_d x + A_o g first: boundary rows round differently (same
 * iterations, history within 1e-10; AIJHIP_MG_UNFUSED=1 keeps PETSc's order).
 * BJACOBI_GAMG = -pc_type bjacobi -sub_pc_type gamg: a hierarchy per rank's
 * diagonal block, no communication inside the PC. Options, reasons and norms
 * as aijhip_ksp.h; defaults as PETSc. */
int aijhip_kspmpi_create(aijhip_mpiaij_t M, aijhip_kspmpi_t *out);
int aijhip_kspmpi_set_tolerances(aijhip_kspmpi_t K, double rtol, double abstol, double dtol, int32_t max_it);
int aijhip_kspmpi_set_pc_type(aijhip_kspmpi_t K, int pc_type);
int aijhip_kspmpi_set_gamg_params(aijhip_kspmpi_t K, const aijhip_gamg_params_t *p);
int aijhip_kspmpi_set_norm_type(aijhip_kspmpi_t K, int norm_type);
/* Iterations launched between two host polls of the device stop flag
 * (default 8). Every kernel of an iteration is a no-op once the flag is set,
 * and every rank polls at the same iterations, so the collectives stay
 * matched. */
int aijhip_kspmpi_set_poll_interval(aijhip_kspmpi_t K, int32_t iters);
/* The poll batch (the iterations between two polls) captured once into a HIP
 * graph and replayed with one launch: 0 off (default), 1 on (RCCL only; the
 * host transport waits on the host inside its exchanges); -1 = the default. The same kernels and collectives in the same order:
 * the results are the direct launches' bits. Re-captured when x, the poll
 * interval, the tolerances / norm or the set-up change. */
int aijhip_kspmpi_set_graph(aijhip_kspmpi_t K, int mode);
/* Batches the last solve replayed from the graph. */
int aijhip_kspmpi_get_graph_batches(aijhip_kspmpi_t K, int32_t *batches);
/* KSPSolve from x = 0 (main_ksp.cpp: VecSet(lhs, 0)); b, x device
 * fp64[mloc]. Returns once the solve has finished on this rank. */
int aijhip_kspmpi_solve(aijhip_kspmpi_t K, const double *b, double *x, void *stream);
int aijhip_kspmpi_get_iteration_number(aijhip_kspmpi_t K, int32_t *its);
int aijhip_kspmpi_get_residual_norm(aijhip_kspmpi_t K, double *rnorm);
int aijhip_kspmpi_get_converged_reason(aijhip_kspmpi_t K, int *reason);
int aijhip_kspmpi_get_residual_history(aijhip_kspmpi_t K, double *hist, int32_t na, int32_t *n);
/* Host synchronisations made by the last solve (polls + the final read). */
int aijhip_kspmpi_get_host_syncs(aijhip_kspmpi_t K, int32_t *n);
/* The preconditioner's multigrid levels after set-up: global rows and
 * global operator entries per level (GAMG across ranks); BJACOBI_GAMG: this
 * rank's block hierarchy; other PCs: the operator alone. Collective for
 * GAMG (nnz is summed over the ranks). */
int aijhip_kspmpi_get_pc_levels(aijhip_kspmpi_t K, int32_t *nlevels, int64_t *rows, int64_t *nnz, int32_t cap);
/* GAMG across ranks, after set-up: this rank's rows of level l's operator
 * (which = 'A') or interpolation (which = 'P', l below the coarsest) with
 * GLOBAL column ids of their level; *rstart = the first global row, *m rows,
 * *nnz entries. Call with ai = NULL for the sizes, then with arrays of
 * m + 1 / nnz / nnz entries. For tests and inspection. */
int aijhip_kspmpi_get_pc_level(aijhip_kspmpi_t K, int32_t l, char which, int64_t *rstart, int32_t *m, int64_t *nnz,
                               int64_t *ai, int64_t *aj, double *aa);
/* Seconds the last set-up took on this rank. */
int aijhip_kspmpi_get_setup_seconds(aijhip_kspmpi_t K, double *seconds);
int aijhip_kspmpi_destroy(aijhip_kspmpi_t K);

#ifdef __cplusplus
}
#endif

#endif /* AIJHIP_MPI_H */
