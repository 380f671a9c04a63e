// mpi_internal.h — the communicator and MatMult_MPIAIJ handles shared by the
// distributed solver (ksp_mpi.hip) and the distributed GAMG (gamg_mpi.hip).
// Not part of the ABI (include/aijhip_mpi.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

#include "aijhip_internal.h"
#include "aijhip_mpi.h"
#include "cg_device.h"

struct aijhip_comm {
    int kind = 0;
    int32_t nranks = 1, rank = 0, device = 0;
    int version = 0;
    ncclComm_t nc = nullptr;
    aijhip_host_allreduce_fn har = nullptr;
    aijhip_host_exchange_fn hex = nullptr;
    aijhip_host_sendrecv_fn hsr = nullptr;  // variable-size set-up exchanges (host transport)
    void *ctx = nullptr;
    double timeout_s = 300.0;
    bool aborted = false;
    double *h_red = nullptr;  // pinned staging of host all-reduces
    hipEvent_t ev_wait = nullptr;
    int64_t waits = 0;  // host waits made (polls, host-transport collectives)
    hipStream_t xs = nullptr;  // set-up exchanges (RCCL), created on first use
};

struct aijhip_mpiaij {
    aijhip_comm *comm = nullptr;
    aijhip_mat *Ad = nullptr, *Ao = nullptr;
    int halo = AIJHIP_HALO_P2P;
    int32_t mloc = 0;
    int64_t n_ghost = 0;
    std::vector<int32_t> send_peer, recv_peer;
    std::vector<int64_t> send_off, recv_off;
    std::vector<int64_t> send_first;  // per send peer: first row if its rows are one contiguous run, else -1
    int32_t gather_len = 0;
    int64_t n_send = 0;     // packed send entries (all-gather: gather_len)
    bool pack_all = false;  // every send row goes through the packed buffer
    int32_t *d_send_rows = nullptr;
    std::vector<int32_t> h_send_rows;  // host copy of the send rows (the distributed GAMG set-up)
    double *d_sendbuf = nullptr, *d_ghost = nullptr;
    double *h_send = nullptr, *h_ghost = nullptr;  // host transport staging (pinned)
    hipStream_t xs = nullptr;
    hipEvent_t ev_x = nullptr, ev_halo = nullptr;
    const double *post_x = nullptr;  // RCCL: the x of the posted exchange, sent by halo_finish
    // RCCL: the exchange on its own stream beside A_d (1, default) or on the
    // compute stream itself, in order (0: no fork / join events; the pack,
    // A_d, the collective and A_o run one after another)
    int overlap = 1;
    hipStream_t post_s = nullptr;  // the stream the posted exchange runs on
    bool posted = false;           // a halo_post not yet matched by its halo_finish
    int o_grid = 1;
    // test hook (AIJHIP_FAULT_AD_RANK at create): this rank's A_d launch
    // reports hipErrorInvalidValue, so the error paths after a post are tested
    bool fault_ad = false;
};

namespace aijhip_mpi {

int mfail(int code, const std::string &msg);
int mhip(hipError_t e, const char *what);
// Block until `s` has drained (timeout + RCCL async-error checks).
int wait_stream(aijhip_comm *C, hipStream_t s);
// In-place sum of n device doubles over all ranks, on `s`.
int comm_allreduce(aijhip_comm *C, double *d_buf, int32_t n, hipStream_t s);
// Sum of one host double over all ranks (every rank gets the same value).
int comm_allreduce_host(aijhip_comm *C, double *v, int32_t n);
// Set-up exchange of 8-byte words: out[q] goes to rank q, in[p] receives
// what rank p sent (sizes travel first; out[rank] is copied to in[rank]).
// Collective: every rank calls it with nranks-long vectors.
int comm_sendrecv(aijhip_comm *C, const std::vector<std::vector<uint64_t>> &out,
                  std::vector<std::vector<uint64_t>> &in);
// The ghost exchange of an operator: post = the fork from `s` and the pack
// kernels on its exchange stream; the caller then launches the diagonal
// product on `s`; finish = the RCCL collective (or the host transport's
// exchange), then `s` waits for the ghosts in M->d_ghost. Every post is
// followed by exactly one finish — on an error path too (halo_abort): the
// peers are already committed to the exchange, and a rank that skipped its
// half would leave them blocked in the collective.
int halo_post(aijhip_mpiaij *M, const double *x, hipStream_t s);
int halo_finish(aijhip_mpiaij *M, hipStream_t s);
// y[row] += the ghost values other ranks hold for this rank's rows: the
// exchange backwards (VecScatter SCATTER_REVERSE, ADD_VALUES), on s, p2p
// plans only. Collective.
int halo_reverse_add(aijhip_mpiaij *M, const double *d_gvals, double *y, hipStream_t s);
// The error path after a successful halo_post: completes the exchange (its
// result ignored) so no peer waits on this rank, and returns rc.
int halo_abort(aijhip_mpiaij *M, hipStream_t s, int rc);
// y = A_d x + A_o g (MatMult_MPIAIJ); part/opart/S/fused: the CG epilogue
// (ksp_mpi.hip); stop: CG's flag for the products.
int mpiaij_apply(aijhip_mpiaij *M, const double *x, double *y, hipStream_t s, double *part, double *opart,
                 const CGState *S, bool fused, const int *stop = nullptr);

}  // namespace aijhip_mpi
