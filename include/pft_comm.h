/*
 * pft_comm.h -- the inter-slab communicator that replaces the reference's MPI traffic on the
 * hot path (SURVEY.md section 2 "Every MPI call site"):
 *   - sync_solution (equation.c:290-326, MPI_Isend/Irecv/Waitall of 2 ghost planes x 3 vars)
 *       -> pft_comm_halo: ONE ghost plane per field and direction (the 7-point stencil reads only
 *          the first ghost layer), RCCL grouped ncclSend/ncclRecv over xGMI on a dedicated HIP
 *          stream, overlapped with the interior sweep;
 *   - MPI_Allreduce(MAX) of eps (hybrid2.c:572) -> pft_comm_allreduce_eps (device buffer, RCCL);
 *   - MPI_Bcast of t/h/delta/... and of the command (hybrid2.c:328-336,616,690) -> pft_comm_bcast.
 *
 * One process per slab: rank r drives GPU `device` and holds Z-slab r (rank 0 = bottom).
 * Transports:
 *   "ipc"      one process per slab on one node (one slab per GPU, or several on one GPU): the
 *              neighbours' slab buffers are IPC-mapped (hipIpcOpenMemHandle, over xGMI between
 *              GPUs), each stage's boundary planes are stored straight into the neighbours' ghost
 *              planes by a put kernel that then raises their flag words, and each compute stream
 *              waits for its own flags (hipStreamWaitValue64): one launch per stage, no collective
 *              library, no host round trip.  The eps max and the broadcasts are host rounds over a
 *              POSIX shared-memory segment.
 *   "rccl"     one process per GPU, RCCL ncclSend/ncclRecv on a priority stream beside the
 *              interior sweep (boundary planes launched first).
 *   "loopback" several slabs in ONE process, one host thread per slab, device-to-device copies.
 *   "self"     one rank.
 * The communicator in use is per host thread (pft_comm_set_current), as the reference solver's
 * MPI state is per process.
 */
#ifndef PFT_COMM_H
#define PFT_COMM_H

#include "pft_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pft_comm pft_comm;

#define PFT_UNIQUE_ID_BYTES 128

int pft_comm_init_self(pft_comm ** c);
/* rank 0 creates the id, every rank passes the same bytes (exchange them out of band, e.g.
   through torch.distributed's store) */
int pft_comm_get_unique_id(void * id_bytes);
int pft_comm_init_rccl(pft_comm ** c, int nranks, int rank, const void * id_bytes, int device);
/* ipc: every rank passes the same POSIX shared-memory name ("/..."; rank 0 creates the segment
   and unlinks the name once all ranks have mapped it) and its HIP device.  Peers are waited for
   up to PFT_IPC_TIMEOUT seconds (environment, default 300); a timeout returns -5000. */
int pft_comm_init_ipc(pft_comm ** c, int nranks, int rank, const char * name, int device);
/* loopback: create once, then each of the nranks threads calls pft_comm_loopback_rank() */
int pft_comm_init_loopback(pft_comm ** group, int nranks);
int pft_comm_loopback_rank(pft_comm * group, int rank, pft_comm ** mine);
int pft_comm_destroy(pft_comm * c);

int pft_comm_rank(const pft_comm * c);
/* 1 when the stage pipeline splits boundary planes from the interior and exchanges halos
   (more than one rank, or the self-exchange diagnostic) */
int pft_comm_splits(const pft_comm * c);
/* diagnostic, 1-rank RCCL or ipc communicator, before a slab is attached: run the multi-rank
   stage pipeline on one GPU, the halo exchange sending the slab's boundary planes to its own
   ghost planes (never read by a single slab) -- the per-rank cost of the N > 1 path without the
   xGMI transfer time (bench.py --self-exchange) */
int pft_comm_set_self_exchange(pft_comm * c, int on);
/* 1: the ipc transport exchanges halos (more than one rank, or the self exchange): every stage is
   one launch over all planes followed by the stream-ordered put + wait (no boundary split) */
int pft_comm_device_halo(const pft_comm * c);
/* 1: each launch whose output is exchanged runs its boundary planes first and the exchange goes
   beside the interior launch (pft_comm_halo_start ... interior ... pft_comm_halo_finish): RCCL,
   loopback, and ipc on the copy engines; 0: one launch, then the exchange (ipc with put kernels) */
int pft_comm_boundary_first(const pft_comm * c);
/* ipc, before a slab is attached: 1 = the exchange on the copy engines (SDMA copies of the planes
   and 8-byte copies raising the flags on the comm stream, pft_slab_halo_put_ce) beside the interior
   launch, instead of a put kernel after the whole-slab launch; env PFT_IPC_CE=1 sets it at init */
int pft_comm_set_copy_engine(pft_comm * c, int on);
int pft_comm_copy_engine(const pft_comm * c);
int pft_comm_size(const pft_comm * c);
const char * pft_comm_kind(const pft_comm * c);

/* per-thread current communicator (RK_MPI_SA_init binds to it; NULL = self) */
int pft_comm_set_current(pft_comm * c);
pft_comm * pft_comm_current(void);

/* attach the slab whose buffers are exchanged */
int pft_comm_attach(pft_comm * c, pft_slab * s);
/* ipc: a rank could not export or map a neighbour's buffers; every rank's attach returns it (or
   its own error) in the same round */
#define PFT_ERR_IPC_ATTACH (-5004)

/* exchange the boundary planes of buffer `buf` (fields [f0, f1)) with the z-neighbours.
   halo_start: ordered after the work already on the slab's compute stream, runs on the slab's
   communication stream, so kernels enqueued on the compute stream afterwards (the interior
   sweep) overlap it; halo_finish: the compute stream waits for the exchange.
   No-ops for a single rank. */
int pft_comm_halo_start(pft_comm * c, int buf, int f0, int f1);
int pft_comm_halo_finish(pft_comm * c);
int pft_comm_halo(pft_comm * c, int buf, int f0, int f1);   /* start + finish */
/* the pair kernels' two-plane halo: planes 1, 2 and n3-1, n3 into the neighbours' ghost and far
   ghost planes (pft_slab_far), start + finish; needs n3 >= 2 on every slab */
int pft_comm_halo_deep(pft_comm * c, int buf, int f0, int f1);
int pft_comm_halo_start_deep(pft_comm * c, int buf, int f0, int f1);   /* ... then pft_comm_halo_finish */
/* eps max over ranks, on the slab's scratch (u64 bits + non-finite flag), stream-ordered
   (rccl, loopback; a no-op for ipc, whose max is pft_comm_eps_host) */
int pft_comm_allreduce_eps(pft_comm * c);
/* ipc: the max over ranks of the error norm the host fetched (and the OR of the non-finite
   flags), one shared-memory round; a no-op for the other transports */
int pft_comm_eps_host(pft_comm * c, double * eps, int * nonfinite);
/* eps max over ranks + its publication to pinned host memory (pft_slab_eps_mark): with RCCL both
   run on the communication stream, off the compute stream's critical path (the speculative
   stage 1 is enqueued right after); a single rank just publishes */
int pft_comm_eps_publish(pft_comm * c);
/* host-level collectives used outside the per-stage path */
int pft_comm_bcast(pft_comm * c, void * data, int bytes, int root);
int pft_comm_allreduce_max_i64(pft_comm * c, long long * v);
int pft_comm_barrier(pft_comm * c);

#ifdef __cplusplus
}
#endif
#endif
