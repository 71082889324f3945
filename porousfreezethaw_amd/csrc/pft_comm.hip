// pft_comm.hip -- inter-slab communication for libpft (see include/pft_comm.h).
//
// Replaces the reference's MPI calls on the hot path (equation.c:290-326 sync_solution,
// RK_MPI_SAsolver_hybrid2.c:572 eps Allreduce, :328-336/:616/:690 Bcasts).  Transports:
//  - ipc: one process per slab on one node.  Each slab's buffers are mapped into its
//    z-neighbours' processes (hipIpcOpenMemHandle; same GPU or a peer GPU over xGMI); a stage's
//    boundary planes are stored straight into the neighbours' ghost planes by a put kernel that
//    then raises their flag words, and each stream waits for its own flags
//    (hipStreamWaitValue64).  Host-level collectives (the eps max, broadcasts) go through a POSIX
//    shared-memory segment.  No collective library, no host round trip per stage.
//  - rccl: the librccl of /opt/rocm, one process per GPU, ncclSend/ncclRecv on a priority stream.
//  - loopback: several slabs in one process (one host thread each), device copies (tests).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "../../include/pft_comm.h"

enum { KIND_SELF = 0, KIND_RCCL = 1, KIND_LOOP = 2, KIND_IPC = 3 };

// ---- ipc rendezvous segment ---------------------------------------------------------------
#define PFT_IPC_MAX 64
#define PFT_IPC_MAGIC 0x7066745f69706331ULL   // "pft_ipc1"

struct IpcSlot {              // one rank's slab, published at attach
  int n3, device;
  char ident[PFT_DEV_IDENT_BYTES];   // its GPU's identity (pft_hip_device_ident)
  int staged;                 // its staged-receive request (PFT_IPC_STAGED): both ends of a link agree
  long fs;
  char handles[PFT_IPC_HANDLE_BYTES];
};

struct IpcRound {             // one rank's part of a host collective round
  unsigned long long seq;     // written last (release): the round this payload belongs to
  unsigned long long v[2];
  long long iv;
  char bytes[256];
};

struct IpcShared {
  unsigned long long magic;
  int nranks;
  IpcSlot slot[PFT_IPC_MAX];
  IpcRound round[2][PFT_IPC_MAX];   // by round parity: round n+2 may reuse round n's records
                                    // only once every rank has posted round n+1
};

struct LoopGroup {
  int n;
  int refs;
  pthread_barrier_t bar;
  pft_slab** slabs;
  unsigned long long* eps;   // 2 per rank
  long long* ivals;          // 1 per rank
  char bbuf[256];
};

struct pft_comm {
  int kind;
  int rank, size;
  int device;
  pft_slab* slab;
  ncclComm_t nccl;
  LoopGroup* grp;
  hipEvent_t ev_ready, ev_done;
  int pending;
  void* dscratch;   // 256 bytes of device memory for host-level collectives
  int self_x;       // diagnostic: 1-rank communicator exchanging with itself
  // ipc
  IpcShared* shm;
  char shm_name[128];
  unsigned long long hseq;   // host collective rounds so far (identical on every rank)
  unsigned long long dseq;   // device halo exchanges so far (identical on every rank)
  double timeout_s;
  int ce_buf, ce_f0, ce_f1, ce_deep;   // the copy-engine exchange marked by halo_start
  int ce;                    // ipc: the halo planes go on the copy engines beside the interior launch
                             // (pft_comm_set_copy_engine; env PFT_IPC_CE)
  void* bcast_pinned;        // rccl: pinned host staging of pft_comm_bcast
  // rccl: every host wait on RCCL work is bounded (PFT_COMM_TIMEOUT, default 300 s) and watches
  // ncclCommGetAsyncError; on expiry or an error the communicator is aborted (ncclCommAbort) and
  // every later call refuses (PFT_ERR_COMM_ABORTED)
  int aborted;
  long halos;                        // exchanges started so far
  long stall_after;                  // test hook PFT_COMM_STALL=n: the n-th exchange's comm stream
  unsigned long long* stall_word;    // waits on this word (uncached device memory), released only
  hipStream_t stall_stream;          // by the abort -- a peer that never arrives, on one GPU
};

static __thread pft_comm* g_current = nullptr;

static double now_s()
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

// spin on a shared-memory word (tight for ~50 us, then yielding), up to c->timeout_s
static int ipc_wait_ge(const pft_comm* c, const unsigned long long* w, unsigned long long v)
{
  if (__atomic_load_n(w, __ATOMIC_ACQUIRE) >= v) return 0;
  const double t0 = now_s();
  for (long it = 0;; ++it) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) >= v) return 0;
    if (it < 20000) {
      __builtin_ia32_pause();
    } else {
      sched_yield();
      if ((it & 1023) == 0 && now_s() - t0 > c->timeout_s) {
        fprintf(stderr, "pft_comm(ipc): rank %d timed out waiting for a peer (%.0f s)\n", c->rank, c->timeout_s);
        return -5000;
      }
    }
  }
}

// one host collective round: post this rank's payload, wait for every rank's; returns the records
static int ipc_round(pft_comm* c, const unsigned long long v[2], long long iv, const void* bytes, int nbytes,
                     IpcRound** recs)
{
  const unsigned long long seq = ++c->hseq;
  IpcRound* R = c->shm->round[seq & 1];
  IpcRound* me = &R[c->rank];
  if (v) {
    me->v[0] = v[0];
    me->v[1] = v[1];
  }
  me->iv = iv;
  if (bytes && nbytes > 0) memcpy(me->bytes, bytes, nbytes);
  __atomic_store_n(&me->seq, seq, __ATOMIC_RELEASE);
  for (int q = 0; q < c->size; ++q) {
    const int rc = ipc_wait_ge(c, &R[q].seq, seq);
    if (rc) return rc;
  }
  *recs = R;
  return 0;
}

// ---- rccl watchdog -------------------------------------------------------------------------
static double comm_timeout_env()
{
  const char* e = getenv("PFT_COMM_TIMEOUT");
  return (e && atof(e) > 0.0) ? atof(e) : 300.0;
}

static int rccl_abort(pft_comm* c, const char* why)
{
  if (c->aborted) return PFT_ERR_COMM_ABORTED;
  fprintf(stderr, "pft_comm(rccl): rank %d: %s: aborting the communicator\n", c->rank, why);
  c->aborted = 1;
  if (c->stall_word) {
    // the test hook's stalled comm stream goes on first, so that nothing still waits on it while
    // the abort frees the communicator's resources
    static const unsigned long long go = ~0ULL >> 1;
    (void)hipMemcpyAsync(c->stall_word, &go, 8, hipMemcpyHostToDevice, c->stall_stream);
    (void)hipStreamSynchronize(c->stall_stream);
  }
  // the abort flag ends RCCL kernels waiting for a peer; the frees inside wait for the device
  (void)ncclCommAbort(c->nccl);
  c->nccl = nullptr;
  (void)hipGetLastError();
  return PFT_ERR_COMM_ABORTED;
}

// pft_slab_watch_fn of an RCCL communicator: its asynchronous error, or the expiry of a host wait
static int rccl_watch(void* ctx, int expired)
{
  pft_comm* c = (pft_comm*)ctx;
  if (c->aborted) return PFT_ERR_COMM_ABORTED;
  ncclResult_t ae = ncclSuccess;
  if (ncclCommGetAsyncError(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
    return rccl_abort(c, ncclGetErrorString(ae));
  if (expired) return rccl_abort(c, "no progress within PFT_COMM_TIMEOUT");
  return 0;
}

// the host waits for stream st, which carries RCCL work: bounded and watched as above
static int rccl_stream_wait(pft_comm* c, hipStream_t st)
{
  double t0 = 0.0;
  for (long it = 0;; ++it) {
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) {
      fprintf(stderr, "pft_comm: hipStreamQuery: %s\n", hipGetErrorString(q));
      (void)hipGetLastError();
      return -1000 - (int)q;
    }
    if (it < 20000) {
      __builtin_ia32_pause();
    } else {
      sched_yield();
      if ((it & 1023) == 0) {
        if (t0 == 0.0) t0 = now_s();
        const int rc = rccl_watch(c, now_s() - t0 > c->timeout_s);
        if (rc) return rc;
      }
    }
  }
}

#define NCCLCHK(x)                                                         \
  do {                                                                     \
    ncclResult_t r_ = (x);                                                 \
    if (r_ != ncclSuccess) {                                               \
      fprintf(stderr, "pft_comm: %s failed: %s\n", #x, ncclGetErrorString(r_)); \
      return -3000 - (int)r_;                                              \
    }                                                                      \
  } while (0)
#define HCHK(x)                                                            \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "pft_comm: %s failed: %s\n", #x, hipGetErrorString(e_)); \
      (void)hipGetLastError();                                             \
      return -1000 - (int)e_;                                              \
    }                                                                      \
  } while (0)

extern "C" {

int pft_comm_init_self(pft_comm** c)
{
  pft_comm* m = (pft_comm*)calloc(1, sizeof(pft_comm));
  m->kind = KIND_SELF;
  m->size = 1;
  *c = m;
  return 0;
}

int pft_comm_get_unique_id(void* id_bytes)
{
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  memcpy(id_bytes, &id, sizeof(id) < PFT_UNIQUE_ID_BYTES ? sizeof(id) : PFT_UNIQUE_ID_BYTES);
  return 0;
}

int pft_comm_init_rccl(pft_comm** c, int nranks, int rank, const void* id_bytes, int device)
{
  *c = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return -2;
  HCHK(hipSetDevice(device));
  pft_comm* m = (pft_comm*)calloc(1, sizeof(pft_comm));
  m->kind = KIND_RCCL;
  m->rank = rank;
  m->size = nranks;
  m->device = device;
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&m->nccl, nranks, id, rank);
  if (r != ncclSuccess) {
    fprintf(stderr, "pft_comm: ncclCommInitRank: %s\n", ncclGetErrorString(r));
    free(m);
    return -3000 - (int)r;
  }
  HCHK(hipEventCreateWithFlags(&m->ev_ready, hipEventDisableTiming));
  HCHK(hipEventCreateWithFlags(&m->ev_done, hipEventDisableTiming));
  HCHK(hipMalloc(&m->dscratch, 256));
  m->timeout_s = comm_timeout_env();
  const char* es = getenv("PFT_COMM_STALL");
  m->stall_after = es ? atol(es) : 0;
  if (m->stall_after > 0) {
    HCHK(hipExtMallocWithFlags((void**)&m->stall_word, 64, hipDeviceMallocUncached));
    HCHK(hipMemset(m->stall_word, 0, 64));
    HCHK(hipStreamCreateWithFlags(&m->stall_stream, hipStreamNonBlocking));
  }
  *c = m;
  return 0;
}

int pft_comm_init_ipc(pft_comm** c, int nranks, int rank, const char* name, int device)
{
  *c = nullptr;
  if (nranks < 1 || nranks > PFT_IPC_MAX || rank < 0 || rank >= nranks || !name || name[0] != '/' ||
      strlen(name) >= 128)
    return -2;
  HCHK(hipSetDevice(device));
  pft_comm* m = (pft_comm*)calloc(1, sizeof(pft_comm));
  m->kind = KIND_IPC;
  m->rank = rank;
  m->size = nranks;
  m->device = device;
  const char* to = getenv("PFT_IPC_TIMEOUT");
  m->timeout_s = to ? atof(to) : 300.0;
  const char* ec = getenv("PFT_IPC_CE");
  m->ce = ec ? atoi(ec) != 0 : 0;
  snprintf(m->shm_name, sizeof(m->shm_name), "%s", name);
  const size_t bytes = sizeof(IpcShared);
  int fd = -1;
  const double t0 = now_s();
  if (rank == 0) {
    fd = shm_open(name, O_RDWR | O_CREAT | O_EXCL, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      fd = -1;
    }
  } else {
    // wait for rank 0 to create and size the segment
    while (true) {
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size == bytes) break;
        close(fd);
        fd = -1;
      }
      if (now_s() - t0 > m->timeout_s) break;
      usleep(1000);
    }
  }
  if (fd < 0) {
    fprintf(stderr, "pft_comm(ipc): rank %d: shared memory %s: %s\n", rank, name, strerror(errno));
    free(m);
    return -5001;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    free(m);
    return -5001;
  }
  m->shm = (IpcShared*)p;
  if (rank == 0) {
    m->shm->nranks = nranks;
    __atomic_store_n(&m->shm->magic, PFT_IPC_MAGIC, __ATOMIC_RELEASE);
  } else {
    int rc = ipc_wait_ge(m, &m->shm->magic, PFT_IPC_MAGIC);
    if (rc || m->shm->nranks != nranks) {
      munmap(p, bytes);
      free(m);
      return rc ? rc : -2;
    }
  }
  // everyone is mapped: rank 0 may unlink the name (the mappings stay), so nothing is left behind
  IpcRound* recs;
  int rc = ipc_round(m, nullptr, 0, nullptr, 0, &recs);
  if (rank == 0) shm_unlink(name);
  if (rc) {
    munmap(p, bytes);
    free(m);
    return rc;
  }
  *c = m;
  return 0;
}

int pft_comm_init_loopback(pft_comm** group, int nranks)
{
  if (nranks < 1) return -2;
  pft_comm* m = (pft_comm*)calloc(1, sizeof(pft_comm));
  m->kind = KIND_LOOP;
  m->rank = -1;
  m->size = nranks;
  LoopGroup* g = (LoopGroup*)calloc(1, sizeof(LoopGroup));
  g->n = nranks;
  pthread_barrier_init(&g->bar, nullptr, nranks);
  g->slabs = (pft_slab**)calloc(nranks, sizeof(pft_slab*));
  g->eps = (unsigned long long*)calloc(2 * nranks, sizeof(unsigned long long));
  g->ivals = (long long*)calloc(nranks, sizeof(long long));
  m->grp = g;
  *group = m;
  return 0;
}

int pft_comm_loopback_rank(pft_comm* group, int rank, pft_comm** mine)
{
  if (!group || group->kind != KIND_LOOP || rank < 0 || rank >= group->size) return -2;
  pft_comm* m = (pft_comm*)calloc(1, sizeof(pft_comm));
  m->kind = KIND_LOOP;
  m->rank = rank;
  m->size = group->size;
  m->grp = group->grp;
  __atomic_add_fetch(&m->grp->refs, 1, __ATOMIC_SEQ_CST);
  *mine = m;
  return 0;
}

int pft_comm_destroy(pft_comm* c)
{
  if (!c) return 0;
  if (g_current == c) g_current = nullptr;
  if (c->kind == KIND_RCCL) {
    if (c->slab) (void)pft_slab_set_watch(c->slab, nullptr, nullptr, 0.0);
    if (!c->aborted) ncclCommDestroy(c->nccl);
    (void)hipEventDestroy(c->ev_ready);
    (void)hipEventDestroy(c->ev_done);
    (void)hipFree(c->dscratch);
    if (c->stall_word) (void)hipFree(c->stall_word);
    if (c->stall_stream) (void)hipStreamDestroy(c->stall_stream);
  }
  if (c->kind == KIND_IPC) {
    if (c->slab) pft_comm_attach(c, nullptr);
    munmap(c->shm, sizeof(IpcShared));
  }
  if (c->bcast_pinned) (void)hipHostFree(c->bcast_pinned);
  if (c->kind == KIND_LOOP && c->rank < 0) {
    pthread_barrier_destroy(&c->grp->bar);
    free(c->grp->slabs);
    free(c->grp->eps);
    free(c->grp->ivals);
    free(c->grp);
  }
  free(c);
  return 0;
}

int pft_comm_rank(const pft_comm* c) { return c ? c->rank : 0; }
int pft_comm_splits(const pft_comm* c) { return c && (c->size > 1 || c->self_x); }
int pft_comm_set_self_exchange(pft_comm* c, int on)
{
  if (!c || (c->kind != KIND_RCCL && c->kind != KIND_IPC) || c->size != 1 || c->slab) return -2;
  c->self_x = on ? 1 : 0;
  return 0;
}
int pft_comm_device_halo(const pft_comm* c) { return c && c->kind == KIND_IPC && (c->size > 1 || c->self_x); }
int pft_comm_boundary_first(const pft_comm* c)
{
  return pft_comm_splits(c) && !(c->kind == KIND_IPC && !c->ce);
}
int pft_comm_set_copy_engine(pft_comm* c, int on)
{
  if (!c || c->kind != KIND_IPC || c->slab) return -2;
  c->ce = on ? 1 : 0;
  return 0;
}
int pft_comm_copy_engine(const pft_comm* c) { return c && c->kind == KIND_IPC && c->ce; }
int pft_comm_size(const pft_comm* c) { return c ? c->size : 1; }
const char* pft_comm_kind(const pft_comm* c)
{
  if (!c || c->kind == KIND_SELF) return "self";
  return c->kind == KIND_RCCL ? "rccl" : c->kind == KIND_IPC ? "ipc" : "loopback";
}

int pft_comm_set_current(pft_comm* c)
{
  g_current = c;
  return 0;
}
pft_comm* pft_comm_current(void) { return g_current; }

// 1 unless the neighbour's GPU is provably ours (equal, non-empty identities): a remote neighbour
// stages its halo through our uncached receive buffer (pft_slab_ipc_set_peer); symmetric, so both
// ends of a link take the same decision
static int ident_remote(const IpcSlot* me, const IpcSlot* peer)
{
  if (!me->ident[0] || !peer->ident[0]) return 1;
  return strncmp(me->ident, peer->ident, sizeof(me->ident)) != 0 || me->device != peer->device;
}

static int ipc_attach(pft_comm* c, pft_slab* s)
{
  // collective: every rank attaches / detaches its slab at the same point of the run
  IpcRound* recs;
  int rc;
  if (c->slab) {
    // nobody may still write into the buffers about to be unmapped (or freed); bounded by the
    // slab's ipc timeout (a lost peer's flag never comes)
    if ((rc = pft_slab_sync(c->slab))) {
      pft_slab_ipc_close(c->slab);
      c->slab = nullptr;
      return rc;
    }
    if ((rc = ipc_round(c, nullptr, 0, nullptr, 0, &recs))) return rc;
    pft_slab_ipc_close(c->slab);
    c->slab = nullptr;
  }
  if (!s) return 0;
  // both rounds carry each rank's local outcome (iv), so that a rank that cannot export or map a
  // neighbour's buffers makes every rank fail here at once -- none is left waiting in a later round
  // until PFT_IPC_TIMEOUT
  IpcSlot* me = &c->shm->slot[c->rank];
  int lrc = pft_slab_ipc_export(s, me->handles);
  me->n3 = pft_slab_nz(s);
  // the GPU's physical id, not the index: ranks whose device numbering differs (HIP_VISIBLE_DEVICES
  // per rank) still see whether a neighbour shares their GPU (pft_slab_ipc_set_peer: staged or not)
  if (!lrc) lrc = pft_hip_device_phys_id(c->device, &me->device);
  // ... and in full (PCI bus id with the function, and the UUID): a neighbour counts as on this
  // GPU only when the two identities are equal -- partitions of one package share a bus:device
  // but not the L2s, and a direct write into their ghost planes could be read stale
  if (!lrc) lrc = pft_hip_device_ident(c->device, me->ident, (int)sizeof(me->ident));
  me->fs = (long)pft_slab_field_stride(s);
  me->staged = pft_ipc_staged_env();
  if ((rc = ipc_round(c, nullptr, lrc ? 1 : 0, nullptr, 0, &recs))) return rc;   // every slot is published
  for (int q = 0; q < c->size; ++q)
    if (recs[q].iv) return lrc ? lrc : PFT_ERR_IPC_ATTACH;
  if (c->self_x) {
    if (!(lrc = pft_slab_ipc_set_peer(s, 0, nullptr, 0, 0, 0, 0))) lrc = pft_slab_ipc_set_peer(s, 1, nullptr, 0, 0, 0, 0);
  } else {
    if (c->rank > 0) {
      const IpcSlot* b = &c->shm->slot[c->rank - 1];
      lrc = pft_slab_ipc_set_peer(s, 0, b->handles, b->n3, b->fs, ident_remote(me, b), b->staged);
    }
    if (!lrc && c->rank < c->size - 1) {
      const IpcSlot* a = &c->shm->slot[c->rank + 1];
      lrc = pft_slab_ipc_set_peer(s, 1, a->handles, a->n3, a->fs, ident_remote(me, a), a->staged);
    }
  }
  if (!lrc) {
    // the ranks on this GPU (this one included): a staged wait spins in few blocks when it shares
    // the GPU with another rank (pft_halo_wait_blocks)
    int same = 0;
    for (int q = 0; q < c->size; ++q) same += !ident_remote(me, &c->shm->slot[q]);
    lrc = pft_slab_set_gpu_ranks(s, same > 0 ? same : 1);
  }
  if (!lrc) lrc = pft_slab_set_boundary_stream(s, c->ce);
  {
    // fault injection (tests/test_ipc_multiprocess.py): this rank fails to map its neighbours
    const char* ef = getenv("PFT_IPC_FAIL_ATTACH");
    if (!lrc && ef && atoi(ef) == 1) lrc = PFT_ERR_IPC_ATTACH;
  }
  // the slots are reused by the next attach only after everyone has read them
  if ((rc = ipc_round(c, nullptr, lrc ? 1 : 0, nullptr, 0, &recs))) return rc;
  for (int q = 0; q < c->size; ++q)
    if (recs[q].iv) {
      pft_slab_ipc_close(s);
      return lrc ? lrc : PFT_ERR_IPC_ATTACH;
    }
  c->slab = s;
  return 0;
}

int pft_comm_attach(pft_comm* c, pft_slab* s)
{
  if (!c) return -2;
  if (c->kind == KIND_IPC) return c->slab == s ? 0 : ipc_attach(c, s);
  if (c->kind == KIND_RCCL && c->slab != s) {
    // the slab's host waits (error norm, sync, up/download) wait on RCCL-fed streams: bounded
    if (c->slab) (void)pft_slab_set_watch(c->slab, nullptr, nullptr, 0.0);
    if (s) (void)pft_slab_set_watch(s, rccl_watch, c, c->timeout_s);
  }
  c->slab = s;
  if (c->kind == KIND_LOOP) c->grp->slabs[c->rank] = s;
  return 0;
}

static void loop_barrier(pft_comm* c) { pthread_barrier_wait(&c->grp->bar); }

static int halo_start(pft_comm* c, int buf, int f0, int f1, bool deep = false)
{
  if (!pft_comm_splits(c)) return 0;
  pft_slab* s = c->slab;
  if (!s) return -2;
  hipStream_t st = (hipStream_t)pft_slab_stream(s);
  const size_t plane = pft_slab_plane(s), fs = pft_slab_field_stride(s);
  const int n3 = pft_slab_nz(s);
  double* b = pft_slab_buffer(s, buf);
  const int below = c->rank > 0 || c->self_x, above = c->rank < c->size - 1 || c->self_x;
  // self exchange (diagnostic, one slab): the boundary planes go to the slab's own ghost planes,
  // which a single slab never reads (mirror bottom wall, Dirichlet top)
  const int pb = c->self_x ? c->rank : c->rank - 1, pa = c->self_x ? c->rank : c->rank + 1;
  if (c->kind == KIND_IPC) {
    const unsigned long long seq = ++c->dseq;
    if (c->ce) {
      // copy engines: mark the compute stream here (after the boundary launch); halo_finish, which
      // the caller reaches after enqueueing the interior launch, enqueues the planes and flags on
      // the copy streams (they start at the mark, beside the interior launch) and then the wait for
      // our own flags -- the interior launch is not held behind the host's copy calls
      int rc = pft_slab_halo_mark(s);
      if (!rc) {
        c->pending = 1;
        c->ce_buf = buf;
        c->ce_f0 = f0;
        c->ce_f1 = f1;
        c->ce_deep = deep ? 1 : 0;
      }
      return rc;
    }
    // stream-ordered on the compute stream: put (boundary planes into the neighbours' ghost
    // planes, then their flags), then wait for our own flags
    int rc = pft_slab_halo_put2(s, buf, f0, f1, deep ? 1 : 0, seq);
    return rc ? rc : pft_slab_halo_wait(s, seq);
  }
  if (c->kind == KIND_RCCL) {
    if (c->aborted) return PFT_ERR_COMM_ABORTED;
    hipStream_t cs = (hipStream_t)pft_slab_comm_stream(s);
    HCHK(hipEventRecord(c->ev_ready, st));
    HCHK(hipStreamWaitEvent(cs, c->ev_ready, 0));
    if (++c->halos == c->stall_after)
      HCHK(hipStreamWaitValue64(cs, c->stall_word, 1, hipStreamWaitValueGte, ~0ULL));
    NCCLCHK(ncclGroupStart());
    // deep: also the second planes into / from the far ghost planes; per peer the sends and the
    // peer's receives pair up in the same order (field by field: ghost plane, then far plane)
    for (int f = f0; f < f1; ++f) {
      double* fld = b + f * fs;
      if (below) {
        NCCLCHK(ncclSend(fld + 1 * plane, plane, ncclFloat64, pb, c->nccl, cs));
        NCCLCHK(ncclRecv(fld + 0 * plane, plane, ncclFloat64, pb, c->nccl, cs));
        if (deep) {
          NCCLCHK(ncclSend(fld + 2 * plane, plane, ncclFloat64, pb, c->nccl, cs));
          NCCLCHK(ncclRecv(pft_slab_far(s, buf, f, 0), plane, ncclFloat64, pb, c->nccl, cs));
        }
      }
      if (above) {
        NCCLCHK(ncclSend(fld + (size_t)n3 * plane, plane, ncclFloat64, pa, c->nccl, cs));
        NCCLCHK(ncclRecv(fld + (size_t)(n3 + 1) * plane, plane, ncclFloat64, pa, c->nccl, cs));
        if (deep) {
          NCCLCHK(ncclSend(fld + (size_t)(n3 - 1) * plane, plane, ncclFloat64, pa, c->nccl, cs));
          NCCLCHK(ncclRecv(pft_slab_far(s, buf, f, 1), plane, ncclFloat64, pa, c->nccl, cs));
        }
      }
    }
    NCCLCHK(ncclGroupEnd());
    HCHK(hipEventRecord(c->ev_done, cs));
    c->pending = 1;
    return 0;
  }
  // loopback: pull the neighbours' boundary planes into our ghost planes
  HCHK(hipStreamSynchronize(st));
  loop_barrier(c);
  for (int f = f0; f < f1; ++f) {
    double* fld = b + f * fs;
    if (below) {
      pft_slab* nb = c->grp->slabs[c->rank - 1];
      const double* src = pft_slab_buffer(nb, buf) + f * pft_slab_field_stride(nb) +
                          (size_t)pft_slab_nz(nb) * pft_slab_plane(nb);
      HCHK(hipMemcpyAsync(fld, src, plane * sizeof(double), hipMemcpyDeviceToDevice, st));
      if (deep)
        HCHK(hipMemcpyAsync(pft_slab_far(s, buf, f, 0), src - pft_slab_plane(nb), plane * sizeof(double),
                            hipMemcpyDeviceToDevice, st));
    }
    if (above) {
      pft_slab* na = c->grp->slabs[c->rank + 1];
      const double* src = pft_slab_buffer(na, buf) + f * pft_slab_field_stride(na) + pft_slab_plane(na);
      HCHK(hipMemcpyAsync(fld + (size_t)(n3 + 1) * plane, src, plane * sizeof(double), hipMemcpyDeviceToDevice, st));
      if (deep)
        HCHK(hipMemcpyAsync(pft_slab_far(s, buf, f, 1), src + pft_slab_plane(na), plane * sizeof(double),
                            hipMemcpyDeviceToDevice, st));
    }
  }
  HCHK(hipStreamSynchronize(st));
  loop_barrier(c);
  return 0;
}

int pft_comm_halo_start(pft_comm* c, int buf, int f0, int f1) { return halo_start(c, buf, f0, f1); }

int pft_comm_halo_finish(pft_comm* c)
{
  if (!pft_comm_splits(c) || !c->pending) return 0;
  c->pending = 0;
  if (c->kind == KIND_IPC) {
    int rc = pft_slab_halo_put_ce(c->slab, c->ce_buf, c->ce_f0, c->ce_f1, c->ce_deep, c->dseq);
    return rc ? rc : pft_slab_halo_wait(c->slab, c->dseq);
  }
  HCHK(hipStreamWaitEvent((hipStream_t)pft_slab_stream(c->slab), c->ev_done, 0));
  return 0;
}

int pft_comm_halo_start_deep(pft_comm* c, int buf, int f0, int f1) { return halo_start(c, buf, f0, f1, true); }

int pft_comm_halo_deep(pft_comm* c, int buf, int f0, int f1)
{
  int rc = halo_start(c, buf, f0, f1, true);
  return rc ? rc : pft_comm_halo_finish(c);
}

int pft_comm_halo(pft_comm* c, int buf, int f0, int f1)
{
  int rc = pft_comm_halo_start(c, buf, f0, f1);
  return rc ? rc : pft_comm_halo_finish(c);
}

int pft_comm_allreduce_eps(pft_comm* c)
{
  if (!pft_comm_splits(c) || c->kind == KIND_IPC) return 0;   // ipc: pft_comm_eps_host
  pft_slab* s = c->slab;
  hipStream_t st = (hipStream_t)pft_slab_stream(s);
  unsigned long long* d = (unsigned long long*)pft_slab_scratch(s);
  if (c->kind == KIND_RCCL) {
    if (c->aborted) return PFT_ERR_COMM_ABORTED;
    // max of non-negative doubles == max of their bit patterns; flag: max of 0/1
    NCCLCHK(ncclAllReduce(d, d, 2, ncclUint64, ncclMax, c->nccl, st));
    return 0;
  }
  unsigned long long v[2];
  HCHK(hipMemcpyAsync(v, d, 16, hipMemcpyDeviceToHost, st));
  HCHK(hipStreamSynchronize(st));
  c->grp->eps[2 * c->rank] = v[0];
  c->grp->eps[2 * c->rank + 1] = v[1];
  loop_barrier(c);
  unsigned long long m0 = 0, m1 = 0;
  for (int r = 0; r < c->size; ++r) {
    if (c->grp->eps[2 * r] > m0) m0 = c->grp->eps[2 * r];
    if (c->grp->eps[2 * r + 1] > m1) m1 = c->grp->eps[2 * r + 1];
  }
  loop_barrier(c);
  v[0] = m0;
  v[1] = m1;
  HCHK(hipMemcpyAsync(d, v, 16, hipMemcpyHostToDevice, st));
  HCHK(hipStreamSynchronize(st));
  return 0;
}

int pft_comm_eps_publish(pft_comm* c)
{
  if (!c || !c->slab) return -2;
  pft_slab* s = c->slab;
  if (!pft_comm_splits(c) || c->kind == KIND_IPC) return pft_slab_eps_mark(s);   // ipc: pft_comm_eps_host
  if (c->kind == KIND_RCCL) {
    // the max over ranks and the publication run on the communication stream, so the compute
    // stream goes on with the speculative stage 1 while RCCL reduces
    if (c->aborted) return PFT_ERR_COMM_ABORTED;
    hipStream_t st = (hipStream_t)pft_slab_stream(s), cs = (hipStream_t)pft_slab_comm_stream(s);
    unsigned long long* d = (unsigned long long*)pft_slab_scratch(s);
    HCHK(hipEventRecord(c->ev_ready, st));
    HCHK(hipStreamWaitEvent(cs, c->ev_ready, 0));
    NCCLCHK(ncclAllReduce(d, d, 2, ncclUint64, ncclMax, c->nccl, cs));
    return pft_slab_eps_mark_on(s, (void*)cs);
  }
  // loopback: the host-side max reads the error norm through the compute stream, which must
  // first take in the comm stream's boundary launch of stage 5
  int rc = pft_slab_order(s, 1);
  if (!rc) rc = pft_comm_allreduce_eps(c);
  return rc ? rc : pft_slab_eps_mark(s);
}

int pft_comm_eps_host(pft_comm* c, double* eps, int* nonfinite)
{
  if (!c || c->kind != KIND_IPC || c->size == 1) return 0;
  // max of non-negative doubles == max of their bit patterns; the non-finite flag: any rank's
  unsigned long long v[2];
  memcpy(&v[0], eps, 8);
  v[1] = (unsigned long long)(nonfinite && *nonfinite);
  IpcRound* R;
  int rc = ipc_round(c, v, 0, nullptr, 0, &R);
  if (rc) return rc;
  unsigned long long m0 = 0, m1 = 0;
  for (int q = 0; q < c->size; ++q) {
    if (R[q].v[0] > m0) m0 = R[q].v[0];
    m1 |= R[q].v[1];
  }
  memcpy(eps, &m0, 8);
  if (nonfinite) *nonfinite = (int)(m1 != 0);
  return 0;
}

int pft_comm_bcast(pft_comm* c, void* data, int bytes, int root)
{
  if (!c || c->size == 1) return 0;
  if (bytes > 256) return -2;
  if (c->kind == KIND_IPC) {
    IpcRound* R;
    int rc = ipc_round(c, nullptr, 0, c->rank == root ? data : nullptr, bytes, &R);
    if (!rc && c->rank != root) memcpy(data, R[root].bytes, bytes);
    return rc;
  }
  if (c->kind == KIND_RCCL) {
    // on the communication stream through pinned host memory: the host waits for that stream
    // only -- not for the compute stream's speculative stage 1 (the comm stream holds at most the
    // boundary planes' exchange of it)
    if (c->aborted) return PFT_ERR_COMM_ABORTED;
    hipStream_t st = c->slab ? (hipStream_t)pft_slab_comm_stream(c->slab) : 0;
    if (!c->bcast_pinned) HCHK(hipHostMalloc(&c->bcast_pinned, 256, hipHostMallocDefault));
    memcpy(c->bcast_pinned, data, bytes);
    HCHK(hipMemcpyAsync(c->dscratch, c->bcast_pinned, bytes, hipMemcpyHostToDevice, st));
    NCCLCHK(ncclBroadcast(c->dscratch, c->dscratch, bytes, ncclUint8, root, c->nccl, st));
    HCHK(hipMemcpyAsync(c->bcast_pinned, c->dscratch, bytes, hipMemcpyDeviceToHost, st));
    const int rc = rccl_stream_wait(c, st);
    if (rc) return rc;
    memcpy(data, c->bcast_pinned, bytes);
    return 0;
  }
  if (c->rank == root) memcpy(c->grp->bbuf, data, bytes);
  loop_barrier(c);
  if (c->rank != root) memcpy(data, c->grp->bbuf, bytes);
  loop_barrier(c);
  return 0;
}

int pft_comm_allreduce_max_i64(pft_comm* c, long long* v)
{
  if (!c || c->size == 1) return 0;
  if (c->kind == KIND_IPC) {
    IpcRound* R;
    int rc = ipc_round(c, nullptr, *v, nullptr, 0, &R);
    if (rc) return rc;
    long long m = R[0].iv;
    for (int q = 1; q < c->size; ++q)
      if (R[q].iv > m) m = R[q].iv;
    *v = m;
    return 0;
  }
  if (c->kind == KIND_RCCL) {
    if (c->aborted) return PFT_ERR_COMM_ABORTED;
    hipStream_t st = c->slab ? (hipStream_t)pft_slab_stream(c->slab) : 0;
    HCHK(hipMemcpyAsync(c->dscratch, v, 8, hipMemcpyHostToDevice, st));
    NCCLCHK(ncclAllReduce(c->dscratch, c->dscratch, 1, ncclInt64, ncclMax, c->nccl, st));
    HCHK(hipMemcpyAsync(v, c->dscratch, 8, hipMemcpyDeviceToHost, st));
    return rccl_stream_wait(c, st);
  }
  c->grp->ivals[c->rank] = *v;
  loop_barrier(c);
  long long m = c->grp->ivals[0];
  for (int r = 1; r < c->size; ++r)
    if (c->grp->ivals[r] > m) m = c->grp->ivals[r];
  loop_barrier(c);
  *v = m;
  return 0;
}

int pft_comm_barrier(pft_comm* c)
{
  long long z = 0;
  return pft_comm_allreduce_max_i64(c, &z);
}

}  // extern "C"
