/*
 * pft_hip.h -- the thin C-ABI shim between libpft's host C code (rk_solver.c, model.c) and
 * the hand-written HIP kernels for gfx950 (porousfreezethaw_amd/csrc/pft_kernels.hip).
 *
 * Conventions: extern "C"; every call returns int (0 = OK, negative = HIP error, mirroring the
 * reference's negative codes); streams are explicit (opaque handles); no exceptions cross the
 * ABI; device buffers are owned by a pft_slab object.  No torch types anywhere.
 *
 * Device layout of one slab (one Z-slab of the reference decomposition, intertrack.c:1776-1800):
 * a "state" is 3 fields (u, p, gl) at stride `fs` doubles; from the buffer pointer a field holds
 * n3+2 planes of n1*n2 doubles, i fastest: plane 0 is the ghost plane below the slab, planes
 * 1..n3 the interior, plane n3+1 the ghost plane above.  The stage kernels read only these (the
 * 7-point stencil reads only the first of the reference's two ghost layers, equation.c:659-724);
 * the pair kernels also read the far ghost planes -1 and n3+2 (the second layer, exchanged at
 * slab interfaces only: pft_slab_far).  x/y mirror and z-wall conditions are folded into the
 * stencil's index logic.
 */
#ifndef PFT_HIP_H
#define PFT_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* model constants, all derived exactly as equation.c:442-447,605-612 and the left-to-right
   products of f_GradP / f_SigmaP1_P (equation.c:367-388) */
typedef struct {
	double h1_2, h2_2, h3_2;         /* (n_d/L_d)^2 (global total_n3 for d = 3) */
	double h1d2, h2d2, h3d2;         /* 0.5 * n_d/L_d */
	double xi2a;                     /* a / (xi*xi) */
	double bam;                      /* (b*alpha)*mu            (GradP, left-to-right prefix) */
	double sam;                      /* (b*sqrt(0.5a)/xi*alpha)*mu (SigmaP1-P prefix) */
	double alpha, L, zeta, u_star;
	double p_eps0, p_eps1, e23, e32; /* Sshape limiter, 3/d^2, 2/d^3 */
	double gamma, mhg;               /* gamma, (-0.5)*gamma */
	double rho_g, rho_i, rho_w;
	double cp_g, cp_i, cp_w;
	double lam_g, lam_i, lam_w;
	double top_temp1, top_temp2, phase_switch_time;
} pft_consts;

typedef struct pft_slab pft_slab;   /* opaque: device buffers + streams of one slab */

typedef struct {
	int n1, n2, n3;          /* interior cells of this slab */
	int has_below;           /* 1: a neighbour slab below (ghost plane 0 is exchanged data) */
	int has_above;           /* 1: a neighbour slab above */
	int calc_mode;           /* 0, 1, 2, 10, 11 */
	int gl_static;           /* 1: the model declares gl static (K_gl == 0): gl is read from x
	                            and neither stored in K nor combined (bit-identical, F4) */
	double eps_mult[3];      /* per-variable error multipliers (chunk_eps_mult) */
} pft_slab_desc;

/* device management */
int pft_hip_device_count(int * n);
int pft_hip_set_device(int dev);
int pft_hip_get_device(int * dev);
/* the GPU's PCI location (domain, bus, device) as one integer: equal across processes exactly when
   they use the same physical GPU (the ipc transport's staged-or-direct decision) */
int pft_hip_device_phys_id(int dev, int * id);
/* the GPU's full identity as text: its PCI bus id string with the function (hipDeviceGetPCIBusId)
   and its UUID (hipDeviceGetUuid), "dddd:bb:dd.f/<32 hex digits>".  Two processes use the same GPU
   -- the same L2s -- only when the strings are equal: partitions of one package (several HIP devices
   at one bus:device) differ in the function or the UUID, and the ipc transport stages its receive
   between them (pft_slab_ipc_set_peer).  len >= PFT_DEV_IDENT_BYTES. */
#define PFT_DEV_IDENT_BYTES 80
int pft_hip_device_ident(int dev, char * buf, int len);
int pft_hip_device_sync(void);
const char * pft_hip_last_error(void);

/* slab lifecycle */
int pft_slab_create(pft_slab ** s, const pft_slab_desc * d, const pft_consts * c);
int pft_slab_destroy(pft_slab * s);
size_t pft_slab_state_bytes(const pft_slab * s);
void * pft_slab_stream(pft_slab * s);      /* hipStream_t of the compute stream */
void * pft_slab_comm_stream(pft_slab * s); /* hipStream_t used for halo exchange */

/* Buffers of a slab: X (solution), XN (candidate x(t+h)), A0/A1 (stage inputs), K1/K3/K4. */
enum { PFT_BUF_X = 0, PFT_BUF_XN, PFT_BUF_A0, PFT_BUF_A1, PFT_BUF_K1, PFT_BUF_K3, PFT_BUF_K4, PFT_BUF_COUNT };
double * pft_slab_buffer(pft_slab * s, int which);
size_t pft_slab_field_stride(const pft_slab * s);     /* fs, in doubles */
size_t pft_slab_plane(const pft_slab * s);            /* n1*n2 */
int pft_slab_nz(const pft_slab * s);                  /* n3 (interior planes) */
void * pft_slab_scratch(pft_slab * s);                /* device: u64 eps bits, u64 non-finite flag */
const pft_slab_desc * pft_slab_get_desc(const pft_slab * s);
/* planes per workgroup z-march (tuning knob); 0 (default) = automatic: the fewest planes per
   workgroup that keep the whole launch resident in one round (occupancy x CUs / tiles chunks) */
int pft_slab_set_kz(pft_slab * s, int kz);
/* stage kernel flavour: 32 or 16 = the fused LDS-tiled kernel with 64x8 / 32x16 cell tiles (n1
   even); 1 (default) = automatic: the fused kernel with a tile fitted to n1 x n2, or the cache
   kernel where that tile would leave most lanes idle; 2 = the fitted tile at any size; 0 = the
   cache-based kernel (any n1; also used for odd n1 and for the aux-array path) */
int pft_slab_set_tile(pft_slab * s, int wx);
/* the kernel flavour (0 cache, 2 fused recompute; 1 is retired) and tile (wx cell pairs x ty
   rows; 0 x 0 for the cache kernel) that stage 1..5 launches on this slab */
int pft_slab_tile_geometry(const pft_slab * s, int stage, int * wx, int * ty);
/* 1 (default): the tiled kernels rebuild every stage input from x and the K's inside the
   stencil (no aux arrays: 39 instead of 72 doubles of traffic per cell-step, bit-identical);
   0: the reference's aux arrays are materialised between stages (cache kernel) */
int pft_slab_set_recompute(pft_slab * s, int on);
/* 1: X and XN hold the same gl field and no gl value is -0.0 or NaN (the caller checked), so
   stage 5 need not store gl's x(t+h) = x + coef*0.0 (== x); cleared by every upload */
int pft_slab_set_gl_keep(pft_slab * s, int on);
int pft_slab_get_gl_keep(const pft_slab * s);   /* 1: stage 5 skips that store */
/* buffer written by stage 1..5 of the step on this slab's path (its boundary planes are what
   the z-neighbours need before the next stage) */
int pft_slab_stage_output(const pft_slab * s, int stage);
/* number of fields (u, p[, gl]) of that buffer the stage writes and the neighbours need; stage 6
   = the speculative stage 1.  gl is left out under gl_static, and for K1..K4 on the recompute
   path, where gl's K's are the literal zeros of dgl (equation.c:731) and never stored */
int pft_slab_stage_fields(const pft_slab * s, int stage);

/* stream order between the slab's two streams: pft_slab_order(s, 0): the comm stream waits for
   the compute stream's work so far, (s, 1): the compute stream waits for the comm stream's */
int pft_slab_order(pft_slab * s, int comm_first);

/* host layout (reference padded, ghost thickness 2) <-> device layout, on the compute stream */
int pft_slab_upload_host(pft_slab * s, int which, const double * host_padded);
int pft_slab_download_host(pft_slab * s, int which, double * host_padded);

/* One Merson stage (stage 1..5) as ONE fused kernel: K = f(stage input) and the pointwise stage
   combine of RK_MPI_SAsolver_hybrid2.c:378-450 (stage 5: error norm :507-524 and the candidate
   update :657-668 into XN).  t_stage: time passed to f (for the Dirichlet value);  coef: h3,
   h6, h8, h, h3 for stages 1..5;  h: the full step (stage 4 combine);  k_begin/k_end: plane
   range (for boundary-first splitting), -1/-1 = all planes. */
int pft_slab_stage(pft_slab * s, int stage, double t_stage, double coef, double h,
                   int k_begin, int k_end);
/* k_begin value selecting the slab's two boundary planes (0 and n3-1) in one launch */
#define PFT_K_BOUNDARY (-2)
/* k_begin value selecting planes 0, 1 and n3-2, n3-1 in one launch (what the z-neighbours' pair
   kernels read: the two-plane halo) */
#define PFT_K_BOUNDARY2 (-3)
/* pair kernels only: the PFT_K_BOUNDARY2 chunks lead the grid of the interior launch [2, n3-2), one
   launch; the copy-engine exchange that follows starts when those workgroups are done
   (pft_slab_boundary_inline) */
#define PFT_K_INLINE (-4)
/* pair kernels only: the whole slab in one launch whose first workgroups are the first and the last
   z-chunk of every tile column (at least three chunks); the copy-engine exchange that follows starts
   when those are done */
#define PFT_K_ENDS_FIRST (-5)

/* K = f(input) only (RK_RightHandSide semantics), input/output buffer indices */
int pft_slab_rhs(pft_slab * s, int in_buf, int out_buf, double t);

/* refresh the model constants / per-variable error multipliers of an existing slab */
int pft_slab_set_consts(pft_slab * s, const pft_consts * c);
int pft_slab_set_eps_mult(pft_slab * s, const double * em3);

/* u_noise field (PrecalculateData, equation.c:450-456), n3*n1*n2 doubles [k][j][i]; NULL clears */
int pft_slab_set_noise(pft_slab * s, const double * host_noise);

/* f1: the default Params' initial condition and the glass beads (intertrack.c:1880-2010 with
   Params:9-21; PrecalculateData, equation.c:459-530) evaluated on the device straight into X and
   XN, bit for bit the host's (pft_model_ic_default + PrecalculateData).  Every term that depends
   on one coordinate only (the walls' tanh, the (x-L1/2)^2 of the ice disc, the node coordinates)
   comes in per-axis tables the host evaluates with the C library; the beads' tanh runs on the
   device as the C library's algorithm (pft_tanh.h).  Tables: [n1] x terms, [n2] y terms, [n3]
   z terms of this slab's planes; beads: 3*nbeads scaled centres, plane_off[n3+1] / plane_beads[]
   the candidate beads of each plane (any superset of the beads whose tanh argument is below 22).
   *gl_unclean: 1 if a gl value is -0.0 or NaN (pft_slab_set_gl_keep). */
typedef struct {
	int n1, n2, n3;
	const double *tx1, *tx2, *px2, *xb;   /* gl wall terms x - L1 + off_x, off_x - x; (x - L1/2)^2; bead x */
	const double *ty1, *ty2, *py2, *yb;
	const double *tz1, *tz2, *pz, *zb;    /* gl terms z - 0.055, off_z - z; ice-disc z window (0/1); bead z */
	double u0, r2;                        /* 293.15 (float_val), (L1/3)^2 */
	int nbeads;                           /* 0: no bead overlay */
	const double * bxyz;
	const int *plane_off, *plane_beads;
	double s, R, reach2;                  /* 0.5/xi_gl, ball_radius, the host's cull distance^2 */
} pft_ic_tables;
int pft_slab_ic_default(pft_slab * s, const pft_ic_tables * t, int * gl_unclean);
/* the beads of t over the gl already in X and XN (u, p kept; t's default-IC terms unused); with
   nbeads = 0 only the gl scan for *gl_unclean */
int pft_slab_ic_beads(pft_slab * s, const pft_ic_tables * t, int * gl_unclean);
/* (f1 for any icond formula: pft_slab_ic_program, declared in pft_frontend.h) */

/* error norm of the last stage 5: reset before the step, fetch after (blocks on the stream) */
int pft_slab_eps_reset(pft_slab * s);
int pft_slab_eps_fetch(pft_slab * s, double * eps, int * nonfinite);

/* HIP-event timing of the stage kernels on the compute stream (benchmark roofline):
   mark(stage, 0|1) records the begin/end event of one stage's launches; collect() adds the
   elapsed milliseconds of every completed begin/end pair to ms[1..5] and counts to n[1..5] */
int pft_slab_timing_mark(pft_slab * s, int stage, int end);
int pft_slab_timing_collect(pft_slab * s, double * ms, long * n);   /* completed pairs only */
int pft_slab_timing_flush(pft_slab * s, double * ms, long * n);     /* waits for all pairs */

/* buffer swap X <-> XN after an accepted step */
int pft_slab_accept(pft_slab * s);
int pft_slab_swap_buffers(pft_slab * s, int a, int b);

/* Speculative stage 1 (recompute path only): K1' = f(t_stage, XN) into A1, enqueued after stage 5
   before the accept decision.  Accepted: swap K1 <-> A1 and skip the next stage 1; rejected: x and t
   are unchanged, so K1 = f(t, x) is still exact and the next stage 1 is skipped as well (the
   reference recomputes the identical K1).  pft_slab_eps_mark() before it publishes the error norm
   to pinned host memory (and resets it for the next step), so that eps_fetch() returns while the
   speculative kernel runs. */
int pft_slab_can_speculate(const pft_slab * s);
int pft_slab_stage_spec(pft_slab * s, double t_stage, int k_begin, int k_end);
int pft_slab_eps_mark(pft_slab * s);
/* Gated steps (f4, one slab, fused stage launches): the launches of the next attempted step are
   enqueued BEFORE this step's error norm is known, so that the GPU waits neither for the host's
   decision nor for its launch latency between steps.  They assume the step is accepted (the caller
   swaps the buffers as pft_slab_accept would for the enqueue, and back) and run on the DEVICE's
   decision: the speculative stage 1 of this step, once it has reduced the error norm, decides the
   step as hybrid2.c:578-611 does (pow from ocml) and writes the next step's t and h, or a skip.
   The host takes its own decision (glibc pow) and keeps the gated step only if both agree bit for
   bit; otherwise it discards it (its outputs are never read) and launches the step again.
     gate_config(final_time, delta, h_min, delta_local, handle_nan)  the solve's constants
     gate_arm(t, h)      the next speculative stage-1 launch decides step (t, h) (ignored when that
                         launch is gated itself: it decides its own step); returns the decision seq
     gate_use(seq | 0)   launches enqueued from now on run only if decision seq accepted the step
     gate_decision(seq, &go, &t, &h)  the device's decision (waits for its publication)
   book_save/load(0|1): the error-norm publication bookkeeping, so that this step's error norm is
   fetched after the next step's launches were enqueued (save 0, enqueue, save 1, load 0, fetch;
   on a kept gated step load 1). */
int pft_slab_gate_config(pft_slab * s, double final_time, double delta, double h_min, int delta_local,
                         int handle_nan);
unsigned long long pft_slab_gate_arm(pft_slab * s, double t, double h);
int pft_slab_gate_use(pft_slab * s, unsigned long long seq);
int pft_slab_gate_decision(pft_slab * s, unsigned long long seq, int * go, double * t, double * h);
/* x^0.2 rounded to nearest from a candidate c within 1 ulp (the device's gate_decide uses it with
   ocml's pow as c): host build of the same code, for the CPU tests */
double pft_pow02_fix(double x, double c);
int pft_slab_book_save(pft_slab * s, int which);
int pft_slab_book_load(pft_slab * s, int which);
/* Pair kernels (one slab, recompute path): stages 2+3 or 4+5 of the step (first = 2 or 4) in ONE
   launch.  Stage A's K is evaluated on the tile and a one-cell ring and never stored; stage B
   writes K3 (first = 2) or the error norm and x(t+h) into XN (first = 4), bit for bit what the
   two stage launches give.  t_a / t_b: the two stage times (Dirichlet value); h: the step; coef:
   h3 for x(t+h).  set_pair: 0 off, 1 (default) automatic (slabs of >= 4 Ki cells per CU), 2 on
   any slab they fit; env PFT_PAIR=0/1/2 overrides.  pair_ok: 1 when this slab runs them (even
   n1, no z-neighbours, the mode allows); pair_geometry: the tile (tx cells x ty rows) */
int pft_slab_set_pair(pft_slab * s, int on);
int pft_slab_pair_ok(const pft_slab * s);
int pft_slab_pair_geometry(const pft_slab * s, int * tx, int * ty);
int pft_slab_pair(pft_slab * s, int first, double t_a, double t_b, double h, double coef);
/* the same on planes [k_begin, k_end) (-1/-1: all; k_begin = PFT_K_BOUNDARY2: the two planes at
   each end, for the N > 1 pipeline that exchanges them beside the interior launch) */
int pft_slab_pair_range(pft_slab * s, int first, double t_a, double t_b, double h, double coef, int k_begin,
                        int k_end);
/* the same publication enqueued on another stream of the slab's device (the communication
   stream, behind the eps max over ranks: pft_comm_eps_publish) */
int pft_slab_eps_mark_on(pft_slab * s, void * stream);
/* 1: a stage-5 launch over the whole slab publishes the error norm itself (its last workgroup
   writes it to pinned host memory, which pft_slab_eps_fetch polls) and pft_slab_eps_mark adds no
   kernel; for the single-rank and ipc paths, where the max over ranks is not a device
   collective */
int pft_slab_set_inkernel_publish(pft_slab * s, int on);

/* generic chunk-table combines for the host-staged path (any RK_MEM_DIST on a flat array) */
int pft_flat_alloc(double ** p, size_t n);
int pft_flat_free(double * p);
int pft_flat_h2d(double * dst, const double * src, size_t n, void * stream);
int pft_flat_d2h(double * dst, const double * src, size_t n, void * stream);
int pft_flat_combine(int stage, int n_chunks, const int * d_start, const int * d_size,
                     const double * d_mult, double coef, double h, const double * x,
                     const double * k1, const double * k2, const double * k3, const double * k4,
                     const double * k5, double * out, double * d_eps2, void * stream);
int pft_stream_sync(void * stream);
/* raw device memory (bytes) for the chunk tables of the host-staged path */
int pft_dev_alloc(void ** p, size_t bytes);
int pft_dev_free(void * p);
int pft_h2d(void * dst, const void * src, size_t bytes, void * stream);
/* diagnostic: plain 8-byte-per-lane device copy (rocprofv3 FETCH_SIZE/WRITE_SIZE calibration) */
int pft_probe_copy(double * dst, const double * src, size_t n, void * stream);

/* ipc transport (pft_comm.h).  Every rank swaps its buffers identically, so a buffer role names
   the same physical allocation on every slab; the neighbours' allocations are mapped once.
   export: the slab's PFT_BUF_COUNT buffer allocations, its flag words and its receive buffer as
   PFT_BUF_COUNT + 2 hipIpcMemHandle_t (64 bytes each, PFT_IPC_HANDLE_BYTES in all);
   set_peer(side 0 = below / 1 = above): open the neighbour's handles (handles = NULL: the slab
   itself, the one-GPU self-exchange diagnostic); n3 / fs are the neighbour's planes and stride;
   halo_put: boundary planes 1 and n3 of buffer `role`, fields [f0, f1), into the neighbours' ghost
   planes, then `seq` into their flag words (a copy and a one-thread signal kernel on the compute
   stream);
   halo_wait: the compute stream waits until both neighbours' flags reach `seq`.
   Staged receive (a neighbour on another GPU, or env PFT_IPC_STAGED=1): the sender writes into the
   receiver's receive buffer -- uncached device memory, so no cache of the receiving GPU holds a
   line of it -- instead of its ghost planes, and after the flag wait the receiver copies it into
   its ghost planes on its own stream (halo_recv_kernel): the halo is then as coherent as any
   kernel-to-kernel hand-off on one GPU, whatever the receiving L2s held of the ghost planes. */
#define PFT_IPC_HANDLE_BYTES (64 * (PFT_BUF_COUNT + 2))
int pft_slab_ipc_export(pft_slab * s, void * handles);
/* 1 when this process asks for staged receive between processes on one GPU (env PFT_IPC_STAGED=1) */
int pft_ipc_staged_env(void);
/* remote: 1 unless the neighbour provably uses this process's GPU (equal pft_hip_device_ident);
   peer_staged: the neighbour's own staged-receive choice (its PFT_IPC_STAGED, published at attach);
   both ends of a link stage when either asks for it, or when the neighbour is remote */
int pft_slab_ipc_set_peer(pft_slab * s, int side, const void * handles, int n3, long fs, int remote,
                          int peer_staged);
int pft_slab_ipc_close(pft_slab * s);
/* how many ranks of the communicator use this slab's GPU (ipc attach, from the identities) */
int pft_slab_set_gpu_ranks(pft_slab * s, int n);
/* workgroups of a staged receive's wait launch (n doubles): every block spins on the neighbours'
   flags first, so the count bounds the CUs a wait holds -- 32 with a staged neighbour on this GPU or
   any other rank sharing it, 128 beside an interior launch, else up to 1024 */
int pft_halo_wait_blocks(long n, int local_staged, int gpu_ranks, int on_boundary_stream);
int pft_slab_halo_put(pft_slab * s, int role, int f0, int f1, unsigned long long seq);
/* the same with deep = 1: also planes 2 and n3-1 into the neighbours' far ghost planes (the pair
   kernels' two-plane halo) */
int pft_slab_halo_put2(pft_slab * s, int role, int f0, int f1, int deep, unsigned long long seq);
/* the same put on the copy engines (SDMA, hipMemcpyDeviceToDeviceNoCU) from the slab's comm stream,
   ordered after the work already on the compute stream: the planes and then the neighbours' flags
   (8-byte copies), no kernel -- beside the interior launch that follows on the compute stream.
   The receiver's side is pft_slab_halo_wait as for halo_put2. */
int pft_slab_halo_put_ce(pft_slab * s, int role, int f0, int f1, int deep, unsigned long long seq);
/* marks the point of the compute stream the next put_ce sends from (an event after the boundary
   launch), so that the host can enqueue the interior launch before the copies: put_ce then waits
   for the mark instead of recording one */
int pft_slab_halo_mark(pft_slab * s);
/* 1: a launch of the boundary planes (k_begin PFT_K_BOUNDARY / PFT_K_BOUNDARY2) runs on a stream of
   its own at the greatest priority, beside the interior launch that follows on the compute stream,
   instead of before it; the copy-engine exchange starts when it ends, and pft_slab_halo_wait makes
   the compute stream wait for it before the next launch (its planes are that launch's input).  The
   boundary launch takes the second set of error-norm shards. */
int pft_slab_set_boundary_stream(pft_slab * s, int on);
/* the pair kernels' inline boundary: PFT_K_INLINE (the copy-engine exchange's boundary placement 4,
   PFT_CE_BND=4), PFT_K_ENDS_FIRST (placement 5), or 0 (a separate boundary launch or none) */
int pft_slab_boundary_inline(const pft_slab * s);
/* the same for the stage launches (their inline boundary can be turned off: PFT_CE_STAGE_INLINE=0) */
int pft_slab_stage_inline(const pft_slab * s);
/* the same for one pair kernel (first = 2: stages 2+3, 4: stages 4+5) */
int pft_slab_pair_inline(const pft_slab * s, int first);
/* far ghost plane of buffer `which`, field q: side 0 = two planes below the slab (the neighbour
   below's plane n3' - 1; plane -1 of the field), side 1 = two above (the neighbour above's plane
   2; plane n3 + 2) */
double * pft_slab_far(pft_slab * s, int which, int q, int side);
/* raise the neighbours' flags to `seq` behind the work on the compute stream (halo_put calls it) */
int pft_slab_halo_signal(pft_slab * s, unsigned long long seq);
int pft_slab_halo_wait(pft_slab * s, unsigned long long seq);
/* The host waits for the compute stream.  With ipc neighbours attached every host wait of the
   slab (this one, up/download, the error-norm fetch) is bounded by PFT_IPC_TIMEOUT seconds
   (default 300): a peer that died or diverged never raises the flag the stream waits on, so on
   expiry the slab releases its own flags, drains the stream and returns PFT_ERR_IPC_TIMEOUT
   (RK_MPI_SA_solve: PFT_SOLVE_DEVICE_ERROR).  A neighbour on another GPU is staged (above). */
#define PFT_ERR_IPC_TIMEOUT (-5002)
int pft_slab_sync(pft_slab * s);
/* A communicator whose work the compute stream waits on (RCCL) bounds the slab's host waits the
   same way: while a watch is set, every host wait (pft_slab_sync, the error-norm fetch, up/download)
   polls, and calls fn(ctx, expired) about every millisecond, expired = 1 once timeout_s has passed
   since the wait began.  A nonzero return (the communicator saw an asynchronous error, or the
   expiry, and aborted: PFT_ERR_COMM_ABORTED) ends the wait with that code, and the slab refuses
   every later wait, exchange and error-norm fetch until it is destroyed.  fn = NULL removes it. */
#define PFT_ERR_COMM_ABORTED (-5003)
typedef int (*pft_slab_watch_fn)(void * ctx, int expired);
int pft_slab_set_watch(pft_slab * s, pft_slab_watch_fn fn, void * ctx, double timeout_s);

/* peer copy of one ghost plane between slabs on the same process (loopback transport) */
int pft_memcpy_d2d_async(void * dst, const void * src, size_t bytes, void * stream);
int pft_event_record_wait(void * from_stream, void * to_stream);

#ifdef __cplusplus
}
#endif
#endif
