#!/usr/bin/env python3
"""Benchmark: Mcells x attempted RK-Merson steps per second on MI355X.

One "step" = one attempted Merson step of RK_MPI_SA_solve (the reference's steps_total):
5 RHS evaluations of the intertrack (u, p, gl) model + 4 stage combines + error norm + the
update, run by libpft's fused device path with the state resident in HBM.

Workload (N = number of GPUs, one process per GPU, Z-slab decomposition, weak scaling):
  default Params (apps/intertrack-hybrid-S-freezing/Params, calc_mode 0 GradP).  "G^3" means
  grid_nodes G, i.e. (G/2) x (G/2) x G cells of the fixed 0.03 x 0.03 x 0.06 m domain.
  N = 1: 400^3 = 200 x 200 x 400 = 16 M cells.
  --shape cube (default): G = 400 N^(1/3) rounded to a multiple of 4, so N = 8 is exactly the
      "800^3 grid, 8-way Z-slab split" configuration (400 x 400 x 800, 100 planes per GPU) and
      every GPU holds ~16 M cells (N = 2: 504^3, N = 4: 636^3).
  --shape tall: the 400^3 slab stacked N times (200 x 200 x 400N, L3 = 0.06 N m): per-GPU work
      identical to N = 1, only the halo exchange is added.
  Initial state: the default Params initial condition (u = 293.15 K, ice cap, glass walls and
  200 glass beads) built by libpft's host model code; t = 0, h = tau = 1 s.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line (contract in the task statement) with `roofline` (dominant stage
kernel, HIP-event timed) and `cpu_baseline` (the CPU oracle port on a bounded sample, N=1 only).
"""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PROBE_STEPS = 3    # attempted steps of the N > 1 setup's delivery check (bench.py main)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import porousfreezethaw_amd as P  # noqa: E402
from porousfreezethaw_amd import params as PR  # noqa: E402

HBM_PEAK_GBPS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6        # FP64 vector: half the guide's 157.3 TF FP32 vector peak (16 FP64 lanes per SIMD and cycle)
# algorithmic HBM bytes per cell of each fused stage kernel: doubles read
# once + written once, perfect stencil reuse.  faithful: u, p, gl all evolved by the solver;
# gl_static: dgl == 0 exploited (PFT_OPT_GL_STATIC)
STAGE_DOUBLES_AUX = {False: {1: 9, 2: 12, 3: 15, 4: 18, 5: 18}, True: {1: 7, 2: 9, 3: 11, 4: 13, 5: 13}}
# recompute path: stage s reads the arrays its input is built from, writes K_s (stage 5: x(t+h));
# gl's K's are the literal zeros of dgl (PFT_GLK_LITERAL, never stored or loaded), so a stage
# reads x of all 3 fields, the K's of u and p, and writes K_s of u and p (stage 5: all of x(t+h));
# stage 2 stores S = K1 + K2, so stage 3 reads x and S (PFT_K12_SUM); stage 5 stores gl's x(t+h)
# only when it is not x itself (pft_slab_get_gl_keep: 11 doubles then, as with gl_static)
STAGE_DOUBLES_RC = {False: {1: 5, 2: 7, 3: 7, 4: 9, 5: 12}, True: {1: 5, 2: 7, 3: 7, 4: 9, 5: 11}}
# pair kernels (one slab, PFT_OPT_PAIR, merson_pair), timed as stages 3 and 5: pair 2+3 reads x and
# K1 and writes K3 (K2 never stored), pair 4+5 reads x, K1, K3 and writes x(t+h) (K4 never stored);
# with the speculative stage 1: 21 doubles per cell-step
PAIR_DOUBLES = {False: {1: 5, 3: 7, 5: 10}, True: {1: 5, 3: 7, 5: 9}}
METRIC = "Mcells·RK-steps/s at 400³ grid, 1/2/4/8 MI355X; % HBM roofline"
PUBLISHED_400_MODE1 = 351.88      # BASELINE.md 1, CC-HR-12nodes SigmaP1-P-smallsigma, 384 cores


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--prewarm-s", type=float, default=0.3,
                    help="before the W counted warm-up steps, run untimed attempted steps for about this "
                         "long so the GPU clock has left its idle level (0: off; DESIGN 5)")
    ap.add_argument("--grid-nodes", type=int, default=400, help="grid_nodes G of the 1-GPU case")
    ap.add_argument("--shape", choices=("cube", "tall", "strong"), default="cube",
                    help="N>1 workload family (module docstring): cube/tall weak scaling; strong = the "
                         "--grid-nodes grid itself split N ways (BASELINE configs[3]: 400^3 4-way)")
    ap.add_argument("--no-strong", action="store_true",
                    help="N>1: skip the strong-split sub-run (config.strong)")
    ap.add_argument("--literal-cube", action="store_true",
                    help="L1 = L2 = L3 = 0.06 m: G x G x G cells (SURVEY 8(d) secondary number)")
    ap.add_argument("--domain", default=None,
                    help="L1,L2,L3 in m (diagnostics): n_d = L_d * grid_nodes / max L, e.g. 0.06,0.06,0.015 "
                         "with --grid-nodes 400 is one rank's 400x400x100 slab of the 800^3 8-way case")
    ap.add_argument("--mode", type=int, default=0, help="calc_mode (0 GradP, 1 SigmaP1-P, 2 Temp)")
    ap.add_argument("--gl-static", action="store_true", help="exploit dgl == 0 (bit-identical)")
    ap.add_argument("--kz", type=int, default=0, help="planes per workgroup z-march (default 0 = automatic)")
    ap.add_argument("--tile", type=int, default=1,
                    help="1: per stage (default), 32 / 16: LDS-tiled kernel, 0: cache-based")
    ap.add_argument("--no-recompute", action="store_true",
                    help="materialise the reference's aux arrays between stages (72 vs 54 doubles/cell-step)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--host-ic", action="store_true",
                    help="initial condition on the host (default: on the device, bit-identical, f1)")
    ap.add_argument("--gate", type=int, default=0, choices=(0, 1),
                    help="gated steps on small single slabs (PFT_OPT_GATE, f4; default off: measured neutral)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="CPU sample: attempted steps (in batches of 2) until this much time has passed")
    ap.add_argument("--no-timing", action="store_true", help="no HIP-event stage timing")
    ap.add_argument("--host-boundary", action="store_true",
                    help="timed call is one RK_MPI_SA_solve-style call: x copied host->device at entry "
                         "and back at exit (PCIe-inclusive rate; never the headline value)")
    ap.add_argument("--transport", choices=("auto", "ipc", "ipc-ce", "rccl"), default="auto",
                    help="N>1 (and --self-exchange) inter-slab transport (pft_comm.h): ipc = IPC-mapped "
                         "neighbour slabs, boundary planes stored into their ghost planes + flag words; "
                         "ipc-ce = the same planes and flags as copy-engine (SDMA) copies beside the interior "
                         "launch; rccl = ncclSend/ncclRecv on a priority stream beside the interior sweep; "
                         "auto (default) = ipc-ce with one GPU per rank, ipc when ranks share a GPU and for "
                         "--self-exchange (DESIGN section 6)")
    ap.add_argument("--self-exchange", action="store_true",
                    help="diagnostic, 1 GPU: run the N>1 path of --transport (ipc: put kernel + flag waits "
                         "per stage; rccl: boundary planes first, halo exchange beside the interior sweep, "
                         "RCCL eps max) with a 1-rank communicator exchanging with itself; never the headline")
    ap.add_argument("--callback", action="store_true",
                    help="install a Service_Callback that reads t and h after every accepted step, as the "
                         "reference driver's RKService does with its default Params (intertrack.c:1072-1116)")
    ap.add_argument("--timing-steps", type=int, default=30,
                    help="attempted steps of the separate, untimed pass that measures the stage kernels with "
                         "HIP events (roofline); 0 = none")
    ap.add_argument("--no-parity", action="store_true",
                    help="N > 1: skip the decomposition-invariance check (rank 0 re-runs the same attempted "
                         "steps on one slab of its own GPU and compares every rank's state bit for bit)")
    ap.add_argument("--probe", type=int, default=0,
                    help="after the run, launch the 8-B/lane copy probe this many times "
                         "(rocprofv3 FETCH_SIZE/WRITE_SIZE calibration, known bytes)")
    return ap.parse_args()


def main():
    a = parse()
    worker = os.environ.get("PFT_BENCH_WORKER") == "1"
    if not worker and (a.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1") or 1) > 1):
        # N > 1: this process only launches and watches the ranks (supervise); it never loads libpft
        sys.exit(supervise(a))
    if worker and os.environ.get("PFT_BENCH_DRYRUN") == "1":
        sys.exit(dryrun_worker(a))
    # stdout carries exactly one JSON line: anything else written to fd 1 (RCCL's version banner
    # at communicator init, library diagnostics) goes to stderr
    json_fd = os.dup(1)
    os.dup2(2, 1)
    rc_path = (not a.no_recompute) and a.tile != 0
    STAGE_DOUBLES = STAGE_DOUBLES_RC if rc_path else STAGE_DOUBLES_AUX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            sys.exit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
        a.gpus = world
    L = P.lib()
    ndev = P.device_count()
    if ndev < 1:
        sys.exit("no HIP device visible (the benchmark has no CPU fallback)")
    dev = local % ndev           # one process per GPU; more ranks than GPUs share round-robin
    transport_auto = a.transport == "auto"
    if a.transport == "auto":
        # one GPU per rank: the exchange on the copy engines beside the interior launch (the planes
        # cross xGMI without CUs; RCCL's kernel waits for the launch that holds every CU, and the
        # put kernel would run after it); ranks sharing a GPU, and the self exchange: the put kernel
        # (a local copy, the cheapest there).  DESIGN.md section 6.
        a.transport = "ipc" if (world > ndev or a.self_exchange) else "ipc-ce"
    dist = None
    comm = None
    if world > 1:
        # a neighbour that never delivers ends the run within a minute (every wait polls; the
        # library's default bound is 300 s), so that a failed first exchange falls back to RCCL and
        # a failure in the timed region exits non-zero before the driver's own limit
        os.environ.setdefault("PFT_IPC_TIMEOUT", "60")
        os.environ.setdefault("PFT_COMM_TIMEOUT", "60")
        # torch.distributed (gloo, host only) is the rendezvous and the barrier; the data path is
        # libpft's communicator (pft_comm.h).  torch never touches the GPU here.
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm, a.transport = make_comm(L, a.transport, world, rank, dev, dist)
    else:
        L.pft_hip_set_device(dev)
        if a.self_exchange:
            comm, a.transport = make_comm(L, a.transport, 1, 0, dev, None)
            assert L.pft_comm_set_self_exchange(comm, 1) == 0
    L.pft_solver_set_option(P.PFT_OPT_DEVICE, dev)
    L.pft_solver_set_option(P.PFT_OPT_GATE, a.gate)

    def barrier():
        if dist is not None:
            dist.barrier()
        L.pft_hip_device_sync()

    # ---- workload -------------------------------------------------------------------------
    gn, base, (n1, n2, total_n3), Ls = workload(a.grid_nodes, world, a.shape, a.literal_cube, a.mode, a.domain)
    prm = P.params_array(base)
    beads = np.load(os.path.join(REPO, "tests", "golden", "beads.npy"))
    t0 = time.time()

    def make_sim():
        return P.Simulation(n1, n2, total_n3, Ls, a.mode, prm, nprocs=world, rank=rank, beads=beads,
                            tau=base["tau"], tau_min=base["tau_min"], delta=base["delta"],
                            gl_static=a.gl_static, kz=a.kz or None, tile=a.tile,
                            recompute=not a.no_recompute, device_ic=not a.host_ic)

    probe_calls = []   # solve calls made by the setup's check (world > 1), replayed by the parity re-run
    if world > 1:
        # The first exchanges (the device IC's ghost planes) run inside the setup.  If the ipc transport
        # the run chose by itself fails there on any rank (mapping a neighbour's buffers across GPUs,
        # say: the attach agrees its outcome across ranks, so all fail together), every rank falls
        # back to RCCL rather than ending without a measurement; the JSON line names the transport.
        sim, fail = None, 0
        try:
            sim = make_sim()
            # the setup's exchange delivered the neighbours' boundary planes bit for bit (a transport
            # that maps but does not deliver -- across GPUs, say -- is caught here, not at the parity
            # check after the timed region)
            if not a.host_ic and not halo_delivered(L, sim, dist, world, rank):
                raise RuntimeError("the ghost planes after the setup exchange differ from the neighbours' planes")
            if not a.host_ic and a.transport in ("ipc", "ipc-ce"):
                # the same after a few attempted steps: the split launches' exchanges (copy engines,
                # boundary stream) -- the first solve call, replayed by the parity re-run like the rest
                rc = sim.solve_ex(base["final_time"], PROBE_STEPS, P.PFT_SOLVE_KEEP_DEVICE)
                probe_calls.append(PROBE_STEPS)
                delivered = halo_delivered(L, sim, dist, world, rank)   # collective: every rank calls it
                if rc != 2 or not delivered:
                    raise RuntimeError(f"after {PROBE_STEPS} attempted steps (rc {rc}) the ghost planes differ "
                                       f"from the neighbours' planes")
        except Exception as e:  # noqa: BLE001
            print(f"rank {rank}: setup over {a.transport} failed: {e}", file=sys.stderr)
            fail = 1
        import torch
        ft = torch.tensor([fail], dtype=torch.int64)
        dist.all_reduce(ft, op=dist.ReduceOp.MAX)
        if int(ft.item()):
            if not (transport_auto and a.transport in ("ipc", "ipc-ce")):
                sys.exit(f"rank {rank}: setup over {a.transport} failed on a rank")
            if sim is not None:
                sim.close()
            else:
                L.RK_MPI_SA_cleanup()
                L.FreePrecalcData()
            L.pft_comm_set_current(None)
            L.pft_comm_destroy(comm)
            print(f"rank {rank}: every rank falls back to RCCL", file=sys.stderr)
            comm, a.transport = make_comm(L, "rccl", world, rank, dev, dist, fallback=False)
            sim = make_sim()
            probe_calls = []
    else:
        sim = make_sim()
    init_s = time.time() - t0
    cells_rank = n1 * n2 * sim.grid.n3
    cells_total = n1 * n2 * total_n3
    final_time = base["final_time"]

    callbacks = []
    if a.callback:
        @P.SERVICE_FN
        def service(final, s):
            callbacks.append((s.contents.t, s.contents.h))   # RKService logs t and tau, then stat()s
            return 0

        sim.system.Service_Callback = C.cast(service, C.c_void_p).value

    # Clock pre-warm.  The GPU leaves its idle clock over the first ~50 ms of load: the same
    # launches take the same cycles but run at 2.1 rising to 2.4-2.5 GHz (GRBM_GUI_ACTIVE per
    # launch, profiles/r03b_clock_ramp_driver_config.txt), so a 20-step window right after start
    # measured 15 853-16 090 where the steady state is 17 592.  Untimed attempted steps of the same
    # solve run until --prewarm-s has passed (every rank takes the same decision: the max over
    # ranks); they are solve calls like the warm-up, replayed by the N > 1 parity re-run.
    calls = list(probe_calls)                  # the capped solve calls, in order (the parity re-run repeats them)
    prewarm_steps = 0
    tp = time.perf_counter()
    while a.prewarm_s > 0 and prewarm_steps < 5000:
        k = max(20, a.warmup)
        rc = sim.solve_ex(final_time, k, P.PFT_SOLVE_KEEP_DEVICE | (P.PFT_SOLVE_REUSE_DEVICE if calls else 0))
        assert rc == 2, rc
        calls.append(k)
        prewarm_steps += k
        L.pft_hip_device_sync()
        el_p = time.perf_counter() - tp
        if dist is not None:
            import torch
            tt = torch.tensor([el_p], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el_p = float(tt.item())
        if el_p >= a.prewarm_s:
            break
    prewarm_s = time.perf_counter() - tp
    # warm-up: uploads x once (when not pre-warmed), builds the kernels' caches; W attempted steps
    calls.append(max(1, a.warmup))
    rc = sim.solve_ex(final_time, calls[-1], P.PFT_SOLVE_KEEP_DEVICE | (P.PFT_SOLVE_REUSE_DEVICE if len(calls) > 1 else 0))
    assert rc == 2, rc
    st0 = sim.system.steps_total
    barrier()
    t1 = time.perf_counter()
    timed_flags = 0 if a.host_boundary else P.PFT_SOLVE_KEEP_DEVICE | P.PFT_SOLVE_REUSE_DEVICE
    rc = sim.solve_ex(final_time, a.steps, timed_flags)
    barrier()
    t2 = time.perf_counter()
    _st = sim.stats()
    gated_steps, gate_misses = int(_st.gated_steps), int(_st.gate_misses)
    assert rc == 2, rc
    calls.append(a.steps)
    steps = sim.system.steps_total - st0
    assert steps == a.steps, (steps, a.steps)
    el = t2 - t1
    if dist is not None:
        import torch
        tt = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    accepted = int(sim.system.steps)
    t_end = sim.t
    # stage kernels timed in a separate pass after the timed region (HIP events on the slab's
    # compute stream, every other attempted step: each timed stage adds an event pair)
    if not a.no_timing and a.timing_steps > 0:
        L.pft_solver_set_option(P.PFT_OPT_TIMING, 2)
        rc = sim.solve_ex(final_time, a.timing_steps, P.PFT_SOLVE_KEEP_DEVICE | P.PFT_SOLVE_REUSE_DEVICE)
        assert rc == 2, rc
        calls.append(a.timing_steps)
        L.pft_solver_set_option(P.PFT_OPT_TIMING, 0)
    stats = sim.stats()
    geo = sim.tile_geometry()
    L.pft_slab_get_gl_keep.argtypes = [C.c_void_p]
    L.pft_solver_slab.restype = C.c_void_p
    gl_keep = bool(rc_path and L.pft_slab_get_gl_keep(L.pft_solver_slab()))
    pairs = bool(stats.pairs)
    if pairs:
        STAGE_DOUBLES = PAIR_DOUBLES
    if gl_keep and not a.gl_static:
        STAGE_DOUBLES = {g: dict(v) for g, v in STAGE_DOUBLES.items()}
        STAGE_DOUBLES[False][5] = 9 if pairs else 11

    # ---- roofline: dominant fused stage kernel, HIP events on the slab's compute stream -----
    roof = None
    if not a.no_timing and stats.stage_n[1] > 0:
        per = {}
        nl = {s: 1 for s in range(1, 6)}
        for s in range(1, 6):
            if stats.stage_n[s] == 0:
                continue                                                 # a pair's first stage
            ms = stats.stage_ms[s] / max(1, stats.stage_n[s]) * nl[s]     # per step
            byts = STAGE_DOUBLES[a.gl_static][s] * 8 * cells_rank
            per[s] = (ms, byts)
        dom = max(per, key=lambda s: per[s][0])
        ms, byts = per[dom]
        achieved = byts / (ms * 1e-3) / 1e9
        traffic, traffic_src, valu_frac, f64 = None, None, None, {}
        pmc = os.path.join(REPO, "profiles", "pmc_summary.json")
        if os.path.exists(pmc):
            try:
                ps = json.load(open(pmc))
                gk = f"glx{int(a.gl_static or gl_keep)}" if pairs else f"gl{int(a.gl_static)}"
                key = f"{'pair' if pairs else 'stage'}{dom}_{gk}_{n1}x{n2}x{sim.grid.n3}_m{a.mode}"
                traffic = ps.get(key, {}).get("hbm_bytes_per_launch")
                valu_frac = ps.get(key, {}).get("valu_issue_frac")
                f64 = {q: ps.get(key, {}).get(q) for q in ("fp64_flop_per_launch", "fp64_pipe_busy_frac")}
                if traffic is not None:
                    # not measured in this run: the calibrated FETCH_SIZE + WRITE_SIZE of that
                    # kernel from the rocprofv3 --pmc passes recorded in the file
                    traffic_src = dict(ps.get("provenance", {}), file="profiles/pmc_summary.json", key=key)
            except (OSError, ValueError):
                traffic = None
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": kernel_name(dom, a, rc_path, n1, pairs, gl_keep),
                # the pair kernels are FP64-VALU-bound (stage A recomputed on a ring, no HBM bytes
                # spared to compute): the fraction of the SIMDs' issue cycles their VALU
                # instructions take, from the same PMC file (SQ_INSTS_VALU, GRBM_GUI_ACTIVE)
                "valu_issue_frac": round(valu_frac, 4) if valu_frac is not None else None,
                # the same kernel against the FP64 vector roof: its FP64 FLOP per launch (PMC, same
                # file: 64 lanes x (ADD + MUL + TRANS + 2 FMA) wave instructions) / this run's
                # launch time, and the FP64 pipe's busy fraction (4 cycles per wave64 instruction)
                "fp64": ({"achieved": round(f64["fp64_flop_per_launch"] / (ms / nl[dom] * 1e-3) / 1e12, 2),
                          "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(f64["fp64_flop_per_launch"] / (ms / nl[dom] * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4),
                          "pipe_busy_frac": round(f64["fp64_pipe_busy_frac"], 4)}
                         if f64.get("fp64_flop_per_launch") else None),
                "algorithmic_bytes_per_launch": byts // nl[dom],
                "avg_launch_ms": round(ms / nl[dom], 4),
                "stages_ms": {str(s): round(per[s][0], 4) for s in per},
                "stages_GBps": {str(s): round(per[s][1] / (per[s][0] * 1e-3) / 1e9, 1) for s in per}}

    value = cells_total * steps / el / 1e6
    # the reference publishes this metric at 400^3 only for the SigmaP1-P model
    # (calc_mode 1): 351.88 Mcells*steps/s on 384 CPU cores.  Quoted for that mode only.
    vs_base = (round(value / PUBLISHED_400_MODE1, 2)
               if (a.mode == 1 and gn == 400 and world == 1 and not a.literal_cube) else None)
    step_bytes = sum(STAGE_DOUBLES[a.gl_static].values()) * 8
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mcells·steps/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if (a.shape == "strong" and world > 1) else "weak",
        "vs_baseline": vs_base,
        "dtype": "f64",
        "data": "synthetic: default Params initial condition (u=293.15 K, ice cap, glass walls, "
                "200 glass beads from the reference's data file), t=0, h=tau=1",
        "config": {"workload": (f"{gn}^3 default Params" if a.shape in ("cube", "strong") or world == 1 else
                                f"{a.grid_nodes}^3 slab x {world} (tall)") +
                               f": {n1}x{n2}x{total_n3} cells, Z-slab split {world}-way "
                               f"({n1}x{n2}x{sim.grid.n3} on rank {rank})",
                   "grid_nodes": gn, "shape": a.shape, "literal_cube": a.literal_cube,
                   "calc_mode": a.mode, "cells": cells_total, "parallelism": f"zslab{world}",
                   "gl_static": a.gl_static, "kz": a.kz or "auto", "tile": a.tile, "recompute": not a.no_recompute,
                   "accepted_steps_total": accepted, "t_end": t_end,
                   "host_boundary": a.host_boundary, "self_exchange": a.self_exchange,
                   "transport": (a.transport if (world > 1 or a.self_exchange) else None),
                   "service_callback": a.callback,
                   "clock_prewarm": {"attempted_steps": prewarm_steps, "seconds": round(prewarm_s, 3)},
                   "gl_store_skipped": gl_keep, "pair_kernels": pairs,
                   "gated_steps": gated_steps, "gate_misses": gate_misses,
                   "tiles": ({str(k): ("cache" if v[0] == 0 else f"{2 * v[1]}x{v[2]} cells")
                              for k, v in geo.items()} if geo else None),
                   "pair_tile": pair_tile_text(L, n1, n2) if pairs else None},
        "roofline": roof,
        # whole step at its algorithmic bytes (21 doubles per cell-step with the pair kernels, 39
        # with one launch per stage), per GPU
        "step_algorithmic_GBps": round(step_bytes * cells_total * steps / el / 1e9 / world, 1),
        "init_s": round(init_s, 2),
        "initial_condition": "host" if a.host_ic else "device",
    }

    if a.probe:
        slab = L.pft_solver_slab()
        L.pft_slab_buffer.restype = C.c_void_p
        L.pft_slab_buffer.argtypes = [C.c_void_p, C.c_int]
        L.pft_slab_state_bytes.restype = C.c_size_t
        L.pft_slab_state_bytes.argtypes = [C.c_void_p]
        L.pft_probe_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        nd = L.pft_slab_state_bytes(slab) // 8
        src, dst = L.pft_slab_buffer(slab, 5), L.pft_slab_buffer(slab, 6)   # K3 -> K4 scratch
        for _ in range(a.probe):
            L.pft_probe_copy(dst, src, nd, L.pft_slab_stream(slab))
        L.pft_hip_device_sync()
        out["probe_bytes_each_way"] = nd * 8

    # ---- CPU baseline (rank 0, N = 1 only): the oracle port, bounded sample -----------------
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(sim, base, a)
    out["cpu_baseline"] = cpu
    mine = slab_digest(sim) if (world > 1 and not a.no_parity) else None
    sim.close()
    if comm is not None:
        L.pft_comm_set_current(None)
        L.pft_comm_destroy(comm)

    # ---- N > 1: decomposition invariance, checked on every run --------------------
    ok = True
    if mine is not None:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        if rank == 0:
            out["parity"] = parity_check(ranks, calls, a, base, (n1, n2, total_n3), Ls, beads, final_time, dev)
            ok = out["parity"]["equal"]
        dist.barrier()                        # the other ranks wait for rank 0's single-slab re-run
    else:
        out["parity"] = None
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()
    if not ok:
        print(f"parity: the {world}-slab run differs from the single-slab run of the same steps", file=sys.stderr)
        sys.exit(PARITY_EXIT)


# ---- N > 1: the ranks as child processes of a supervisor ------------------------------------
# `bench.py --gpus N` started as ONE process (no RANK / WORLD_SIZE) spawns the N ranks itself;
# started by torch.distributed.run, each of its N processes supervises one rank.  Either way the
# ranks are fresh child processes (PFT_BENCH_WORKER=1) with their own rendezvous port, and the
# supervisors never load libpft or touch a GPU.  That buys two things:
#   - the run cannot fail for launch reasons: a plain `python bench.py --gpus 4` measures;
#   - a failed attempt is retried in FRESH processes: when the transport is auto (ipc-ce across
#     GPUs, ipc when ranks share one) or ipc-ce and any rank fails -- an exchange that never
#     arrives (the bounded waits end it), a device error, a parity mismatch -- every rank is
#     started again over RCCL.  The JSON line records every attempt ("launch").
# With N > 1 a second set of ranks then times the reference's 400^3 grid split N ways (BASELINE
# configs[3] at N = 4: 200 x 200 x 100 per rank) with its own parity re-run: config.strong.
PARITY_EXIT = 3


def _child_env(rank, local, world, port, transport):
    # (not torch.distributed.run's agent store: the ranks rendezvous on their own port)
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(PFT_BENCH_WORKER="1", RANK=str(rank), LOCAL_RANK=str(local), WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("LOCAL_WORLD_SIZE", str(world))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PFT_BENCH_ATTEMPT_TRANSPORT"] = transport
    return env


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_children(specs, timeout_s, grace_s=30.0):
    """start the child ranks (argv, env, capture_stdout) and wait for all of them; once one has
    failed, the others get grace_s to end by themselves (a failed rank closes its gloo sockets, which
    ends its peers' collectives) before they are killed, as is every child still running after
    timeout_s.  Returns (exit codes, captured stdout of the capturing child)."""
    import subprocess
    procs = []
    for argv, env, cap in specs:
        procs.append(subprocess.Popen(argv, env=env, stdout=subprocess.PIPE if cap else sys.stderr,
                                      stderr=None, start_new_session=True))
    out = {}
    import threading

    def drain(i, p):
        out[i] = p.stdout.read()

    readers = [threading.Thread(target=drain, args=(i, p), daemon=True) for i, p in enumerate(procs) if p.stdout]
    for t in readers:
        t.start()
    t0 = time.time()
    failed_at = None
    while True:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            break
        if failed_at is None and any(c not in (None, 0) for c in codes):
            failed_at = time.time()
        now = time.time()
        if now - t0 > timeout_s or (failed_at is not None and now - failed_at > grace_s):
            for p in procs:
                if p.poll() is None:
                    print(f"bench supervisor: killing rank process {p.pid} "
                          f"({'time limit' if now - t0 > timeout_s else 'a peer failed'})", file=sys.stderr)
                    try:
                        os.killpg(p.pid, 9)
                    except OSError:
                        pass
            for p in procs:
                p.wait()
            break
        time.sleep(0.2)
    for t in readers:
        t.join(timeout=10)
    codes = [p.returncode for p in procs]
    cap = next((out.get(i, b"") for i, (argv, env, c) in enumerate(specs) if c), b"")
    return codes, cap.decode(errors="replace")


def _last_json(text):
    for line in reversed(text.strip().splitlines()):
        try:
            return json.loads(line)
        except ValueError:
            continue
    return None


def supervise(a):
    """the N > 1 launcher (comment block above): returns the process exit code"""
    world_env = int(os.environ.get("WORLD_SIZE", "1") or 1)
    launched = world_env > 1                  # torch.distributed.run: one supervisor per rank
    world = world_env if launched else a.gpus
    rank = int(os.environ.get("RANK", "0")) if launched else 0
    local = int(os.environ.get("LOCAL_RANK", str(rank))) if launched else 0
    # stdout carries the one JSON line and nothing else: everything else written to fd 1 from here
    # on (the gloo library's connection notes under torch.distributed.run) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    dist = None
    if launched:
        import torch.distributed as dist      # gloo: host only, the supervisors' own rendezvous
        dist.init_process_group("gloo", rank=rank, world_size=world)
    script = [sys.executable, "-u", os.path.abspath(__file__)]
    argv0 = [x for x in sys.argv[1:]]
    timeout_s = float(os.environ.get("PFT_BENCH_CHILD_TIMEOUT", "1200"))

    def attempt(extra):
        """one set of N child ranks with these extra arguments: (every rank ok, rank 0's JSON, codes)"""
        port = [_free_port() if rank == 0 else 0]
        if dist is not None:
            dist.broadcast_object_list(port, src=0)
        tr = extra[extra.index("--transport") + 1] if "--transport" in extra else a.transport
        if launched:
            specs = [(script + argv0 + extra, _child_env(rank, local, world, port[0], tr), rank == 0)]
        else:
            specs = [(script + argv0 + extra, _child_env(r, r, world, port[0], tr), r == 0) for r in range(world)]
        codes, text = _run_children(specs, timeout_s)
        if dist is not None:
            allc = [None] * world
            dist.all_gather_object(allc, codes[0])
            codes = allc
        line = _last_json(text) if rank == 0 else None
        ok = all(c == 0 for c in codes) and (rank != 0 or line is not None)
        if dist is not None:
            import torch
            t = torch.tensor([0 if ok else 1], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ok = not int(t.item())
        print(f"bench supervisor (rank {rank}): {' '.join(extra) or 'as given'}: rank exit codes {codes}", file=sys.stderr)
        return ok, line, codes

    plans = [a.transport] + (["rccl"] if a.transport in ("auto", "ipc-ce") else [])
    attempts, out, success = [], None, False
    for tr in plans:
        ok, line, codes = attempt(["--transport", tr])
        attempts.append({"transport": tr, "exit_codes": codes, "ok": ok})
        if ok:
            out, success = line, True        # (every rank agrees on ok; only rank 0 has the line)
            break
        if tr != plans[-1]:
            print(f"bench supervisor (rank {rank}): the run over '{tr}' failed on a rank; every rank starts again "
                  f"over RCCL in fresh processes", file=sys.stderr)
    strong = None
    if success and world > 1 and not a.no_strong and a.shape != "strong" and not a.self_exchange:
        # BASELINE configs[3] (at N = 4): the 400^3 grid split N ways, over the transport the main run used
        tr = (out or {}).get("config", {}).get("transport") or "auto" if rank == 0 else "auto"
        trl = [tr]
        if dist is not None:
            dist.broadcast_object_list(trl, src=0)
        sok, sline, scodes = attempt(["--transport", trl[0], "--shape", "strong", "--no-cpu"])
        if rank == 0:
            if sok and sline:
                c = sline.get("config", {})
                strong = {"workload": c.get("workload"), "scaling": "strong", "value": sline.get("value"),
                          "unit": sline.get("unit"), "ms_per_step": sline.get("ms_per_step"),
                          "steps": sline.get("steps"), "cells": c.get("cells"), "transport": c.get("transport"),
                          "parity": sline.get("parity"), "roofline": sline.get("roofline")}
            else:
                strong = {"error": f"the strong-split run failed (rank exit codes {scodes})"}
    if dist is not None:
        dist.destroy_process_group()
    if rank != 0:
        return 0 if success else 1
    if out is None:
        print(f"bench supervisor: no attempt succeeded: {attempts}", file=sys.stderr)
        return 1
    out["launch"] = {"mode": "torchrun (one supervisor per rank, one child rank each)" if launched
                     else "self-spawn (one supervisor, N child ranks)", "attempts": attempts}
    if strong is not None:
        out.setdefault("config", {})["strong"] = strong
    json_out.write(json.dumps(out) + "\n")
    json_out.flush()
    return 0


def dryrun_worker(a):
    """test hook (PFT_BENCH_DRYRUN=1, tests/test_bench_launch.py): a child rank that does the
    rendezvous and a barrier and prints a stand-in line, without a GPU.  PFT_BENCH_DRYRUN_FAIL =
    "<rank>:<transport>" makes that rank exit non-zero when its attempt uses that transport."""
    import torch.distributed as dist
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    tr = os.environ.get("PFT_BENCH_ATTEMPT_TRANSPORT", a.transport)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fail = os.environ.get("PFT_BENCH_DRYRUN_FAIL", "")
    if fail and fail.split(":")[0] == str(rank) and fail.split(":")[1] == tr:
        print(f"dryrun rank {rank}: failing on purpose over {tr}", file=sys.stderr)
        os._exit(5)
    names = [None] * world
    dist.all_gather_object(names, {"rank": rank, "pid": os.getpid(), "local": int(os.environ.get("LOCAL_RANK", "-1"))})
    dist.barrier()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "dryrun": True, "n_gpus": world,
                          "config": {"transport": tr, "shape": a.shape, "ranks": names}}))
    dist.destroy_process_group()
    return 0


def halo_delivered(L, sim, dist, world, rank):
    """after the setup (the IC and its one-plane exchange of X), every rank's ghost planes hold its
    z-neighbours' boundary planes bit for bit (u, p, gl of X).  Collective over gloo; every rank gets
    the same answer."""
    import torch
    L.pft_solver_slab.restype = C.c_void_p
    L.pft_slab_buffer.restype = C.c_void_p
    L.pft_slab_buffer.argtypes = [C.c_void_p, C.c_int]
    L.pft_slab_plane.restype = C.c_size_t
    L.pft_slab_plane.argtypes = [C.c_void_p]
    L.pft_slab_field_stride.restype = C.c_size_t
    L.pft_slab_field_stride.argtypes = [C.c_void_p]
    L.pft_slab_nz.argtypes = [C.c_void_p]
    L.pft_flat_d2h.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    L.pft_stream_sync.argtypes = [C.c_void_p]
    slab = L.pft_solver_slab()
    ok = 1
    planes = {}
    try:
        L.pft_hip_device_sync()
        base, P_, fs, n3 = L.pft_slab_buffer(slab, 0), L.pft_slab_plane(slab), L.pft_slab_field_stride(slab), L.pft_slab_nz(slab)
        for name, k in (("g0", 0), ("b1", 1), ("bn", n3), ("gn", n3 + 1)):
            a = np.empty((3, P_))
            for q in range(3):
                if L.pft_flat_d2h(a[q].ctypes.data, base + 8 * (q * fs + k * P_), P_, None):
                    ok = 0
            planes[name] = a
        L.pft_stream_sync(None)
    except Exception:  # noqa: BLE001
        ok = 0
    rec = {"ok": ok, "sha": {k: hashlib.sha256(v.tobytes()).hexdigest() for k, v in planes.items()}}
    allrec = [None] * world
    dist.all_gather_object(allrec, rec)
    good = all(r["ok"] for r in allrec)
    for r in range(world):
        if r > 0 and good:
            good = allrec[r]["sha"]["g0"] == allrec[r - 1]["sha"]["bn"]
        if r < world - 1 and good:
            good = allrec[r]["sha"]["gn"] == allrec[r + 1]["sha"]["b1"]
    return good


def slab_digest(sim):
    """this rank's trajectory position and the SHA-256 of its interior (u, p, gl planes of the slab)"""
    sim.download()
    g = sim.grid
    x = sim.interior()
    if os.environ.get("PFT_BENCH_PARITY_PERTURB") == str(g.rank):
        # diagnostic: one value of this rank's state off by one ulp, so that the check must fail
        x.reshape(-1)[x.size // 2] = np.nextafter(x.reshape(-1)[x.size // 2], np.inf)
    return slab_record(x, sim.t, sim.h, sim.system.steps, sim.system.steps_total, g.first_row, g.n3)


def slab_record(x, t, h, steps, steps_total, first_row, n3):
    """what a rank hands to rank 0 for the parity check: (t, h, steps, steps_total) exactly, its
    Z-slab's place, and the SHA-256 of its interior state x[field][k][j][i]"""
    return {"t": float(t).hex(), "h": float(h).hex(), "steps": int(steps), "steps_total": int(steps_total),
            "first_row": int(first_row), "n3": int(n3),
            "sha256": hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()}


def compare_records(ranks, x, t, h, steps, steps_total):
    """every rank's record against the single-slab state x (all planes) and trajectory position:
    the list of mismatching ranks and fields (empty: the decomposition changed no bit)"""
    bad = []
    for r, m in enumerate(ranks):
        f, n = m["first_row"], m["n3"]
        want = slab_record(x[:, f:f + n], t, h, steps, steps_total, f, n)
        diff = [k for k in want if want[k] != m[k]]
        if diff:
            bad.append({"rank": r, "fields": diff})
    return bad


def parity_check(ranks, calls, a, base, dims, Ls, beads, final_time, dev):
    """Rank 0 re-runs the N-slab benchmark's exact solve calls (the same attempted-step caps, from the
    same initial condition) on ONE slab on its own GPU, and compares every rank's (t, h, steps,
    steps_total) and the SHA-256 of its planes with the single slab's.  The reference's results do
    not depend on the decomposition (bitwise across rank counts), so any difference --
    a wrong halo pairing, a stale ghost plane -- fails the run."""
    L = P.lib()
    t0 = time.time()
    n1, n2, total_n3 = dims
    L.pft_comm_set_current(None)
    L.pft_hip_set_device(dev)
    ref = P.Simulation(n1, n2, total_n3, Ls, a.mode, P.params_array(base), nprocs=1, rank=0, beads=beads,
                       tau=base["tau"], tau_min=base["tau_min"], delta=base["delta"], gl_static=a.gl_static,
                       kz=a.kz or None, tile=a.tile, recompute=not a.no_recompute, device_ic=not a.host_ic)
    for i, k in enumerate(calls):
        flags = P.PFT_SOLVE_KEEP_DEVICE | (P.PFT_SOLVE_REUSE_DEVICE if i else 0)
        rc = ref.solve_ex(final_time, k, flags)
        assert rc == 2, rc
    ref.download()
    x = ref.interior()
    pairs = bool(ref.stats().pairs)
    bad = compare_records(ranks, x, ref.t, ref.h, ref.system.steps, ref.system.steps_total)
    ref.close()
    return {"equal": not bad, "attempted_steps": int(sum(calls)), "calls": calls, "ranks": len(ranks),
            "reference": "one slab on rank 0's GPU, same initial condition and solve calls"
                         + (" (pair kernels)" if pairs else ""),
            "mismatches": bad, "seconds": round(time.time() - t0, 1)}


def make_comm(L, transport, world, rank, dev, dist, fallback=True):
    """libpft communicator of this rank (pft_comm.h), bound to this thread, and the transport it
    uses.  The rendezvous data (ipc: a shared-memory name, rccl: the unique id) goes through
    torch.distributed's gloo store.  If the RCCL communicator fails to initialise on any rank
    (every rank learns it through gloo), all ranks fall back to the ipc transport -- across GPUs its
    staged receive -- so that an N > 1 run still measures, and checks its parity, rather than
    ending; the JSON line then names the transport that ran."""
    comm = C.c_void_p()
    if transport in ("ipc", "ipc-ce"):
        name = [f"/pft_bench_{os.getpid()}_{int(time.time() * 1e6) % 10**9}"]
        if dist is not None:
            dist.broadcast_object_list(name, src=0)
        rc = L.pft_comm_init_ipc(C.byref(comm), world, rank, name[0].encode(), dev)
        if rc == 0 and transport == "ipc-ce":
            # the halo planes on the copy engines beside the interior launch (pft_comm_set_copy_engine)
            assert L.pft_comm_set_copy_engine(comm, 1) == 0
    else:
        uid = (C.c_char * 128)()
        if rank == 0:
            assert L.pft_comm_get_unique_id(uid) == 0
        if dist is not None:
            obj = [bytes(uid)]
            dist.broadcast_object_list(obj, src=0)
            uid = (C.c_char * 128).from_buffer_copy(obj[0])
            if fallback:
                # ncclCommInitRank is collective: a rank that would fail before entering it (its
                # device cannot be set) would leave the others inside it for good, so every rank's
                # local precheck is agreed first, and a failure anywhere goes to ipc before RCCL
                import torch
                pre = torch.tensor([0 if L.pft_hip_set_device(dev) == 0 else 1], dtype=torch.int64)
                dist.all_reduce(pre, op=dist.ReduceOp.MAX)
                if int(pre.item()):
                    print(f"rank {rank}: a rank cannot set its device for RCCL; every rank falls back to the "
                          f"ipc transport", file=sys.stderr)
                    return make_comm(L, "ipc", world, rank, dev, dist, fallback=False)
        rc = L.pft_comm_init_rccl(C.byref(comm), world, rank, uid, dev)
        if dist is not None and fallback:
            import torch
            bad = torch.tensor([1 if rc else 0], dtype=torch.int64)
            dist.all_reduce(bad, op=dist.ReduceOp.MAX)
            if int(bad.item()):
                if rc == 0:
                    L.pft_comm_destroy(comm)
                print(f"rank {rank}: the RCCL communicator failed to initialise on a rank ({rc} here); "
                      f"every rank falls back to the ipc transport", file=sys.stderr)
                return make_comm(L, "ipc", world, rank, dev, dist, fallback=False)
    if rc:
        sys.exit(f"rank {rank}: pft_comm_init_{transport} failed ({rc})")
    L.pft_comm_set_current(comm)
    return comm, transport


def workload(grid_nodes, world, shape="cube", literal_cube=False, mode=0, domain=None):
    """(G, Params dict, (n1, n2, total_n3), (L1, L2, L3)) of the N = world benchmark case"""
    Lc = (PR.float_val("0.06"),) * 3 if literal_cube else None
    if domain:
        Lc = tuple(PR.float_val(v) for v in domain.split(","))
    if shape == "strong":
        # the grid itself, its n3 planes split over the ranks (intertrack.c:1776-1800)
        base = PR.default_params(grid_nodes=grid_nodes, calc_mode=mode, L=Lc)
        return grid_nodes, base, (base["n1"], base["n2"], base["n3"]), (base["L1"], base["L2"], base["L3"])
    if shape == "cube" and world > 1:
        gn = int(round(grid_nodes * world ** (1.0 / 3.0) / 4.0)) * 4
        base = PR.default_params(grid_nodes=gn, calc_mode=mode, L=Lc)
        return gn, base, (base["n1"], base["n2"], base["n3"]), (base["L1"], base["L2"], base["L3"])
    base = PR.default_params(grid_nodes=grid_nodes, calc_mode=mode, L=Lc)
    return (grid_nodes, base, (base["n1"], base["n2"], base["n3"] * world),
            (base["L1"], base["L2"], base["L3"] * world))


def pair_tile_text(L, n1, n2):
    """the pair kernels' tile on this slab (pft_slab_pair_geometry) and the tiles per plane"""
    tx, ty = C.c_int(), C.c_int()
    L.pft_solver_slab.restype = C.c_void_p
    L.pft_slab_pair_geometry.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    if L.pft_slab_pair_geometry(L.pft_solver_slab(), C.byref(tx), C.byref(ty)):
        return None
    nt = ((n1 + tx.value - 1) // tx.value) * ((n2 + ty.value - 1) // ty.value)
    return f"{tx.value}x{ty.value} cells, {nt} tiles per plane"


def kernel_name(stage, a, rc_path, n1, pairs=False, glx=False):
    """the stage kernel libpft launches for these options (pft_kernels.hip launch_stage, run_pair);
    a pair kernel's third parameter is GLX (gl's inputs read from x: gl_static, or gl_keep)"""
    gls = "true" if a.gl_static else "false"
    if pairs and stage in (3, 5):
        return f"merson_pair<{stage - 1}, {a.mode}, {'true' if (a.gl_static or glx) else 'false'}>"
    if a.tile == 0 or n1 % 2 or not rc_path:
        return f"merson_stage<{stage}, {a.mode}, {gls}>"
    return f"merson_fused<{stage}, {a.mode}, {gls}>"


def cpu_baseline(sim, base, a):
    """Time the CPU restatement of the reference (oracle/pft_oracle.c: plain C, OpenMP over
    z-planes, the reference's arithmetic) on the same 400^3 state for a few attempted steps."""
    try:
        import _oracle as O
    except Exception as e:  # noqa: BLE001
        return {"error": f"oracle unavailable: {e}"}
    if not os.path.exists(O.LIB_PATH):
        return {"error": "oracle not built"}
    g = sim.grid
    info = {"n1": g.n1, "n2": g.n2, "n3": g.total_n3, "L1": g.L1, "L2": g.L2, "L3": g.L3}
    sim.download()
    x0 = sim.interior()
    prm = P.params_array(base)
    og = O.make_grid(info)
    xp = O.pad(og, x0)
    t, h = C.c_double(sim.t), C.c_double(sim.h)
    s, stt = C.c_long(0), C.c_long(0)

    def run(nsteps):
        # the cap counts this call's attempted steps; (t, h) carry the trajectory on
        t0 = time.perf_counter()
        O.lib().pft_or_solve(C.byref(og), O.ptr(prm), a.mode, base["final_time"], C.byref(t), C.byref(h),
                             base["tau_min"], base["delta"], 0, O.ptr(xp), C.byref(s), C.byref(stt),
                             nsteps, O.EXCHANGE_FN(), O.ALLREDUCE_FN(), None)
        return time.perf_counter() - t0

    run(1)                                           # first touch of the oracle's arrays (not counted)
    per_step = run(3) / 3.0                          # sizes the sample (not counted)
    n = max(2, int(a.cpu_seconds / per_step))
    stt.value = 0
    el = run(n)
    cores = int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1)))
    cells = g.n1 * g.n2 * g.total_n3
    value = cells * stt.value / el / 1e6
    out = {"value": round(value, 3), "unit": "Mcells·steps/s", "cores": cores, "kind": "port",
           "sample": f"{stt.value} attempted steps of the same {g.n1}x{g.n2}x{g.total_n3} state (after 3 untimed), "
                     f"oracle/pft_oracle.c (gcc -O2, OpenMP {cores} threads), {el:.1f} s"}
    # the port's speed relative to the reference itself, measured on the same cores and state in the
    # build container (scripts/calibrate_cpu.py: the reference compiled in place, P MPI ranks x 1
    # thread, vs the port on P threads, same attempted steps, bitwise-equal result)
    cal = os.path.join(REPO, "profiles", "r02_cpu_calibration.json")
    if os.path.exists(cal):
        c = json.load(open(cal))
        out["reference_equivalent"] = {
            "value": round(value * c["reference_over_port"], 3), "factor": c["reference_over_port"],
            "calibration": f"profiles/r02_cpu_calibration.json: reference {c['reference']['Mcells_steps_per_s']} vs "
                           f"port {c['port']['Mcells_steps_per_s']} Mcells*steps/s on {c['cores']} cores, {c['grid']}"}
    return out


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException:   # noqa: BLE001
        # a failed solve (a lost peer: the solver's bounded waits return PFT_SOLVE_DEVICE_ERROR)
        # ends this rank at once with a non-zero status; its closed gloo sockets end the others'
        # collectives instead of leaving them to time out
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        os._exit(1)
