#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REFERENCE ITSELF.

Test infrastructure only.  Runs oracle/_ref/pft_ref (the reference's equation.c/model.c,
RK_MPI_SAsolver_hybrid2.c and Params front end compiled in place by oracle/Makefile, see
oracle/ref_harness.c) on modified copies of the reference's default Params
(apps/intertrack-hybrid-S-freezing/Params) and stores inputs + outputs as compressed npz
fixtures.  Needs /root/reference and MPICH; the fixtures themselves travel, the reference
does not.  Re-run with:  make -C oracle ref && python tests/golden/gen_golden.py

Cases (SURVEY.md section 4.2 KATs 1-4):
  g20      default Params at grid_nodes 20 (10x10x20): parameters, IC (formula + glass
           beads), RHS at t=0 and after phase_switch_time for calc_mode 0/1/2/10/11,
           trajectory to several snapshot times (mode 0 and 1; mode 2 with p IC = 0);
           trajectory also run on 3 ranks and checked byte-identical (F6).
  ragged   L1=0.036, L2=0.024, grid_nodes 30 -> 18x12x30, random state (seed 20251015),
           RHS for all modes on 1 and 4 ranks (ranks hold 8/8/7/7 planes), plus every
           rank's padded input array after bcond_setup+sync_solution (boundary KAT),
           and single-step solves (accepted and rejected-first).
  ctl      control-flow KATs on g20: NaN give-up (3 variants), NaN retries then recovery, and
           a Service_Callback break + resume, with the (steps, t, h) the callback saw per step
  g100     BASELINE configs[0]: default Params at grid_nodes 100 (50x50x100): parameters, the
           SHA-256 of the IC and of a mode-0 trajectory to two snapshot times (checked identical
           on 2 ranks), plus the middle and top z-planes of each state (a state is 6 MB).
  g20nf    the g20 trajectory record for calc_mode 10 and 11 (to t = 36, 360, 720 s), checked
           identical on 3 ranks.
  g200     BASELINE configs[1]: grid_nodes 200 (100x100x200), the same record for calc_mode 0 to
           t = 0.01 and 0.03 s (35 and 65 attempted steps) and calc_mode 1 to t = 0.03 s; run on
           8 MPI ranks and checked identical on 3.
  gnoise   the g20 grid with u_noise_amp = 0.5 K (every published Params has 0): the noise field
           the reference draws (glibc rand() from seed 1, equation.c:450-456), the RHS of the four
           models that add it (calc_mode 0/10 GradP, 1/11 SigmaP1-P, equation.c:676-687) at t = 0,
           and the mode-0 and mode-1 trajectories to t = 36 and 360 s.  One MPI rank: rand() runs
           per rank, so the field depends on the decomposition.
  g400     BASELINE configs[2]: grid_nodes 400 (200x200x400, 16 M cells), calc_mode 0 to
           t = 0.002 and 0.005 s (about 45 and 67 attempted steps); run on 8 MPI ranks and checked
           identical on 5 (about 3 minutes of the build container's 8 cores).

    python tests/golden/gen_golden.py [case ...]     (default: all)
"""
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_APP = "/root/reference/apps/intertrack-hybrid-S-freezing"
PFT_REF = os.path.join(REPO, "oracle", "_ref", "pft_ref")
MPIRUN = "/opt/conda/bin/mpirun"
SEED = 20251015
ENV = dict(os.environ, OMP_NUM_THREADS="1", OMP_SCHEDULE="static", OMP_PROC_BIND="FALSE")


def params_text(replace):
    src = open(os.path.join(REF_APP, "Params")).read()
    for key, val in replace.items():
        if key.startswith("icond "):
            pat = re.compile(r"^" + re.escape(key) + r"\s*=.*$", re.M)
            src, n = pat.subn(f'{key} = "{val}"', src)
        else:
            pat = re.compile(r"^" + re.escape(key) + r"[ \t]+.*$", re.M)
            src, n = pat.subn(f"{key}\t{val}", src)
        assert n == 1, (key, n)
    return src


class Work:
    def __init__(self, replace):
        self.dir = tempfile.mkdtemp(prefix="pftgold_")
        os.symlink(os.path.join(REF_APP, "data"), os.path.join(self.dir, "data"))
        with open(os.path.join(self.dir, "Params"), "w") as f:
            f.write(params_text(replace))

    def run(self, nranks, *args, timeout=600):
        out = os.path.join(self.dir, f"out{nranks}_{abs(hash(args)) % 10**8}")
        os.makedirs(out, exist_ok=True)
        cmd = [PFT_REF, args[0], "Params", out] + [str(a) for a in args[1:]]
        if nranks > 1:
            cmd = [MPIRUN, "-np", str(nranks)] + cmd
        subprocess.run(cmd, cwd=self.dir, env=ENV, check=True, timeout=timeout,
                       stdout=subprocess.DEVNULL)
        return out

    def close(self):
        shutil.rmtree(self.dir, ignore_errors=True)


def read_params(out):
    p = {}
    for line in open(os.path.join(out, "params.txt")):
        k, v = line.split()
        p[k] = int(v) if re.fullmatch(r"-?\d+", v) else float.fromhex(v)
    return p


def hexify(p):
    return {k: (v.hex() if isinstance(v, float) else v) for k, v in p.items()}


def load(path, shape):
    return np.fromfile(path, dtype="<f8").reshape(shape)


def random_state(n1, n2, n3, rng):
    p = rng.uniform(0.0, 1.0, size=(n3, n2, n1))
    g = rng.uniform(0.0, 1.0, size=(n3, n2, n1))
    # smooth gl a little so it looks like a phase field, keep it in [0,1]
    for ax in range(3):
        g = 0.5 * g + 0.25 * (np.roll(g, 1, ax) + np.roll(g, -1, ax))
    u = 273.15 + rng.uniform(-20.0, 20.0, size=(n3, n2, n1))
    return np.stack([u, p, g]).astype("<f8")


def traj(out, ncalls, shape):
    rows = [l.split() for l in open(os.path.join(out, "traj.txt"))]
    meta = [[float.fromhex(r[0]).hex(), float.fromhex(r[1]).hex(), int(r[2]), int(r[3]), int(r[4])]
            for r in rows]
    states = [load(os.path.join(out, f"state{i}.f64"), shape) for i in range(ncalls)]
    return meta, states


def case_g20():
    arrays, meta = {}, {"case": "g20", "source": "reference Params, grid_nodes 20"}
    w = Work({"grid_nodes": 20})
    try:
        out = w.run(1, "setup")
        p = read_params(out)
        n1, n2, n3 = p["n1"], p["n2"], p["n3"]
        shape = (3, n3, n2, n1)
        ic = load(os.path.join(out, "ic.f64"), shape)
        arrays["ic"] = ic
        meta["params"] = hexify(p)
        ic_path = os.path.join(w.dir, "ic.f64")
        ic.tofile(ic_path)
        # RHS at t = 0 and after the phase switch for every model
        for mode in (0, 1, 2, 10, 11):
            wm = Work({"grid_nodes": 20, "calc_mode": mode})
            try:
                for tag, t in (("t0", 0.0), ("t1", 20000.0)):
                    o = wm.run(1, "rhs", ic_path, t)
                    arrays[f"rhs_m{mode}_{tag}"] = load(os.path.join(o, "rhs.f64"), shape)
            finally:
                wm.close()
        meta["rhs_times"] = {"t0": 0.0, "t1": 20000.0}
        # trajectories: from IC at t=0, h=tau=1 to several snapshot times (intertrack.c:2272)
        times = [36.0, 360.0, 720.0]
        meta["traj_times"] = times
        for mode, rep in ((0, {}), (1, {}), (2, {"icond p": "0"})):
            r = {"grid_nodes": 20, "calc_mode": mode}
            r.update(rep)
            wm = Work(r)
            try:
                o = wm.run(1, "setup")
                ic_m = load(os.path.join(o, "ic.f64"), shape)
                icp = os.path.join(wm.dir, "icm.f64")
                ic_m.tofile(icp)
                o1 = wm.run(1, "solve", icp, 0.0, 1.0, *times)
                tm, st = traj(o1, len(times), shape)
                o3 = wm.run(3, "solve", icp, 0.0, 1.0, *times)
                tm3, st3 = traj(o3, len(times), shape)
                assert tm == tm3 and all(np.array_equal(a, b) for a, b in zip(st, st3)), \
                    f"decomposition invariance broken for mode {mode}"
                arrays[f"traj_m{mode}_ic"] = ic_m
                for i, s in enumerate(st):
                    arrays[f"traj_m{mode}_state{i}"] = s
                meta[f"traj_m{mode}"] = tm
            finally:
                wm.close()
    finally:
        w.close()
    return arrays, meta


def case_g20nf():
    """g20's trajectory record for the two remaining models, calc_mode 10 and 11 (the RHS without
    the heat-flux term, equation.c:650-731 with du = 0), from the default IC to the same snapshot
    times, checked identical on 3 ranks"""
    arrays, meta = {}, {"case": "g20nf", "source": "reference Params, grid_nodes 20, calc_mode 10 and 11"}
    times = [36.0, 360.0, 720.0]
    meta["traj_times"] = times
    for mode in (10, 11):
        wm = Work({"grid_nodes": 20, "calc_mode": mode})
        try:
            o = wm.run(1, "setup")
            p = read_params(o)
            shape = (3, p["n3"], p["n2"], p["n1"])
            ic_m = load(os.path.join(o, "ic.f64"), shape)
            icp = os.path.join(wm.dir, "icm.f64")
            ic_m.tofile(icp)
            o1 = wm.run(1, "solve", icp, 0.0, 1.0, *times)
            tm, st = traj(o1, len(times), shape)
            o3 = wm.run(3, "solve", icp, 0.0, 1.0, *times)
            tm3, st3 = traj(o3, len(times), shape)
            assert tm == tm3 and all(np.array_equal(a, b) for a, b in zip(st, st3)), \
                f"decomposition invariance broken for mode {mode}"
            arrays[f"traj_m{mode}_ic"] = ic_m
            for i, x in enumerate(st):
                arrays[f"traj_m{mode}_state{i}"] = x
            meta[f"traj_m{mode}"] = tm
            meta[f"m{mode}_params"] = hexify(p)
        finally:
            wm.close()
    return arrays, meta


NOISE_AMP = 0.5


def case_gnoise():
    arrays, meta = {}, {"case": "gnoise", "source": f"reference Params, grid_nodes 20, u_noise_amp {NOISE_AMP}",
                        "u_noise_amp": NOISE_AMP}
    times = [36.0, 360.0]
    meta["traj_times"] = times
    noise = None
    for mode in (0, 1, 10, 11):
        w = Work({"grid_nodes": 20, "calc_mode": mode, "u_noise_amp": NOISE_AMP})
        try:
            o = w.run(1, "setup")
            p = read_params(o)
            shape = (3, p["n3"], p["n2"], p["n1"])
            ic = load(os.path.join(o, "ic.f64"), shape)
            icp = os.path.join(w.dir, "ic.f64")
            ic.tofile(icp)
            if mode == 0:
                meta["params"] = hexify(p)
                arrays["ic"] = ic
            else:
                assert np.array_equal(ic, arrays["ic"])
            meta[f"m{mode}_params"] = hexify(p)
            if mode in (0, 1):
                o1 = w.run(1, "solve", icp, 0.0, 1.0, *times)
                tm, st = traj(o1, len(times), shape)
                for i, x in enumerate(st):
                    arrays[f"traj_m{mode}_state{i}"] = x
                meta[f"traj_m{mode}"] = tm
            # the RHS at the mode-0 state of t = 360 s, where p is mixed (the IC's pure 0 / 1 phases
            # switch the SigmaP1-P source term, and with it the noise, off)
            sp = os.path.join(w.dir, "s.f64")
            arrays["traj_m0_state1"].tofile(sp)
            o = w.run(1, "rhs", sp, times[1])
            arrays[f"rhs_m{mode}"] = load(os.path.join(o, "rhs.f64"), shape)
            nz = np.fromfile(os.path.join(o, "noise_rank0.f64"), dtype="<f8").reshape(shape[1:])
            if noise is None:
                noise = nz
                arrays["noise"] = nz
            else:
                assert np.array_equal(nz, noise)
        finally:
            w.close()
    meta["rhs_state"] = "traj_m0_state1"
    meta["rhs_time"] = times[1]
    return arrays, meta


def sha256(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


G100_TIMES = [3.0, 10.0]


def case_g100():
    arrays, meta = {}, {"case": "g100", "source": "reference Params, grid_nodes 100"}
    w = Work({"grid_nodes": 100})
    try:
        out = w.run(1, "setup")
        p = read_params(out)
        shape = (3, p["n3"], p["n2"], p["n1"])
        ic = load(os.path.join(out, "ic.f64"), shape)
        meta["params"] = hexify(p)
        meta["ic_sha256"] = sha256(ic)
        icp = os.path.join(w.dir, "ic.f64")
        ic.tofile(icp)
        o = w.run(1, "solve", icp, 0.0, 1.0, *G100_TIMES)
        tm, st = traj(o, len(G100_TIMES), shape)
        o2 = w.run(2, "solve", icp, 0.0, 1.0, *G100_TIMES)
        tm2, st2 = traj(o2, len(G100_TIMES), shape)
        assert tm == tm2 and all(np.array_equal(a, b) for a, b in zip(st, st2)), "decomposition invariance"
        meta["traj_times"] = G100_TIMES
        meta["traj_m0"] = tm
        meta["traj_m0_sha256"] = [sha256(x) for x in st]
        for i, x in enumerate(st):
            arrays[f"traj_m0_state{i}_mid"] = x[:, shape[1] // 2]
            arrays[f"traj_m0_state{i}_top"] = x[:, -1]
    finally:
        w.close()
    return arrays, meta


def case_large(name, gn, runs, nranks, check_ranks):
    """a full-size BASELINE grid: per calc_mode, the reference's trajectory to `times` on nranks
    MPI ranks (re-checked on check_ranks), stored as digests plus the middle and top planes"""
    arrays, meta = {}, {"case": name, "source": f"reference Params, grid_nodes {gn}",
                        "mpi_ranks": nranks, "checked_on_ranks": check_ranks}
    for mode, times in runs:
        w = Work({"grid_nodes": gn, "calc_mode": mode})
        try:
            out = w.run(nranks, "setup", timeout=3600)
            p = read_params(out)
            shape = (3, p["n3"], p["n2"], p["n1"])
            ic = load(os.path.join(out, "ic.f64"), shape)
            if mode == runs[0][0]:
                meta["params"] = hexify(p)
            meta[f"m{mode}_params"] = hexify(p)
            meta[f"m{mode}_ic_sha256"] = sha256(ic)
            icp = os.path.join(w.dir, "ic.f64")
            ic.tofile(icp)
            o = w.run(nranks, "solve", icp, 0.0, 1.0, *times, timeout=3600)
            tm, st = traj(o, len(times), shape)
            o2 = w.run(check_ranks, "solve", icp, 0.0, 1.0, *times, timeout=3600)
            tm2, st2 = traj(o2, len(times), shape)
            assert tm == tm2 and all(np.array_equal(a, b) for a, b in zip(st, st2)), "decomposition invariance"
            meta[f"traj_m{mode}_times"] = times
            meta[f"traj_m{mode}"] = tm
            meta[f"traj_m{mode}_sha256"] = [sha256(x) for x in st]
            for i, x in enumerate(st):
                arrays[f"traj_m{mode}_state{i}_mid"] = x[:, shape[1] // 2]
                arrays[f"traj_m{mode}_state{i}_top"] = x[:, -1]
        finally:
            w.close()
    return arrays, meta


def case_g200():
    return case_large("g200", 200, [(0, [0.01, 0.03]), (1, [0.03])], 8, 3)


def case_g400():
    return case_large("g400", 400, [(0, [0.002, 0.005])], 8, 5)


def traj_ext(out, ncalls, shape):
    """solvex rows: t, h, steps, steps_total, rc, check_NAN; cb.txt rows: steps, t, h"""
    rows = [l.split() for l in open(os.path.join(out, "traj.txt"))]
    meta = [[float.fromhex(r[0]).hex(), float.fromhex(r[1]).hex(), int(r[2]), int(r[3]), int(r[4]), int(r[5])]
            for r in rows]
    cb = []
    if os.path.exists(os.path.join(out, "cb.txt")):
        cb = [[int(r[0]), float.fromhex(r[1]).hex(), float.fromhex(r[2]).hex()]
              for r in (l.split() for l in open(os.path.join(out, "cb.txt")))]
    states = [load(os.path.join(out, f"state{i}.f64"), shape) for i in range(ncalls)]
    return meta, cb, states


def case_ctl():
    """Control-flow KATs of RK_MPI_SA_solve (hybrid2.c) on the g20 grid, mode 0, run through the
    reference's solvex harness command:
      nan_giveup_*  a NaN in the state with RK_MPI_SA_handle_NAN(1): h/10 retries until
                    h/(T-t) < 1e-11, return -4 (hybrid2.c:464-504, 624-646), for three (t0, h0, T)
      nan_retry     h0 = 1e8 s: the first attempts overflow to inf/NaN in the stage values, h/10
                    retries until the error norm is finite, then ordinary steps; a Service_Callback
                    logs (steps, t, h) after every accepted step and interrupts at the 10th
      cb_break      h0 = 1, T = 36: the callback interrupts at its 25th call (return 1, t and
                    h = new_h left in the system, hybrid2.c:697-705), the second call resumes to
                    T; the log holds every accepted step of both calls"""
    arrays, meta = {}, {"case": "ctl", "source": "reference Params, grid_nodes 20, solvex"}
    w = Work({"grid_nodes": 20})
    try:
        out = w.run(1, "setup")
        p = read_params(out)
        shape = (3, p["n3"], p["n2"], p["n1"])
        ic = load(os.path.join(out, "ic.f64"), shape)
        meta["params"] = hexify(p)
        arrays["ic"] = ic
        runs = {}
        nan_ic = ic.copy()
        nan_ic[0, 5, 5, 5] = np.nan
        inf_ic = ic.copy()
        inf_ic[1, 13, 2, 7] = np.inf
        # name: (state, t0, h0, handle_nan, break_at, [T...])
        spec = {
            "nan_giveup_a": (nan_ic, 0.0, 1.0, 1, -1, [36.0]),
            "nan_giveup_b": (nan_ic, 100.0, 5.0, 1, -1, [1e5]),
            "nan_giveup_c": (inf_ic, 7.0, 0.25, 1, -1, [7.5]),
            "nan_retry": (ic, 0.0, 1e8, 1, 10, [1e9]),
            "cb_break": (ic, 0.0, 1.0, 0, 25, [36.0, 36.0]),
        }
        for name, (st, t0, h0, hn, brk, Ts) in spec.items():
            sp = os.path.join(w.dir, name + ".f64")
            st.tofile(sp)
            o = w.run(1, "solvex", sp, t0, h0, hn, brk, *Ts)
            tm, cb, states = traj_ext(o, len(Ts), shape)
            if name in ("nan_retry", "cb_break"):
                o3 = w.run(3, "solvex", sp, t0, h0, hn, brk, *Ts)
                tm3, cb3, states3 = traj_ext(o3, len(Ts), shape)
                assert tm == tm3 and cb == cb3 and all(np.array_equal(a, b) for a, b in zip(states, states3))
            runs[name] = {"t0": t0, "h0": h0, "handle_nan": hn, "break_at": brk, "T": Ts, "traj": tm, "cb": cb}
            if name.startswith("nan_giveup"):
                arrays[name + "_ic"] = st
            for i, s in enumerate(states):
                arrays[f"{name}_state{i}"] = s
        meta["runs"] = runs
    finally:
        w.close()
    return arrays, meta


def case_ragged():
    arrays, meta = {}, {"case": "ragged", "source": "reference Params, L1=0.036 L2=0.024 grid_nodes 30"}
    rep = {"L1": 0.036, "L2": 0.024, "grid_nodes": 30}
    w = Work(rep)
    try:
        out = w.run(1, "setup")
        p = read_params(out)
        n1, n2, n3 = p["n1"], p["n2"], p["n3"]
        shape = (3, n3, n2, n1)
        meta["params"] = hexify(p)
        st = random_state(n1, n2, n3, np.random.default_rng(SEED))
        arrays["state"] = st
        sp = os.path.join(w.dir, "state.f64")
        st.tofile(sp)
        for mode in (0, 1, 2, 10, 11):
            wm = Work(dict(rep, calc_mode=mode))
            try:
                for tag, t in (("t0", 100.0), ("t1", 20000.0)):
                    o1 = wm.run(1, "rhs", sp, t)
                    o4 = wm.run(4, "rhs", sp, t)
                    a1 = load(os.path.join(o1, "rhs.f64"), shape)
                    a4 = load(os.path.join(o4, "rhs.f64"), shape)
                    assert np.array_equal(a1, a4), f"rhs decomposition mismatch mode {mode}"
                    arrays[f"rhs_m{mode}_{tag}"] = a1
                    if mode == 0:
                        for r in range(4):
                            arrays[f"w4_{tag}_rank{r}"] = np.fromfile(
                                os.path.join(o4, f"w_rank{r}.f64"), dtype="<f8")
                        arrays[f"w1_{tag}_rank0"] = np.fromfile(os.path.join(o1, "w_rank0.f64"), dtype="<f8")
            finally:
                wm.close()
        meta["rhs_times"] = {"t0": 100.0, "t1": 20000.0}
        # single steps: small h (accepted at once) and a large h (rejected first, then accepted)
        for tag, (t0, h0, T) in {"small": (100.0, 1e-3, 100.001), "large": (100.0, 5.0, 105.0)}.items():
            o = w.run(1, "solve", sp, t0, h0, T)
            tm, sts = traj(o, 1, shape)
            o4 = w.run(4, "solve", sp, t0, h0, T)
            tm4, sts4 = traj(o4, 1, shape)
            assert tm == tm4 and np.array_equal(sts[0], sts4[0])
            arrays[f"step_{tag}"] = sts[0]
            meta[f"step_{tag}"] = {"t0": t0, "h0": h0, "T": T, "result": tm[0]}
    finally:
        w.close()
    return arrays, meta


def main():
    if not os.path.exists(PFT_REF):
        sys.exit("build the reference harness first: make -C oracle ref")
    cases = {"g20": case_g20, "ragged": case_ragged, "g100": case_g100, "ctl": case_ctl, "g200": case_g200,
             "g400": case_g400, "g20nf": case_g20nf, "gnoise": case_gnoise}
    for name in sys.argv[1:] or list(cases):
        arrays, meta = cases[name]()
        name = meta["case"]
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print(name, {k: v.shape for k, v in arrays.items()})
    # the bead centres (data/spheres_positions.txt, data file used by equation.c:35,459-530)
    beads = np.loadtxt(os.path.join(REF_APP, "data", "spheres_positions.txt"))
    np.save(os.path.join(HERE, "beads.npy"), beads.astype("<f8"))


if __name__ == "__main__":
    main()
