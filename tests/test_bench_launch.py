"""bench.py's N > 1 launcher (bench.py `supervise`), on the CPU.

`bench.py --gpus N` started as ONE plain process spawns the N ranks itself (child processes with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, before any HIP call: the supervisor never loads
libpft); started by torch.distributed.run, each launched process supervises one child rank.  A
failed attempt over auto / ipc-ce is retried over RCCL in fresh processes; a failure with no retry
left ends the run with a non-zero status.  The child ranks here are the launcher's dry-run hook
(PFT_BENCH_DRYRUN=1: rendezvous, gather, barrier, a stand-in line -- no GPU), which also fails a
chosen rank on a chosen transport (PFT_BENCH_DRYRUN_FAIL=rank:transport).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, fail=None, torchrun=0, timeout=180):
    env = dict(os.environ, PFT_BENCH_DRYRUN="1", PFT_BENCH_CHILD_TIMEOUT="90", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "PFT_BENCH_WORKER", "PFT_BENCH_DRYRUN_FAIL"):
        env.pop(k, None)
    if fail:
        env["PFT_BENCH_DRYRUN_FAIL"] = fail
    if torchrun:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH] + args
    else:
        cmd = [sys.executable, BENCH] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_plain_launch_spawns_n_ranks():
    """a plain `bench.py --gpus 3`: three child ranks with distinct processes and ranks 0..2, rank 0's
    line forwarded on stdout with the launch record; then the strong-split set of ranks"""
    r, out = _run(["--gpus", "3", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert out["dryrun"] and out["n_gpus"] == 3
    ranks = out["config"]["ranks"]
    assert [q["rank"] for q in ranks] == [0, 1, 2]
    assert [q["local"] for q in ranks] == [0, 1, 2]
    assert len({q["pid"] for q in ranks}) == 3 and os.getpid() not in {q["pid"] for q in ranks}
    assert out["launch"]["mode"].startswith("self-spawn")
    assert out["launch"]["attempts"] == [{"transport": "auto", "exit_codes": [0, 0, 0], "ok": True}]
    assert out["config"]["strong"]["scaling"] == "strong"
    assert r.stdout.count("\n") == 1                    # exactly one line on stdout


def test_plain_launch_propagates_a_rank_failure():
    """no retry left (RCCL named): a rank that fails makes the whole run fail, nothing printed"""
    r, out = _run(["--gpus", "2", "--transport", "rccl", "--no-strong"], fail="1:rccl")
    assert r.returncode != 0
    assert out is None
    assert "rank exit codes [" in r.stderr and "no attempt succeeded" in r.stderr


def test_plain_launch_falls_back_to_rccl_in_fresh_processes():
    """auto fails on rank 1: every rank starts again over RCCL, in new processes, and the line says so"""
    r, out = _run(["--gpus", "2", "--no-strong"], fail="1:auto")
    assert r.returncode == 0, r.stderr[-3000:]
    att = out["launch"]["attempts"]
    assert [a["transport"] for a in att] == ["auto", "rccl"]
    assert att[0]["ok"] is False and att[0]["exit_codes"][1] == 5
    assert att[1] == {"transport": "rccl", "exit_codes": [0, 0], "ok": True}
    assert out["config"]["transport"] == "rccl"


def test_torchrun_launch_supervises_one_rank_each():
    """the driver's launch (torch.distributed.run, N processes): each supervises one child rank with a
    rendezvous of its own; an ipc-ce failure on one rank moves every rank to RCCL"""
    r, out = _run(["--gpus", "2", "--transport", "ipc-ce", "--no-strong"], fail="0:ipc-ce", torchrun=2)
    assert r.returncode == 0, r.stderr[-3000:]
    assert out["launch"]["mode"].startswith("torchrun")
    assert [a["transport"] for a in out["launch"]["attempts"]] == ["ipc-ce", "rccl"]
    assert sorted(q["rank"] for q in out["config"]["ranks"]) == [0, 1]
    # stdout is the JSON line alone (the gloo library's connection notes go to stderr)
    assert json.loads(r.stdout) == out


def test_torchrun_launch_propagates_a_rank_failure():
    r, out = _run(["--gpus", "2", "--transport", "rccl", "--no-strong"], fail="0:rccl", torchrun=2)
    assert r.returncode != 0
    assert out is None
