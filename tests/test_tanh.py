"""f1: the device initial condition computes tanh (glass walls and beads, equation.c:459-530) with
libpft's restatement of the host C library's algorithm (porousfreezethaw_amd/csrc/pft_tanh.h),
so that the device IC is the host IC bit for bit.  Here the restatement, compiled for the CPU
without contraction, is compared with the C library on 10^7 arguments."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_restated_tanh_equals_c_library(tmp_path):
    exe = tmp_path / "tanh_check"
    subprocess.run(["gcc", "-O2", "-std=c99", "-ffp-contract=off", "-fno-fast-math",
                    os.path.join(HERE, "native", "tanh_check.c"), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "10000000"], check=True, capture_output=True, text=True).stdout.split()
    n, bad_tanh, bad_expm1 = map(int, out)
    assert n == 10_000_000
    assert bad_tanh == 0 and bad_expm1 == 0, f"{bad_tanh} tanh / {bad_expm1} expm1 results differ"
