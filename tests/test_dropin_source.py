"""The drop-in, checked on the real driver's own text (CPU; reads /root/reference as text only and
skips where it is absent, e.g. on the GPU box).

The real intertrack.c is not compiled here: it includes <netcdf.h> unconditionally
(intertrack.c:111), the image has no NetCDF, and a stand-in header for building reference code is
ruled out by this project's build rules.  What a compile and link of the swapped driver would
establish is checked instead on its source:

1. intertrack.c:633 is the one `#include "equation.c"` the swap replaces by
   `#include "pft_equation_adapter.c"`, and nothing else in the driver includes equation.c;
2. every symbol equation.c defines that the driver uses after that line is provided by the swap:
   defined (or macro-redirected) in include/pft_equation_adapter.c, or declared in libpft's headers
   and exported by libpft.so -- no undefined symbol at link time;
3. every driver identifier the adapter reads is declared at file scope of intertrack.c before
   line 633 -- the adapter compiles where equation.c compiled;
4. every RK_MPI_SA_* entry point the driver calls is declared in libpft's RK_MPI_SAsolver.h with
   the reference header's parameter list and exported by libpft.so.

tests/test_reference_abi.py compiles libpft against the reference's own solver header, and
tests/test_adapter.py compiles the adapter into a mock driver and runs its call sequence.
"""
import os
import re
import subprocess

import pytest

import _oracle as O

REPO = O.REPO
APP = "/root/reference/apps/intertrack-hybrid-S-freezing"
DRIVER = os.path.join(APP, "intertrack.c")
EQUATION = os.path.join(APP, "equation.c")
REF_SOLVER_H = "/root/reference/include/RK_MPI_SAsolver.h"
ADAPTER = os.path.join(REPO, "include", "pft_equation_adapter.c")
LIB = os.path.join(REPO, "porousfreezethaw_amd", "lib", "libpft.so")

pytestmark = pytest.mark.skipif(not os.path.exists(DRIVER), reason="reference sources not present")

# the driver statics the adapter reads (include/pft_equation_adapter.c:14-15)
DRIVER_GLOBALS = ["n1", "n2", "total_n3", "L1", "L2", "L3", "calc_mode", "param", "solution",
                  "MPIrank", "MPIprocs", "MPIrankmap"]


def strip_c(src):
    """comments and string/char literals removed, line structure kept"""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append(re.sub(r"[^\n]", " ", src[i:j]))
            i = j
        elif src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            i = j
        elif c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == "\\" else 1
            out.append(c + " " * (min(j, n - 1) - i - 1) + c)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def file_scope_lines(src):
    """(line number, text) of the lines that start at brace depth 0"""
    depth, res = 0, []
    for no, line in enumerate(src.split("\n"), 1):
        if depth == 0:
            res.append((no, line))
        depth += line.count("{") - line.count("}")
    return res


def equation_symbols():
    """names equation.c defines at file scope (functions and variables)"""
    src = strip_c(open(EQUATION, errors="replace").read())
    names = set()
    for _, line in file_scope_lines(src):
        if line.startswith(("#", " ", "\t")) or not line.strip():
            continue
        m = re.match(r"^(?:static\s+)?(?:inline\s+)?(?:const\s+)?[A-Za-z_]\w*[\s\*]+\**\s*([A-Za-z_]\w*)\s*[\(\[=;,]",
                     line)
        if m:
            names.add(m.group(1))
    return names


def exported():
    r = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True)
    return {ln.split()[-1] for ln in r.stdout.splitlines() if ln.strip()}


def header_declared():
    names = set()
    for h in os.listdir(os.path.join(REPO, "include")):
        if h.endswith(".h"):
            src = strip_c(open(os.path.join(REPO, "include", h)).read())
            names |= set(re.findall(r"\b([A-Za-z_]\w*)\s*\(", src))
    return names


def test_one_line_swap_point():
    lines = open(DRIVER, errors="replace").read().split("\n")
    inc = [i + 1 for i, ln in enumerate(lines) if re.match(r'\s*#\s*include\s+"equation\.c"', ln)]
    assert inc == [633]


def test_every_equation_symbol_the_driver_uses_is_provided():
    src = strip_c(open(DRIVER, errors="replace").read()).split("\n")
    after = "\n".join(src[633:])
    used = sorted(n for n in equation_symbols() if re.search(rf"\b{re.escape(n)}\b", after))
    assert {"AllocPrecalcData", "PrecalculateData", "bcond_thickness"} <= set(used), used
    adapter = strip_c(open(ADAPTER).read())
    provided_in_adapter = set(re.findall(r"#define\s+([A-Za-z_]\w*)", adapter)) | \
        set(re.findall(r"^static\s+[^;(]*?\b([A-Za-z_]\w*)\s*=", adapter, re.M))
    lib_syms, declared = exported(), header_declared()
    missing = [n for n in used if n not in provided_in_adapter and not (n in declared and n in lib_syms)]
    assert not missing, f"driver uses equation.c symbols the swap does not provide: {missing}"


def test_adapter_reads_only_driver_globals_declared_before_the_swap():
    src = strip_c(open(DRIVER, errors="replace").read())
    prefix = "\n".join(src.split("\n")[:632])
    decl = [ln for _, ln in file_scope_lines(prefix) if not ln.lstrip().startswith("#")]
    adapter = strip_c(open(ADAPTER).read())
    for g in DRIVER_GLOBALS:
        assert re.search(rf"\b{g}\b", adapter), g
        hits = [ln for ln in decl if re.search(rf"\b{g}\b", ln) and "(" not in ln.split(g)[0]]
        assert hits, f"{g}: not declared at file scope of intertrack.c before line 633"


def _prototypes(path):
    src = strip_c(open(path, errors="replace").read())
    src = re.sub(r"\s+", " ", src)
    out = {}
    for m in re.finditer(r"\b(RK_MPI_SA_\w+)\s*\(([^()]*)\)\s*;", src):
        params = [re.sub(r"\s*\*\s*", "*", p.strip()) for p in m.group(2).split(",")]
        params = [re.sub(r"(?<=[\s*])[A-Za-z_]\w*$", "", p).strip() for p in params]   # parameter names
        out[m.group(1)] = params
    return out


def test_driver_solver_calls_match_libpft():
    src = strip_c(open(DRIVER, errors="replace").read())
    called = sorted(set(re.findall(r"\b(RK_MPI_SA_\w+)\s*\(", src)))
    assert {"RK_MPI_SA_init", "RK_MPI_SA_check_mem", "RK_MPI_SA_solve", "RK_MPI_SA_cleanup"} <= set(called)
    ours = _prototypes(os.path.join(REPO, "include", "RK_MPI_SAsolver.h"))
    ref = _prototypes(REF_SOLVER_H) if os.path.exists(REF_SOLVER_H) else None
    lib_syms = exported()
    for f in called:
        assert f in lib_syms, f"{f} not exported by libpft.so"
        assert f in ours, f"{f} not declared in include/RK_MPI_SAsolver.h"
        if ref is not None:
            assert ours[f] == ref[f], (f, ours[f], ref[f])
