"""The Julia binding (julia/PamgHIP) against the C-ABI header, without Julia (not in the image).

Every ``ccall((:sym, libpamg), RetT, (ArgT, ...), args...)`` in the package and its
PartitionedArrays extension is parsed and checked against ``include/pamg.h``: the symbol is
declared, the argument-type tuple has the prototype's arity, each Julia type is the ABI
equivalent of the C parameter type, the return type matches, and the call passes as many
arguments as it declares. The package must bind every entry point of the header except the
few listed in UNBOUND (each with its reason) — the Julia counterpart of tests/test_abi.py.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pamg.h")
JL = [os.path.join(ROOT, "julia", "PamgHIP", "src", "PamgHIP.jl"),
      os.path.join(ROOT, "julia", "PamgHIP", "ext", "PamgHIPPartitionedArraysExt.jl")]

UNBOUND = {
    # debug transport: a host callback serving all ranks of ONE process; Julia's debug backend
    # runs the parts in one task (synchronous callbacks would deadlock), MPI runs use RCCL
    "pamg_comm_init_host",
}

OPAQUE = {"pamg_ctx", "pamg_plan", "pamg_vec", "pamg_mat", "pamg_hier", "pamg_hcsr", "pamg_world"}
SCALAR = {"int": {"Cint", "Int32"}, "int32_t": {"Int32", "Cint"}, "int64_t": {"Int64"},
          "uint64_t": {"UInt64"}, "double": {"Cdouble", "Float64"}, "uint8_t": {"UInt8"},
          "unsigned char": {"UInt8"}, "char": {"UInt8", "Cchar"}}


def _split_top(s, sep=","):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def c_prototypes():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(pamg_\w+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, params = m.group(1).strip(), m.group(2), m.group(3).strip()
        if "typedef" in ret:
            continue
        plist = [] if params in ("", "void") else [p.strip() for p in params.split(",")]
        protos[name] = (ret, plist)
    return protos


def c_param_type(p: str):
    """(base, pointer depth) of a C parameter declaration ('const int64_t* rowptr')."""
    p = re.sub(r"\bconst\b", " ", p)
    arr = p.count("[")
    p = re.sub(r"\[[^\]]*\]", "", p)
    depth = p.count("*") + arr
    words = p.replace("*", " ").split()
    base = " ".join(words[:-1]) if len(words) > 1 else words[0]
    return base, depth


def jl_type(t: str):
    """(base, pointer depth) of a Julia ccall type ('Ptr{Ptr{Cvoid}}')."""
    t = t.strip()
    depth = 0
    while t.startswith("Ptr{") and t.endswith("}"):
        t = t[4:-1]
        depth += 1
    if t == "Cstring":
        return "Cstring", 1
    return t, depth


def compatible(c: str, j: str) -> bool:
    cb, cd = c_param_type(c) if not isinstance(c, tuple) else c
    jb, jd = jl_type(j)
    if cb == "pamg_host_comm_fn":
        return jb == "Cvoid" and jd == 1
    if cb in OPAQUE or cb == "void":
        return jb == "Cvoid" and jd == cd  # handles / untyped buffers are Ptr{Cvoid}
    if cb == "char" and cd == 1:
        return (jb, jd) in {("Cstring", 1), ("UInt8", 1)}
    return cd == jd and jb in SCALAR.get(cb, set())


def julia_ccalls():
    calls = []
    for path in JL:
        src = open(path).read()
        src = re.sub(r"#[^\n]*", "", src)  # comments
        for m in re.finditer(r"ccall\(\(:(pamg_\w+),\s*libpamg\)", src):
            # the whole ccall( ... ) expression
            i, depth = m.start() + len("ccall"), 0
            for k in range(i, len(src)):
                depth += {"(": 1, ")": -1}.get(src[k], 0)
                if depth == 0:
                    break
            body = src[i + 1:k]
            parts = _split_top(body)
            ret, types = parts[1], parts[2]
            assert types.startswith("(") and types.endswith(")"), (m.group(1), types)
            tl = _split_top(types[1:-1])
            calls.append((os.path.basename(path), m.group(1), ret, tl, parts[3:]))
    return calls


def test_every_ccall_matches_the_header():
    protos = c_prototypes()
    calls = julia_ccalls()
    assert len(calls) > 60
    for fname, sym, ret, types, args in calls:
        assert sym in protos, f"{fname}: {sym} is not declared in include/pamg.h"
        cret, cparams = protos[sym]
        assert len(types) == len(cparams), f"{fname}: {sym} binds {len(types)} args, header has {len(cparams)}"
        assert len(args) == len(types), f"{fname}: {sym} passes {len(args)} values for {len(types)} types"
        for k, (c, j) in enumerate(zip(cparams, types)):
            assert compatible(c, j), f"{fname}: {sym} arg {k}: Julia {j} vs C '{c}'"
        want = "Cstring" if cret.replace("const", "").strip() in ("char*", "char *") else "Cint"
        if cret.strip() == "int":
            want = "Cint"
        assert ret == want, f"{fname}: {sym} returns {ret}, header says {cret}"


def test_the_binding_covers_the_header():
    protos = c_prototypes()
    bound = {c[1] for c in julia_ccalls()}
    missing = set(protos) - bound - UNBOUND
    assert not missing, f"entry points without a Julia binding: {sorted(missing)}"
    assert not (UNBOUND & bound), "UNBOUND lists a symbol that is bound"


@pytest.mark.parametrize("c,j,ok", [("const int64_t* rowptr", "Ptr{Int64}", True),
                                    ("const int64_t* rowptr", "Ptr{Int32}", False),
                                    ("pamg_ctx** out", "Ptr{Ptr{Cvoid}}", True),
                                    ("pamg_ctx* ctx", "Ptr{Ptr{Cvoid}}", False),
                                    ("const unsigned char id[128]", "Ptr{UInt8}", True),
                                    ("double omega", "Cdouble", True), ("int set", "Int64", False),
                                    ("const char* key", "Cstring", True)])
def test_type_rules(c, j, ok):
    assert compatible(c, j) == ok


# PartitionedArrays' / LinearAlgebra's generic-function surface an AMG solver calls unqualified
# (the PartitionedArrays tables): PamgHIP must not export a generic of its own
# under any of these names, or `using PartitionedArrays, PamgHIP` makes the solver's calls
# ambiguous.
PA_SURFACE = {"consistent!", "assemble!", "own_values", "ghost_values", "local_values", "partition",
              "exchange", "exchange!", "mul!", "dot", "norm", "axpy!", "axpby!", "ldiv!", "fill!",
              "copy!", "copyto!", "similar", "PVector", "PSparseMatrix", "PRange", "own_to_local",
              "ghost_to_local", "local_to_global", "global_to_local", "uniform_partition",
              "variable_partition", "gather", "scatter", "reduction", "wait", "fetch"}


def _strip_comments(src):
    src = re.sub(r'"""(.*?)"""', '""', src, flags=re.S)
    return re.sub(r"#[^\n]*", "", src)


def test_pamghip_exports_no_partitionedarrays_name():
    src = _strip_comments(open(JL[0]).read())
    m = re.search(r"\bexport\b(.*?)\n(?!\s)", src, flags=re.S)
    exported = {w.strip() for w in m.group(1).replace("\n", " ").split(",") if w.strip()}
    assert "DeviceVector" in exported and "download_own" in exported
    clash = exported & PA_SURFACE
    assert not clash, f"PamgHIP exports PartitionedArrays/LinearAlgebra names: {sorted(clash)}"
    # and defines no unqualified generic of those names either (exported or not)
    defs = set(re.findall(r"^function\s+([A-Za-z_][\w!]*)\s*\(", src, flags=re.M))
    defs |= set(re.findall(r"^([A-Za-z_][\w!]*)\s*\([^\n]*\)\s*=", src, flags=re.M))
    assert not (defs & PA_SURFACE), sorted(defs & PA_SURFACE)


def test_device_vector_is_not_an_abstract_vector():
    """A DeviceVector lives on the GPU: the AbstractVector fallbacks (getindex per element)
    would download it once per element."""
    src = _strip_comments(open(JL[0]).read())
    assert re.search(r"mutable struct DeviceVector\s*\n", src)
    assert "DeviceVector <:" not in src
    assert not re.search(r"Base\.getindex\(\s*v::DeviceVector", src)


def test_extension_methods_extend_the_owning_generics():
    """Every method the extension defines on its distributed types is a method of the owning
    package's generic (PartitionedArrays., LinearAlgebra., Base., PamgHIP.), never a new
    function of the same name; consistent! returns a waitable Task; no invented
    PartitionedArrays names."""
    src = _strip_comments(open(JL[1]).read())
    types = ("HIPPVector", "HIPPSparseMatrix", "HIPPVCycle")
    heads = re.findall(r"^function\s+([\w\.!]+)\s*\(([^\n]*)\)", src, flags=re.M)
    heads += re.findall(r"^([\w\.!]+)\s*\(([^\n=]*)\)\s*=", src, flags=re.M)
    checked = 0
    for name, args in heads:
        if not any(f"::{t}" in args for t in types) or name in types:
            continue
        checked += 1
        assert re.match(r"^(PartitionedArrays|LinearAlgebra|Base|PamgHIP)\.", name), \
            f"extension method {name}({args}) is not a qualified extension"
    assert checked >= 12, checked
    for needed in ("PartitionedArrays.consistent!", "PartitionedArrays.own_values", "PartitionedArrays.partition",
                   "LinearAlgebra.mul!", "LinearAlgebra.dot", "LinearAlgebra.norm", "LinearAlgebra.axpy!",
                   "LinearAlgebra.ldiv!"):
        assert re.search(rf"^(function\s+)?{re.escape(needed)}\(", src, flags=re.M), needed
    body = src[src.index("function PartitionedArrays.consistent!"):]
    body = body[:body.index("\nend")]
    assert "@async" in body
    assert "PartitionedArrays.Future" not in src
    # the distributed setup driver exists and uses the split-format blocks of v0.5 local matrices
    assert re.search(r"^function HIPPVCycle\(ctxs, A::PSparseMatrix", src, flags=re.M)
    assert "own_own_values(A)" in src and "own_ghost_values(A)" in src
