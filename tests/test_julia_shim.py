"""The committed Julia host binding (julia/MD2HIP.jl) against the C-ABI it binds (CPU only).

Julia is not installed here, so the shim cannot be executed; these checks pin what
can be checked without it:
  * every `ccall((:md2_..., lib), ...)` names a symbol the library exports and include/md2.h
    declares;
  * every Julia struct that mirrors a C struct (ModelCfg, LossCfg, LossOut, WarpCfg, ConvDesc)
    has the same field sequence, element counts and byte layout as the typedef in include/md2.h;
  * every ccall's argument-type tuple has as many entries as the C prototype has parameters;
  * the rrules cover the op-level pullbacks the shim exposes;
  * train_loss keeps the reference's return convention (src/training.jl:36,71-77): a host scalar
    loss and host visualisation arrays, and its pullback's θ tangent is an array in m.θ's own
    layout reached through ``m.θ`` (Flux.params / implicit-gradient callers, scripts/script.jl:84-86)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = os.path.join(ROOT, "julia", "MD2HIP.jl")
HDR = os.path.join(ROOT, "include", "md2.h")
LIB = os.path.join(ROOT, "monodepth2.jl_amd", "lib", "libmd2hip.so")

C_SIZES = {"int": 4, "float": 4, "long long": 8, "size_t": 8, "ptr": 8}
JL_SIZES = {"Cint": 4, "Cfloat": 4, "Clonglong": 8, "Csize_t": 8}
PAIRS = {"ModelCfg": "md2_model_cfg", "LossCfg": "md2_loss_cfg", "LossOut": "md2_loss_out",
         "WarpCfg": "md2_warp_cfg", "ConvDesc": "md2_conv_desc"}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def _c_struct(hdr, name):
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), hdr, re.S).group(1)
    fields = []
    for decl in _strip_c_comments(body).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        m = re.match(r"(unsigned\s+)?(signed\s+)?(long long|int|float|char|size_t)\s*(\*?)\s*(.*)", decl)
        base, star, names = m.group(3), m.group(4), m.group(5)
        for nm in names.split(","):
            nm = nm.strip()
            is_ptr = bool(star) or nm.startswith("*")
            nm = nm.lstrip("*").strip()
            count = 1
            arr = re.match(r"(\w+)\[(\w+)\]", nm)
            if arr:
                nm, count = arr.group(1), arr.group(2)
                count = 5 if count == "MD2_MAX_SCALES" else int(count)
            size = 8 if is_ptr else C_SIZES[base]
            fields.append((nm, size, count))
    return fields


def _jl_struct(src, name):
    body = re.search(r"struct %s\s*(?:#[^\n]*)?\n(.*?)\nend" % name, src, re.S).group(1)
    fields = []
    for part in re.split(r"[;\n]", body):
        part = part.split("#")[0].strip()
        if not part:
            continue
        nm, ty = [t.strip() for t in part.split("::")]
        count = 1
        tup = re.match(r"NTuple\{(\d+),\s*(.+)\}", ty)
        if tup:
            count, ty = int(tup.group(1)), tup.group(2).strip()
        size = 8 if ty.startswith("Ptr") else JL_SIZES[ty]
        fields.append((nm, size, count))
    return fields


def _layout(fields):
    off, out = 0, []
    for _, size, count in fields:
        off = (off + size - 1) // size * size
        out.append(off)
        off += size * count
    align = max(f[1] for f in fields)
    return out, (off + align - 1) // align * align


@pytest.fixture(scope="module")
def sources():
    with open(JL) as f:
        jl = f.read()
    with open(HDR) as f:
        hdr = f.read()
    return jl, hdr


@pytest.mark.parametrize("jl_name,c_name", sorted(PAIRS.items()))
def test_struct_layouts_match(sources, jl_name, c_name):
    jl, hdr = sources
    cf, jf = _c_struct(hdr, c_name), _jl_struct(jl, jl_name)
    assert [(s, n) for _, s, n in cf] == [(s, n) for _, s, n in jf], (cf, jf)
    assert _layout(cf) == _layout(jf)


def _c_prototypes(hdr):
    protos = {}
    for m in re.finditer(r"\b(?:int|size_t|const char\*)\s+(md2_\w+)\((.*?)\);", _strip_c_comments(hdr), re.S):
        args = m.group(2).strip()
        protos[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return protos


def _jl_ccalls(jl):
    calls = []
    for m in re.finditer(r"ccall\(\(:(md2_\w+),\s*lib\),\s*\w+,\s*\(", jl):
        # the argument-type tuple: balanced parentheses from the match end
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(jl[i], 0)
            i += 1
        types = jl[m.end():i - 1]
        depth, n, cur = 0, 0, ""
        for ch in types + ",":
            if ch in "({":
                depth += 1
            elif ch in ")}":
                depth -= 1
            if ch == "," and depth == 0:
                n += bool(cur.strip())
                cur = ""
            else:
                cur += ch
        calls.append((m.group(1), n))
    return calls


def test_ccalls_match_header_and_library(sources):
    jl, hdr = sources
    protos = _c_prototypes(hdr)
    calls = _jl_ccalls(jl)
    assert len(calls) >= 30
    lib = ctypes.CDLL(LIB) if os.path.exists(LIB) else None
    for name, nargs in calls:
        assert name in protos, f"{name} is not declared in include/md2.h"
        assert nargs == protos[name], (name, nargs, protos[name])
        if lib is not None:
            assert hasattr(lib, name), f"{name} is not exported by libmd2hip.so"


def test_rrules_cover_the_op_level_pullbacks(sources):
    jl, _ = sources
    for op in ("_train_loss", "SSIM", "Backproject", "Project", "grid_sample_border", "smooth_loss",
               "warp_photometric", "so3_compose"):
        assert re.search(r"ChainRulesCore\.rrule\((?:::typeof\()?\(?\w*::?%s" % op, jl) or \
            re.search(r"ChainRulesCore\.rrule\(\w+::%s" % op, jl) or \
            re.search(r"ChainRulesCore\.rrule\(::typeof\(%s\)" % op, jl), op


def _function_body(jl, header_regex):
    m = re.search(header_regex, jl)
    assert m, header_regex
    depth, i = 1, m.end()
    # Julia blocks: count function/if/for/while/let/begin/do ... end pairs crudely by keywords
    for tok in re.finditer(r"\b(function|if|for|while|let|begin|do|try)\b|\bend\b", jl[i:]):
        depth += -1 if tok.group(0) == "end" else 1
        if depth == 0:
            return jl[m.start():i + tok.end()]
    raise AssertionError("unbalanced " + header_regex)


def test_train_loss_return_convention(sources):
    jl, _ = sources
    # train_loss passes m.θ through traced code, so Zygote's implicit Params see the gradient
    tl = _function_body(jl, r"function train_loss\(m::HIPModel")
    assert re.search(r"_train_loss\(m, m\.θ,", tl)
    # the cache / params the caller passes must be the ones the executor was built for
    assert "check_config(m, cache, params)" in tl
    cc = _function_body(jl, r"function check_config\(m::HIPModel")
    for field in ("batch_size", "target_size", "min_depth", "max_depth", "disparity_smoothness",
                  "automasking", "target_id", "source_ids", "scales", "cache.K", "cache.invK"):
        assert field in cc, field
    assert "error(" in cc
    body = _function_body(jl, r"function _train_loss\(m::HIPModel")
    # the loss is a host scalar: copied out of the device vector before returning
    assert re.search(r"l = Array\(loss\)\[1\]", body)
    assert "return (l, nothing, nothing, nothing)" in body
    # visualisation outputs are host arrays (cpu(...) in the reference)
    ret = body[body.rindex("return (l,"):]
    assert ret.count("Array(") == 4, ret
    # the rrule: θ tangent = a fresh array in θ's layout (the library gradient), m itself untangented
    rr = _function_body(jl, r"function ChainRulesCore\.rrule\(::typeof\(_train_loss\)")
    assert re.search(r"return \(NoTangent\(\), NoTangent\(\), copy\(m\.∇θ\),", rr)
    assert "Tangent{HIPModel}" not in rr
    # Flux.params(m) is exactly [m.θ]
    assert re.search(r"Flux\.@functor HIPModel \(θ,\)", jl)
    assert re.search(r"Flux\.trainable\(m::HIPModel\) = \(θ = m\.θ,\)", jl)
    # after an update of θ outside the library the packed weights are refreshed before use
    assert "m.packed || repack!(m)" in body


def test_abi_version_pinned_in_every_binding():
    """The header's MD2_ABI_VERSION is what both bindings refuse to run without."""
    hdr = open(HDR).read()
    v = int(re.search(r"#define MD2_ABI_VERSION (\d+)", hdr).group(1))
    jl = open(JL).read()
    assert int(re.search(r"const ABI_VERSION = (\d+)", jl).group(1)) == v
    assert "function __init__()" in jl and "md2_abi_version" in jl
    import sys
    sys.path.insert(0, os.path.join(ROOT, "monodepth2.jl_amd"))
    from md2hip import _lib
    assert _lib.ABI_VERSION == v


def test_comm_init_waits_with_a_timeout(sources):
    jl, _ = sources
    body = _function_body(jl, r"function comm_init\(")
    assert "timeout_s" in body and re.search(r"time\(\) - t0 > timeout_s && error\(", body)
