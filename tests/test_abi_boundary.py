"""The drop-in boundary cannot drift: every prototype in include/csmom.h is parsed and checked
against the ctypes table the package binds (csmom._lib.SIGNATURES) and against the ctypes
snippets a maintainer copies from INTEGRATION.md (argtypes lists and call sites).  CPU only:
nothing here touches a GPU."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "csmom.h"
INTEGRATION = ROOT / "INTEGRATION.md"


def _strip_comments(txt):
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    return re.sub(r"//[^\n]*", " ", txt)


def header_prototypes():
    """{name: (return C type, [param C types])} of every csm_* declaration."""
    txt = _strip_comments(HEADER.read_text())
    out = {}
    for m in re.finditer(r"(const\s+char\s*\*|int64_t|int)\s+(csm_\w+)\s*\(([^)]*)\)\s*;", txt):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ps = [p.strip() for p in params.split(",")] if params.strip() not in ("", "void") else []
        types = []
        for p in ps:
            p = re.sub(r"\s+", " ", p)
            p = re.sub(r"\s*\w+$", "", p) if not p.endswith("*") else p   # drop the name
            types.append(p.replace(" *", "*").strip())
        out[name] = (re.sub(r"\s+", "", ret), types)
    return out


def c_to_ctypes(t):
    t = t.replace(" ", "")
    if t in ("constchar*",):
        return ctypes.c_char_p
    if t == "csm_ctx**":
        return "ctx_out"
    if t.endswith("*") or "*const*" in t:
        return ctypes.c_void_p
    return {"int": ctypes.c_int, "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64,
            "uint64_t": ctypes.c_uint64, "double": ctypes.c_double,
            "constchar*": ctypes.c_char_p}[t]


def kind(t):
    """Comparable class of a ctypes type: pointer, C string, ctx out-pointer, or
    (signed/unsigned/float, size)."""
    if t == "ctx_out" or getattr(t, "_type_", None) is ctypes.c_void_p:
        return "ctx_out"
    if t is ctypes.c_void_p:
        return "ptr"
    if t is ctypes.c_char_p:
        return "str"
    if t is ctypes.c_double:
        return ("f", 8)
    signed = t(-1).value == -1
    return ("i" if signed else "u", ctypes.sizeof(t))


def same(a, b):
    return kind(a) == kind(b)


def test_header_parses():
    protos = header_prototypes()
    assert len(protos) >= 40
    assert protos["csm_pipeline"][1][0] == "csm_ctx*"
    assert len(protos["csm_pipeline"][1]) == 21


def test_ctypes_table_matches_header():
    from csmom import _lib
    protos = header_prototypes()
    assert set(_lib.SIGNATURES) == set(protos), (set(_lib.SIGNATURES) ^ set(protos))
    for name, (ret, params) in protos.items():
        res, args = _lib.SIGNATURES[name]
        assert len(args) == len(params), (name, len(args), len(params))
        for i, (c, py) in enumerate(zip(params, args)):
            assert same(c_to_ctypes(c), py), (name, i, c, py)
        assert same(c_to_ctypes(ret), res), (name, ret)


def _integration_blocks():
    txt = INTEGRATION.read_text()
    return re.findall(r"```python\n(.*?)```", txt, flags=re.S)


def _split_args(s):
    """Top-level comma split of a call's argument text."""
    depth, cur, out = 0, "", []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _calls(code, name):
    """Argument lists of every `lib.<name>(...)` call in code."""
    out = []
    for m in re.finditer(r"lib\." + name + r"\(", code):
        i, depth = m.end(), 1
        j = i
        while depth:
            depth += {"(": 1, ")": -1}.get(code[j], 0)
            j += 1
        out.append(_split_args(code[i:j - 1]))
    return out


def test_integration_snippets_match_header():
    protos = header_prototypes()
    env = {"ctypes": ctypes, "P_": ctypes.c_void_p, "I32": ctypes.c_int32, "I64": ctypes.c_int64,
           "F64": ctypes.c_double, "U64": ctypes.c_uint64}
    blocks = _integration_blocks()
    assert blocks
    seen_argtypes = seen_calls = 0
    for code in blocks:
        code = re.sub(r"#[^\n]*", "", code)
        for m in re.finditer(r"lib\.(csm_\w+)\.argtypes\s*=\s*(\[.*?\])", code, flags=re.S):
            name = m.group(1)
            assert name in protos, name
            args = eval(m.group(2), env)   # noqa: S307 -- the repo's own documentation
            params = protos[name][1]
            assert len(args) == len(params), (name, len(args), len(params))
            for i, (c, py) in enumerate(zip(params, args)):
                assert same(c_to_ctypes(c), py), (name, i, c, py)
            seen_argtypes += 1
        for name in protos:
            for args in _calls(code, name):
                assert len(args) == len(protos[name][1]), (name, len(args), args)
                seen_calls += 1
    assert seen_argtypes >= 6 and seen_calls >= 6


def test_library_exports_match_header():
    import csmom
    try:
        raw = ctypes.CDLL(str(csmom.lib_path()))
    except OSError as e:   # pragma: no cover
        pytest.skip(f"library not loadable here: {e}")
    for name in header_prototypes():
        assert hasattr(raw, name), name
