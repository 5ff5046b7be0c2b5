"""CPU tests of the C ABI boundary: librankops.so loads, exports every function declared in
include/*.h, the ctypes struct layouts match what a C compiler makes of the header,
and argument validation fails loudly (no device work is started on invalid input)."""
import ctypes
import glob
import os
import re
import subprocess
import tempfile

import pytest

import helpers as H
from rankops import _lib

HEADER = os.path.join(H.REPO, "include", "rankops.h")
HEADERS = sorted(glob.glob(os.path.join(H.REPO, "include", "*.h")))


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rk_[a-z_0-9]+)\s*\(", text, flags=re.M))
    return sorted(names)


def test_library_loads_and_exports_header():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes prototypes cover exactly the declared set
    assert sorted(_lib.SIGNATURES) == names
    assert lib.rk_abi_version() == _lib.ABI_VERSION


def test_exports_are_visible_in_dynamic_symbol_table():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    syms = {line.split()[-1] for line in out.stdout.splitlines() if line.strip()}
    for n in declared_functions():
        assert n in syms, n


STRUCTS = {"rk_segment": _lib.Segment, "rk_epilogue": _lib.Epilogue, "rk_mlp_layer": _lib.MlpLayer}


def test_struct_layouts_match_c_compiler():
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, cls in STRUCTS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "layout.c"), os.path.join(d, "layout")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c99", "-Wall", "-o", exe, src], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {}
    for line in out:
        parts = line.split()
        if len(parts) == 3:
            got[(parts[0], parts[1])] = int(parts[2])
    for cname, cls in STRUCTS.items():
        assert got[(cname, "size")] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert got[(cname, fname)] == getattr(cls, fname).offset, (cname, fname)


def test_invalid_arguments_fail_before_any_launch():
    lib = _lib.load()
    ep = _lib.Epilogue()
    assert lib.rk_linear(None, 0, None, 0, None, 0, 10, 4, 4, ctypes.byref(ep), None, 0, None) == 1
    assert "rk_linear" in _lib.last_error()
    assert lib.rk_concat_gather(None, 0, 8, None, 0, None) == 1
    assert lib.rk_fm_gather(None, None, 40, 8, 8, None, 0, None, None, None) == 4  # > 32 fields: unsupported
    segs = (_lib.Segment * 1)()
    assert lib.rk_afm_forward(segs, 1, 8, 4, None, 0, 0, None, None, None, None, 16, None, None, None, None,
                              None, None, None) == 4
    layer = (_lib.MlpLayer * 1)()
    layer[0].n = 600
    head = _lib.Epilogue()
    head.head_w = 1
    head.head_b = 1
    assert lib.rk_mlp_forward(16, 64, 32, 64, layer, 1, ctypes.byref(head), None, 0, None) == 4
    rows, cols = ctypes.c_int64(), ctypes.c_int64()
    assert lib.rk_mlp_packed_size(50, 114, ctypes.byref(rows), ctypes.byref(cols)) == 0
    assert (rows.value, cols.value) == (64, 128)


def test_error_flags_need_init():
    lib = _lib.load()
    flags = ctypes.c_uint32(0)
    assert lib.rk_error_flags(63, ctypes.byref(flags), 0) == 1


def test_python_layer_refuses_cpu_tensors():
    import torch
    import rankops
    m = H.build("dcn", {})
    inp = H.make_inputs("dcn", {}, 4)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        H.call_model(m, "dcn", inp)
    with pytest.raises(RuntimeError, match="ROCm GPU"):  # DCN trains on the engine, still GPU-only
        H.call_model(m.train(), "dcn", inp)
    bst = H.build("bst", {"T": 8}).train()  # train mode without autograd: refused, never a silent fallback
    with torch.no_grad(), pytest.raises(NotImplementedError):
        H.call_model(bst, "bst", H.make_inputs("bst", {"T": 8}, 4))
    with pytest.raises(RuntimeError, match="ROCm GPU"):  # BST trains on the engine: GPU-only
        H.call_model(bst, "bst", H.make_inputs("bst", {"T": 8}, 4))
    afm = H.build("afm", {}).train()  # trains on the engine: GPU-only like the forward
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        H.call_model(afm, "afm", H.make_inputs("afm", {}, 4))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        rankops.cross_layer(torch.zeros(2, 50), torch.zeros(2, 50), 0)
