"""CPU checks of the C-ABI boundary (include/lthm.h <-> liblthm_hip.so <-> ctypes).

No compute calls: the library is loaded and inspected only.  Struct layouts
are compared field by field against a probe compiled by gcc from the header
itself, which is what a cgo / JNI / ctypes integrator binds.
"""
import ctypes
import os
import re
import subprocess

import pytest
import torch

from recommendations_amd import _lib


def test_every_header_symbol_is_exported():
    lib = _lib.load()
    protos = _lib.parse_header()
    assert len(protos) >= 30 and "lthm_kshift_fwd" in protos and "lthm_gemm" in protos
    missing = [n for n in protos if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_matches_header():
    lib = _lib.load()
    with open(_lib.HEADER) as f:
        want = int(re.search(r"#define\s+LTHM_ABI_VERSION\s+(\d+)", f.read()).group(1))
    assert lib.lthm_abi_version() == want


def test_device_count_never_fails():
    n = _lib.load().lthm_device_count()
    assert n >= 0
    if not torch.cuda.is_available():
        assert n == 0


def test_struct_layouts_match_c(tmp_path):
    structs = _lib.STRUCTS
    assert {"lthm_gemm_desc", "lthm_attn_desc", "lthm_ptower_desc", "lthm_tokens_desc",
            "lthm_contrastive_desc"} <= set(structs)
    lines = ['#include "%s"' % _lib.HEADER, "#include <stdio.h>", "#include <stddef.h>", "int main(void) {"]
    for name, cls in structs.items():
        lines.append(f'  printf("{name} sizeof %zu\\n", sizeof({name}));')
        for fname, _ in cls._fields_:
            lines.append(f'  printf("{name} {fname} %zu\\n", offsetof({name}, {fname}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, out):
        sname, field, val = line.split()
        cls = structs[sname]
        got = ctypes.sizeof(cls) if field == "sizeof" else getattr(cls, field).offset
        assert got == int(val), (sname, field, got, val)


def test_header_compiles_as_cxx(tmp_path):
    src = tmp_path / "probe.cpp"
    src.write_text('#include "%s"\nint (*volatile f)(void) = lthm_abi_version;\nint main() { return f ? 0 : 1; }\n' % _lib.HEADER)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", str(src)], check=True)


def test_product_path_refuses_cpu_tensors():
    from recommendations_amd import kernels as K
    with pytest.raises(RuntimeError, match="MI355X"):
        K.kshift(torch.zeros((4, 1), dtype=torch.int64), torch.zeros((10, 8)), 10, 4, 0)
