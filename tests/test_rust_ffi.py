"""The Rust FFI crate (rust/dcf-hip) cannot be compiled here (no cargo or
rustc in the image), so this checks what can be checked without it: its extern block
declares every function of include/dcf_hip.h with the same parameter count, and no
function the header lacks."""
import os
import re

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dcf_hip.h")
FFI = os.path.join(ROOT, "rust", "dcf-hip", "src", "ffi.rs")


def _arity(params: str) -> int:
    params = params.strip()
    if params in ("", "void"):
        return 0
    return params.count(",") + 1


def header_sigs():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return {m.group(1): _arity(m.group(2))
            for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(dcf_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.M)}


def rust_sigs():
    src = open(FFI).read()
    block = src[src.index('extern "C"'):]
    return {m.group(1): _arity(m.group(2)) for m in re.finditer(r"pub fn (dcf_\w+)\s*\(([^)]*)\)", block, flags=re.S)}


def test_rust_ffi_matches_header():
    h, r = header_sigs(), rust_sigs()
    assert h, "no functions parsed from the header"
    assert set(h) == set(r), (set(h) ^ set(r))
    for name, n in h.items():
        assert r[name] == n, (name, n, r[name])


def test_rust_crate_files_present():
    for f in ("Cargo.toml", "build.rs", "src/lib.rs", "src/ffi.rs", "tests/reference_tests.rs"):
        assert os.path.exists(os.path.join(ROOT, "rust", "dcf-hip", f)), f
    lib = open(os.path.join(ROOT, "rust", "dcf-hip", "src", "lib.rs")).read()
    assert "impl<const N: usize, const LAMBDA: usize> Dcf<N, LAMBDA> for DcfHip<N, LAMBDA>" in lib
