"""C-ABI checks that need no GPU: the library builds for gfx950, loads, exports
every function include/dcf_hip.h declares, and its pure-host helpers / argument
validation behave.  No kernel is launched here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT
from tests.golden.make_golden import REF_ALPHAS, REF_BETA, REF_KEYS

HEADER = os.path.join(ROOT, "include", "dcf_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^[A-Za-z_][\w \*]*?\b(dcf_\w+)\s*\(", src, flags=re.M))


def test_header_declares_expected_api():
    from dcf_amd import _lib
    assert header_functions() == set(_lib.EXPORTS)


def test_library_exports_every_header_symbol(hip_lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", hip_lib._name]).decode()
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = header_functions() - syms
    assert not missing, missing
    for name in header_functions():
        assert getattr(hip_lib, name) is not None


def test_library_is_gfx950_code_object(hip_lib):
    out = subprocess.check_output(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                                   f"--input={hip_lib._name}"], stderr=subprocess.STDOUT).decode() \
        if os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler") else ""
    if out:
        assert "gfx950" in out


def test_version_and_layout_helpers(hip_lib):
    assert b"gfx950" in hip_lib.dcf_version() and b"0.2.0" in hip_lib.dcf_version()  # INTEGRATION.md "ABI version"
    for nb, lam, K in ((16, 16, 1), (4, 16, 7), (3, 32, 5), (2, 16384, 1)):
        n = 8 * nb
        off = hip_lib.dcf_cwb_np1_offset(nb, lam, K)
        assert off == (2 * n * K * lam + n * K + 15) // 16 * 16
        assert hip_lib.dcf_cwb_bytes(nb, lam, K) == off + K * lam
    assert hip_lib.dcf_cwb_bytes(16, 16, 1) == 4240


def test_multikey_launch_split_keeps_indices_32_bit(hip_lib):
    """the multi-key stream engine's point, work-unit and CW-digest-row indices are
    32-bit (kernels_stream.h StreamLane::ci / pt), so each launch holds at most
    min(2^24, 2^31 / P, 2^30 / 8N) keys: 2 * (key * 8N + level + 1) and key * P stay below 2^31."""
    assert hip_lib.dcf_eval_keys_per_launch(0, 64) == 0 and hip_lib.dcf_eval_keys_per_launch(16, 0) == 0
    for nb in (1, 4, 16, 17, 32, 64, 159):
        for ppk in (1, 32, 64, 255, 256, 4096, 1 << 20, 1 << 30, (1 << 31) + 5):
            kpl = hip_lib.dcf_eval_keys_per_launch(nb, ppk)
            n = 8 * nb
            assert kpl == max(1, min(1 << 24, (1 << 31) // ppk, (1 << 30) // n)), (nb, ppk)
            if kpl > 1:
                assert 2 * (kpl * n) <= 1 << 31 and kpl * ppk <= 1 << 31
    assert hip_lib.dcf_eval_keys_per_launch(32, 1) == (1 << 30) // 256  # N = 32: 4 Mi keys, not 2^24


def test_argument_validation_without_gpu(hip_lib):
    h = ctypes.c_void_p()
    keys = b"\x00" * (32 * 18)
    assert hip_lib.dcf_hirose_prg_new(keys, 18, 24, 0, ctypes.byref(h)) == -2   # lambda % 16
    assert hip_lib.dcf_hirose_prg_new(keys, 17, 32, 0, ctypes.byref(h)) == -3   # prg.rs:51 panic
    assert hip_lib.dcf_hirose_prg_new(keys, 0, 16, 0, ctypes.byref(h)) == -3
    assert hip_lib.dcf_hirose_prg_new(None, 2, 16, 0, ctypes.byref(h)) == -1
    assert b"cipher" in hip_lib.dcf_last_error() or hip_lib.dcf_last_error() != b""
    assert hip_lib.dcf_eval(None, 16, 0, None, 0, None, None, 0, None, 0) == -1
    assert hip_lib.dcf_gen_batch_device(None, 16, 1, None, None, None, None, 0, None, None) == -1


def test_share_cwb_roundtrip_matches_oracle_layout(hip_lib):
    import dcf_amd
    P = O.OraclePrg(REF_KEYS, 16)
    s0s = [b"\x11" * 16, b"\x22" * 16]
    k = O.gen(P, REF_ALPHAS[2], REF_BETA, s0s[0], s0s[1], 0)
    share = dcf_amd.Share(s0s, [dcf_amd.Cw(k.cw_s[i].tobytes(), k.cw_v[i].tobytes(), bool(k.cw_t[i] & 1),
                                           bool(k.cw_t[i] & 2)) for i in range(128)], k.cw_np1.tobytes())
    cwb = dcf_amd.share_to_cwb(share, 16, 16)
    raw = k.cw_s.tobytes() + k.cw_v.tobytes() + k.cw_t.tobytes()
    assert cwb == raw + bytes((-len(raw)) % 16) + k.cw_np1.tobytes()
    back = dcf_amd.cwb_to_share(cwb, 16, 16, s0s)
    assert back == share
    bad = dcf_amd.Share(s0s, share.cws[:-1], share.cw_np1)
    with pytest.raises(dcf_amd.DcfError):  # assert_eq!(k.cws.len(), N * 8), lib.rs:165
        dcf_amd.share_to_cwb(bad, 16, 16)


def test_product_has_no_oracle_dependency():
    """The product package must not import, link or load the oracle."""
    pkg = os.path.join(ROOT, "dcf_amd")
    bad = re.compile(r"(import\s+oracle|from\s+oracle|dcf_oracle|orc_[a-z_]+\(|oracle/)")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".hpp", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not bad.search(txt), f
    so = os.path.join(pkg, "libdcf_hip.so")
    if os.path.exists(so):
        assert b"dcf_oracle" not in open(so, "rb").read()


def test_single_hip_runtime_in_process(hip_lib):
    """torch and libdcf_hip.so must share one libamdhip64 (two runtimes -> 'no device')."""
    maps = {line.split()[-1] for line in open("/proc/self/maps") if "libamdhip64" in line}
    assert len(maps) == 1, maps
