"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end for ``oracle/build/libdcf_oracle.so`` (the C restatement of the
xymeng16/dcf hot path in ``oracle/dcf_oracle.c``).  Imported only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, as the
checker; the product (``dcf_amd``) never imports it.

Parity status: PARITY UNPINNED against bytes produced by the reference itself (the
Rust crate cannot be built here and its tests hold no output vectors).  What pins
it: the FIPS-197 AES-256 known-answer vector, libcrypto, the independent
restatement in ``oracle/pyref.py`` (every golden vector is written only when both
agree) and the reference's own reconstruction tests (lib.rs:372-442,
prg.rs:86-96).  See DESIGN.md "Oracle".
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DCF_ORACLE_LIB: another build of the same source (scripts/host_sanitize.sh: ASan + UBSan)
_LIB_PATH = os.environ.get("DCF_ORACLE_LIB") or os.path.join(_HERE, "build", "libdcf_oracle.so")
_lib = None

LT_BETA = 0
GT_BETA = 1


def build() -> str:
    """Compile the oracle (gcc) if it is missing or stale."""
    src = os.path.join(_HERE, "dcf_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_prg_new.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(P)]
        L.orc_prg_new.restype = ctypes.c_int
        L.orc_mmo_prg_new.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(P)]
        L.orc_mmo_prg_new.restype = ctypes.c_int
        L.orc_aes128_expand.argtypes = [u8p, u8p]
        L.orc_aes128_expand.restype = None
        L.orc_aes128_encrypt_portable.argtypes = [u8p, u8p, u8p]
        L.orc_aes128_encrypt_portable.restype = None
        L.orc_prg_free.argtypes = [P]
        L.orc_prg_free.restype = None
        L.orc_prg_uses_aesni.argtypes = [P]
        L.orc_prg_uses_aesni.restype = ctypes.c_int
        L.orc_prg_gen.argtypes = [P, u8p, u8p, u8p, u8p, u8p, u8p]
        L.orc_prg_gen.restype = ctypes.c_int
        L.orc_aes256_expand.argtypes = [u8p, u8p]
        L.orc_aes256_expand.restype = None
        L.orc_aes256_encrypt_portable.argtypes = [u8p, u8p, u8p]
        L.orc_aes256_encrypt_portable.restype = None
        L.orc_gen.argtypes = [P, ctypes.c_size_t, u8p, u8p, u8p, u8p, ctypes.c_int, u8p, u8p, u8p, u8p]
        L.orc_gen.restype = ctypes.c_int
        L.orc_eval.argtypes = [P, ctypes.c_size_t, ctypes.c_int, u8p, u8p, u8p, u8p, u8p, u8p,
                               ctypes.c_size_t, u8p, ctypes.c_int]
        L.orc_eval.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _u8(b) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(bytes(b), dtype=np.uint8)) if isinstance(b, (bytes, bytearray)) \
        else np.ascontiguousarray(b, dtype=np.uint8)


def aes256_encrypt(key: bytes, block: bytes) -> bytes:
    rk = np.zeros(240, np.uint8)
    k = _u8(key)
    lib().orc_aes256_expand(_p(k), _p(rk))
    out = np.zeros(16, np.uint8)
    lib().orc_aes256_encrypt_portable(_p(rk), _p(_u8(block)), _p(out))
    return out.tobytes()


def aes128_encrypt(key: bytes, block: bytes) -> bytes:
    rk = np.zeros(176, np.uint8)
    lib().orc_aes128_expand(_p(_u8(key)), _p(rk))
    out = np.zeros(16, np.uint8)
    lib().orc_aes128_encrypt_portable(_p(rk), _p(_u8(block)), _p(out))
    return out.tobytes()


class OraclePrg:
    """Aes256HirosePrg<LAMBDA, CIPHER_N> (prg.rs:22-74)."""
    KEY_BYTES = 32

    def __init__(self, keys, lam: int, allow_aesni: bool = True):
        keys = [bytes(k) for k in keys]
        assert all(len(k) == self.KEY_BYTES for k in keys)
        self.lam = lam
        self.cipher_n = len(keys)
        self._keys = _u8(b"".join(keys))
        h = ctypes.c_void_p()
        rc = self._new(_p(self._keys), self.cipher_n, lam, int(allow_aesni), ctypes.byref(h))
        if rc != 0:
            raise ValueError(f"prg constructor failed rc={rc}")
        self._h = h

    @staticmethod
    def _new(*args):
        return lib().orc_prg_new(*args)

    @property
    def uses_aesni(self) -> bool:
        return bool(lib().orc_prg_uses_aesni(self._h))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_prg_free(self._h)
            self._h = None

    def gen(self, seed: bytes):
        """Returns [(s_l, v_l, t_l), (s_r, v_r, t_r)] like Prg::gen (lib.rs:52-54)."""
        lam = self.lam
        outs = [np.zeros(lam, np.uint8) for _ in range(4)]
        t = np.zeros(2, np.uint8)
        rc = lib().orc_prg_gen(self._h, _p(_u8(seed)), *[_p(o) for o in outs], _p(t))
        assert rc == 0
        return [(outs[0].tobytes(), outs[1].tobytes(), bool(t[0])),
                (outs[2].tobytes(), outs[3].tobytes(), bool(t[1]))]


class OracleMmoPrg(OraclePrg):
    """Aes128MatyasMeyerOseasPrg<LAMBDA, CIPHER_N> (BASELINE.json north_star; not in the
    reference, parity unpinned): CIPHER_N >= 4 * LAMBDA / 16 AES-128 keys."""
    KEY_BYTES = 16

    @staticmethod
    def _new(*args):
        return lib().orc_mmo_prg_new(*args)


class OracleKey:
    """Correction words of one key in the SoA layout of include/dcf_hip.h."""

    def __init__(self, n_bytes: int, lam: int):
        n = 8 * n_bytes
        self.n_bytes, self.lam = n_bytes, lam
        self.cw_s = np.zeros((n, lam), np.uint8)
        self.cw_v = np.zeros((n, lam), np.uint8)
        self.cw_t = np.zeros(n, np.uint8)
        self.cw_np1 = np.zeros(lam, np.uint8)


def gen(prg: OraclePrg, alpha: bytes, beta: bytes, s0_0: bytes, s0_1: bytes, bound: int) -> OracleKey:
    """DcfImpl::gen (lib.rs:86-161)."""
    n_bytes = len(alpha)
    k = OracleKey(n_bytes, prg.lam)
    rc = lib().orc_gen(prg._h, n_bytes, _p(_u8(alpha)), _p(_u8(beta)), _p(_u8(s0_0)), _p(_u8(s0_1)), int(bound),
                       _p(k.cw_s), _p(k.cw_v), _p(k.cw_t), _p(k.cw_np1))
    if rc != 0:
        raise ValueError(f"orc_gen rc={rc}")
    return k


def eval_(prg: OraclePrg, party: int, key: OracleKey, s0: bytes, xs: np.ndarray, nthreads: int = 1) -> np.ndarray:
    """DcfImpl::eval (lib.rs:163-204).  xs: (m, N) uint8 -> ys: (m, lambda) uint8."""
    xs = np.ascontiguousarray(xs, dtype=np.uint8)
    m = xs.shape[0]
    assert xs.shape[1] == key.n_bytes
    ys = np.zeros((m, prg.lam), np.uint8)
    rc = lib().orc_eval(prg._h, key.n_bytes, int(party), _p(_u8(s0)), _p(key.cw_s), _p(key.cw_v), _p(key.cw_t),
                        _p(key.cw_np1), _p(xs) if m else None, m, _p(ys) if m else None, int(nthreads))
    if rc != 0:
        raise ValueError(f"orc_eval rc={rc}")
    return ys
