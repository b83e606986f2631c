"""ORACLE (second, independent restatement) — TEST INFRASTRUCTURE ONLY.

A pure-Python restatement of the xymeng16/dcf PRG / gen / eval that shares no
code with ``oracle/dcf_oracle.c``: AES-256 comes from OpenSSL libcrypto
(EVP aes-256-ecb, via ctypes), the DCF logic is written directly from the Rust
source.  Used only in ``-m "not gpu"`` tests to cross-check the C oracle and to
(re)generate the committed golden vectors (tests/golden/make_golden.py).
Small inputs only: it is a Python loop.
"""
from __future__ import annotations

import ctypes
import ctypes.util

_crypto = None


def _libcrypto():
    global _crypto
    if _crypto is None:
        name = ctypes.util.find_library("crypto")
        if not name:
            raise RuntimeError("libcrypto not found")
        c = ctypes.CDLL(name)
        c.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        c.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        c.EVP_aes_256_ecb.restype = ctypes.c_void_p
        c.EVP_aes_128_ecb.restype = ctypes.c_void_p
        c.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                         ctypes.c_char_p]
        c.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
        c.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                        ctypes.c_char_p, ctypes.c_int]
        _crypto = c
    return _crypto


class Aes256Ecb:
    def __init__(self, key: bytes):
        assert len(key) in (16, 32)
        c = _libcrypto()
        self._c = c
        self._ctx = c.EVP_CIPHER_CTX_new()
        cipher = c.EVP_aes_256_ecb() if len(key) == 32 else c.EVP_aes_128_ecb()
        assert c.EVP_EncryptInit_ex(self._ctx, cipher, None, key, None) == 1
        c.EVP_CIPHER_CTX_set_padding(self._ctx, 0)

    def encrypt(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(len(data) + 32)
        n = ctypes.c_int(0)
        assert self._c.EVP_EncryptUpdate(self._ctx, out, ctypes.byref(n), data, len(data)) == 1
        return out.raw[: n.value]

    def __del__(self):
        if getattr(self, "_ctx", None):
            self._c.EVP_CIPHER_CTX_free(self._ctx)
            self._ctx = None


def _xor(*arrs: bytes) -> bytes:
    out = bytearray(len(arrs[0]))
    for a in arrs:
        for i, b in enumerate(a):
            out[i] ^= b
    return bytes(out)


class HirosePrg:
    """Aes256HirosePrg (prg.rs:22-74), generic LAMBDA."""

    def __init__(self, keys, lam: int):
        self.lam = lam
        self.ciphers = [Aes256Ecb(bytes(k)) for k in keys]

    def gen(self, seed: bytes):
        lam = self.lam
        seed_p = bytes(b ^ 0xFF for b in seed)
        buf0 = [bytearray(lam), bytearray(lam)]
        buf1 = [bytearray(lam), bytearray(lam)]
        for i, j in zip(range(2), range(lam // 16)):
            c = self.ciphers[i * 16 + j]
            out = c.encrypt(seed[j * 16:(j + 1) * 16] + seed_p[j * 16:(j + 1) * 16])
            buf0[i][j * 16:(j + 1) * 16] = out[:16]
            buf1[i][j * 16:(j + 1) * 16] = out[16:]
        buf0 = [bytearray(_xor(b, seed)) for b in buf0]
        buf1 = [bytearray(_xor(b, seed_p)) for b in buf1]
        bit0 = bool(buf0[0][0] & 1)
        bit1 = bool(buf1[0][0] & 1)
        for b in buf0 + buf1:
            b[lam - 1] &= 0xFE
        return [(bytes(buf0[0]), bytes(buf1[0]), bit0), (bytes(buf0[1]), bytes(buf1[1]), bit1)]


class MmoPrg:
    """Aes128MatyasMeyerOseasPrg (ours; the reference has none): out_b = AES128_{k_b}(seed) ^ seed
    blockwise for b = s_L, v_L, s_R, v_R; t from bit 0 of byte 0 of s_L / s_R; the last
    byte's bit 0 cleared as in prg.rs:63-68."""

    def __init__(self, keys, lam: int):
        self.lam = lam
        self.ciphers = [Aes256Ecb(bytes(k)) for k in keys]  # 16-byte keys -> AES-128

    def gen(self, seed: bytes):
        lam, nb = self.lam, self.lam // 16
        outs = []
        for b in range(4):
            o = bytearray()
            for j in range(nb):
                blk = seed[16 * j:16 * (j + 1)]
                o += _xor(self.ciphers[b * nb + j].encrypt(blk), blk)
            outs.append(o)
        tl, tr = bool(outs[0][0] & 1), bool(outs[2][0] & 1)
        for o in outs:
            o[lam - 1] &= 0xFE
        return [(bytes(outs[0]), bytes(outs[1]), tl), (bytes(outs[2]), bytes(outs[3]), tr)]


def _bit_msb0(b: bytes, i: int) -> bool:
    return bool((b[i // 8] >> (7 - i % 8)) & 1)


def gen(prg: HirosePrg, alpha: bytes, beta: bytes, s0s, bound: int):
    """DcfImpl::gen (lib.rs:86-161).  bound 0 = LtBeta, 1 = GtBeta.
    Returns (cws, cw_np1) with cws a list of (s, v, tl, tr)."""
    lam, n = prg.lam, 8 * len(alpha)
    v_alpha = bytes(lam)
    ss = [bytes(s0s[0]), bytes(s0s[1])]
    ts = [False, True]
    cws = []
    zero = bytes(lam)
    for i in range(1, n + 1):
        (s0l, v0l, t0l), (s0r, v0r, t0r) = prg.gen(ss[0])
        (s1l, v1l, t1l), (s1r, v1r, t1r) = prg.gen(ss[1])
        a = _bit_msb0(alpha, i - 1)
        keep, lose = (1, 0) if a else (0, 1)
        s_cw = _xor([s0l, s0r][lose], [s1l, s1r][lose])
        v_cw = _xor([v0l, v0r][lose], [v1l, v1r][lose], v_alpha)
        if (bound == 0 and lose == 0) or (bound == 1 and lose == 1):
            v_cw = _xor(v_cw, beta)
        v_alpha = _xor(v_alpha, [v0l, v0r][keep], [v1l, v1r][keep], v_cw)
        tl_cw = t0l ^ t1l ^ a ^ True
        tr_cw = t0r ^ t1r ^ a
        cws.append((s_cw, v_cw, tl_cw, tr_cw))
        tk = [tl_cw, tr_cw][keep]
        ns = [_xor([s0l, s0r][keep], s_cw if ts[0] else zero), _xor([s1l, s1r][keep], s_cw if ts[1] else zero)]
        nt = [[t0l, t0r][keep] ^ (ts[0] & tk), [t1l, t1r][keep] ^ (ts[1] & tk)]
        ss, ts = ns, nt
    cw_np1 = _xor(ss[0], ss[1], v_alpha)
    return cws, cw_np1


def eval_(prg: HirosePrg, b: bool, s0: bytes, cws, cw_np1: bytes, xs):
    """DcfImpl::eval (lib.rs:163-204) for a list of byte strings xs."""
    lam = prg.lam
    zero = bytes(lam)
    ys = []
    for x in xs:
        s, t, v = bytes(s0), bool(b), bytes(lam)
        for i in range(1, len(cws) + 1):
            cs, cv, ctl, ctr = cws[i - 1]
            (sl, vl, tl), (sr, vr, tr) = prg.gen(s)
            sl = _xor(sl, cs if t else zero)
            sr = _xor(sr, cs if t else zero)
            tl ^= t & ctl
            tr ^= t & ctr
            if _bit_msb0(x, i - 1):
                v = _xor(v, vr, cv if t else zero)
                s, t = sr, tr
            else:
                v = _xor(v, vl, cv if t else zero)
                s, t = sl, tl
        v = _xor(v, s, cw_np1 if t else zero)
        ys.append(v)
    return ys
