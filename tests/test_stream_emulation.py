"""CPU emulation of one stream of k_eval16_stream (dcf_amd/csrc/kernels_stream.h, single key, x words
in registers, no shared prefix) against the second oracle restatement (oracle/pyref.py,
lib.rs:163-204): the per-step B / A slot schedule and B reuse after a right step at t = 0.
Word-level transcription of the kernel's update (same masks and order), so a schedule bug shows
up here as wrong bytes or a level past 8N — the GPU tests pin the kernel itself.  run=True
transcribes the DCF_REUSE_RUN form: after a reused right step that left t = 0, a whole run of right
steps (and the left step ending it) takes no AES slot."""
import random

import pytest

from oracle import pyref

M3 = 0xFEFFFFFF  # kMaskLast: bit 0 of byte 15 in little-endian word 3
F = 0xFFFFFFFF


def _w(b: bytes):
    return [int.from_bytes(b[4 * i:4 * i + 4], "little") for i in range(4)]


def _b(w):
    return b"".join(x.to_bytes(4, "little") for x in w)


def _bswap(x):
    return int.from_bytes(x.to_bytes(4, "little"), "big")


def stream_eval(aes, party, s0, cws, np1, x, counts, run=False):
    nb = len(x)
    nlev = 8 * nb
    raw = x + bytes((-nb) % 4) + bytes(16)
    xw = [int.from_bytes(raw[4 * k:4 * k + 4], "little") if 4 * k < nb else 0 for k in range(4)]
    cw = [(_w(c[0]), _w(c[1]), int(c[2]) | (int(c[3]) << 1)) for c in cws]
    s, v, t = _w(s0), [0, 0, 0, 0], int(party)
    ph, lev, cur, fresh = 0, 0, 0, True
    enc = lambda w: _w(aes.encrypt(_b(w)))  # noqa: E731
    msk = [F, F, F, M3]

    def next_word():
        nonlocal cur
        cur = _bswap(xw[0])
        xw[0], xw[1], xw[2] = xw[1], xw[2], xw[3]

    while lev < nlev:
        counts[0] += 1
        cs, cv, ct = cw[lev]
        c2 = lev + (1 if lev + 1 < nlev else 0)
        cs2, cv2, ct2 = cw[c2]
        maybe = ph == 0 and t == 0 and not fresh and (cur >> 31) != 0 and lev + 1 < nlev
        inv = (ph - 1) & F
        st = enc([w ^ inv for w in s])
        if fresh:
            next_word()
            fresh = False
        p, xb = ph, cur >> 31
        adv = p | xb
        keepB = (xb - 1) & F
        tm, am, pm = (-t) & F, (-adv) & F, (-p) & F
        d = [st[j] ^ s[j] ^ inv for j in range(4)]
        d0 = d[0]
        reuse = maybe and (s[3] & ~M3 & F) == 0
        for j in range(4):
            inn = s[j] ^ inv
            vhat = (inn ^ (st[j] & keepB)) & msk[j]
            v[j] ^= inv & (vhat ^ (tm & cv[j]))
            sx = s[j] ^ (st[j] & pm)
            sn = (sx & msk[j]) ^ (tm & cs[j])
            s[j] = (am & sn) | (~am & F & s[j])
        tb = (d0 ^ (t & (ct >> xb))) & 1
        t = tb if adv else t
        ph = adv ^ 1
        nl = lev + adv
        cur = (cur << adv) & F
        if adv and (nl & 31) == 0:
            next_word()
        # reuse (branch-free form)
        xb2, t1 = cur >> 31, t
        tm1 = (-t1) & F
        rm = F if reuse else 0
        rr = rm & ((-xb2) & F)
        for j in range(4):
            v[j] ^= rm & ((((~s[j] & F) if xb2 else d[j]) & msk[j]) ^ (tm1 & cv2[j]))
            s[j] ^= rr & tm1 & cs2[j]
        if rr:
            t = (d0 ^ (t1 & (ct2 >> 1))) & 1
        if reuse and not xb2:
            ph = 1
        nl += rr & 1
        cur = (cur << (rr & 1)) & F
        if rr and (nl & 31) == 0:
            next_word()
        if run:  # DCF_REUSE_RUN
            go = bool(rr) and t1 == 0 and (nl & 31) != 0 and nl < nlev
            k = min(32 - ((~cur) & F).bit_length(), nlev - nl) if go else 0
            ko = F if k & 1 else 0
            nl += k
            cur = (cur << k) & F
            lm = F if (go and nl < nlev and (nl & 31) != 0) else 0
            for j in range(4):
                v[j] ^= ((ko & ~s[j] & F) ^ (lm & d[j])) & msk[j]
            if lm:
                ph = 1
            if go and k and (nl & 31) == 0 and nl < nlev:
                next_word()
        assert nl <= nlev, (nl, nlev)
        lev = nl
    np_ = _w(np1)
    return _b([v[j] ^ s[j] ^ (np_[j] if t else 0) for j in range(4)])


@pytest.mark.parametrize("run", [False, True], ids=["reuse1", "reuse_run"])
@pytest.mark.parametrize("nb", [1, 2, 3, 4, 5, 8, 16])
def test_stream_schedule_matches_oracle(nb, run):
    rnd = random.Random(0x57E4 + nb)
    lam = 16
    keys = [rnd.randbytes(32) for _ in range(2)]
    prg = pyref.HirosePrg(keys, lam)
    aes = pyref.Aes256Ecb(keys[0])
    alpha, beta = rnd.randbytes(nb), rnd.randbytes(lam)
    s0s = [rnd.randbytes(lam), rnd.randbytes(lam)]
    cws, np1 = pyref.gen(prg, alpha, beta, s0s, nb % 2)
    m = 48 if nb == 16 else 40
    # random points, points ending in a run of 1 bits (a reused right step can end the walk there),
    # all-ones / all-zeros, alpha
    xs = [rnd.randbytes(nb) for _ in range(m)] + [rnd.randbytes(nb - 1) + b"\xff" for _ in range(m)]
    xs += [b"\xff" * nb, bytes(nb), alpha, bytes(max(0, nb - 1)) + b"\x7f", b"\x0f" * nb]
    xs += [bytes([0x80 | rnd.getrandbits(7)]) + b"\xff" * (nb - 1) for _ in range(8)]  # long right runs
    counts = [0]
    for party in (0, 1):
        ref = pyref.eval_(prg, bool(party), s0s[party], cws, np1, xs)
        got = [stream_eval(aes, party, s0s[party], cws, np1, x, counts, run) for x in xs]
        assert got == ref
    assert counts[0] < 2 * len(xs) * 2 * 8 * nb
