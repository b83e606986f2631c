"""Oracle checks (CPU only): the C restatement against FIPS-197, libcrypto, the
independent Python restatement, the committed golden vectors and the
reference's own tests (lib.rs:372-442, prg.rs:86-96) with fixed seeds."""
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from oracle import pyref as R
from tests.golden.make_golden import REF_ALPHAS, REF_BETA, REF_KEYS, REF_PRG_SEED, detbytes


def test_aes256_fips197_and_kat(golden):
    for v in golden("aes256_kat"):
        key, pt, ct = (bytes.fromhex(v[k]) for k in ("key", "pt", "ct"))
        assert O.aes256_encrypt(key, pt) == ct
        assert R.Aes256Ecb(key).encrypt(pt) == ct


@pytest.mark.parametrize("name,lam", [("prg16", 16), ("prg32", 32)])
@pytest.mark.parametrize("aesni", [True, False])
def test_prg_golden(golden, name, lam, aesni):
    g = golden(name)
    P = O.OraclePrg([bytes.fromhex(k) for k in g["keys"]], lam, allow_aesni=aesni)
    for r in g["rows"]:
        (sl, vl, tl), (sr, vr, tr) = P.gen(bytes.fromhex(r["seed"]))
        assert (sl.hex(), vl.hex(), tl, sr.hex(), vr.hex(), tr) == (r["sl"], r["vl"], r["tl"], r["sr"], r["vr"], r["tr"])


def test_prg_quirks_lambda16():
    """prg.rs:42-73 at LAMBDA=16: right child is the seed itself (masked), key 1 unused."""
    P = O.OraclePrg(REF_KEYS, 16)
    P2 = O.OraclePrg([REF_KEYS[0], bytes(32)], 16)  # ciphers[1] never read
    seed = REF_PRG_SEED
    (sl, vl, tl), (sr, vr, tr) = P.gen(seed)
    assert P2.gen(seed) == P.gen(seed)
    m = bytearray(seed)
    m[15] &= 0xFE
    assert sr == bytes(m)
    assert vr == bytes((b ^ 0xFF) for b in m[:15]) + bytes([(seed[15] ^ 0xFF) & 0xFE])
    assert sl[15] & 1 == 0 and vl[15] & 1 == 0


def test_prg_not_zeros():
    """prg.rs:86-96."""
    P = O.OraclePrg(REF_KEYS, 16)
    out = P.gen(REF_PRG_SEED)
    for i in range(2):
        assert out[i][0] != bytes(16) and out[i][1] != bytes(16)
        assert bytes(a ^ b for a, b in zip(out[i][0], REF_PRG_SEED)) != bytes(16)
        assert bytes(a ^ b for a, b in zip(out[i][1], REF_PRG_SEED)) != bytes(16)


def test_cipher_n_too_small_rejected():
    """The reference panics at ciphers[i*16+j] (prg.rs:51)."""
    with pytest.raises(ValueError):
        O.OraclePrg([bytes(32)] * 17, 32)
    with pytest.raises(ValueError):
        O.OraclePrg([bytes(32)] * 2, 24)


def _key_to_cwb(k):
    cwb = k.cw_s.tobytes() + k.cw_v.tobytes() + k.cw_t.tobytes()
    return cwb + bytes((-len(cwb)) % 16) + k.cw_np1.tobytes()


def test_dcf_golden_cases(golden):
    for c in golden("dcf_cases"):
        lam, nb = c["lambda"], c["n_bytes"]
        if "keys" in c:
            keys = [bytes.fromhex(k) for k in c["keys"]]
            xs = [bytes.fromhex(x) for x in c["xs"]]
        else:
            keys = [detbytes(c["keys_fmt"].format(i=i), 32) for i in range(c["cipher_n"])]
            xs = [detbytes(c["xs_fmt"].format(i=i), nb) for i in range(c["m"])]
        P = O.OraclePrg(keys, lam)
        s0s = [bytes.fromhex(s) for s in c["s0s"]]
        k = O.gen(P, bytes.fromhex(c["alpha"]), bytes.fromhex(c["beta"]), s0s[0], s0s[1], c["bound"])
        assert hashlib.sha256(_key_to_cwb(k)).hexdigest() == c["cwb_sha256"], c["name"]
        xa = np.frombuffer(b"".join(xs), np.uint8).reshape(-1, nb)
        y0 = O.eval_(P, 0, k, s0s[0], xa, nthreads=2)
        y1 = O.eval_(P, 1, k, s0s[1], xa, nthreads=1)
        assert hashlib.sha256(y0.tobytes()).hexdigest() == c["y0_sha256"], c["name"]
        assert hashlib.sha256(y1.tobytes()).hexdigest() == c["y1_sha256"], c["name"]


@pytest.mark.parametrize("bound,expect", [(0, [1, 1, 0, 0, 0]), (1, [0, 0, 0, 1, 1])])
def test_reference_reconstruction_kat(bound, expect):
    """lib.rs:372-395 (LtBeta) and lib.rs:397-420 (GtBeta), seeds fixed, plus the
    not-zeros check of lib.rs:422-442."""
    P = O.OraclePrg(REF_KEYS, 16)
    for trial in range(4):
        s0s = [detbytes(f"kat/{trial}/0", 16), detbytes(f"kat/{trial}/1", 16)]
        k = O.gen(P, REF_ALPHAS[2], REF_BETA, s0s[0], s0s[1], bound)
        xa = np.frombuffer(b"".join(REF_ALPHAS), np.uint8).reshape(5, 16)
        y0 = O.eval_(P, 0, k, s0s[0], xa)
        y1 = O.eval_(P, 1, k, s0s[1], xa)
        for i, e in enumerate(expect):
            assert (y0[i] ^ y1[i]).tobytes() == (REF_BETA if e else bytes(16))
        assert y0[2].tobytes() != bytes(16) and y1[2].tobytes() != bytes(16)


def test_c_oracle_matches_python_restatement_random():
    rng = np.random.default_rng(7)
    for lam, nkeys in ((16, 2), (48, 18)):
        keys = [rng.bytes(32) for _ in range(nkeys)]
        P, Q = O.OraclePrg(keys, lam), R.HirosePrg(keys, lam)
        for nb in (1, 2):
            alpha, beta = rng.bytes(nb), rng.bytes(lam)
            s0s = [rng.bytes(lam), rng.bytes(lam)]
            for bound in (0, 1):
                k = O.gen(P, alpha, beta, s0s[0], s0s[1], bound)
                cws, np1 = R.gen(Q, alpha, beta, s0s, bound)
                assert np1 == k.cw_np1.tobytes()
                xs = [rng.bytes(nb) for _ in range(6)]
                y = O.eval_(P, 1, k, s0s[1], np.frombuffer(b"".join(xs), np.uint8).reshape(-1, nb))
                assert [r.tobytes() for r in y] == R.eval_(Q, True, s0s[1], cws, np1, xs)


def test_eval_threads_and_empty():
    P = O.OraclePrg(REF_KEYS, 16)
    k = O.gen(P, REF_ALPHAS[0], REF_BETA, bytes(16), b"\x01" * 16, 0)
    xa = np.frombuffer(detbytes("thr", 16 * 37), np.uint8).reshape(37, 16)
    assert (O.eval_(P, 0, k, bytes(16), xa, 1) == O.eval_(P, 0, k, bytes(16), xa, 5)).all()
    assert O.eval_(P, 0, k, bytes(16), xa[:0]).shape == (0, 16)
