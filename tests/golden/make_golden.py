"""Generate the committed golden vectors under tests/golden/.

Two independent CPU restatements of the reference must agree before anything is
written: the C oracle (oracle/dcf_oracle.c, portable AES and AES-NI) and the
Python/libcrypto restatement (oracle/pyref.py).  The AES layer is additionally
pinned to FIPS-197 C.3.  Constants marked "reference" are decoded from the
reference's own tests (lib.rs:359-370, prg.rs:80-84).

Inputs that are not reference constants come from `detbytes` (SHA-256 in
counter mode), so any test can regenerate them without storing them.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402
from oracle import pyref as R  # noqa: E402

# ---- reference constants (lib.rs:359-370, prg.rs:80-84) ----
REF_KEYS = [
    bytes.fromhex("6a391b5fb358f333ac57151b0831324bb349b990721c4eb5ee3957d3bb40c664"),
    bytes.fromhex("9b15c80fb7bc21719e89b8f70ea0539d4efa0c3b16e4988262fc6479b58c7bc2"),
]
REF_ALPHAS = [
    bytes.fromhex("4ba957f5dd05e9fc3f04f6fb556fa843"),
    bytes.fromhex("c2474bdac6bb999846712266b78c7355"),
    bytes.fromhex("c2474bdac6bb999846712266b78c7356"),
    bytes.fromhex("c2474bdac6bb999846712266b78c7357"),
    bytes.fromhex("ef9697d78f8aa441500ab335b56bff97"),
]
REF_BETA = bytes.fromhex("03119712438ae92381a8dea88f20c0bb")
REF_PRG_SEED = bytes.fromhex("2a4c8f2579125a942a458f242b4e4819")

FIPS197_C3 = {
    "key": bytes(range(32)).hex(),
    "pt": "00112233445566778899aabbccddeeff",
    "ct": "8ea2b7ca516745bfeafc49904b496089",
}


def detbytes(tag: str, n: int) -> bytes:
    out = bytearray()
    ctr = 0
    while len(out) < n:
        out += hashlib.sha256(f"{tag}/{ctr}".encode()).digest()
        ctr += 1
    return bytes(out[:n])


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


FIPS197_C1 = {
    "key": bytes(range(16)).hex(),
    "pt": "00112233445566778899aabbccddeeff",
    "ct": "69c4e0d86a7b0430d8cdb78070b4c55a",
}


def dcf_case(name, keys, lam, n_bytes, alpha, beta, s0s, bound, xs, full=True, mmo=False):
    """Run gen + eval of both parties on both restatements; return a fixture dict."""
    OP, RP = (O.OracleMmoPrg, R.MmoPrg) if mmo else (O.OraclePrg, R.HirosePrg)
    P = OP(keys, lam)
    k = O.gen(P, alpha, beta, s0s[0], s0s[1], bound)
    xa = np.frombuffer(b"".join(xs), np.uint8).reshape(len(xs), n_bytes)
    y0 = O.eval_(P, 0, k, s0s[0], xa, nthreads=4)
    y1 = O.eval_(P, 1, k, s0s[1], xa, nthreads=4)
    # portable AES path must agree with AES-NI
    Pp = OP(keys, lam, allow_aesni=False)
    assert (O.eval_(Pp, 0, k, s0s[0], xa[:4]) == y0[:4]).all()
    # independent restatement (small cases in full, large ones on a prefix)
    Q = RP(keys, lam)
    if lam * n_bytes <= 256:
        cws, np1 = R.gen(Q, alpha, beta, s0s, bound)
        assert np1 == k.cw_np1.tobytes()
        for i, (s, v, tl, tr) in enumerate(cws):
            assert s == k.cw_s[i].tobytes() and v == k.cw_v[i].tobytes()
            assert int(tl) | (int(tr) << 1) == int(k.cw_t[i])
        ry0 = R.eval_(Q, False, s0s[0], cws, np1, [bytes(x) for x in xs[:8]])
        assert ry0 == [y.tobytes() for y in y0[:8]]
    # reconstruction property (lib.rs:372-420)
    a = int.from_bytes(alpha, "big")
    for x, u, w in zip(xs, y0, y1):
        xv = int.from_bytes(x, "big")
        hit = (xv < a) if bound == 0 else (xv > a)
        assert (u ^ w).tobytes() == (beta if hit else bytes(lam)), name
    cwb = (k.cw_s.tobytes() + k.cw_v.tobytes() + k.cw_t.tobytes())
    cwb += bytes((-len(cwb)) % 16) + k.cw_np1.tobytes()
    d = {
        "name": name, "lambda": lam, "n_bytes": n_bytes, "bound": bound,
        "cipher_n": len(keys), "alpha": alpha.hex(), "beta": beta.hex(),
        "s0s": [s.hex() for s in s0s], "m": len(xs),
        "cwb_sha256": sha(cwb), "y0_sha256": sha(y0.tobytes()), "y1_sha256": sha(y1.tobytes()),
    }
    if full:
        d.update({
            "keys": [kk.hex() for kk in keys], "cwb": cwb.hex(), "xs": [x.hex() for x in xs],
            "y0": [y.tobytes().hex() for y in y0], "y1": [y.tobytes().hex() for y in y1],
        })
    else:
        d["y0_head"] = [y.tobytes()[:64].hex() for y in y0[:4]]
    return d


def mmo_vectors():
    """Aes128MatyasMeyerOseasPrg fixtures.  PARITY UNPINNED: the reference has no MMO
    PRG (its definition is ours, include/dcf_hip.h); these vectors pin our GPU path
    to two agreeing CPU restatements and AES-128 to FIPS-197 C.1."""
    kat = [FIPS197_C1]
    for i in range(8):
        key, pt = detbytes(f"aes128/key/{i}", 16), detbytes(f"aes128/pt/{i}", 16)
        ct = R.Aes256Ecb(key).encrypt(pt)  # 16-byte key -> EVP aes-128-ecb
        assert O.aes128_encrypt(key, pt) == ct
        kat.append({"key": key.hex(), "pt": pt.hex(), "ct": ct.hex()})
    assert O.aes128_encrypt(bytes(range(16)), bytes.fromhex(FIPS197_C1["pt"])).hex() == FIPS197_C1["ct"]
    keys = [detbytes(f"mmo16/key/{i}", 16) for i in range(4)]
    P, Q = O.OracleMmoPrg(keys, 16), R.MmoPrg(keys, 16)
    rows = []
    for i in range(32):
        sd = detbytes(f"mmo16/seed/{i}", 16)
        g = P.gen(sd)
        assert g == Q.gen(sd)
        (sl, vl, tl), (sr, vr, tr) = g
        rows.append({"seed": sd.hex(), "sl": sl.hex(), "vl": vl.hex(), "tl": tl, "sr": sr.hex(), "vr": vr.hex(),
                     "tr": tr})
    cases = []
    for nb, bound in ((16, 0), (16, 1), (4, 0), (3, 1)):
        alpha = detbytes(f"mmo/n{nb}/alpha", nb)
        xs = [alpha] + [detbytes(f"mmo/n{nb}/x/{i}", nb) for i in range(47)]
        cases.append(dcf_case(f"mmo_n{nb}_{'lt' if bound == 0 else 'gt'}", keys, 16, nb, alpha,
                              detbytes(f"mmo/n{nb}/beta", 16),
                              [detbytes(f"mmo/n{nb}/s0/0", 16), detbytes(f"mmo/n{nb}/s0/1", 16)], bound, xs,
                              mmo=True))
    return {"parity": "unpinned: no MMO PRG in the reference; C oracle == Python/libcrypto restatement",
            "aes128_kat": kat, "keys": [k.hex() for k in keys], "prg_rows": rows, "cases": cases}


def main():
    if sys.argv[1:] == ["--mmo"]:
        with open(os.path.join(HERE, "mmo16.json"), "w") as f:
            json.dump(mmo_vectors(), f, indent=1)
            f.write("\n")
        print("wrote mmo16")
        return
    out = {"mmo16": mmo_vectors()}
    # AES-256 known answers: FIPS-197 C.3 + libcrypto on derived keys/blocks
    kat = [FIPS197_C3]
    for i in range(8):
        key, pt = detbytes(f"aes/key/{i}", 32), detbytes(f"aes/pt/{i}", 16)
        ct = R.Aes256Ecb(key).encrypt(pt)
        assert O.aes256_encrypt(key, pt) == ct
        kat.append({"key": key.hex(), "pt": pt.hex(), "ct": ct.hex()})
    assert O.aes256_encrypt(bytes(range(32)), bytes.fromhex(FIPS197_C3["pt"])).hex() == FIPS197_C3["ct"]
    out["aes256_kat"] = kat

    # PRG vectors, LAMBDA = 16 (reference KEYS and SEED, prg.rs:80-84) + derived seeds
    P, Q = O.OraclePrg(REF_KEYS, 16), R.HirosePrg(REF_KEYS, 16)
    seeds = [REF_PRG_SEED] + [detbytes(f"prg16/seed/{i}", 16) for i in range(31)]
    rows = []
    for s in seeds:
        g = P.gen(s)
        assert g == Q.gen(s)
        (sl, vl, tl), (sr, vr, tr) = g
        rows.append({"seed": s.hex(), "sl": sl.hex(), "vl": vl.hex(), "tl": tl, "sr": sr.hex(), "vr": vr.hex(),
                     "tr": tr})
    out["prg16"] = {"keys": [k.hex() for k in REF_KEYS], "rows": rows}

    # PRG vectors, LAMBDA = 32 with 18 derived keys (ciphers 0 and 17 are read)
    keys32 = [detbytes(f"prg32/key/{i}", 32) for i in range(18)]
    P, Q = O.OraclePrg(keys32, 32), R.HirosePrg(keys32, 32)
    rows = []
    for i in range(8):
        s = detbytes(f"prg32/seed/{i}", 32)
        g = P.gen(s)
        assert g == Q.gen(s)
        (sl, vl, tl), (sr, vr, tr) = g
        rows.append({"seed": s.hex(), "sl": sl.hex(), "vl": vl.hex(), "tl": tl, "sr": sr.hex(), "vr": vr.hex(),
                     "tr": tr})
    out["prg32"] = {"keys": [k.hex() for k in keys32], "rows": rows}

    cases = []
    # Reference test shape: N = LAMBDA = 16, KEYS, alpha = ALPHAS[2], BETA (lib.rs:372-420);
    # fixed seeds replace thread_rng().  Points: the 5 ALPHAS + 59 derived points.
    s0s = [detbytes("ref16/s0/0", 16), detbytes("ref16/s0/1", 16)]
    xs = REF_ALPHAS + [detbytes(f"ref16/x/{i}", 16) for i in range(59)]
    for bound in (0, 1):
        cases.append(dcf_case(f"ref16_{'lt' if bound == 0 else 'gt'}", REF_KEYS, 16, 16, REF_ALPHAS[2], REF_BETA,
                              s0s, bound, xs))
    # N = 4 (the 32-bit-input config), points around alpha and random
    alpha = detbytes("n4/alpha", 4)
    a = int.from_bytes(alpha, "big")
    xs = [((a + d) % (1 << 32)).to_bytes(4, "big") for d in (-2, -1, 0, 1, 2)]
    xs += [detbytes(f"n4/x/{i}", 4) for i in range(59)] + [bytes(4), b"\xff" * 4]
    cases.append(dcf_case("n4_lt", REF_KEYS, 16, 4, alpha, detbytes("n4/beta", 16),
                          [detbytes("n4/s0/0", 16), detbytes("n4/s0/1", 16)], 0, xs))
    # odd N (byte path of the x loader): N = 3 and N = 5
    for nb in (1, 3, 5):
        alpha = detbytes(f"n{nb}/alpha", nb)
        xs = [alpha] + [detbytes(f"n{nb}/x/{i}", nb) for i in range(40)]
        cases.append(dcf_case(f"n{nb}_gt", REF_KEYS, 16, nb, alpha, detbytes(f"n{nb}/beta", 16),
                              [detbytes(f"n{nb}/s0/0", 16), detbytes(f"n{nb}/s0/1", 16)], 1, xs))
    # LAMBDA = 32, 18 keys, N = 2
    cases.append(dcf_case("l32_n2_lt", keys32, 32, 2, detbytes("l32/alpha", 2), detbytes("l32/beta", 32),
                          [detbytes("l32/s0/0", 32), detbytes("l32/s0/1", 32)], 0,
                          [detbytes(f"l32/x/{i}", 2) for i in range(24)]))
    # LAMBDA = 16384 (benches/dcf_large_lambda.rs:8-35 shape) at N = 2: hashes only
    keysL = [detbytes(f"l16384/keys/{i}", 32) for i in range(2048)]
    cases.append(dcf_case("l16384_n2_lt", keysL, 16384, 2, detbytes("l16384/alpha", 2),
                          detbytes("l16384/beta", 16384),
                          [detbytes("l16384/s0/0", 16384), detbytes("l16384/s0/1", 16384)], 0,
                          [detbytes(f"l16384/x/{i}", 2) for i in range(16)], full=False))
    cases[-1].update({"keys_fmt": "l16384/keys/{i}", "xs_fmt": "l16384/x/{i}", "alpha_tag": "l16384/alpha",
                      "beta_tag": "l16384/beta", "s0_tags": ["l16384/s0/0", "l16384/s0/1"]})
    out["dcf_cases"] = cases

    for name, obj in out.items():
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(obj, f, indent=1)
            f.write("\n")
    print("wrote", ", ".join(out))


if __name__ == "__main__":
    main()
