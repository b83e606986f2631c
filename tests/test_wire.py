"""Key wire formats: bincode 1.x and serde_json forms of
`Share` (lib.rs:217-340).  Host-only code, no GPU.  The expected bincode bytes
are built here independently from the bincode 1.x spec (fixint LE, u64
lengths); no Rust toolchain exists to produce reference bytes ("parity
unpinned" beyond the spec)."""
import struct

import numpy as np
import pytest

import dcf_amd
from dcf_amd import wire
from oracle import oracle as O
from tests.golden.make_golden import REF_ALPHAS, REF_BETA, REF_KEYS


def _oracle_share(nb=16, lam=16, keys=REF_KEYS):
    P = O.OraclePrg(keys, lam)
    rng = np.random.default_rng(3)
    s0s = [rng.bytes(lam), rng.bytes(lam)]
    alpha = REF_ALPHAS[2][:nb] if lam == 16 else rng.bytes(nb)
    k = O.gen(P, alpha, REF_BETA if lam == 16 else rng.bytes(lam), s0s[0], s0s[1], 0)
    cws = [dcf_amd.Cw(k.cw_s[i].tobytes(), k.cw_v[i].tobytes(), bool(k.cw_t[i] & 1), bool(k.cw_t[i] & 2))
           for i in range(8 * nb)]
    return dcf_amd.Share(s0s, cws, k.cw_np1.tobytes())


def _spec_bincode(k, lam):
    out = struct.pack("<Q", len(k.s0s))
    for s in k.s0s:
        out += struct.pack("<Q", lam) + s
    out += struct.pack("<Q", len(k.cws))
    for c in k.cws:
        out += struct.pack("<Q", lam) + c.s + struct.pack("<Q", lam) + c.v + bytes([c.tl, c.tr])
    return out + struct.pack("<Q", lam) + k.cw_np1


@pytest.mark.parametrize("nb,lam", [(16, 16), (2, 16), (1, 32)])
def test_bincode_matches_spec_and_roundtrips(hip_lib, nb, lam):
    keys = REF_KEYS if lam == 16 else [bytes([i]) * 32 for i in range(18)]
    k = _oracle_share(nb, lam, keys)
    b = wire.share_to_bincode(k, nb, lam)
    assert b == _spec_bincode(k, lam)
    assert len(b) == hip_lib.dcf_share_bincode_bytes(nb, lam, 2)
    assert wire.share_from_bincode(b, nb, lam) == k
    k1 = dcf_amd.Share([k.s0s[1]], k.cws, k.cw_np1)  # eval-side share (lib.rs:385)
    assert wire.share_from_bincode(wire.share_to_bincode(k1, nb, lam), nb, lam) == k1


def test_bincode_rejects_malformed(hip_lib):
    k = _oracle_share()
    b = bytearray(wire.share_to_bincode(k, 16, 16))
    with pytest.raises(dcf_amd.DcfError):
        wire.share_from_bincode(bytes(b[:-1]), 16, 16)  # truncated
    with pytest.raises(dcf_amd.DcfError):
        wire.share_from_bincode(bytes(b) + b"\x00", 16, 16)  # trailing
    bad = bytearray(b)
    bad[8] = 15  # first seed declared 15 bytes: copy_from_slice would panic (lib.rs:319-321)
    with pytest.raises(dcf_amd.DcfError):
        wire.share_from_bincode(bytes(bad), 16, 16)
    bad = bytearray(b)
    off = 8 + 2 * (8 + 16) + 8 + (8 + 16) * 2
    assert bad[off] in (0, 1)
    bad[off] = 2  # bool byte must be 0/1
    with pytest.raises(dcf_amd.DcfError):
        wire.share_from_bincode(bytes(bad), 16, 16)
    with pytest.raises(dcf_amd.DcfError):
        wire.share_from_bincode(bytes(b), 15, 16)  # cws.len() != 8N


def test_json_forms(hip_lib):
    k = _oracle_share()
    j = wire.share_to_json(k)
    assert j.startswith('{"s0s":[[') and '"tl":' in j
    assert wire.share_from_json(j, 16, 16) == k
    seq = '[%s,%s,%s]' % (str([list(s) for s in k.s0s]).replace(" ", ""),
                          str([[list(c.s), list(c.v), c.tl, c.tr] for c in k.cws]).replace(" ", "")
                          .replace("True", "true").replace("False", "false"),
                          str(list(k.cw_np1)).replace(" ", ""))
    assert wire.share_from_json(seq, 16, 16) == k


@pytest.mark.parametrize("nb,lam", [(16, 16), (1, 32)])
def test_bincode_decode_mutation_fuzz(hip_lib, nb, lam):
    """dcf_share_from_bincode on corrupted input (seeded mutations of a valid key: byte flips,
    truncations, appended bytes and arbitrary u64 length fields): every call either fails with a
    DcfError or returns a Share whose encoding is exactly the input (the decoder accepts only
    canonical bincode).  Run under a host sanitizer by scripts/host_sanitize.sh."""
    keys = REF_KEYS if lam == 16 else [bytes([i]) * 32 for i in range(18)]
    good = wire.share_to_bincode(_oracle_share(nb, lam, keys), nb, lam)
    rng = np.random.default_rng(11 + lam)
    # offsets of the u64 length fields: vec len, 2 seeds, cws len, 2 per cw, cw_np1
    lens = [0, 8, 16 + lam, 24 + 2 * lam]
    o = 32 + 2 * lam
    for _ in range(8 * nb):
        lens += [o, o + 8 + lam]
        o += 2 * (8 + lam) + 2
    lens.append(o)
    assert o + 8 + lam == len(good)
    accepted = 0
    for i in range(1500):
        b = bytearray(good)
        kind = i % 4
        if kind == 0:  # flip 1-3 bytes anywhere
            for p in rng.integers(0, len(b), rng.integers(1, 4)):
                b[p] ^= int(rng.integers(1, 256))
        elif kind == 1:  # truncate
            b = b[:int(rng.integers(0, len(b)))]
        elif kind == 2:  # extend
            b += rng.bytes(int(rng.integers(1, 64)))
        else:  # a length field set to a small, boundary or huge value
            p = lens[int(rng.integers(0, len(lens)))]
            vals = [0, 1, lam - 1, lam + 1, 8 * nb + 1, 2**31, 2**63, 2**64 - 1]
            v = vals[int(rng.integers(0, len(vals)))]
            b[p:p + 8] = struct.pack("<Q", v)
        try:
            k = wire.share_from_bincode(bytes(b), nb, lam)
        except dcf_amd.DcfError:
            continue
        accepted += 1
        assert wire.share_to_bincode(k, nb, lam) == bytes(b)
    assert accepted < 1500 // 4  # most corruptions are rejected; byte flips inside payloads are not
