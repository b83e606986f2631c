"""CPU emulation of the latency kernels' lane algorithm (dcf_amd/csrc/kernels_lat.h) against
the oracle: the per-lane column AES (DPP quad_perm rotations bring columns j+1..j+3), the
16-lane-row AES of k_eval16_row (one lookup per lane, quad / stride-4 XOR reductions), the
octet's A/B exchange (row_ror 4 / 12) and the gen row's block exchange (row_ror 4 / 8 / 12),
with DPP semantics dst[i] = src[(i - n) mod 16] (row_ror:n) and dst[j] = src[sel[j]] within a
quad (quad_perm).  This pins the lane decomposition on CPU; the GPU tests
(tests/test_lat_threads.py) pin the kernels themselves."""
import numpy as np

from oracle import oracle as O


def _tables():
    exp, log = [0] * 256, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x ^= (x << 1) ^ (0x1B if x & 0x80 else 0)
        x &= 0xFF
    sbox = []
    for v in range(256):
        inv = exp[(255 - log[v]) % 255] if v else 0
        s = inv
        for k in range(1, 5):
            s ^= ((inv << k) | (inv >> (8 - k))) & 0xFF
        sbox.append(s ^ 0x63)

    def xt(a):
        return ((a << 1) ^ (0x1B if a & 0x80 else 0)) & 0xFF
    T0 = [xt(s) | (s << 8) | (s << 16) | ((xt(s) ^ s) << 24) for s in sbox]
    rot = lambda w, k: ((w << (8 * k)) | (w >> (32 - 8 * k))) & 0xFFFFFFFF if k else w  # noqa: E731
    return sbox, [[rot(t, k) for t in T0] for k in range(4)]


SBOX, T = _tables()


def _expand256(key: bytes):
    b = list(key)
    rcon = 1
    for i in range(8, 60):
        t = b[4 * i - 4:4 * i]
        if i % 8 == 0:
            t = [SBOX[t[1]] ^ rcon, SBOX[t[2]], SBOX[t[3]], SBOX[t[0]]]
            rcon = ((rcon << 1) ^ (0x1B if rcon & 0x80 else 0)) & 0xFF
        elif i % 8 == 4:
            t = [SBOX[c] for c in t]
        b += [b[4 * (i - 8) + k] ^ t[k] for k in range(4)]
    return [int.from_bytes(bytes(b[4 * i:4 * i + 4]), "little") for i in range(60)]


def _byte(w, k):
    return (w >> (8 * k)) & 0xFF


def _quad(vals, sel):
    """quad_perm on a list of lanes: dst[i] = src[quad_base + sel[i & 3]]."""
    return [vals[(i & ~3) + sel[i & 3]] for i in range(len(vals))]


def _ror(vals, n):
    """row_ror:n on a list of lanes (rows of 16)."""
    return [vals[(i & ~15) + (((i & 15) - n) % 16)] for i in range(len(vals))]


ROT1, ROT2, ROT3, BC0 = (1, 2, 3, 0), (2, 3, 0, 1), (3, 0, 1, 2), (0, 0, 0, 0)


LATE_DPP = True  # kernels_lat.h aes256_col: rotate the lookup results instead of the inputs


def aes_cols(st, rk):
    """aes256_col for every lane of `st` (lane i holds column i & 3 of its quad's block)."""
    kw = lambda r, i: rk[4 * r + (i & 3)]  # noqa: E731
    st = [s ^ kw(0, i) for i, s in enumerate(st)]
    for r in range(1, 14):
        if LATE_DPP:  # each lane looks up its own word's four bytes; the results rotate
            a = [T[0][_byte(w, 0)] for w in st]
            c, d, e = ([T[k][_byte(w, k)] for w in st] for k in (1, 2, 3))
            c1, d2, e3 = _quad(c, ROT1), _quad(d, ROT2), _quad(e, ROT3)
            st = [a[i] ^ kw(r, i) ^ c1[i] ^ d2[i] ^ e3[i] for i in range(len(st))]
            continue
        w1, w2, w3 = _quad(st, ROT1), _quad(st, ROT2), _quad(st, ROT3)
        st = [T[0][_byte(st[i], 0)] ^ T[1][_byte(w1[i], 1)] ^ T[2][_byte(w2[i], 2)] ^ T[3][_byte(w3[i], 3)] ^ kw(r, i)
              for i in range(len(st))]
    w1, w2, w3 = _quad(st, ROT1), _quad(st, ROT2), _quad(st, ROT3)
    return [(SBOX[_byte(st[i], 0)] | SBOX[_byte(w1[i], 1)] << 8 | SBOX[_byte(w2[i], 2)] << 16 |
             SBOX[_byte(w3[i], 3)] << 24) ^ kw(14, i) for i in range(len(st))]


M32 = 0xFFFFFFFF
MASK_LAST = 0xFEFFFFFF


def oct_eval(rk, cws, cwv, cwt, np1, s0, party, xs):
    """k_eval16_oct for a list of points (8 lanes each)."""
    nb = len(xs[0])
    n = 8 * nb
    L = 8 * len(xs)
    j = [i & 3 for i in range(L)]
    b = [(i >> 2) & 1 for i in range(L)]
    s = [int.from_bytes(s0[4 * j[i]:4 * j[i] + 4], "little") for i in range(L)]
    v, t = [0] * L, [party] * L
    xbits = [int.from_bytes(bytes(x), "big") for x in xs]
    for lev in range(n):
        mine = aes_cols([s[i] ^ (M32 if b[i] else 0) for i in range(L)], rk)
        r4, r12 = _ror(mine, 4), _ror(mine, 12)
        tn0 = []
        A, B = [], []
        for i in range(L):
            other = r4[i] if b[i] else r12[i]
            A.append(other if b[i] else mine[i])
            B.append(mine[i] if b[i] else other)
        for i in range(L):
            xb = (xbits[i >> 3] >> (n - 1 - lev)) & 1
            tl, tr = (A[i] ^ s[i]) & 1, (B[i] ^ ~s[i]) & 1
            tn0.append((tr if xb else tl) ^ (t[i] & (cwt[lev] >> xb) & 1))
        tn = _quad(tn0, BC0)
        for i in range(L):
            xb = (xbits[i >> 3] >> (n - 1 - lev)) & 1
            keep_a = (xb - 1) & M32
            tm = (-t[i]) & M32
            msk = MASK_LAST if j[i] == 3 else M32
            cs = int.from_bytes(cws[lev][4 * j[i]:4 * j[i] + 4], "little")
            cv = int.from_bytes(cwv[lev][4 * j[i]:4 * j[i] + 4], "little")
            v[i] ^= ((~s[i] ^ (B[i] & keep_a)) & msk) ^ (tm & cv)
            v[i] &= M32
            s[i] = (((s[i] ^ (A[i] & keep_a)) & msk) ^ (tm & cs)) & M32
            t[i] = tn[i]
    ys = []
    for p in range(len(xs)):
        words = [v[8 * p + jj] ^ s[8 * p + jj] ^ ((-t[8 * p + jj]) & M32 & int.from_bytes(np1[4 * jj:4 * jj + 4], "little"))
                 for jj in range(4)]
        ys.append(b"".join(w.to_bytes(4, "little") for w in words))
    return ys


def col_gen(rk, alpha, beta, s0_0, s0_1, bound):
    """k_gen16_col for one key (one row of 16 lanes)."""
    nb = len(alpha)
    n = 8 * nb
    q = [(i >> 2) & 3 for i in range(16)]
    j = [i & 3 for i in range(16)]
    w = lambda bb, i: int.from_bytes(bb[4 * j[i]:4 * j[i] + 4], "little")  # noqa: E731
    s0w, s1w, be = [w(s0_0, i) for i in range(16)], [w(s0_1, i) for i in range(16)], [w(beta, i) for i in range(16)]
    va, t0, t1 = [0] * 16, [0] * 16, [1] * 16
    abits = int.from_bytes(alpha, "big")
    cws, cwv, cwt = [], [], []
    for lev in range(n):
        mine = aes_cols([(s1w[i] if q[i] >> 1 else s0w[i]) ^ (M32 if q[i] & 1 else 0) for i in range(16)], rk)
        r4, r8, r12 = _ror(mine, 4), _ror(mine, 8), _ror(mine, 12)
        a = (abits >> (n - 1 - lev)) & 1
        scw_l, vcw_l, tp0 = [0] * 16, [0] * 16, [0] * 16
        new0, new1 = [0] * 16, [0] * 16
        for i in range(16):
            X = []
            for tb in range(4):
                d = (q[i] - tb) & 3
                X.append([mine, r4, r8, r12][d][i])
            A0, B0, A1, B1 = X
            msk = MASK_LAST if j[i] == 3 else M32
            am = (-a) & M32
            bm = am if bound == 0 else (~am & M32)
            n0, n1 = (~s0w[i]) & M32, (~s1w[i]) & M32
            sl0, vl0, sr0, vr0 = (A0 ^ s0w[i]) & msk, (B0 ^ n0) & msk, s0w[i] & msk, n0 & msk
            sl1, vl1, sr1, vr1 = (A1 ^ s1w[i]) & msk, (B1 ^ n1) & msk, s1w[i] & msk, n1 & msk
            scw = (sl0 if a else sr0) ^ (sl1 if a else sr1)
            vcw = (vl0 if a else vr0) ^ (vl1 if a else vr1) ^ va[i] ^ (bm & be[i])
            va[i] ^= (vr0 if a else vl0) ^ (vr1 if a else vl1) ^ vcw
            tl0, tr0, tl1, tr1 = (A0 ^ s0w[i]) & 1, (B0 ^ n0) & 1, (A1 ^ s1w[i]) & 1, (B1 ^ n1) & 1
            tlcw, trcw = tl0 ^ tl1 ^ a ^ 1, tr0 ^ tr1 ^ a
            tkcw = trcw if a else tlcw
            nt0, nt1 = (tr0 if a else tl0) ^ (t0[i] & tkcw), (tr1 if a else tl1) ^ (t1[i] & tkcw)
            tp0[i] = tlcw | (trcw << 1) | (nt0 << 2) | (nt1 << 3)
            m0, m1 = (-t0[i]) & M32, (-t1[i]) & M32
            new0[i] = (sr0 if a else sl0) ^ (m0 & scw)
            new1[i] = (sr1 if a else sl1) ^ (m1 & scw)
            scw_l[i], vcw_l[i] = scw, vcw
        tp = _quad(tp0, BC0)
        s0w, s1w = new0, new1
        t0 = [(x >> 2) & 1 for x in tp]
        t1 = [(x >> 3) & 1 for x in tp]
        cws.append(b"".join(scw_l[jj].to_bytes(4, "little") for jj in range(4)))   # quad 0 stores
        cwv.append(b"".join(vcw_l[4 + jj].to_bytes(4, "little") for jj in range(4)))  # quad 1 stores
        cwt.append(tp[8] & 3)                                                      # quad 2, lane 0
    np1 = b"".join((s0w[jj] ^ s1w[jj] ^ va[jj]).to_bytes(4, "little") for jj in range(4))
    return cws, cwv, cwt, np1


def test_column_aes_matches_fips197():
    # FIPS-197 C.3: AES-256, both round forms of aes256_col
    global LATE_DPP
    key = bytes(range(32))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    rk = _expand256(key)
    st = [int.from_bytes(pt[4 * (i & 3):4 * (i & 3) + 4], "little") for i in range(4)]
    for late in (True, False):
        LATE_DPP = late
        out = b"".join(w.to_bytes(4, "little") for w in aes_cols(st, rk))
        assert out.hex() == "8ea2b7ca516745bfeafc49904b496089"
    LATE_DPP = True


def test_oct_and_col_lane_algorithm_vs_oracle():
    rng = np.random.default_rng(3)
    for nb in (1, 2):
        keys = [rng.bytes(32) for _ in range(2)]
        P = O.OraclePrg(keys, 16)
        rk = _expand256(keys[0])
        for bound in (0, 1):
            alpha, beta, s0, s1 = rng.bytes(nb), rng.bytes(16), rng.bytes(16), rng.bytes(16)
            ok = O.gen(P, alpha, beta, s0, s1, bound)
            cws, cwv, cwt, np1 = col_gen(rk, alpha, beta, s0, s1, bound)
            assert [bytes(r) for r in ok.cw_s] == cws
            assert [bytes(r) for r in ok.cw_v] == cwv
            assert [int(c) for c in ok.cw_t] == cwt
            assert bytes(ok.cw_np1) == np1
            xs = [rng.bytes(nb) for _ in range(3)] + [alpha]
            for party, sp in ((0, s0), (1, s1)):
                want = O.eval_(P, party, ok, sp, np.frombuffer(b"".join(xs), np.uint8).reshape(-1, nb))
                got = oct_eval(rk, [bytes(r) for r in ok.cw_s], [bytes(r) for r in ok.cw_v], [int(c) for c in ok.cw_t],
                               bytes(ok.cw_np1), sp, party, xs)
                assert [bytes(r) for r in want] == got


def aes_col16(st, rk):
    """aes256_col16 for one 16-lane row: lane p holds column p&3 of the block (layout A) on entry
    and exit; DPP row_ror:n is dst[i] = src[(i - n) mod 16]."""
    p = list(range(16))
    a, b = [i & 3 for i in p], [i >> 2 for i in p]
    kA, kB = [(a[i] - b[i]) & 3 for i in p], [(b[i] - a[i]) & 3 for i in p]
    st = [st[i] ^ rk[a[i]] for i in p]
    for r in range(1, 14):
        if r & 1:  # from layout A: lane p looks up T_k[byte k] of its column for output column p>>2
            x = [T[kA[i]][_byte(st[i], kA[i])] for i in p]
            x = [x[i] ^ x[i ^ 1] for i in p]          # quad_perm [1,0,3,2]
            x = [x[i] ^ x[i ^ 2] for i in p]          # quad_perm [2,3,0,1]
            st = [x[i] ^ rk[4 * r + b[i]] for i in p]
        else:      # from layout B: stride-4 reduction over the row
            x = [T[kB[i]][_byte(st[i], kB[i])] for i in p]
            x = [x[i] ^ x[(i - 4) % 16] for i in p]   # row_ror:4
            x = [x[i] ^ x[(i - 8) % 16] for i in p]   # row_ror:8
            st = [x[i] ^ rk[4 * r + a[i]] for i in p]
    x = [T[(kB[i] + 2) & 3][_byte(st[i], kB[i])] & (0xFF << (8 * kB[i])) for i in p]
    x = [x[i] ^ x[(i - 4) % 16] for i in p]
    x = [x[i] ^ x[(i - 8) % 16] for i in p]
    return [x[i] ^ rk[56 + a[i]] for i in p]


def test_col16_aes_matches_fips197():
    key = bytes(range(32))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    rk = _expand256(key)
    out = aes_col16([int.from_bytes(pt[4 * (i & 3):4 * (i & 3) + 4], "little") for i in range(16)], rk)
    for q in range(4):  # every quad holds the whole block
        assert b"".join(w.to_bytes(4, "little") for w in out[4 * q:4 * q + 4]).hex() == "8ea2b7ca516745bfeafc49904b496089"
