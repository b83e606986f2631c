"""Host-side mirror of the `dcf` crate's operator and plugin interface.

Same names, argument meaning and error behaviour as the Rust crate
(xymeng16/dcf v0.2.2), with the compute on MI355X through the C ABI:

  Rust (reference)                                   here
  -------------------------------------------------  ------------------------------
  trait Dcf<N, LAMBDA> { gen, eval }  lib.rs:24-35   DcfImpl.gen / DcfImpl.eval
  struct CmpFn { alpha, beta }        lib.rs:41-46   CmpFn
  trait Prg / Aes256HirosePrg::new    lib.rs:52, prg.rs:27  Aes256HirosePrg(keys, lam)
  Aes128MatyasMeyerOseasPrg (north_star; not in the crate)  Aes128MatyasMeyerOseasPrg(keys, lam)
  DcfImpl::new(prg)                   lib.rs:74      DcfImpl(n_bytes, lam, prg)
  struct Cw { s, v, tl, tr }          lib.rs:209     Cw
  struct Share { s0s, cws, cw_np1 }   lib.rs:275     Share
  enum BoundState { LtBeta, GtBeta }  lib.rs:342     BoundState

Const generics `N` / `LAMBDA` become constructor arguments.  Panics of the
reference (`assert_eq!(k.cws.len(), N * 8)`, lib.rs:165; the cipher index at
prg.rs:51) surface as `DcfError`/`ValueError`; the silent zip truncation of
lib.rs:196 becomes an error.

Batch entry points (`eval_device`, `eval_multikey_device`, `gen_batch_device`)
take torch uint8 tensors resident on the prg's device and run on the current
stream.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np

from . import _lib
from ._lib import DcfError, check


class BoundState(enum.IntEnum):
    """lib.rs:342-349."""
    LtBeta = 0  # f(x) = beta iff x < alpha
    GtBeta = 1  # f(x) = beta iff x > alpha


@dataclass
class CmpFn:
    """lib.rs:41-46: alpha (N bytes), beta (LAMBDA bytes)."""
    alpha: bytes
    beta: bytes


@dataclass
class Cw:
    """lib.rs:209-214."""
    s: bytes
    v: bytes
    tl: bool
    tr: bool


@dataclass
class Share:
    """lib.rs:275-283.  gen returns both seeds; eval reads s0s[0] (lib.rs:168)."""
    s0s: List[bytes]
    cws: List[Cw] = field(default_factory=list)
    cw_np1: bytes = b""


def cwb_bytes(n_bytes: int, lam: int, num_keys: int = 1) -> int:
    return int(_lib.load().dcf_cwb_bytes(n_bytes, lam, num_keys))


def cwb_np1_offset(n_bytes: int, lam: int, num_keys: int = 1) -> int:
    return int(_lib.load().dcf_cwb_np1_offset(n_bytes, lam, num_keys))


def share_to_cwb(k: Share, n_bytes: int, lam: int) -> bytes:
    """Pack `Share.cws` / `cw_np1` into the single-key CWB layout (include/dcf_hip.h)."""
    n = 8 * n_bytes
    if len(k.cws) != n:  # lib.rs:165
        raise DcfError(-8, f"k.cws.len() = {len(k.cws)} != N * 8 = {n}")
    buf = bytearray(cwb_bytes(n_bytes, lam, 1))
    for i, cw in enumerate(k.cws):
        if len(cw.s) != lam or len(cw.v) != lam:
            raise DcfError(-8, "correction word of the wrong length")
        buf[i * lam:(i + 1) * lam] = cw.s
        buf[n * lam + i * lam:n * lam + (i + 1) * lam] = cw.v
        buf[2 * n * lam + i] = int(bool(cw.tl)) | (int(bool(cw.tr)) << 1)
    off = cwb_np1_offset(n_bytes, lam, 1)
    buf[off:off + lam] = k.cw_np1
    return bytes(buf)


def cwb_to_share(cwb: bytes, n_bytes: int, lam: int, s0s: Sequence[bytes]) -> Share:
    n = 8 * n_bytes
    cws = []
    for i in range(n):
        t = cwb[2 * n * lam + i]
        cws.append(Cw(bytes(cwb[i * lam:(i + 1) * lam]), bytes(cwb[n * lam + i * lam:n * lam + (i + 1) * lam]),
                      bool(t & 1), bool(t & 2)))
    off = cwb_np1_offset(n_bytes, lam, 1)
    return Share([bytes(s) for s in s0s], cws, bytes(cwb[off:off + lam]))


def _ptr(b) -> ctypes.c_void_p:
    if isinstance(b, np.ndarray):
        assert b.flags["C_CONTIGUOUS"]
        return ctypes.c_void_p(b.ctypes.data)
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)


def _tptr(t) -> ctypes.c_void_p:
    """Device pointer of a contiguous torch uint8 tensor."""
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _dev(t, name: str, device: int, shape=None, numel=None):
    """Validate a device buffer before its pointer crosses the C ABI, which takes no
    lengths for device buffers: a wrong dtype, device, row width or size would make a
    kernel read or write out of bounds.  Returns the pointer."""
    import torch
    if not isinstance(t, torch.Tensor):
        raise DcfError(-1, f"{name} must be a torch tensor")
    if t.dtype != torch.uint8:
        raise DcfError(-1, f"{name} must be uint8, got {t.dtype}")
    if t.device.type != "cuda" or t.device.index != device:
        raise DcfError(-1, f"{name} must be on cuda:{device}, got {t.device}")
    if not t.is_contiguous():
        raise DcfError(-1, f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise DcfError(-5, f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    if numel is not None and t.numel() != numel:
        raise DcfError(-5, f"{name} has {t.numel()} bytes, expected {numel}")
    return ctypes.c_void_p(t.data_ptr())


def _stream(device_index: int):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device_index).cuda_stream)


class Aes256HirosePrg:
    """`Aes256HirosePrg::<LAMBDA, CIPHER_N>::new(keys)` (prg.rs:27-33), resident on one GPU.

    keys: CIPHER_N 32-byte AES-256 keys.  LAMBDA = 16 reads cipher 0 only;
    LAMBDA >= 32 reads ciphers 0 and 17 (the diagonal zip, prg.rs:48-51), so it
    needs CIPHER_N >= 18 (the reference panics otherwise).
    """

    def __init__(self, keys: Sequence[bytes], lam: int = 16, device: int = 0):
        keys = [bytes(k) for k in keys]
        if any(len(k) != 32 for k in keys):
            raise ValueError("AES-256 keys are 32 bytes")
        L = _lib.load()
        blob = b"".join(keys)
        h = ctypes.c_void_p()
        check(L.dcf_hirose_prg_new(_ptr(blob), len(keys), lam, device, ctypes.byref(h)))
        self._h = h
        self.lam = lam
        self.cipher_n = len(keys)
        self.device = device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.dcf_prg_free(h)
            self._h = None

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def set_eval_mode(self, mode: int) -> None:
        """AES engine for LAMBDA = 16 eval: 0 auto, 1 lockstep LDS T-table, 4 stream (LDS T-table,
        per-lane block scheduling).  Identical bytes for every mode (dcf_prg_set_eval_mode)."""
        check(_lib.load().dcf_prg_set_eval_mode(self._h, int(mode)))

    def set_prefix_levels(self, levels: int) -> None:
        """Shared-prefix depth for single-key LAMBDA = 16 eval (Hirose: stream engine; MMO):
        -1 automatic (default), 0 off, > 0 that depth.  Output bytes are identical."""
        check(_lib.load().dcf_prg_set_prefix_levels(self._h, int(levels)))

    def set_prefix_max_bytes(self, max_bytes: int) -> None:
        """Cap the device memory of the automatic shared-prefix table (0 = no cap)."""
        check(_lib.load().dcf_prg_set_prefix_max_bytes(self._h, int(max_bytes)))

    def device_bytes(self) -> int:
        """Device memory this prg currently holds (tables, prefix table, scratch, staging)."""
        return int(_lib.load().dcf_prg_device_bytes(self._h))

    def eval_prefix_levels(self, n_bytes: int, num_keys: int, points_per_key: int) -> int:
        """The prefix depth an eval of this shape uses (0 = none)."""
        r = _lib.load().dcf_eval_prefix_levels(self._h, int(n_bytes), int(num_keys), int(points_per_key))
        if r < 0:
            check(r)
        return r

    def last_eval_blocks(self) -> int:
        """AES blocks the last stream-engine eval encrypted for live points, counted on the
        device (no prefix table build).  Call after synchronizing the eval's stream."""
        n = ctypes.c_uint64(0)
        check(_lib.load().dcf_prg_last_eval_blocks(self._h, ctypes.byref(n)))
        return int(n.value)

    def host_pinned_bytes(self) -> int:
        """Pinned host memory this prg holds for the host-pointer entry points."""
        return int(_lib.load().dcf_prg_host_pinned_bytes(self._h))

    def workspaces(self) -> int:
        """Workspaces in the prg's pool (the most calls that were in flight at once)."""
        return int(_lib.load().dcf_prg_workspaces(self._h))

    def trim(self) -> int:
        """Free the workspaces no call holds (device scratch, prefix tables, pinned staging);
        returns how many were freed."""
        n = int(_lib.load().dcf_prg_trim(self._h))
        if n < 0:
            check(n)
        return n

    def set_phase_timing(self, on: bool) -> None:
        """Record HIP events around every eval's preparation and walk (measurement hook)."""
        check(_lib.load().dcf_prg_set_phase_timing(self._h, int(bool(on))))

    def last_eval_phases(self):
        """(prep_ms, walk_ms, prefix_levels) of the last timed eval; sync its stream first."""
        a, b, d = ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
        check(_lib.load().dcf_prg_last_eval_phases(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(d)))
        return float(a.value), float(b.value), int(d.value)

    def gen(self, seed: bytes):
        """`Prg::gen` (lib.rs:52-54) for one seed — the GPU PRG kernel, not a CPU path."""
        return self.gen_many([seed])[0]

    def gen_many(self, seeds: Sequence[bytes]):
        lam = self.lam
        m = len(seeds)
        blob = b"".join(bytes(s) for s in seeds)
        if len(blob) != m * lam:
            raise ValueError("seed of the wrong length")
        out = np.zeros((m, 4 * lam + 2), np.uint8)
        check(_lib.load().dcf_prg_gen(self._h, _ptr(blob), m, _ptr(out)))
        res = []
        for r in out:
            b = r.tobytes()
            res.append([(b[0:lam], b[lam:2 * lam], bool(b[4 * lam])),
                        (b[2 * lam:3 * lam], b[3 * lam:4 * lam], bool(b[4 * lam + 1]))])
        return res


class Aes128MatyasMeyerOseasPrg(Aes256HirosePrg):
    """`Aes128MatyasMeyerOseasPrg::<LAMBDA, CIPHER_N>::new(keys)`, the PRG BASELINE.json's
    north_star names, resident on one GPU.  The reference crate has no such PRG, so its
    definition is ours (include/dcf_hip.h, dcf_mmo_prg_new; parity unpinned):
    out_b = AES128_{keys[b]}(seed) ^ seed for b = s_L, v_L, s_R, v_R; t from bit 0 of
    byte 0 of s_L / s_R; bit 0 of the last byte cleared (prg.rs:63-68's convention).

    keys: CIPHER_N >= 4 16-byte AES-128 keys; LAMBDA = 16.
    """

    def __init__(self, keys: Sequence[bytes], lam: int = 16, device: int = 0):
        keys = [bytes(k) for k in keys]
        if any(len(k) != 16 for k in keys):
            raise ValueError("AES-128 keys are 16 bytes")
        L = _lib.load()
        blob = b"".join(keys)
        h = ctypes.c_void_p()
        check(L.dcf_mmo_prg_new(_ptr(blob), len(keys), lam, device, ctypes.byref(h)))
        self._h = h
        self.lam = lam
        self.cipher_n = len(keys)
        self.device = device


class DcfImpl:
    """`DcfImpl<N, LAMBDA, P>` (lib.rs:63-205) on MI355X, P = Aes256HirosePrg or
    Aes128MatyasMeyerOseasPrg."""

    def __init__(self, n_bytes: int, lam: int, prg: Aes256HirosePrg):
        if prg.lam != lam:
            raise ValueError("prg LAMBDA mismatch")
        if n_bytes <= 0:
            raise ValueError("N must be positive")
        self.n_bytes = n_bytes
        self.lam = lam
        self.prg = prg

    # ---- Dcf trait (lib.rs:24-35), host buffers ----
    def gen(self, f: CmpFn, s0s: Sequence[bytes], bound: BoundState) -> Share:
        """`Dcf::gen` (lib.rs:86-161)."""
        lam, nb = self.lam, self.n_bytes
        if len(f.alpha) != nb or len(f.beta) != lam or len(s0s) != 2 or any(len(s) != lam for s in s0s):
            raise ValueError("argument lengths do not match N / LAMBDA")
        out = np.zeros(cwb_bytes(nb, lam, 1), np.uint8)
        check(_lib.load().dcf_gen(self.prg.handle, nb, _ptr(bytes(f.alpha)), _ptr(bytes(f.beta)),
                                  _ptr(bytes(s0s[0])), _ptr(bytes(s0s[1])), int(bound), _ptr(out)))
        return cwb_to_share(out.tobytes(), nb, lam, [bytes(s0s[0]), bytes(s0s[1])])

    def eval(self, b: bool, k: Share, xs, ys=None):
        """`Dcf::eval` (lib.rs:163-204).  xs: sequence of N-byte strings or an (m, N)
        uint8 array; ys (optional, (m, LAMBDA) uint8 array) is overwritten in place.
        Returns ys."""
        lam, nb = self.lam, self.n_bytes
        cwb = share_to_cwb(k, nb, lam)
        xa = self._as_points(xs)
        m = xa.shape[0]
        if ys is None:
            ys = np.zeros((m, lam), np.uint8)
        if not (isinstance(ys, np.ndarray) and ys.dtype == np.uint8 and ys.flags["C_CONTIGUOUS"]):
            raise TypeError("ys must be a contiguous uint8 numpy array")
        if ys.size != m * lam:
            raise DcfError(-5, f"xs.len() = {m} does not match ys")
        check(_lib.load().dcf_eval(self.prg.handle, nb, int(bool(b)), _ptr(cwb), len(cwb), _ptr(bytes(k.s0s[0])),
                                   _ptr(xa), m, _ptr(ys), ys.size))
        return ys

    def _as_points(self, xs) -> np.ndarray:
        nb = self.n_bytes
        if isinstance(xs, np.ndarray):
            xa = np.ascontiguousarray(xs, dtype=np.uint8).reshape(-1, nb) if xs.size else np.zeros((0, nb), np.uint8)
        else:
            blob = b"".join(bytes(x) for x in xs)
            if len(blob) != len(xs) * nb:
                raise ValueError("point of the wrong length")
            xa = np.frombuffer(blob, np.uint8).reshape(-1, nb).copy() if xs else np.zeros((0, nb), np.uint8)
        return xa

    # ---- batch / device entry points (torch uint8 tensors on self.prg.device) ----
    def gen_batch_device(self, alpha, beta, s0_0, s0_1, bound: BoundState, cwb_out=None):
        """K independent `Dcf::gen` calls in one launch.  alpha: (K, N), beta/s0_0/s0_1: (K, LAMBDA).
        Returns the K-key CWB tensor (include/dcf_hip.h layout)."""
        import torch
        lam, nb, dev = self.lam, self.n_bytes, self.prg.device
        K = alpha.shape[0] if alpha.dim() == 2 else -1
        pa = _dev(alpha, "alpha", dev, shape=(K, nb))
        pb = _dev(beta, "beta", dev, shape=(K, lam))
        p0 = _dev(s0_0, "s0_0", dev, shape=(K, lam))
        p1 = _dev(s0_1, "s0_1", dev, shape=(K, lam))
        if cwb_out is None:
            cwb_out = torch.empty(cwb_bytes(nb, lam, K), dtype=torch.uint8, device=alpha.device)
        po = _dev(cwb_out, "cwb_out", dev, numel=cwb_bytes(nb, lam, K))
        check(_lib.load().dcf_gen_batch_device(self.prg.handle, nb, K, pa, pb, p0, p1, int(bound), po,
                                               _stream(dev)))
        return cwb_out

    def eval_device(self, b: bool, cwb, s0, xs, ys=None):
        """One key over m points: xs (m, N) -> ys (m, LAMBDA), device tensors."""
        import torch
        lam, nb, dev = self.lam, self.n_bytes, self.prg.device
        m = xs.shape[0] if xs.dim() == 2 else -1
        px = _dev(xs, "xs", dev, shape=(m, nb))
        pk = _dev(cwb, "cwb", dev, numel=cwb_bytes(nb, lam, 1))
        ps = _dev(s0, "s0", dev, numel=lam)
        if ys is None:
            ys = torch.empty((m, lam), dtype=torch.uint8, device=xs.device)
        py = _dev(ys, "ys", dev, numel=m * lam)
        check(_lib.load().dcf_eval_device(self.prg.handle, nb, int(bool(b)), pk, ps, px, m, py, _stream(dev)))
        return ys

    def eval_multikey_device(self, b: bool, cwb, s0s, xs, points_per_key: int, ys=None):
        """K keys x P points: xs (K*P, N), s0s (K, LAMBDA) -> ys (K*P, LAMBDA)."""
        import torch
        lam, nb, dev = self.lam, self.n_bytes, self.prg.device
        K = s0s.shape[0] if s0s.dim() == 2 else -1
        ps = _dev(s0s, "s0s", dev, shape=(K, lam))
        px = _dev(xs, "xs", dev, shape=(K * points_per_key, nb))
        pk = _dev(cwb, "cwb", dev, numel=cwb_bytes(nb, lam, K))
        if ys is None:
            ys = torch.empty((xs.shape[0], lam), dtype=torch.uint8, device=xs.device)
        py = _dev(ys, "ys", dev, numel=K * points_per_key * lam)
        check(_lib.load().dcf_eval_multikey_device(self.prg.handle, nb, K, points_per_key, int(bool(b)),
                                                   pk, ps, px, py, _stream(dev)))
        return ys

    def eval_full_domain_device(self, b: bool, cwb, s0, ys=None):
        """`Dcf::eval` at every x in [0, 2^(8N)) (increasing, big-endian x): (2^(8N), LAMBDA) device tensor."""
        import torch
        lam, nb, dev = self.lam, self.n_bytes, self.prg.device
        npts = 1 << (8 * nb)
        pk = _dev(cwb, "cwb", dev, numel=cwb_bytes(nb, lam, 1))
        ps = _dev(s0, "s0", dev, numel=lam)
        if ys is None:
            ys = torch.empty((npts, lam), dtype=torch.uint8, device=cwb.device)
        py = _dev(ys, "ys", dev, numel=npts * lam)
        check(_lib.load().dcf_eval_full_domain_device(self.prg.handle, nb, int(bool(b)), pk, ps, py, _stream(dev)))
        return ys


def point_slice(total: int, G: int, g: int):
    """dcf_point_slice: contiguous slice (start, count) of `total` points for slice g of G."""
    st, ct = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.load().dcf_point_slice(int(total), int(G), int(g), ctypes.byref(st), ctypes.byref(ct))
    return int(st.value), int(ct.value)


class MultiGpuDcf:
    """`Dcf::eval` of one key over G GPUs in one call (dcf_eval_multi_gpu[_device]): one
    `DcfImpl` per device, all over PRGs built from the same keys; points are split into G
    contiguous slices (point_slice).  The reference spreads eval over host cores inside one
    call (lib.rs:194-199); this spreads it over devices, with no collective."""

    def __init__(self, impls: Sequence[DcfImpl]):
        if not impls:
            raise ValueError("need at least one DcfImpl")
        self.impls = list(impls)
        self.n_bytes, self.lam = impls[0].n_bytes, impls[0].lam
        if any(d.n_bytes != self.n_bytes or d.lam != self.lam for d in impls):
            raise ValueError("DcfImpls disagree on N / LAMBDA")
        self._prgs = (ctypes.c_void_p * len(impls))(*[d.prg.handle.value for d in impls])

    def eval(self, b: bool, k: Share, xs, ys=None):
        """Host buffers: like DcfImpl.eval, slices evaluated concurrently on every device."""
        lam, nb = self.lam, self.n_bytes
        cwb = share_to_cwb(k, nb, lam)
        xa = self.impls[0]._as_points(xs)
        m = xa.shape[0]
        if ys is None:
            ys = np.zeros((m, lam), np.uint8)
        if not (isinstance(ys, np.ndarray) and ys.dtype == np.uint8 and ys.flags["C_CONTIGUOUS"]):
            raise TypeError("ys must be a contiguous uint8 numpy array")
        if ys.size != m * lam:
            raise DcfError(-5, f"xs.len() = {m} does not match ys")
        check(_lib.load().dcf_eval_multi_gpu(self._prgs, len(self.impls), nb, int(bool(b)), _ptr(cwb), len(cwb),
                                             _ptr(bytes(k.s0s[0])), _ptr(xa), m, _ptr(ys), ys.size))
        return ys

    def eval_device(self, b: bool, cwb: bytes, s0: bytes, xs_slices, ys_slices=None, gather=None):
        """Device slices: xs_slices[g] (m_g, N) on impls[g]'s device -> ys_slices[g];
        cwb / s0 are host bytes (copied to every device once).  gather: None, or a tensor
        on impls[0]'s device of (sum m_g, LAMBDA) that receives every slice in order.
        Queued on each device's current stream; synchronizes them before returning."""
        import torch
        lam, nb, G = self.lam, self.n_bytes, len(self.impls)
        if len(xs_slices) != G:
            raise DcfError(-5, "one xs slice per device")
        if ys_slices is None:
            ys_slices = [torch.empty((x.shape[0], lam), dtype=torch.uint8, device=x.device) for x in xs_slices]
        ms = (ctypes.c_size_t * G)()
        xp, yp, sp = (ctypes.c_void_p * G)(), (ctypes.c_void_p * G)(), (ctypes.c_void_p * G)()
        for g, (d, x, y) in enumerate(zip(self.impls, xs_slices, ys_slices)):
            m = x.shape[0] if x.dim() == 2 else -1
            xp[g] = _dev(x, f"xs[{g}]", d.prg.device, shape=(m, nb)).value
            yp[g] = _dev(y, f"ys[{g}]", d.prg.device, numel=m * lam).value
            ms[g] = m
            sp[g] = _stream(d.prg.device).value
        gp = None
        if gather is not None:
            gp = _dev(gather, "gather", self.impls[0].prg.device, numel=sum(ms) * lam)
        cwb = bytes(cwb)
        if len(cwb) != cwb_bytes(nb, lam, 1):
            raise DcfError(-8, "key size does not match 8*N levels (lib.rs:165)")
        check(_lib.load().dcf_eval_multi_gpu_device(self._prgs, G, nb, int(bool(b)), _ptr(cwb), len(cwb),
                                                    _ptr(bytes(s0)), xp, ms, yp, sp, gp))
        for d in self.impls:
            torch.cuda.current_stream(d.prg.device).synchronize()
        return ys_slices
