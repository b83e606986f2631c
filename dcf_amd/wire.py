"""Key wire formats of the reference's `Share` / `Cw` (lib.rs:217-340).

* bincode 1.x (`bincode::serialize`, the crate's declared serialiser,
  Cargo.toml:44): handled by the C ABI (`dcf_share_to_bincode` /
  `dcf_share_from_bincode`, layout in include/dcf_hip.h) — host-only code.
* serde_json: `Share` serialises as {"s0s": [[..], ..], "cws": [{"s": [..],
  "v": [..], "tl": b, "tr": b}, ..], "cw_np1": [..]} (arrays as Vec<u8>,
  lib.rs:223-226, 291-294).  The reference can only *deserialise* sequences
  (visit_seq, lib.rs:245, 313), so it cannot read its own JSON objects back;
  `share_from_json` here accepts both the object and the sequence forms.
"""
from __future__ import annotations

import ctypes
import json
from typing import Union

import numpy as np

from . import _lib
from ._lib import DcfError, check
from .dcf import Cw, Share, cwb_bytes, cwb_to_share, share_to_cwb


def share_to_bincode(k: Share, n_bytes: int, lam: int) -> bytes:
    L = _lib.load()
    cwb = share_to_cwb(k, n_bytes, lam)
    seeds = b"".join(bytes(s) for s in k.s0s)
    if len(seeds) != len(k.s0s) * lam:
        raise DcfError(-8, "seed of the wrong length")
    n = int(L.dcf_share_bincode_bytes(n_bytes, lam, len(k.s0s)))
    out = ctypes.create_string_buffer(n)
    check(L.dcf_share_to_bincode(n_bytes, lam, cwb, seeds if seeds else None, len(k.s0s), out, n))
    return out.raw


def share_from_bincode(data: bytes, n_bytes: int, lam: int, max_s0s: int = 16) -> Share:
    L = _lib.load()
    cwb = ctypes.create_string_buffer(cwb_bytes(n_bytes, lam, 1))
    seeds = ctypes.create_string_buffer(max_s0s * lam)
    ns = ctypes.c_size_t(0)
    check(L.dcf_share_from_bincode(n_bytes, lam, bytes(data), len(data), cwb, seeds, max_s0s, ctypes.byref(ns)))
    s0s = [seeds.raw[i * lam:(i + 1) * lam] for i in range(ns.value)]
    return cwb_to_share(cwb.raw, n_bytes, lam, s0s)


def share_to_json(k: Share) -> str:
    """serde_json form of `Share` (struct -> object, [u8; L] -> Vec<u8> -> array)."""
    return json.dumps({
        "s0s": [list(bytes(s)) for s in k.s0s],
        "cws": [{"s": list(bytes(c.s)), "v": list(bytes(c.v)), "tl": bool(c.tl), "tr": bool(c.tr)} for c in k.cws],
        "cw_np1": list(bytes(k.cw_np1)),
    }, separators=(",", ":"))


def _u8(a, lam: int) -> bytes:
    b = bytes(np.asarray(a, dtype=np.int64).astype(np.uint8)) if not isinstance(a, (bytes, bytearray)) else bytes(a)
    if len(b) != lam or any(int(x) > 255 or int(x) < 0 for x in a):
        raise DcfError(-8, "array of the wrong length or non-byte element")
    return b


def share_from_json(text: Union[str, bytes], n_bytes: int, lam: int) -> Share:
    obj = json.loads(text)
    if isinstance(obj, list):  # sequence form (what visit_seq accepts)
        obj = {"s0s": obj[0], "cws": obj[1], "cw_np1": obj[2]}
    cws = []
    for c in obj["cws"]:
        if isinstance(c, list):
            c = {"s": c[0], "v": c[1], "tl": c[2], "tr": c[3]}
        if not isinstance(c["tl"], bool) or not isinstance(c["tr"], bool):
            raise DcfError(-8, "Cw.tl / Cw.tr must be booleans")
        cws.append(Cw(_u8(c["s"], lam), _u8(c["v"], lam), c["tl"], c["tr"]))
    if len(cws) != 8 * n_bytes:
        raise DcfError(-8, "cws.len() != N * 8 (lib.rs:165)")
    return Share([_u8(s, lam) for s in obj["s0s"]], cws, _u8(obj["cw_np1"], lam))
