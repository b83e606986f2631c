"""bench.py's roofline arithmetic (no GPU): block counts and peaks the JSON line reports."""
import importlib.util
import os

import pytest

from tests.conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_reference_block_counts(bench):
    # prg.rs:48-53 once per level (lib.rs:176): 2 AES-256 blocks at LAMBDA = 16, 4 at LAMBDA >= 32
    assert bench.blocks_per_eval(16, 16) == 256
    assert bench.blocks_per_eval(4, 16) == 64
    assert bench.blocks_per_eval(16, 16384) == 512


def test_peaks(bench):
    # T-table: 256 CUs x 32 ds_read_b32 lookups/clk x 2.4 GHz / 224 lookups per block
    assert bench.PEAK_TT_BLOCKS == pytest.approx(256 * 32 * 2.4e9 / 224)
    assert bench.engine_peak("stream") == bench.PEAK_TT_BLOCKS
    assert bench.engine_peak("mmo") == pytest.approx(256 * 2.4e9 / (160 / 32 + 11 / 16))
    assert bench.engine_peak("ttable") == bench.engine_peak("ttable-small") == bench.PEAK_TT_BLOCKS


def test_wide_roofline_bound(bench):
    m, lam = 1 << 22, 16384
    r = bench.wide_roofline(m, 16, lam, kern_s=0.05, exec_bpe=320, bpe=512, kernel="k", engine="stream-head")
    t_min = m * 320 / bench.PEAK_TT_BLOCKS + m * lam / bench.HBM_WRITE_BPS
    assert r["peak"] == pytest.approx(m / t_min / 1e6)
    assert r["frac"] == pytest.approx(t_min / 0.05)
    assert r["unit"] == "M evals/s" and r["bound"] == "lds+hbm"


def test_zero_bits_below_prefix(bench):
    # the stream engine's A blocks: 0 bits of x below a shared prefix of `skip` levels
    import numpy as np
    import torch
    rng = np.random.default_rng(3)
    x = rng.integers(0, 256, (777, 5), dtype=np.uint8)
    for skip in (0, 1, 7, 8, 9, 15, 24, 33, 39):
        want = int((np.unpackbits(x, axis=1)[:, skip:] == 0).sum())
        assert bench.zero_bits(torch.from_numpy(x), skip) == want, skip
