"""bench.py's per-config defaults (CPU): configs[3] streams a whole 125 Mbp contig per chunk in
the serial pass (one ~64 GB key buffer) and 2^25 positions with --overlap (two buffers),
configs[4] 2^23 positions at 96 samples; an explicit --chunk is kept."""
import sys

import pytest


def _parse(argv, monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    return bench.parse()


@pytest.mark.parametrize("argv,chunk,samples", [
    ([], 1 << 25, 12),
    (["--config", "3"], 1 << 27, 24),
    (["--config", "3", "--overlap"], 1 << 25, 24),
    (["--config", "3", "--chunk", str(1 << 26)], 1 << 26, 24),
    (["--config", "3", "--chunk", str(1 << 25)], 1 << 25, 24),   # explicit 2^25 kept (was the argparse default)
    (["--config", "4", "--chunk", str(1 << 25)], 1 << 25, 96),
    (["--config", "4"], 1 << 23, 96),
])
def test_config_defaults(monkeypatch, argv, chunk, samples):
    a = _parse(argv, monkeypatch)
    assert a.chunk == chunk and a.samples == samples
    assert a.chunk % 64 == 0   # whole 64-position blocks (genome.GenomePass)
    if a.config == 3 and len(argv) == 2:
        assert a.chunk >= a.contig_len   # the default serial pass: one chunk per contig


def test_traffic_split_bounds_the_hbm_share():
    """A counted traffic above what HBM can deliver in the launch's time is labelled as at least
    that excess served by the Infinity Cache (configs[3]'s 104.7 GB in 15.385 ms
    is 6.81 TB/s counted, above the 6.29 TB/s achievable)."""
    import bench
    s = bench.traffic_split(104_700_000_000, 15.385)
    assert s["counted_GBps"] > bench.HBM_ACHIEVABLE_GBS
    assert s["hbm_bytes_at_most"] == int(6290e9 * 15.385e-3)
    assert s["hbm_bytes_at_most"] + s["infinity_cache_bytes_at_least"] == 104_700_000_000
    s = bench.traffic_split(20_370_000_000, 3.4142)   # configs[2]: within what HBM can deliver
    assert s["infinity_cache_bytes_at_least"] == 0
    assert bench.traffic_split(None, 3.0) is None


@pytest.mark.parametrize("v", [0, 1, 2, 3, 16, 17, 18, 33, 181, 400])
def test_zns_chain_floor_counts_the_kernels_padded_adds(v):
    """window_stats.zns_chain: the longest chain's dependent adds as window_zns_kernel issues them
    (each row of pairs (a, a+1..V-1) padded to a multiple of 16: zns_rounds in stats_kernel.hip),
    against a direct count over the rows."""
    import torch

    import bench
    z = bench.zns_chain_floor(torch.tensor([3, v, 1], dtype=torch.int32))
    assert z["longest_chain_sites"] == max(v, 3)
    vv = max(v, 3)
    rows = [vv - 1 - a for a in range(vv - 1)]              # row a holds pairs (a, a+1 .. V-1)
    assert z["pairs"] == sum(rows)
    assert z["adds_padded"] == sum(-(-r // 16) * 16 for r in rows)
    assert z["floor_ms_at_7_cycles_2p4GHz"] == round(z["adds_padded"] * 7 / 2.4e9 * 1e3, 4)
