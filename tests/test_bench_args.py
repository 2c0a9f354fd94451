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
