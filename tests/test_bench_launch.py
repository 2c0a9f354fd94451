"""bench.py's multi-GPU entry on CPU: `--gpus N` without a launcher starts N rank processes
itself (subprocess, before any HIP call), they meet in gloo, and rank 0's line says n_gpus N;
under a launcher WORLD_SIZE must equal --gpus; a non-product library is refused unless
--allow-variant."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(argv, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=REPO)


def _line(p):
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (p.stdout, p.stderr[-2000:])
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus,config", [(2, 2), (2, 3), (4, 3), (3, 4)])
def test_gpus_n_launches_n_ranks(gpus, config):
    p = _run(["--gpus", str(gpus), "--dry-run", "--config", str(config)])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p)
    assert d["n_gpus"] == gpus and d["dry_run"] and d["value"] is None
    assert sorted(r["rank"] for r in d["ranks"]) == list(range(gpus))
    assert d["windows_covered"]
    if config == 2:
        assert all(r["sites"] == 50_000_000 for r in d["ranks"])   # weak scaling: a contig per rank
    if config == 3:
        assert sum(r["sites"] for r in d["ranks"]) == 24 * 125_000_000   # strong scaling: the genome split


def test_single_process_dry_run():
    d = _line(_run(["--dry-run"]))
    assert d["n_gpus"] == 1 and len(d["ranks"]) == 1


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0 and "must agree" in p.stderr


def test_failing_rank_fails_the_launch():
    # rank 1 dies before the barrier: the launcher returns its status and terminates rank 0, which
    # would otherwise wait in the barrier for ever
    p = _run(["--gpus", "2", "--dry-run"], {"BENCH_DRY_FAIL_RANK": "1"}, timeout=120)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_variant_build_refused(monkeypatch):
    import bench
    from popbam_amd import _lib

    class Fake:
        @staticmethod
        def pbg_build_info():
            return b"experiment"

    monkeypatch.setattr(_lib, "load", lambda *a, **k: Fake)
    with pytest.raises(SystemExit) as e:
        bench.build_info(False)
    assert "experiment" in str(e.value)
    assert bench.build_info(True)["kind"] == "experiment"


@pytest.mark.gpu
def test_gpus_2_on_one_gpu():
    """Both ranks of `--gpus 2` on the box's one GPU (LOCAL_RANK mod device count): a real weak-scaled
    configs[2]-shaped run at a small --sites, timed over both ranks, parity-sampled on rank 0."""
    p = _run(["--gpus", "2", "--sites", "2000000", "--steps", "3", "--warmup", "1", "--cpu-sample", "0",
              "--parity-windows", "4"], timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["build"]["kind"] == "product"
    assert d["parity_sampled"] and d["rows_crosscheck"]["identical"]
