"""Statistics of the benchmark's synthetic pileup (CPU, the oracle's restatement of the
generator, pbg_common.h synth_*): the r05 data model (template pages shared by a 16,384-position
span, per-task error draws) must keep the workload the r04 model gave -- per-read error rate
1/128 (tasks showing a non-reference key ~8.4 % at 12 samples, depth ~10) and segregating
sites per 10 kb window spread like independent sites (r04: sd ~15 around ~180 at 12 samples),
not clustered by span (template-entry errors shared by a page gave sd ~120)."""
import numpy as np

import harness


def _batch_stats(n, lo, hi, seed=0xC0FFEE01):
    from popbam_amd import workload
    params = workload.default_params(n, 2)
    p = harness.oracle_params_from(params)
    b = harness.synth_batch(seed, lo, hi, n, 10, params.max_depth, 0)
    dep = b["depth"].astype(np.int64).reshape(-1)
    base = (b["reads"] >> np.uint32(16)) & np.uint32(0xF)
    refcode = np.array([1, 2, 4, 8], np.uint32)[np.searchsorted(np.array([65, 67, 71, 84]), b["ref"])]
    refper = np.repeat(np.repeat(refcode, n), dep)
    off = np.concatenate([[0], np.cumsum(dep)])
    mism = np.add.reduceat((base != refper).astype(np.int64), off[:-1])
    mism[dep == 0] = 0
    _, _, _, flags = harness.oracle_call(p, b)
    return mism, (flags & 4) > 0


def test_error_rate_and_segregating_sites_match_the_r04_model():
    mism, seg = [], []
    for lo in range(0, 200_000, 50_000):
        m, s = _batch_stats(12, lo, lo + 50_000)
        mism.append(m)
        seg.append(s)
    mism, seg = np.concatenate(mism), np.concatenate(seg)
    frac = float((mism > 0).mean())
    assert 0.078 < frac < 0.088, frac            # r04 model: 0.0837; r05: 0.0824
    w = seg.reshape(-1, 10_000).sum(axis=1)
    assert 150 < w.mean() < 210, w.mean()         # r04: 181, r05: 178
    assert w.std() < 2.0 * np.sqrt(w.mean()), (w.mean(), w.std())   # independent sites: ~sqrt(mean)
