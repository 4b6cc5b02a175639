"""The N=1 headline workload pinned to the oracle (bench.py's `mix`: 60x,
log-uniform 5-500 kb gaps, seed 1000): a subset of its own windows -- the
widest gaps (>= 470 kb, 1,100-1,400 reads) beside ordinary ones -- run with no
environment overrides, so the paths the bench takes on its own run
unforced: K12's dense site path (call positions spanning more than the
2^19-position bitmap), the greedy loop's candidate slot-list cache (the wide
windows' slot lists do not fit the main kernel's LDS budget), and the u8
count pairs of the slot table (every site covered by < 256 reads at 60x).  Every
window's decision, 2x2 tables, join, which_way, score, site and read counts
and every read's tag must equal the oracle's bit for bit; Fisher p within
rtol 1e-6 (the reference's f64 kt_fisher_exact, blockjoin.c:3926).
Reference: haplotag_region_given_bam, blockjoin.c:4217-4335."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# the bench's N=1 workload (bench.py WORKLOADS["mix"]) and its seed
SPEC = dict(n_windows=1024, coverage=60, gap=50_000, seed=1000, gap_mix=True, skip_frac=0.10, nosite_frac=0.05)
WIDE = [218, 422, 691, 830, 580, 52, 884]     # gaps 477-499 kb (830 is a T7-skipped window)
ORDINARY = list(range(10))


@pytest.fixture(scope="module")
def headline_subset():
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    return make_aln_batch(AlnSpec(**SPEC), windows=sorted(WIDE + ORDINARY), workers=16)


def _clean_env(monkeypatch):
    for k in list(os.environ):
        if k.startswith("PF_"):
            monkeypatch.delenv(k)


def _compare(out, ref, wsel=None):
    wsel = np.arange(ref.decision.shape[0]) if wsel is None else np.asarray(wsel)
    for f in ("decision", "dir_table", "dir_join", "dir_which_way", "dir_score", "win_n_sites", "win_n_reads"):
        assert np.array_equal(getattr(out, f), getattr(ref, f)[wsel]), f
    np.testing.assert_allclose(out.dir_fisher_p, ref.dir_fisher_p[wsel], rtol=1e-6, atol=0)


def test_headline_subset_natural_paths(oracle_lib, gpu_ctx, headline_subset, monkeypatch):
    from pomfret_amd import Config, LoadConfig
    _clean_env(monkeypatch)
    aln = headline_subset
    cfg, lcfg = Config.from_coverage(60, given=False), LoadConfig()
    gaps = aln.win_end.astype(np.int64) - aln.win_start.astype(np.int64)
    wide = np.flatnonzero(gaps >= 400_000)
    assert wide.size == len(WIDE)
    db = gpu_ctx.upload_aln(cfg, aln, lcfg)
    out = db.run()
    ref = oracle_lib.methphase_aln(cfg, lcfg, aln, n_threads=16)
    _compare(out, ref)
    # read tags: the oracle's loader then its worker (methphase_aln leaves them unset)
    wb = oracle_lib.load_reads(lcfg, aln)[0]
    ref_t = oracle_lib.methphase(cfg, wb, n_threads=16)
    _compare(out, ref_t)
    assert np.array_equal(out.read_hp, ref_t.read_hp)
    # every problem ran in the main greedy kernel (no heavy split), and the
    # wide windows' slot lists (2 B per methmer) exceed its budget: they ran on
    # the candidate slot-list cache (k3_greedy_slim CACHE).  Round 5: the
    # budget is the four-per-CU one (a quarter of the CU's 160 KB less the
    # kernel's 3,760 B of static LDS) and every problem fits it: paths 1 and 2
    # only below, nothing deferred to the fallback kernel
    assert len(db.heavy_problems()) == 0
    bud = db.k3_budget()
    assert bud["lds"] == 37200 and bud["resident"] >= 4 * 200 and bud["resident"] % 4 == 0, bud
    st = db.stats()
    assert all(int(st[w, d, 4]) * 2 > 37200 for w in wide for d in (0, 1) if out.win_n_sites[w] > 0)
    paths = db.k3_paths()
    assert all(paths[w, d] == 2 for w in wide for d in (0, 1) if out.win_n_sites[w] > 0), paths[wide]
    assert set(paths[out.win_n_sites > 0].ravel().tolist()) <= {1, 2}
    # the wide windows' call positions span beyond one 2^19-position segment
    # of K12's bitmaps: since round 5 they take the fast path over two
    # segments, one after the other (pf_batch_k12_paths 2), and no window of
    # the mix goes to the dense path (3)
    k12 = db.k12_paths()
    off, pos, _, _, _ = db.debug_calls()
    ro = np.searchsorted(db.read_recs(), aln.win_rec_off.astype(np.int64))
    for w in wide:
        c0, c1 = int(off[ro[w]]), int(off[ro[w + 1]])
        if c1 > c0 and out.win_n_sites[w] > 0:
            assert int(pos[c0:c1].max()) - int(pos[c0:c1].min()) >= 1 << 19, w
            assert k12[w] == 2, (w, int(k12[w]))
    assert set(k12[out.win_n_sites > 0].tolist()) <= {1, 2}, np.unique(k12, return_counts=True)
    # at 60x no position is covered by 256 reads (so by 256 reads' methmer
    # spans): every problem's slot table holds u8 count pairs (k3_run's bound)
    wro = wb.win_read_off.astype(np.int64)
    for w in range(aln.n_windows):
        s, e = wb.read_start[wro[w]:wro[w + 1]].astype(np.int64), wb.read_end[wro[w]:wro[w + 1]].astype(np.int64)
        ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        assert np.cumsum(ev[:, 1]).max(initial=0) < 256, w
    decided = ref.decision >= 0
    assert decided[wide].sum() >= 4 and decided.sum() >= 10
    db.free()


def test_headline_subset_two_contexts(oracle_lib, gpu_ctx, headline_subset, monkeypatch):
    """The bench's headline shape: the windows dealt heaviest first over two
    contexts, launched together, pipelined two deep -- equal to the oracle."""
    from pomfret_amd import Config, Context, LoadConfig
    from pomfret_amd.shard import aln_window_costs, split_groups
    _clean_env(monkeypatch)
    aln = headline_subset
    cfg, lcfg = Config.from_coverage(60, given=False), LoadConfig()
    wb = oracle_lib.load_reads(lcfg, aln)[0]
    ref = oracle_lib.methphase(cfg, wb, n_threads=16)
    ro = wb.win_read_off.astype(np.int64)          # T7-skipped windows keep their reads
    idx = np.arange(aln.n_windows)
    parts = [bw for _, bw in split_groups([(idx, idx)], 2, aln_window_costs(aln))]
    ctx2 = Context(0)
    try:
        dbs = [c.upload_aln(cfg, aln.select(p), lcfg) for c, p in zip((gpu_ctx, ctx2), parts)]
        outs = [[d.run(), d.run()] for d in dbs]
        steps = 4
        for d in dbs:
            d.launch()
        for k in range(steps):
            if k + 1 < steps:
                for d in dbs:
                    d.launch()
            for d, o in zip(dbs, outs):
                d.finish(o[k % 2])
        for p, o in zip(parts, outs):
            got = o[(steps - 1) % 2]
            _compare(got, ref, p)
            assert np.array_equal(got.read_hp, np.concatenate([ref.read_hp[ro[w]:ro[w + 1]] for w in p]))
        for d in dbs:
            d.free()
    finally:
        ctx2.close()
